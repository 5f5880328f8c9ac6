"""CPU code under AddressSanitizer + UndefinedBehaviorSanitizer ("race detection /
sanitizers"; host code only — GPU sanitizers are not available on this pool).

Four builds, each compiled here with -fsanitize=address,undefined -fno-sanitize-recover=all and
run on inputs that reach the code's edges:
  * the C restatement (oracle/sm_oracle.c, sm_oracle_agg.c; test infrastructure) through every
    pipeline it implements, tests/cpp/sanitize_oracle.c;
  * the host NL tree (csrc/sm_nl_tree.cpp) against the oracle's, tests/cpp/nl_tree_check.cpp;
  * the C++ facade's PNG / PNM reader (include/stereo_matching.hpp: smamd::imread), which parses
    untrusted files — valid images of every colour type, crafted IHDR sizes, truncated files,
    corrupt and short IDAT streams, bad CRCs, random bytes.  The reference's answer to an
    unreadable image is an error message and exit (main_.cpp:108-112, h:1741-1742); here imread
    returns an empty Mat;
  * the C-ABI's host side (csrc/sm_capi.cpp, host code sanitized with hipcc -Xarch_host) without a
    GPU: parameter validation, null / out-of-range arguments, calErr, tests/cpp/capi_host_check.cpp.
"""
import os
import shutil
import struct
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
CSRC = os.path.join(ROOT, "mystereomatching_amd", "csrc")
INC = os.path.join(ROOT, "include")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
HIPCC = "/opt/rocm/bin/hipcc"


def _run(cmd, **kw):
    r = subprocess.run(cmd, capture_output=True, text=True, **kw)
    assert r.returncode == 0, " ".join(cmd)[:300] + "\n" + r.stderr[-4000:]
    return r


def _clean(r):
    out = r.stdout + r.stderr
    assert "runtime error" not in out and "AddressSanitizer" not in out and "LeakSanitizer" not in out, out[-4000:]


def test_oracle_sanitized(tmp_path):
    exe = str(tmp_path / "sanitize_oracle")
    _run(["gcc", *SAN, "-ffp-contract=off", "-fno-fast-math", "-std=gnu11", f"-I{ORACLE}",
          os.path.join(ROOT, "tests", "cpp", "sanitize_oracle.c"), os.path.join(ORACLE, "sm_oracle.c"),
          os.path.join(ORACLE, "sm_oracle_agg.c"), "-o", exe, "-lm"])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    _clean(r)
    last = r.stdout.strip().splitlines()[-1]
    assert last.startswith("ok ") and int(last.split()[1]) > 400, last


def test_nl_tree_sanitized(tmp_path):
    exe = str(tmp_path / "nl_tree_check")
    _run(["g++", *SAN, "-std=c++17", "-ffp-contract=off", f"-I{CSRC}", f"-I{ORACLE}",
          os.path.join(ROOT, "tests", "cpp", "nl_tree_check.cpp"), os.path.join(CSRC, "sm_nl_tree.cpp"),
          "-x", "c", os.path.join(ORACLE, "sm_oracle_agg.c"), os.path.join(ORACLE, "sm_oracle.c"), "-x", "none",
          "-o", exe, "-lm"])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    _clean(r)
    assert r.stdout.startswith("ok "), r.stdout[-500:]


PNG_READ = r"""
#include "stereo_matching.hpp"
#include <cstdio>
using namespace smamd;
std::string StereoMatching::costcalculation = "censusGrad", StereoMatching::aggregation = "CBCA",
            StereoMatching::optimization = "sgm", StereoMatching::object = "";
const std::string StereoMatching::root = "";
int main(int argc, char** argv) {
    for (int i = 1; i < argc; i++) {
        Mat c = imread(argv[i], 1), g = imread(argv[i], 0);
        unsigned long sum = 0;   // touch every byte the reader returned
        if (!c.empty()) for (size_t k = 0; k < (size_t)c.rows * c.step; k++) sum += c.data[k];
        if (!g.empty()) for (size_t k = 0; k < (size_t)g.rows * g.step; k++) sum += g.data[k];
        std::printf("%s %d %d %d %lu\n", c.empty() ? "E" : "R", c.rows, c.cols, c.channels(), sum);
    }
    return 0;
}
"""


def _chunk(t, d, crc=None):
    c = zlib.crc32(t + d) & 0xffffffff if crc is None else crc
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", c)


def _png(w, h, depth, ctype, raw, crc=None, ihdr_extra=b""):
    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0) + ihdr_extra
    return b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", raw, crc) + _chunk(b"IEND", b"")


def test_imread_sanitized(tmp_path):
    from PIL import Image
    src = tmp_path / "png_read.cpp"
    src.write_text(PNG_READ)
    exe = str(tmp_path / "png_read")
    _run(["g++", *SAN, "-std=c++17", f"-I{INC}", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", str(src), "-o", exe, "-lz"])
    rng = np.random.default_rng(5)
    H, W = 11, 17
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    files, expect_ok = [], []

    def add(name, data, ok):
        p = tmp_path / name
        p.write_bytes(data)
        files.append(str(p))
        expect_ok.append(ok)

    # valid images of every colour type and depth PIL writes
    for name, im in [("rgb", Image.fromarray(rgb)), ("rgba", Image.fromarray(np.dstack([rgb, rgb[..., :1]]), "RGBA")),
                     ("gray", Image.fromarray(rgb[..., 0])), ("g16", Image.fromarray(rgb[..., 0].astype(np.uint16) * 257)),
                     ("b1", Image.fromarray(rgb[..., 0] > 127)), ("pal", Image.fromarray(rgb).quantize(colors=13))]:
        im.save(tmp_path / f"{name}.png")
        good = (tmp_path / f"{name}.png").read_bytes()
        add(f"{name}_ok.png", good, True)
        # every truncation point of the file and a few corrupted bytes: a result or an empty Mat,
        # never a read past the buffer
        for cut in sorted(set(int(x) for x in np.linspace(8, len(good) - 1, 24))):
            add(f"{name}_cut{cut}.png", good[:cut], None)
        for k in range(12):
            bad = bytearray(good)
            pos = int(rng.integers(8, len(bad)))
            bad[pos] ^= int(rng.integers(1, 256))
            add(f"{name}_flip{k}.png", bytes(bad), None)
    # IDAT streams that inflate to fewer / more bytes than the header needs, bad filter bytes,
    # zero-length and non-zlib data, a wrong CRC
    row = 1 + W * 3
    full = bytes(H * row)
    add("short_idat.png", _png(W, H, 8, 2, zlib.compress(full[: row * (H - 1)])), False)
    add("long_idat.png", _png(W, H, 8, 2, zlib.compress(full + bytes(100))), None)
    add("bad_filter.png", _png(W, H, 8, 2, zlib.compress(bytes([7] + [0] * (row - 1)) * H)), None)
    add("empty_idat.png", _png(W, H, 8, 2, b""), False)
    add("not_zlib.png", _png(W, H, 8, 2, bytes(rng.integers(0, 256, 300, dtype=np.uint8))), False)
    add("bad_crc.png", _png(W, H, 8, 2, zlib.compress(full), crc=0x12345678), None)
    add("truncated_zlib.png", _png(W, H, 8, 2, zlib.compress(full)[:-9]), False)
    # crafted IHDR sizes (wrapping products, above the pixel cap, zero) and odd header fields
    for i, (w, h, depth, ctype) in enumerate([(0xFFFFFFFF, 0xFFFFFFFF, 8, 2), (0x80000000, 2, 8, 2), (0x10000, 0x10000, 8, 2),
                                              (0x7FFFFFFF, 3, 16, 6), (1, 0, 8, 2), (0, 1, 8, 2), (3, 3, 3, 2), (3, 3, 8, 5),
                                              (3, 3, 16, 3), (3, 3, 4, 6)]):
        add(f"ihdr{i}.png", _png(w, h, depth, ctype, zlib.compress(bytes(64))), False)
    add("short_ihdr.png", b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", b"\x00\x00\x00\x03"), False)
    add("huge_chunk_len.png", b"\x89PNG\r\n\x1a\n" + struct.pack(">I", 0xFFFFFFF0) + b"IHDR" + bytes(13), False)
    # PNM: valid, truncated, oversized header, garbage
    add("ok.ppm", f"P6\n{W} {H}\n255\n".encode() + rgb.tobytes(), True)
    add("cut.ppm", f"P6\n{W} {H}\n255\n".encode() + rgb.tobytes()[:50], False)
    add("huge.ppm", b"P6\n4294967295 4294967295\n255\n" + bytes(10), False)
    add("neg.pgm", b"P5\n-3 4\n255\n" + bytes(12), False)
    add("maxval.pgm", b"P5\n3 4\n65535\n" + bytes(24), None)
    add("garbage.bin", bytes(rng.integers(0, 256, 2000, dtype=np.uint8)), False)
    add("empty.png", b"", False)
    r = subprocess.run([exe] + files, capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    _clean(r)
    lines = r.stdout.split("\n")[:len(files)]
    for f, ok, line in zip(files, expect_ok, lines):
        if ok is True:
            assert line.startswith(f"R {H} {W} "), (f, line)
        elif ok is False:
            assert line.startswith("E"), (f, line)


@pytest.mark.skipif(not os.path.exists(HIPCC) or not os.path.isdir(os.path.join(CSRC, "build")),
                    reason="needs hipcc and the library's kernel objects (build())")
def test_capi_host_sanitized(tmp_path):
    objs = [os.path.join(CSRC, "build", f"{s}.o") for s in
            ("sm_kernels", "sm_cbca", "sm_sgm", "sm_refine", "sm_pyramid", "sm_so", "sm_gf", "sm_gf_cv", "sm_nl",
             "sm_nl_mst", "sm_nl_walk")]
    if not all(os.path.exists(o) for o in objs):
        pytest.skip("kernel objects not built")
    capi_o, chk_o, exe = (str(tmp_path / n) for n in ("capi_san.o", "chk.o", "capi_host_check"))
    # host code sanitized, device code as shipped (GPU sanitizers are not available on this pool)
    _run([HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fPIC", "-ffp-contract=off", "-w",
          "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
          "-Xarch_host", "-fno-sanitize-recover=all", "-c", os.path.join(CSRC, "sm_capi.cpp"), "-o", capi_o])
    clang = "/opt/rocm/lib/llvm/bin/clang++"
    _run([clang, "-std=c++17", *SAN, f"-I{INC}", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-c",
          os.path.join(ROOT, "tests", "cpp", "capi_host_check.cpp"), "-o", chk_o])
    _run([HIPCC, "--offload-arch=gfx950", "-fsanitize=address,undefined", "-fno-gpu-sanitize", chk_o, capi_o, *objs,
          "-o", exe])
    # (the HIP runtime's own allocations at exit are not this code's: leak checking off here)
    env = dict(ENV, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-4000:]
    _clean(r)
    assert r.stdout.strip().splitlines()[-1].startswith("ok "), r.stdout[-500:]
