"""The C++ drop-in (include/stereo_matching.hpp) against main_.cpp's own use of class StereoMatching.

CPU (no GPU calls): tests/cpp/main_shaped.cpp — main_.cpp:15-19 and 85-178 with `using namespace
smamd` in place of `using namespace cv` — compiles unchanged against the facade (9-argument ctor
with DT and masks, openCSV / closeCSV / saveTime, SolveAll over StereoMatching**, pyrDown on u8 and
f32 images, DP[0] as a Mat); the host-only Mat / imread / convertTo logic matches numpy; the driver
reports unreadable images the way main_.cpp:108-112 does.
GPU: the prebuilt driver (build() makes tests/cpp/build/main_shaped) runs a synthetic pair written
as PPM / PGM files, and its DP[0] equals the oracle's map; its calErr line equals
evaluate.cal_err on the same DT and mask.  tools/build/sm_main's 16-bit PGM is checked the same way.
"""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "mystereomatching_amd")
CXX = ["g++", "-O1", "-std=c++17", "-Wall", "-Wextra", "-Werror", f"-I{INC}", "-I/opt/rocm/include",
       "-D__HIP_PLATFORM_AMD__"]


def _compile(src, out, link=True):
    cmd = CXX + [src, "-o", out]
    if link:
        cmd += [f"-L{LIBDIR}", "-lsm_hip", f"-Wl,-rpath,{LIBDIR}"]
    cmd += ["-lz"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]


def write_ppm(path, bgr):
    h, w, _ = bgr.shape
    with open(path, "wb") as f:
        f.write(f"P6\n{w} {h}\n255\n".encode())
        f.write(np.ascontiguousarray(bgr[..., ::-1]).tobytes())


def write_pgm(path, g):
    h, w = g.shape
    with open(path, "wb") as f:
        f.write(f"P5\n{w} {h}\n255\n".encode())
        f.write(np.ascontiguousarray(g, np.uint8).tobytes())


def write_png(path, a):
    from PIL import Image
    Image.fromarray(np.ascontiguousarray(a)).save(path)


def write_dataset(d, pair, reduce):
    """A Middlebury-2003-style object folder as main_.cpp:85-107 reads it (teddy naming)."""
    os.makedirs(d, exist_ok=True)
    write_png(os.path.join(d, "im2.png"), pair["lbgr"][..., ::-1])
    write_png(os.path.join(d, "im6.png"), pair["rbgr"][..., ::-1])
    dt8 = np.clip(np.rint(pair["gt"] * reduce), 0, 255).astype(np.uint8)
    write_png(os.path.join(d, "disp2.png"), dt8)
    write_png(os.path.join(d, "all.png"), pair["all"])
    write_png(os.path.join(d, "nonocc.png"), pair["nonocc"])
    write_png(os.path.join(d, "disc.png"), pair["nonocc"])
    return dt8


def test_main_shaped_translation_unit_compiles(tmp_path):
    _compile(os.path.join(ROOT, "tests", "cpp", "main_shaped.cpp"), str(tmp_path / "main_shaped"))
    _compile(os.path.join(ROOT, "tools", "sm_main.cpp"), str(tmp_path / "sm_main"))


MAT_CHECK = r"""
#include "stereo_matching.hpp"
#include <cstdio>
using namespace smamd;
std::string StereoMatching::costcalculation = "censusGrad", StereoMatching::aggregation = "CBCA",
            StereoMatching::optimization = "sgm", StereoMatching::object = "";
const std::string StereoMatching::root = "";
int main(int, char** argv) {
    Mat c = imread(argv[1], 1), g = imread(argv[1], 0), p = imread(argv[2], 0), bad = imread(argv[3], 1);
    if (!bad.empty() || c.channels() != 3 || g.channels() != 1 || p.channels() != 1) return 5;
    Mat shallow = p;                       // shares the buffer (cv::Mat header copy)
    p.convertTo(p, CV_32F, 1.0 / 3);       // main_.cpp:129: a new buffer for p
    std::fwrite(c.data, 1, (size_t)c.rows * c.step, stdout);
    std::fwrite(g.data, 1, (size_t)g.rows * g.step, stdout);
    std::fwrite(shallow.data, 1, (size_t)shallow.rows * shallow.step, stdout);
    std::fwrite(p.data, 1, (size_t)p.rows * p.step, stdout);
    return (p.depth() == CV_32F && shallow.depth() == CV_8U && p.data != shallow.data) ? 0 : 6;
}
"""


def test_mat_imread_convert_host_logic(tmp_path):
    from mystereomatching_amd import synthetic as S
    src = tmp_path / "mat_check.cpp"
    src.write_text(MAT_CHECK)
    exe = str(tmp_path / "mat_check")
    _compile(str(src), exe, link=False)
    rng = np.random.default_rng(5)
    bgr = rng.integers(0, 256, (7, 11, 3), dtype=np.uint8)
    gray = rng.integers(0, 256, (5, 9), dtype=np.uint8)
    write_ppm(tmp_path / "c.ppm", bgr)
    write_pgm(tmp_path / "g.pgm", gray)
    r = subprocess.run([exe, str(tmp_path / "c.ppm"), str(tmp_path / "g.pgm"), str(tmp_path / "none.ppm")],
                       capture_output=True)
    assert r.returncode == 0, r.returncode
    out = np.frombuffer(r.stdout, np.uint8)
    n1, n2, n3 = bgr.size, 7 * 11, gray.size
    np.testing.assert_array_equal(out[:n1].reshape(bgr.shape), bgr)
    np.testing.assert_array_equal(out[n1:n1 + n2].reshape(7, 11), S.bgr_to_gray(bgr))
    np.testing.assert_array_equal(out[n1 + n2:n1 + n2 + n3].reshape(gray.shape), gray)
    f = out[n1 + n2 + n3:].view(np.float32).reshape(gray.shape)
    np.testing.assert_array_equal(f, gray.astype(np.float32) * np.float32(1.0 / 3))


def test_main_shaped_reports_unreadable_images(tmp_path):
    exe = os.path.join(ROOT, "tests", "cpp", "build", "main_shaped")
    if not os.path.exists(exe):
        _compile(os.path.join(ROOT, "tests", "cpp", "main_shaped.cpp"), str(tmp_path / "main_shaped"))
        exe = str(tmp_path / "main_shaped")
    r = subprocess.run([exe, str(tmp_path / "missing"), "15", "4", str(tmp_path / "o.i16")],
                       capture_output=True, text=True)
    assert r.returncode == 255 and "can't read original img" in r.stdout   # main_.cpp:108-112 (return -1)


@pytest.mark.gpu
def test_main_shaped_driver_matches_oracle(tmp_path, oracle):
    from mystereomatching_amd import synthetic as S
    from mystereomatching_amd.evaluate import cal_err
    exe = os.path.join(ROOT, "tests", "cpp", "build", "main_shaped")
    assert os.path.exists(exe), "build() makes tests/cpp/build/main_shaped"
    H, W, md, reduce = 120, 168, 47, 4
    pair = S.make_pair(H, W, md + 1, 31)
    dt8 = write_dataset(str(tmp_path / "ds"), pair, reduce)
    out = tmp_path / "dp.i16"
    r = subprocess.run([exe, str(tmp_path / "ds"), str(md), str(reduce), str(out)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    got = np.fromfile(out, np.int16).reshape(H, W)
    want = oracle.run(pair, oracle.config(H, W, md))["disp"]
    np.testing.assert_array_equal(got, want)
    # calErr over the stored DT and masks (h:1748-1825), DT = imread(disp) * (1 / reduce) (main:129)
    dt = dt8.astype(np.float32) * np.float32(1.0 / reduce)
    m = re.search(r"nonocc\terrorRatio: (\S+) epe: (\S+)", r.stdout)
    assert m, r.stdout[-2000:]
    pbm, rms = cal_err(got, dt, pair["nonocc"], 1.0)
    assert float(m.group(1)) == pytest.approx(pbm, rel=1e-5, abs=1e-6)
    assert float(m.group(2)) == pytest.approx(rms, rel=1e-5, abs=1e-6)


@pytest.mark.gpu
def test_sm_main_tool_matches_oracle(tmp_path, oracle):
    from mystereomatching_amd import synthetic as S
    exe = os.path.join(ROOT, "tools", "build", "sm_main")
    assert os.path.exists(exe), "build() makes tools/build/sm_main"
    H, W, md = 96, 130, 31
    pair = S.make_pair(H, W, md + 1, 32)
    write_ppm(tmp_path / "l.ppm", pair["lbgr"])
    write_ppm(tmp_path / "r.ppm", pair["rbgr"])
    r = subprocess.run([exe, str(tmp_path / "l.ppm"), str(tmp_path / "r.ppm"), str(md), str(tmp_path / "o.pgm")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    raw = (tmp_path / "o.pgm").read_bytes()
    hdr = f"P5\n{W} {H}\n65535\n".encode()
    assert raw.startswith(hdr)
    got = np.frombuffer(raw[len(hdr):], ">u2").reshape(H, W).astype(np.int32)
    want = oracle.run(pair, oracle.config(H, W, md))["disp"].astype(np.int32)
    np.testing.assert_array_equal(got, np.maximum(want, 0))


PNG_CHECK = r"""
#include "stereo_matching.hpp"
#include <cstdio>
using namespace smamd;
std::string StereoMatching::costcalculation = "censusGrad", StereoMatching::aggregation = "CBCA",
            StereoMatching::optimization = "sgm", StereoMatching::object = "";
const std::string StereoMatching::root = "";
int main(int argc, char** argv) {
    for (int i = 1; i < argc; i++) {
        Mat c = imread(argv[i], 1), g = imread(argv[i], 0);
        if (c.empty() || g.empty()) { std::printf("E %d\n", i); continue; }
        std::fwrite(c.data, 1, (size_t)c.rows * c.step, stdout);
        std::fwrite(g.data, 1, (size_t)g.rows * g.step, stdout);
    }
    return 0;
}
"""


def _png_with_header(w, h, depth=8, ctype=2, idat=b""):
    import struct
    import zlib

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)
    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0)
    return b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", idat) + chunk(b"IEND", b"")


def test_imread_png_rejects_oversized_headers(tmp_path):
    """Crafted IHDR sizes (round-3 ADVICE): sizes whose products wrap 32 / 64-bit buffer sizes,
    sizes above the 2^28-pixel cap, and a header far larger than its compressed data must give an
    empty Mat (imread's failure result, main_.cpp:108), never a short buffer or an exception."""
    import zlib
    src = tmp_path / "png_check.cpp"
    src.write_text(PNG_CHECK)
    exe = str(tmp_path / "png_check")
    _compile(str(src), exe, link=False)
    small = zlib.compress(bytes(4 * (1 + 3 * 4)))
    cases = [(0xFFFFFFFF, 0xFFFFFFFF, 8, 2), (0x80000000, 2, 8, 2), (0x10000, 0x10000, 8, 2),
             (0x7FFFFFFF, 3, 16, 6), (1 << 15, 1 << 14, 8, 0), (20000, 13000, 16, 6), (1, 0, 8, 2)]
    files = []
    for i, (w, h, depth, ctype) in enumerate(cases):
        f = tmp_path / f"bad{i}.png"
        f.write_bytes(_png_with_header(w, h, depth, ctype, small))
        files.append(str(f))
    r = subprocess.run([exe] + files, capture_output=True, timeout=60)
    assert r.returncode == 0, r.stderr[:300]
    assert r.stdout.decode().split() == sum((["E", str(i + 1)] for i in range(len(cases))), [])


def test_imread_png(tmp_path):
    """smamd::imread on PNG files written by PIL: RGB, RGBA, gray, 16-bit gray, 1/4-bit gray and
    palette images, several filter choices -- BGR for flags 1 and libpng's rgb_to_gray for flags 0,
    as OpenCV's PNG decoder delivers them (main_.cpp:92-107 reads *.png)."""
    from PIL import Image
    from mystereomatching_amd import synthetic as S
    src = tmp_path / "png_check.cpp"
    src.write_text(PNG_CHECK)
    exe = str(tmp_path / "png_check")
    _compile(str(src), exe, link=False)
    rng = np.random.default_rng(11)
    H, W = 13, 21
    rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    rgb[:, :7] = rgb[:, 7:8]                       # flat runs: Sub / Up / Paeth filters get used
    gray = rng.integers(0, 256, (H, W), dtype=np.uint8)
    g16 = rng.integers(0, 65536, (H, W), dtype=np.uint16)
    bits1 = rng.integers(0, 2, (H, W), dtype=np.uint8)
    g4 = rng.integers(0, 16, (H, W), dtype=np.uint8)
    cases = []   # (file, expected RGB)
    Image.fromarray(rgb).save(tmp_path / "rgb.png"); cases.append(("rgb.png", rgb))
    Image.fromarray(rgb).save(tmp_path / "rgb9.png", compress_level=9, optimize=True); cases.append(("rgb9.png", rgb))
    rgba = np.dstack([rgb, rng.integers(0, 256, (H, W), dtype=np.uint8)])
    Image.fromarray(rgba, "RGBA").save(tmp_path / "rgba.png"); cases.append(("rgba.png", rgb))
    Image.fromarray(gray).save(tmp_path / "gray.png"); cases.append(("gray.png", np.dstack([gray] * 3)))
    Image.fromarray(g16).save(tmp_path / "g16.png"); g16h = (g16 >> 8).astype(np.uint8)
    cases.append(("g16.png", np.dstack([g16h] * 3)))
    Image.fromarray(bits1 * 255).convert("1").save(tmp_path / "b1.png"); cases.append(("b1.png", np.dstack([bits1 * 255] * 3)))
    pal = Image.fromarray(rgb).quantize(colors=16)
    pal.save(tmp_path / "pal.png"); cases.append(("pal.png", np.asarray(pal.convert("RGB"))))
    r = subprocess.run([exe] + [str(tmp_path / f) for f, _ in cases], capture_output=True)
    assert r.returncode == 0 and not r.stdout.startswith(b"E"), r.stdout[:200]
    out = np.frombuffer(r.stdout, np.uint8)
    pos = 0
    for f, want in cases:
        bgr = out[pos:pos + H * W * 3].reshape(H, W, 3)
        pos += H * W * 3
        g = out[pos:pos + H * W].reshape(H, W)
        pos += H * W
        np.testing.assert_array_equal(bgr, want[..., ::-1], err_msg=f)
        np.testing.assert_array_equal(g, S.bgr_to_gray(np.ascontiguousarray(want[..., ::-1])), err_msg=f)
    assert pos == out.size
