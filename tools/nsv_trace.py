#!/usr/bin/env python3
"""Where the two-wave V NORM_SCAN sweep's time goes: runs one full-resolution step through a
diagnostic build (tools/build_variants.sh tr "-DSM_CB_NSV_TRACE=1") and prints, per wave role,
the mean shader-clock cycles per tile of each phase (sm_cbca.hip NsvTrace marks).

usage: python tools/nsv_trace.py [--lib tools/abvar/libsm_hip_tr.so] [--workload fullres]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WAVE0 = ["loads+wait+A values (+NsW mailbox)", "wait B1(n-1) read", "A writes+lgkm+barrier"]
WAVE1 = ["loads+wait+pass isect", "wait A(n) written", "B1 issue+lgkm+barrier", "B2 (+write wait)",
         "C reads+wait+stores"]
WAVE1_PIPE = ["X2->X1: B2, C issue, addr, X1 wait", "X1->X2: B1 reads, C stores, loads, isect"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools", "abvar", "libsm_hip_tr.so"))
    ap.add_argument("--workload", default="fullres")
    ap.add_argument("--pipe", action="store_true", help="the library runs SM_CB_NSV2_PIPE (two marks per tile)")
    a = ap.parse_args()
    os.environ["SM_HIP_LIB"] = a.lib
    import bench
    from mystereomatching_amd import StereoBatch
    from mystereomatching_amd import synthetic as S
    H, W, md, paths, B, _ = bench.WORKLOADS[a.workload]
    batch = S.make_batch(B, H, W, md + 1)
    sb = StereoBatch(md, H, W, B, device=0, sgm_paths=paths, num_streams=1)
    sb.upload(batch["lbgr"], batch["rbgr"], batch["lgray"], batch["rgray"])
    sb.profile(True)
    for _ in range(3):
        sb.run(0.3, download=False)
    sb.synchronize()
    prof = sb.profile_read()
    ms = prof["cbca_v_norm_scan"]["total_ms"] / prof["cbca_v_norm_scan"]["launches"]
    lib = C.CDLL(a.lib)
    lib.sm_debug_nsv_trace.restype = C.c_int
    nblk = W * ((md + 1) // 64) * B
    buf = np.zeros((min(nblk, 1 << 16), 2, 8), np.uint64)
    got = lib.sm_debug_nsv_trace(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), buf.shape[0])
    assert got > 0, "sm_debug_nsv_trace failed"
    tiles = buf[:, 1, 7].astype(np.float64)
    print(f"{a.workload}: {nblk} lines, NsV2 {ms:.3f} ms per launch (HIP events), tiles per line {tiles.mean():.1f}")
    for w, names in ((0, WAVE0), (1, WAVE1_PIPE if a.pipe else WAVE1)):
        per = buf[:, w, :len(names)].astype(np.float64) / tiles[:, None]
        tot = per.sum(axis=1)
        print(f"wave {w}: {tot.mean():.0f} cycles per tile (p10 {np.percentile(tot, 10):.0f}, p90 {np.percentile(tot, 90):.0f})")
        for i, nm in enumerate(names):
            print(f"   {nm:28s} {per[:, i].mean():8.1f}  ({100 * per[:, i].mean() / tot.mean():4.1f} %)")
    # clock calibration: a line's cycles vs the launch time (lines run 3 per CU, 256 CUs)
    rounds = nblk / (3 * 256)
    line_cycles = (buf[:, 1, :(2 if a.pipe else 5)].astype(np.float64).sum(axis=1)).mean()
    print(f"implied clock: {line_cycles * rounds / (ms * 1e-3) / 1e9:.2f} GHz if {rounds:.2f} rounds of 3 lines per CU")
    sb.close()


if __name__ == "__main__":
    main()
