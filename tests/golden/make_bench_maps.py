"""Generates tests/golden/bench_maps_<workload>.npz: the oracle's int16 map of EVERY pair of a
bench.py workload's batch (rank 0's pairs 0 .. B-1), so that bench.py can compare the maps its
timed loop (the default pipelined two-group schedule) produced, pair by pair, and the GPU tests can
run whole batches through that schedule against them.

PARITY UNPINNED (see make_golden.py): the maps are the CPU restatement's (oracle/sm_oracle.c).
Each record holds the generator arguments, the sha256 of every regenerated input image (checked
first, so an RNG drift is not mistaken for a kernel bug) and the stacked maps [B, H, W].

Workloads (bench.py WORKLOADS; BASELINE.json configs):
  fullres  configs[3]  3000x2000 D = 256, 2 pairs, censusGrad + CBCA(2) + SolveAll + SGM 4-path
  hd       configs[4]  1920x1080 D = 256, 8 pairs (one GPU's shard), same pipeline
  kitti    configs[2]  1242x375 D = 192, 4 pairs, 8-path SGM
  teddy    configs[1]  450x375 D = 64, 16 pairs
Run:  python tests/golden/make_bench_maps.py [workload ...]     (full resolution: ~70 s and ~25 GB
      of host memory per pair on one core; the pairs run one at a time)
"""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from mystereomatching_amd import synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

# workload: (H, W, max_disp, sgm_paths, pairs) -- the same numbers as bench.py WORKLOADS
CASES = {
    "fullres": (2000, 3000, 255, 4, 2),
    "hd": (1080, 1920, 255, 4, 8),
    "kitti": (375, 1242, 191, 8, 4),
    "teddy": (375, 450, 63, 4, 16),
}
KEYS = ("lbgr", "rbgr", "lgray", "rgray")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def make(name, out_dir):
    H, W, md, paths, B = CASES[name]
    cfg = O.config(H, W, md, sgm_paths=paths)
    maps, rec, t0 = [], {}, time.perf_counter()
    for i in range(B):
        pair = S.make_pair(H, W, md + 1, i)
        maps.append(O.run_ex(pair, cfg)["disp"])
        for k in KEYS:
            rec[f"sha_{k}_{i}"] = sha(pair[k])
        print(f"{name} pair {i}: {time.perf_counter() - t0:.1f} s", flush=True)
    disp = np.stack(maps)
    rec.update(H=H, W=W, max_disp=md, sgm_paths=paths, pairs=B, disp=disp, sha_disp=sha(disp),
               oracle_seconds=time.perf_counter() - t0)
    np.savez_compressed(os.path.join(out_dir, f"bench_maps_{name}.npz"), **rec)
    print(f"bench_maps_{name}: {B} x {W}x{H} D={md + 1} sha {rec['sha_disp'][:16]}", flush=True)


def main():
    out_dir = os.path.dirname(os.path.abspath(__file__))
    for name in (sys.argv[1:] or list(CASES)):
        make(name, out_dir)


if __name__ == "__main__":
    main()
