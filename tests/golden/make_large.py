"""Generates tests/golden/large_*.npz: oracle disparity maps at the BASELINE configs' own shapes.

PARITY UNPINNED (see make_golden.py): the maps are the CPU restatement's (oracle/sm_oracle.c)
output, which is what the GPU path must reproduce bit for bit.  These shapes are too slow or too
large for the oracle inside a GPU test (full resolution: ~25 GB and ~80 s on one core here), so
the oracle runs once in the build container and the fixture stores

  * the generator arguments (H, W, max_disp, synthetic pair index) and the sha256 of each
    regenerated input image (the GPU test checks them first, so an RNG drift is not mistaken
    for a kernel bug),
  * the pipeline configuration (cost method, aggregation, optimisation, SGM paths, refine),
  * the sha256 of the oracle's int16 map and the map itself (zlib-compressed npz).

Cases (BASELINE.json configs):
  configs[3]  Middlebury-2014 full resolution 3000x2000 D = 256, censusGrad + CBCA + SGM 4-path
  configs[4]  1920x1080 D = 256 (one pair of the 64-pair batch), same pipeline
  configs[0]  Cones-shaped 450x375 Census cost + SGM (no aggregation), D = 60 (maxdisp 59, main:39) and D = 64
  configs[1]  Teddy-shaped 450x375 D = 64 with Do_refine (both views, LR check, region vote,
              proper interpolation, median: cpp:1138-1511) and with optimization "so" (cpp:6272-6394)
Run:  python tests/golden/make_large.py [name ...]      (all cases when no name is given)
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

# name: (H, W, max_disp, pair index, oracle/sm_params overrides)
# override keys are field names shared by smo_config and sm_params
CASES = {
    "large_fullres_d256": (2000, 3000, 255, 0, dict(cost_method=0, aggregation=1, optimization=1, sgm_paths=4)),
    "large_hd1080_d256": (1080, 1920, 255, 0, dict(cost_method=0, aggregation=1, optimization=1, sgm_paths=4)),
    "large_cones_census_sgm_d60": (375, 450, 59, 1, dict(cost_method=1, aggregation=0, optimization=1, sgm_paths=4)),
    "large_cones_census_sgm_d64": (375, 450, 63, 1, dict(cost_method=1, aggregation=0, optimization=1, sgm_paths=4)),
    "large_teddy_refine_d64": (375, 450, 63, 0, dict(cost_method=0, aggregation=1, optimization=1, sgm_paths=4,
                                                      do_refine=1)),
    "large_teddy_so_d64": (375, 450, 63, 0, dict(cost_method=0, aggregation=1, optimization=2, sgm_paths=4)),
    "large_kitti_8path_d192": (375, 1242, 191, 0, dict(cost_method=0, aggregation=1, optimization=1, sgm_paths=8)),
}
KEYS = ("lbgr", "rbgr", "lgray", "rgray")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def make(name, out_dir):
    H, W, md, idx, ov = CASES[name]
    pair = S.make_pair(H, W, md + 1, idx)
    cfg = O.config(H, W, md, **ov)
    t = time.perf_counter()
    disp = O.run_ex(pair, cfg)["disp"]
    dt = time.perf_counter() - t
    rec = dict(H=H, W=W, max_disp=md, index=idx, disp=disp, sha_disp=sha(disp), oracle_seconds=dt)
    rec.update({"ov_" + k: v for k, v in ov.items()})
    for k in KEYS:
        rec["sha_" + k] = sha(pair[k])
    np.savez_compressed(os.path.join(out_dir, name + ".npz"), **rec)
    print(f"{name}: {W}x{H} D={md + 1} {ov} oracle {dt:.1f} s sha {rec['sha_disp'][:16]}", flush=True)


def main():
    out_dir = os.path.dirname(os.path.abspath(__file__))
    for name in (sys.argv[1:] or list(CASES)):
        make(name, out_dir)


if __name__ == "__main__":
    main()
