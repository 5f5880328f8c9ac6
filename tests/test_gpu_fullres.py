"""GPU at BASELINE configs[3] size (Middlebury-2014 full resolution, 3000x2000, D = 256), where the
CPU oracle is too slow and too large to run inside a test: size-independent properties instead.

* two independent code paths agree bit for bit on the int16 map and on the final volume: the
  batch entry point (sm_run: SolveAll fused into the last CBCA sweep, WTA fused into the last SGM
  path) and the reference-ordered API (costCalculate, SolveAll as its own pass, dispOptimize with
  the summed volume kept);
* the batch path is deterministic (run twice);
* the map holds disparities in [-1, D - 1] and reproduces the synthetic ground truth (bad-2.0 on
  non-occluded pixels), the reference's evaluator being the one the bench reports.
The oracle itself is pinned at every smaller size (test_gpu_parity.py, KITTI 375x1242 D = 192).
"""
import numpy as np
import pytest

from mystereomatching_amd import SolveAll, StereoBatch, StereoMatching
from mystereomatching_amd import synthetic as S
from mystereomatching_amd.evaluate import cal_err

pytestmark = pytest.mark.gpu

KEYS = ("lbgr", "rbgr", "lgray", "rgray")


def test_fullres_paths_agree_and_deterministic():
    H, W, md = 2000, 3000, 255
    pair = S.make_pair(H, W, md + 1, 7)
    sb = StereoBatch(md, H, W, 1, device=0)
    try:
        sb.upload(*(pair[k][None] for k in KEYS))
        d1 = sb.run(0.3)[0]
        d2 = sb.run(0.3)[0]
    finally:
        sb.close()
    np.testing.assert_array_equal(d1, d2)
    assert d1.min() >= -1 and d1.max() <= md

    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = "censusGrad", "CBCA", "sgm"
    prm = StereoMatching.Parameters(md, H, W)
    sm = StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], pair["gt"], None, pair["nonocc"],
                        None, prm, device=0)
    sm.costCalculate()
    SolveAll([sm], 1, 0.3)
    dp = sm.dispOptimize()
    np.testing.assert_array_equal(dp, d1)

    bad2 = cal_err(d1, pair["gt"], pair["nonocc"], 2.0)[0]
    assert bad2 < 0.05, f"bad-2.0 nonocc = {bad2:.4f}"
