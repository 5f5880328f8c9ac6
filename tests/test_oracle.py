"""The C oracle against the independent numpy restatement (tests/pyref.py) on small inputs.

Both restate the reference (PARITY UNPINNED: no reference binary or fixtures exist); agreement
of two independent restatements is the pin available here.  Bit-exact comparisons throughout.
"""
import numpy as np
import pytest

from mystereomatching_amd import synthetic as S
from tests import pyref


def tiny_pair(H, W, D, idx, smooth=False):
    p = S.make_pair(H, W, D, idx)
    if smooth:  # quantise colours so cross arms grow long
        for k in ("lbgr", "rbgr"):
            p[k] = (p[k] // 64 * 64).astype(np.uint8)
        p["lgray"], p["rgray"] = S.bgr_to_gray(p["lbgr"]), S.bgr_to_gray(p["rbgr"])
    return p


CASES = [(9, 13, 5, 0, False), (12, 17, 8, 1, True), (7, 20, 12, 2, False), (16, 11, 6, 3, True)]


@pytest.mark.parametrize("H,W,D,idx,smooth", CASES)
def test_census_codes(oracle, H, W, D, idx, smooth):
    p = tiny_pair(H, W, D, idx, smooth)
    cfg = oracle.config(H, W, D - 1)
    for g in ("lgray", "rgray"):
        np.testing.assert_array_equal(oracle.census(p[g], cfg), pyref.census_words(pyref.census(p[g])))


@pytest.mark.parametrize("H,W,D,idx,smooth", CASES)
def test_arms(oracle, H, W, D, idx, smooth):
    p = tiny_pair(H, W, D, idx, smooth)
    cfg = oracle.config(H, W, D - 1)
    for k in ("lbgr", "rbgr"):
        np.testing.assert_array_equal(oracle.arms(p[k], cfg), pyref.arms(p[k]))


@pytest.mark.parametrize("cost", ["censusGrad", "Census", "ADCensus", "AD"])
@pytest.mark.parametrize("H,W,D,idx,smooth", CASES[:3])
def test_pipeline_bitexact(oracle, cost, H, W, D, idx, smooth):
    p = tiny_pair(H, W, D, idx, smooth)
    cfg = oracle.config(H, W, D - 1, cost=cost)
    got = oracle.run(p, cfg, dumps=True)
    ref = pyref.pipeline(p, D - 1, cost=cost)
    for k in ("cost", "agg", "final"):
        np.testing.assert_array_equal(got[k].view(np.uint32), ref[k].view(np.uint32), err_msg=k)
    np.testing.assert_array_equal(got["disp"], ref["disp"])


def test_right_view_cost(oracle):
    H, W, D = 10, 14, 7
    p = tiny_pair(H, W, D, 5)
    cfg = oracle.config(H, W, D - 1)
    got = oracle.cost_volume(p, cfg, view=1)
    bl, br = pyref.census(p["lgray"]), pyref.census(p["rgray"])
    gx0, gy0 = pyref.grads(p["lgray"])
    gx1, gy1 = pyref.grads(p["rgray"])
    ref = pyref.fuse(pyref.census_cost(bl, br, D, view=1),
                     pyref.grad_cost(gx0, gx1, gy0, gy1, pyref.arms(p["rbgr"]), D, view=1), 13, 1)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_sgm_8_paths(oracle):
    H, W, D = 9, 12, 6
    p = tiny_pair(H, W, D, 6)
    cfg = oracle.config(H, W, D - 1, sgm_paths=8)
    got = oracle.run(p, cfg, dumps=True)
    ref = pyref.pipeline(p, D - 1, paths=8)
    np.testing.assert_array_equal(got["final"].view(np.uint32), ref["final"].view(np.uint32))
    np.testing.assert_array_equal(got["disp"], ref["disp"])


def test_solve_all_weight(oracle):
    # OpenCV 1x1 float invert: (float)(1.0 / (double)(1 + 0.3f)) = 0x3f44ec4f
    w = np.float32(oracle.solve_all_weight(0.3))
    assert w.view(np.uint32) == 0x3F44EC4F


def test_reflect101(oracle):
    lib = oracle.load()
    for n in (1, 2, 3, 5):
        for p in range(-9, 14):
            assert lib.smo_reflect101(p, n) == pyref.reflect101(p, n)
