"""GPU parity of the cross-scale pyramid (PY_LEV > 1) against the oracle.

main_.cpp:131-158 builds one StereoMatching per level from pyrDown'ed images (maxdisp_{p+1} =
maxdisp_p / 2 + 1, disSc = 2^p), runs costCalculate on each, then SolveAll(smPsy, PY_LEV, 0.3)
combines the levels into level 0 before dispOptimize.  Bit-exact against oracle.run_pyr.
"""
import numpy as np
import pytest

from mystereomatching_amd import SolveAll, StereoMatching, pyrDown
from mystereomatching_amd import synthetic as S

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(375, 450, 3), (375, 450), (21, 34, 3), (2, 2), (3, 5, 3), (188, 225)])
def test_pyr_down(oracle, shape):
    img = np.random.default_rng(sum(shape)).integers(0, 256, size=shape, dtype=np.uint8)
    np.testing.assert_array_equal(pyrDown(img), oracle.pyr_down(img))


def _pyr_down_f32_ref(a):
    """OpenCV's scalar pyrDown_ order for float (FltCast<float, 8>): row pass then column pass,
    s0*6 + (s-1 + s+1)*4 + s-2 + s+2, then * 1/256; BORDER_REFLECT_101 (last bit unpinned)."""
    a = a.astype(np.float32)
    H, W = a.shape
    ry = np.array([abs(i) if i < 0 else (2 * H - 2 - i if i >= H else i) for i in range(-2, 2 * ((H + 1) // 2) + 1)])
    rx = np.array([abs(i) if i < 0 else (2 * W - 2 - i if i >= W else i) for i in range(-2, 2 * ((W + 1) // 2) + 1)])
    if H == 1:
        ry[:] = 0
    if W == 1:
        rx[:] = 0
    dc, dr = (W + 1) // 2, (H + 1) // 2
    cx = [rx[2 * np.arange(dc) + j] for j in range(5)]
    f6, f4 = np.float32(6), np.float32(4)
    rows = []
    for y in range(dr):
        r = []
        for k in range(5):
            row = a[ry[2 * y + k]]
            r.append(row[cx[2]] * f6 + (row[cx[1]] + row[cx[3]]) * f4 + row[cx[0]] + row[cx[4]])
        rows.append((r[2] * f6 + (r[1] + r[3]) * f4 + r[0] + r[4]) * np.float32(1 / 256))
    return np.stack(rows).astype(np.float32)


@pytest.mark.parametrize("shape", [(375, 450), (21, 34), (3, 5), (188, 225)])
def test_pyr_down_f32(shape):
    """pyrDown(DT, DT) of the float ground truth (main_.cpp:149)."""
    rng = np.random.default_rng(sum(shape))
    img = (rng.integers(0, 256, size=shape).astype(np.float32) * np.float32(1 / 3))
    np.testing.assert_array_equal(pyrDown(img), _pyr_down_f32_ref(img))


def run_pyramid(pair, max_disp, L, refine=False):
    """main_.cpp:131-166 through the mirror API."""
    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = "censusGrad", "CBCA", "sgm"
    StereoMatching.Do_refine = refine
    try:
        imgs = {k: pair[k] for k in ("lbgr", "rbgr", "lgray", "rgray")}
        levels, md, sc = [], max_disp, 1
        for p in range(L):
            H, W = imgs["lgray"].shape
            prm = StereoMatching.Parameters(md, H, W, 13, 1, 2, 109, 10, "", sc)
            sm = StereoMatching(imgs["lbgr"], imgs["rbgr"], imgs["lgray"], imgs["rgray"], None, None, None, None, prm)
            sm.costCalculate()
            levels.append(sm)
            md, sc = md // 2 + 1, sc * 2
            imgs = {k: pyrDown(v) for k, v in imgs.items()}
        SolveAll(levels, L, 0.3)
        dp = levels[0].dispOptimize()
        if refine:
            dp = levels[0].refine()
        return dp
    finally:
        StereoMatching.Do_refine = False


@pytest.mark.parametrize("L,H,W,md,refine", [(2, 60, 83, 23, False), (3, 75, 90, 31, False), (2, 48, 70, 63, True),
                                             (3, 61, 77, 15, True), (4, 75, 90, 31, False), (5, 100, 121, 31, True),
                                             (8, 300, 260, 63, False)])
def test_pyramid_pipeline(oracle, L, H, W, md, refine):
    pair = S.make_pair(H, W, md + 1, 300 + L + H)
    cfg = oracle.config(H, W, md, do_refine=int(refine))
    ref = oracle.run_pyr(pair, cfg, L)
    np.testing.assert_array_equal(run_pyramid(pair, md, L, refine), ref)


def test_pyramid_teddy_size(oracle):
    H, W, md = 375, 450, 63
    pair = S.make_pair(H, W, md + 1, 5)
    ref = oracle.run_pyr(pair, oracle.config(H, W, md), 2)
    np.testing.assert_array_equal(run_pyramid(pair, md, 2), ref)


def test_pyramid_validation():
    H, W, md = 40, 50, 15
    pair = S.make_pair(H, W, md + 1, 1)
    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = "censusGrad", "CBCA", "sgm"
    a = StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], None, None, None, None,
                       StereoMatching.Parameters(md, H, W))
    b = StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], None, None, None, None,
                       StereoMatching.Parameters(md, H, W, disSc=2))   # wrong size for level 1
    a.costCalculate()
    b.costCalculate()
    with pytest.raises(Exception, match="pyrDown"):
        SolveAll([a, b], 2, 0.3)
    with pytest.raises(Exception, match="PY_LVL"):
        SolveAll([a] + [b] * 8, 9, 0.3)     # PY_LVL in [1, 8] (sm_capi.h)
