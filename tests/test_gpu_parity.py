"""GPU parity: libsm_hip.so (through the C-ABI) against the CPU oracle, bit-exact.

Every comparison is on float bit patterns (volumes) or int16 (disparity): the whole path is
IEEE-deterministic, so the bar is bit-exactness, not a tolerance (north_star allows 1e-4 for
the float CBCA; we do not need it).
"""
import ctypes as C
import glob
import hashlib
import os

import numpy as np
import pytest

from mystereomatching_amd import StereoBatch, StereoMatching, SolveAll, _capi
from mystereomatching_amd import synthetic as S

pytestmark = pytest.mark.gpu

GOLDEN = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
                if not os.path.basename(p).startswith(("large_", "bench_maps_")))   # those: test_gpu_large_fixtures.py


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def make_sm(pair, max_disp, cost="censusGrad", agg="CBCA", opt="sgm", paths=4, keep=True, **kw):
    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = cost, agg, opt
    H, W = pair["lgray"].shape
    prm = StereoMatching.Parameters(max_disp, H, W)
    prm.sgm_scanNum = paths
    for k, v in kw.items():
        setattr(prm, k, v)
    return StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], pair.get("gt"),
                          None, pair.get("nonocc"), None, prm, keep_final_volume=keep)


def run_reference_order(pair, max_disp, **kw):
    """main_.cpp:139-163 order through the mirror API; returns stage volumes + DP[0]."""
    sm = make_sm(pair, max_disp, **kw)
    sm.costCalculate()
    agg = sm.vm[0]
    SolveAll([sm], 1, 0.3)
    dp = sm.dispOptimize()
    final = sm.vm[0]
    return sm, agg, final, dp


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_golden(path):
    g = np.load(path)
    pair = {k: g[k] for k in ("lbgr", "rbgr", "lgray", "rgray")}
    sm, agg, final, dp = run_reference_order(pair, int(g["max_disp"]), cost=str(g["cost"]), paths=int(g["paths"]))
    np.testing.assert_array_equal(dp, g["disp"])
    assert sha(agg) == str(g["sha_agg"])
    assert sha(final) == str(g["sha_final"])
    if "agg_vol" in g.files:
        np.testing.assert_array_equal(bits(agg), bits(g["agg_vol"]))


@pytest.mark.parametrize("cost", ["censusGrad", "Census", "ADCensus", "AD"])
def test_cost_volume_and_stages(oracle, cost):
    H, W, md = 41, 67, 23
    pair = S.make_pair(H, W, md + 1, 11)
    cfg = oracle.config(H, W, md, cost=cost)
    ref = oracle.run(pair, cfg, dumps=True, right=True)
    # raw cost volume: aggregation off, WTA only
    sm = make_sm(pair, md, cost=cost, agg="", opt="")
    sm.costCalculate()
    np.testing.assert_array_equal(bits(sm.vm[0]), bits(ref["cost"]))
    _, agg, final, dp = run_reference_order(pair, md, cost=cost)
    np.testing.assert_array_equal(bits(agg), bits(ref["agg"]))
    np.testing.assert_array_equal(bits(final), bits(ref["final"]))
    np.testing.assert_array_equal(dp, ref["disp"])


@pytest.mark.parametrize("rv,ru,ring,cost,md", [(1, 1, 0, 1, 23), (2, 3, 1, 0, 99), (3, 4, 0, 2, 23),
                                                 (4, 4, 1, 0, 23), (4, 5, 1, 0, 70), (4, 5, 1, 2, 99),
                                                 (2, 2, 0, 0, 23), (2, 2, 0, 1, 70), (2, 2, 0, 2, 130)])
def test_census_windows(oracle, rv, ru, ring, cost, md):
    """Census widths of 1-4 32-bit words (cost-kernel record layouts), D <= 64 and D > 64, both views."""
    H, W = 23, 97
    pair = S.make_pair(H, W, md + 1, 60 + rv * 7 + ru)
    cfg = oracle.config(H, W, md, cost=cost, census_rv=rv, census_ru=ru, census_ring=ring)
    lib = _capi.load()
    p = _capi.default_params(md, H, W, aggregation=0, optimization=0, compute_right_view=1, cost_method=cost)
    p.census_rv, p.census_ru, p.census_ring = rv, ru, ring
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        a = {k: np.ascontiguousarray(pair[k]) for k in ("lbgr", "rbgr", "lgray", "rgray")}
        _capi.check(lib, ctx, lib.sm_set_images(ctx, _capi.ptr(a["lbgr"]), _capi.ptr(a["rbgr"]), W * 3,
                                                _capi.ptr(a["lgray"]), _capi.ptr(a["rgray"]), W))
        _capi.check(lib, ctx, lib.sm_cost_calculate(ctx))
        for view in (0, 1):
            got = np.empty((H, W, md + 1), np.float32)
            _capi.check(lib, ctx, lib.sm_get_volume(ctx, view, _capi.ptr(got)))
            np.testing.assert_array_equal(bits(got), bits(oracle.cost_volume(pair, cfg, view=view)))
    finally:
        lib.sm_destroy(ctx)


@pytest.mark.parametrize("lam_g,trunc,adaptive,md", [(1.0, 500.0, 1, 23), (20.0, 500.0, 1, 23), (28.0, 500.0, 0, 70),
                                                     (30.0, 500.0, 1, 23), (60.0, 500.0, 1, 70), (1.0, 10.0, 1, 23),
                                                     (1.0, 20.0, 0, 99), (0.5, 3.0, 1, 23)])
def test_grad_cost_constants(oracle, lam_g, trunc, adaptive, md):
    """censusGrad cost volume of both views under lamG / gradient truncation / weighting choices
    on either side of the select-free kernel's bound (-0.999 T / lamG < -17.5, k_cost NOSEL)."""
    H, W = 19, 88
    pair = S.make_pair(H, W, md + 1, 90 + md)
    cfg = oracle.config(H, W, md, lam_g=lam_g, grad_trunc=trunc, grad_adaptive=adaptive)
    lib = _capi.load()
    p = _capi.default_params(md, H, W, aggregation=0, optimization=0, compute_right_view=1)
    p.lam_g, p.grad_trunc, p.grad_adaptive = lam_g, trunc, adaptive
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        a = {k: np.ascontiguousarray(pair[k]) for k in ("lbgr", "rbgr", "lgray", "rgray")}
        _capi.check(lib, ctx, lib.sm_set_images(ctx, _capi.ptr(a["lbgr"]), _capi.ptr(a["rbgr"]), W * 3,
                                                _capi.ptr(a["lgray"]), _capi.ptr(a["rgray"]), W))
        _capi.check(lib, ctx, lib.sm_cost_calculate(ctx))
        for view in (0, 1):
            got = np.empty((H, W, md + 1), np.float32)
            _capi.check(lib, ctx, lib.sm_get_volume(ctx, view, _capi.ptr(got)))
            np.testing.assert_array_equal(bits(got), bits(oracle.cost_volume(pair, cfg, view=view)))
    finally:
        lib.sm_destroy(ctx)


def _extreme_pair(H, W, md, seed):
    """Gray levels 0 / 255 only (every gradient at its bound: +-127.5 inside, +-255 on the border
    rows and columns), the right image a shifted copy with a few flipped pixels."""
    rng = np.random.default_rng(seed)
    lg = (rng.integers(0, 2, (H, W)) * 255).astype(np.uint8)
    rg = np.roll(lg, -min(md, W - 1) // 3, axis=1)
    flip = rng.random((H, W)) < 0.2
    rg = np.where(flip, 255 - rg, rg).astype(np.uint8)
    pair = {"lgray": lg, "rgray": rg,
            "lbgr": np.repeat(lg[:, :, None], 3, axis=2).copy(), "rbgr": np.repeat(rg[:, :, None], 3, axis=2).copy()}
    return pair


@pytest.mark.parametrize("trunc,adaptive,md,W", [(500.0, 1, 255, 300), (382.5, 1, 255, 300), (382.0, 1, 255, 300),
                                                  (700.0, 0, 255, 300), (900.0, 1, 191, 260), (500.0, 0, 127, 200),
                                                  (500.0, 1, 70, 120), (383.0, 1, 23, 64), (500.0, 1, 255, 2)])
def test_grad_cost_extremes(oracle, trunc, adaptive, md, W):
    """censusGrad cost volume on 0 / 255 images, whose gradients sit at their bounds, around the
    FAST elements' truncation bound (T >= 382.5, k_cost) and for T above the sentinel's range:
    both views, the unrolled D = 128 / 192 / 256 kernels, D > 64 and D <= 64, and a 2-pixel row."""
    H = 9
    pair = _extreme_pair(H, W, md, 7 + md + W)
    cfg = oracle.config(H, W, md, grad_trunc=trunc, grad_adaptive=adaptive)
    lib = _capi.load()
    p = _capi.default_params(md, H, W, aggregation=0, optimization=0, compute_right_view=1)
    p.grad_trunc, p.grad_adaptive = trunc, adaptive
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        a = {k: np.ascontiguousarray(pair[k]) for k in ("lbgr", "rbgr", "lgray", "rgray")}
        _capi.check(lib, ctx, lib.sm_set_images(ctx, _capi.ptr(a["lbgr"]), _capi.ptr(a["rbgr"]), W * 3,
                                                _capi.ptr(a["lgray"]), _capi.ptr(a["rgray"]), W))
        _capi.check(lib, ctx, lib.sm_cost_calculate(ctx))
        for view in (0, 1):
            got = np.empty((H, W, md + 1), np.float32)
            _capi.check(lib, ctx, lib.sm_get_volume(ctx, view, _capi.ptr(got)))
            np.testing.assert_array_equal(bits(got), bits(oracle.cost_volume(pair, cfg, view=view)))
    finally:
        lib.sm_destroy(ctx)


def test_right_view_volume(oracle):
    H, W, md = 33, 52, 19
    pair = S.make_pair(H, W, md + 1, 12)
    cfg = oracle.config(H, W, md)
    ref = oracle.cost_volume(pair, cfg, view=1)
    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = "censusGrad", "", ""
    lib = _capi.load()
    p = _capi.default_params(md, H, W, aggregation=0, optimization=0, compute_right_view=1)
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        a = {k: np.ascontiguousarray(pair[k]) for k in ("lbgr", "rbgr", "lgray", "rgray")}
        _capi.check(lib, ctx, lib.sm_set_images(ctx, _capi.ptr(a["lbgr"]), _capi.ptr(a["rbgr"]), W * 3,
                                                _capi.ptr(a["lgray"]), _capi.ptr(a["rgray"]), W))
        _capi.check(lib, ctx, lib.sm_cost_calculate(ctx))
        got = np.empty((H, W, md + 1), np.float32)
        _capi.check(lib, ctx, lib.sm_get_volume(ctx, 1, _capi.ptr(got)))
    finally:
        lib.sm_destroy(ctx)
    np.testing.assert_array_equal(bits(got), bits(ref))


@pytest.mark.parametrize("cost,md,paths", [("censusGrad", 63, 4), ("Census", 40, 8), ("ADCensus", 100, 4)])
def test_census_5x5_maps(oracle, cost, md, paths):
    """north_star's 5 x 5 census (census_rv = census_ru = 2, no ring bits: the generic census
    path, not the unrolled 7 x 9 + ring default): census codes of both views and the final maps
    through the whole pipeline, against the oracle."""
    H, W = 47, 133
    pair = S.make_pair(H, W, md + 1, 880 + md)
    cfg = oracle.config(H, W, md, cost=cost, census_rv=2, census_ru=2, census_ring=0, sgm_paths=paths)
    ref = oracle.run(pair, cfg, dumps=True)
    sb = StereoBatch(md, H, W, 1, cost_method=cost, census_rv=2, census_ru=2, census_ring=0, sgm_paths=paths,
                     keep_final_volume=1)
    try:
        sb.upload(*(pair[k][None] for k in ("lbgr", "rbgr", "lgray", "rgray")))
        np.testing.assert_array_equal(sb.run(0.3)[0], ref["disp"])
        got = np.empty((H, W, md + 1), np.float32)
        lib = _capi.load()
        _capi.check(lib, sb._ctx, lib.sm_get_volume(sb._ctx, 0, _capi.ptr(got)))
        np.testing.assert_array_equal(bits(got), bits(ref["final"]))
        for view, g in ((0, "lgray"), (1, "rgray")):
            codes = np.zeros((H, W, 2), np.uint64)
            _capi.check(lib, sb._ctx, lib.sm_get_census(sb._ctx, view, _capi.ptr(codes)))
            want = oracle.census(pair[g], cfg)
            np.testing.assert_array_equal(codes[..., :want.shape[2]], want)
    finally:
        sb.close()


def test_contexts_with_different_cost_constants(oracle):
    """Contexts on one device keep their own exponent tables (round-2 ADVICE: no __constant__ LUT
    shared across contexts): censusGrad with lamCen 13 and 5, ADCensus with lamCen 30 / lamAD 10
    and with 11 / 4, created together and run interleaved; each context's raw cost volume
    (gen_vm_from2vm_exp, cpp:3566-3590) and final map must equal the oracle's for ITS constants."""
    H, W, md = 33, 71, 31
    pair = S.make_pair(H, W, md + 1, 905)
    cases = [("censusGrad", dict(lam_cen=13.0)), ("censusGrad", dict(lam_cen=5.0)),
             ("ADCensus", dict(lam_cen_adc=30.0, lam_ad=10.0)), ("ADCensus", dict(lam_cen_adc=11.0, lam_ad=4.0))]
    lib = _capi.load()
    ctxs = []
    try:
        for cost, kw in cases:   # raw volumes: aggregation and SGM off (WTA keeps vm)
            ctxs.append(StereoBatch(md, H, W, 1, cost_method=cost, aggregation=0, optimization=0, **kw))
            ctxs.append(StereoBatch(md, H, W, 1, cost_method=cost, **kw))
        for sb in ctxs:
            sb.upload(*(pair[k][None] for k in ("lbgr", "rbgr", "lgray", "rgray")))
        for rnd in range(2):   # interleaved: a table left behind by another context would show
            for i, sb in enumerate(ctxs):
                cost, kw = cases[i // 2]
                if i % 2 == 0:
                    sb.run(0.3)
                    got = np.empty((H, W, md + 1), np.float32)
                    _capi.check(lib, sb._ctx, lib.sm_get_volume(sb._ctx, 0, _capi.ptr(got)))
                    # sm_run applies SolveAll's scale to the unaggregated volume: compare with the
                    # oracle's final volume of the same WTA-only pipeline
                    cfg = oracle.config(H, W, md, cost=cost, aggregation=0, optimization=0, **kw)
                    ref = oracle.run(pair, cfg, dumps=True)
                    np.testing.assert_array_equal(bits(got), bits(ref["final"]), err_msg=f"{cost} {kw}")
                    np.testing.assert_array_equal(sb.download()[0], ref["disp"])
                else:
                    cfg = oracle.config(H, W, md, cost=cost, **kw)
                    np.testing.assert_array_equal(sb.run(0.3)[0], oracle.run(pair, cfg)["disp"], err_msg=f"{cost} {kw}")
    finally:
        for sb in ctxs:
            sb.close()


def test_census_and_arms(oracle):
    H, W, md = 29, 45, 15
    pair = S.make_pair(H, W, md + 1, 13)
    cfg = oracle.config(H, W, md)
    sm = make_sm(pair, md)
    sm.costCalculate()
    for view, g, c in ((0, "lgray", "lbgr"), (1, "rgray", "rbgr")):
        codes = sm.census_codes(view)
        np.testing.assert_array_equal(codes, oracle.census(pair[g], cfg))
        np.testing.assert_array_equal(sm.HVL[view], oracle.arms(pair[c], cfg))


@pytest.mark.parametrize("L,L_out,cT,cT_out,minL", [(17, 34, 20, 6, 1), (5, 10, 12, 30, 2), (40, 80, 20, 6, 1),
                                                     (17, 64, 0, 255, 0), (0, 3, -1, 300, 1)])
def test_arm_parameters(oracle, L, L_out, cT, cT_out, minL):
    """Cross arms under other calHorVerDis arguments (cpp:5371): LDS-strip walks (L_out <= 64) and
    global-memory walks (L_out > 64), thresholds at the guard-bit test's ends, minL fallbacks."""
    H, W, md = 70, 90, 15
    pair = S.make_pair(H, W, md + 1, 33)
    for k in ("lbgr", "rbgr"):   # mix flat and textured regions so both long and short arms occur
        pair[k][: H // 2] = (pair[k][: H // 2] // 96 * 96).astype(np.uint8)
    pair["lgray"], pair["rgray"] = S.bgr_to_gray(pair["lbgr"]), S.bgr_to_gray(pair["rbgr"])
    cfg = oracle.config(H, W, md, arm_L=L, arm_L_out=L_out, arm_cT=cT, arm_cT_out=cT_out, arm_minL=minL)
    sm = make_sm(pair, md, cbca_crossL=[L, 0, 0], cbca_crossL_out=[L_out, 0, 0], cbca_cTresh=[cT, 0, 0],
                 cbca_cTresh_out=[cT_out, 0, 0], cbca_minArmL=minL)
    sm.costCalculate()
    for view, c in ((0, "lbgr"), (1, "rbgr")):
        np.testing.assert_array_equal(sm.HVL[view], oracle.arms(pair[c], cfg))
    ref = oracle.run(pair, cfg, dumps=True)
    np.testing.assert_array_equal(bits(sm.vm[0]), bits(ref["agg"]))


@pytest.mark.parametrize("H,W,L_out", [(5, 300, 34), (140, 70, 34), (67, 513, 64), (130, 260, 17), (66, 257, 0)])
def test_prep_tiles_arms_codes_flags(oracle, H, W, L_out):
    """The split prep (k_prep_h: 256 x 4 tiles, k_prep_v: 64 x 64 tiles) across several tiles in
    both directions: census codes and arms of both views, and the SGM penalty flags of all eight
    directions through the final 8-path volume."""
    md = 15
    pair = S.make_pair(H, W, md + 1, 70 + H)
    for k in ("lbgr", "rbgr"):   # flat and textured regions: arms of every length
        pair[k][: H // 2] = (pair[k][: H // 2] // 96 * 96).astype(np.uint8)
    pair["lgray"], pair["rgray"] = S.bgr_to_gray(pair["lbgr"]), S.bgr_to_gray(pair["rbgr"])
    L = min(17, L_out)
    cfg = oracle.config(H, W, md, sgm_paths=8, arm_L=L, arm_L_out=L_out)
    sm = make_sm(pair, md, paths=8, cbca_crossL=[L, 0, 0], cbca_crossL_out=[L_out, 0, 0])
    sm.costCalculate()
    for view, g, c in ((0, "lgray", "lbgr"), (1, "rgray", "rbgr")):
        np.testing.assert_array_equal(sm.census_codes(view), oracle.census(pair[g], cfg))
        np.testing.assert_array_equal(sm.HVL[view], oracle.arms(pair[c], cfg))
    ref = oracle.run(pair, cfg, dumps=True)
    np.testing.assert_array_equal(bits(sm.vm[0]), bits(ref["agg"]))
    _, agg, final, dp = run_reference_order(pair, md, paths=8, cbca_crossL=[L, 0, 0], cbca_crossL_out=[L_out, 0, 0])
    np.testing.assert_array_equal(bits(final), bits(ref["final"]))
    np.testing.assert_array_equal(dp, ref["disp"])


@pytest.mark.parametrize("H,W,md,paths", [(2, 2, 0, 4), (3, 70, 63, 4), (70, 3, 5, 8), (17, 23, 64, 8),
                                          (25, 31, 127, 4), (13, 90, 191, 8), (9, 40, 255, 4),
                                          (11, 37, 199, 8), (7, 30, 130, 4)])
def test_shapes_and_edge_cases(oracle, H, W, md, paths):
    """Tiny/ragged images, D not a multiple of 64 (or of 4), D > W, D = 1, 8 paths; every SGM
    kernel layout (rows for D <= 128, dwordx4 lanes for 128 < D <= 256 with D % 4 == 0, scalar lanes)."""
    pair = S.make_pair(H, W, md + 1, 14 + H)
    cfg = oracle.config(H, W, md, sgm_paths=paths)
    ref = oracle.run(pair, cfg, dumps=True)
    _, agg, final, dp = run_reference_order(pair, md, paths=paths)
    np.testing.assert_array_equal(bits(agg), bits(ref["agg"]))
    np.testing.assert_array_equal(bits(final), bits(ref["final"]))
    np.testing.assert_array_equal(dp, ref["disp"])


@pytest.mark.parametrize("H,W,md,paths", [(2, 2, 131, 4), (2, 9, 255, 4), (8, 8, 199, 4), (9, 17, 255, 4),
                                           (16, 24, 131, 4), (17, 33, 255, 4), (23, 7, 199, 4), (40, 41, 255, 4),
                                           (9, 17, 63, 4), (17, 10, 127, 4), (8, 8, 99, 4), (16, 9, 59, 4),
                                           (5, 13, 3, 4), (12, 19, 255, 8), (10, 11, 63, 8), (9, 9, 119, 8),
                                           (24, 32, 15, 4), (29, 41, 15, 4), (41, 67, 23, 4), (20, 90, 191, 8),
                                           (2, 2, 131, 8), (9, 17, 255, 8), (23, 7, 199, 8), (40, 41, 255, 8),
                                           (17, 33, 135, 8), (64, 5, 143, 8)])
def test_sgm_checkpointed_pairs(oracle, H, W, md, paths):
    """SGM with D % 4 == 0 runs paths 0 / 1 and 2 / 3 as checkpointed pairs (k_sgm_ck: segments of
    8 steps, 4 with 8 disparities per lane): one line per wave for 128 < D <= 256, four lines
    per wave below; lines shorter than, equal to and one longer than a segment, ragged tails, D
    below the layout's full width (lanes past D must enter every segment with FLT_MAX: the
    d + 1 neighbour of the last disparity — the shapes D = 16, 24 found that), 8 paths (the
    second pair adds into the running sum; with D > 128 the diagonal pair (4, 6) is checkpointed
    too, L5 stored between them: diagonals of 1 .. min(H, W) steps, H < W and H > W, the last
    path a sweep).  The summed volume (keep_final) and the map bit-exact, and the map
    again through the batch path (no final volume)."""
    pair = S.make_pair(H, W, md + 1, 50 + H + W)
    cfg = oracle.config(H, W, md, sgm_paths=paths)
    ref = oracle.run(pair, cfg, dumps=True)
    _, agg, final, dp = run_reference_order(pair, md, paths=paths)
    np.testing.assert_array_equal(bits(agg), bits(ref["agg"]))
    np.testing.assert_array_equal(bits(final), bits(ref["final"]))
    np.testing.assert_array_equal(dp, ref["disp"])
    sb = StereoBatch(md, H, W, 2, sgm_paths=paths)
    sb.upload(*(np.stack([pair[k], pair[k]]) for k in ("lbgr", "rbgr", "lgray", "rgray")))
    disp = sb.run(0.3)
    sb.close()
    np.testing.assert_array_equal(disp[0], ref["disp"])
    np.testing.assert_array_equal(disp[1], ref["disp"])


def test_flat_images_long_arms(oracle):
    """Uniform regions: arms saturate at L_out = 34, prefix sums run long."""
    H, W, md = 60, 90, 31
    pair = S.make_pair(H, W, md + 1, 20)
    for k in ("lbgr", "rbgr"):
        pair[k] = (pair[k] // 128 * 128).astype(np.uint8)
    pair["lgray"], pair["rgray"] = S.bgr_to_gray(pair["lbgr"]), S.bgr_to_gray(pair["rbgr"])
    cfg = oracle.config(H, W, md)
    ref = oracle.run(pair, cfg, dumps=True)
    _, agg, final, dp = run_reference_order(pair, md)
    np.testing.assert_array_equal(bits(agg), bits(ref["agg"]))
    np.testing.assert_array_equal(dp, ref["disp"])


def test_batch_matches_single_and_oracle(oracle):
    H, W, md, n = 48, 64, 31, 5
    b = S.make_batch(n, H, W, md + 1, first_index=30)
    sb = StereoBatch(md, H, W, n)
    sb.upload(b["lbgr"], b["rbgr"], b["lgray"], b["rgray"])
    disp = sb.run(0.3)
    disp2 = sb.run(0.3)
    np.testing.assert_array_equal(disp, disp2)  # deterministic
    cfg = oracle.config(H, W, md)
    for i in range(n):
        pair = {k: b[k][i] for k in ("lbgr", "rbgr", "lgray", "rgray")}
        np.testing.assert_array_equal(disp[i], oracle.run(pair, cfg)["disp"])
    sb.close()


def test_kitti_size_8path(oracle):
    """KITTI-2015 shape (configs[2]): 375x1242, D=192, 8-path SGM, bit-exact map."""
    H, W, md = 375, 1242, 191
    pair = S.make_pair(H, W, md + 1, 40)
    cfg = oracle.config(H, W, md, sgm_paths=8)
    ref = oracle.run(pair, cfg)
    sb = StereoBatch(md, H, W, 1, sgm_paths=8)
    sb.upload(pair["lbgr"][None], pair["rbgr"][None], pair["lgray"][None], pair["rgray"][None])
    disp = sb.run(0.3)[0]
    np.testing.assert_array_equal(disp, ref["disp"])
    sb.close()


def test_device_expf_exhaustive(oracle):
    """Device expf == host libm expf on every negative float down to the underflow bound."""
    lib = _capi.load()
    p = _capi.default_params(15, 8, 8)
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        first, last = 0x80000000, 0xC2D00000
        chunk = 1 << 25
        out = np.empty(chunk, np.float32)
        b = first
        bad = 0
        while b <= last:
            n = min(chunk, last - b + 1)
            _capi.check(lib, ctx, lib.sm_expf_device_range(ctx, b, n, _capi.ptr(out)))
            ref = oracle.expf_range(b, n)
            bad += int(np.count_nonzero(out[:n].view(np.uint32) != ref.view(np.uint32)))
            b += n
        assert bad == 0
    finally:
        lib.sm_destroy(ctx)


@pytest.mark.parametrize("exp2", [0, -110, -60, 40, 120])
def test_div_area_exhaustive(exp2):
    """CBCA's 4-instruction area division equals IEEE a / b for every mantissa of a at the
    exponent and every area b up to the largest a config allows ((2*84+1)^2 = 28561; the default
    arms give 4761).  Exponents >= -110 behave alike (no underflow), so exponent 0 with all b is
    the proof's check; the others sample the range ends."""
    lib = _capi.load()
    p = _capi.default_params(15, 8, 8)
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        bad = C.c_uint64(0)
        bmax = 28561 if exp2 == 0 else 4761
        _capi.check(lib, ctx, lib.sm_div_area_check(ctx, exp2, bmax, C.byref(bad)))
        assert bad.value == 0
    finally:
        lib.sm_destroy(ctx)


def test_state_errors():
    lib = _capi.load()
    p = _capi.default_params(15, 16, 16)
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        assert lib.sm_cost_calculate(ctx) == _capi.SM_ESTATE
        assert lib.sm_disp_optimize(ctx, None) == _capi.SM_ESTATE
        assert b"must follow" in lib.sm_last_error(ctx)
        a = np.zeros((16, 16, 3), np.uint8)
        g = np.zeros((16, 16), np.uint8)
        assert lib.sm_set_images(ctx, _capi.ptr(a), _capi.ptr(a), 16, _capi.ptr(g), _capi.ptr(g), 16) == _capi.SM_EINVAL
        assert lib.sm_set_images(ctx, _capi.ptr(a), _capi.ptr(a), 48, _capi.ptr(g), _capi.ptr(g), 16) == _capi.SM_OK
        assert lib.sm_solve_all(ctx, 1, 0.3) == _capi.SM_ESTATE
        assert lib.sm_cost_calculate(ctx) == _capi.SM_OK
        assert lib.sm_solve_all(ctx, 2, 0.3) == _capi.SM_EINVAL
    finally:
        lib.sm_destroy(ctx)


@pytest.mark.parametrize("iters,md", [(1, 40), (2, 40), (3, 70), (4, 130), (2, 255)])
def test_fuse_norm_scan_volume(oracle, iters, md):
    """sm_params.fuse_norm_scan = 1: iteration k's normalising sweep and iteration k+1's scan run
    as one CB_NORM_SCAN sweep (two prefix rings).  The aggregated volume (cbca_core,
    cpp:5585-5666) and the map must equal the oracle's bit for bit for 1-4 iterations (0-3 fused
    sweeps, both directions) and D up to 256."""
    H, W = 37, 61
    pair = S.make_pair(H, W, md + 1, 500 + iters)
    cfg = oracle.config(H, W, md, cbca_iters=iters)
    ref = oracle.run(pair, cfg, dumps=True)
    lib = _capi.load()
    p = _capi.default_params(md, H, W, cbca_iterations=iters, fuse_norm_scan=1, keep_final_volume=1)
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        a = {k: np.ascontiguousarray(pair[k]) for k in ("lbgr", "rbgr", "lgray", "rgray")}
        _capi.check(lib, ctx, lib.sm_set_images(ctx, _capi.ptr(a["lbgr"]), _capi.ptr(a["rbgr"]), W * 3,
                                                _capi.ptr(a["lgray"]), _capi.ptr(a["rgray"]), W))
        _capi.check(lib, ctx, lib.sm_cost_calculate(ctx))
        got = np.empty((H, W, md + 1), np.float32)
        _capi.check(lib, ctx, lib.sm_get_volume(ctx, 0, _capi.ptr(got)))
        np.testing.assert_array_equal(bits(got), bits(ref["agg"]))
        _capi.check(lib, ctx, lib.sm_solve_all(ctx, 1, 0.3))
        dp = np.empty((H, W), np.int16)
        _capi.check(lib, ctx, lib.sm_disp_optimize(ctx, _capi.ptr(dp)))
        np.testing.assert_array_equal(dp, ref["disp"])
    finally:
        lib.sm_destroy(ctx)


def test_fuse_norm_scan_batch_and_right_view(oracle):
    """fuse_norm_scan through sm_run: batched pairs with Do_refine (the right view's CBCA runs the
    RV instantiation of the fused sweep), maps equal to the oracle's refined maps."""
    H, W, md, n = 45, 70, 31, 3
    b = S.make_batch(n, H, W, md + 1, first_index=520)
    sb = StereoBatch(md, H, W, n, fuse_norm_scan=1, do_refine=1)
    try:
        sb.upload(b["lbgr"], b["rbgr"], b["lgray"], b["rgray"])
        disp = sb.run(0.3)
    finally:
        sb.close()
    cfg = oracle.config(H, W, md, do_refine=1)
    for i in range(n):
        pair = {k: b[k][i] for k in ("lbgr", "rbgr", "lgray", "rgray")}
        np.testing.assert_array_equal(disp[i], oracle.run_ex(pair, cfg)["disp"])


@pytest.mark.parametrize("H,W,md,iters,fuse,refine", [
    (200, 90, 63, 2, 1, 0), (200, 90, 63, 1, 1, 0), (160, 150, 127, 3, 1, 0), (150, 120, 63, 4, 1, 0),
    (130, 110, 63, 4, 0, 0), (90, 140, 191, 2, 1, 1), (70, 75, 255, 2, 0, 1), (40, 300, 63, 2, 1, 0),
    # the shipping two-wave V sweep (k_cbca_nsv2, both views through Do_refine) on lines shorter
    # than 2 lag + T = 75 rows: every tile's arm rows run past the line end into the tail pad
    # (the round-5 work-in-progress fault), D = 256 and 128, iteration 0 (no
    # tiny-dividend test) and iteration 2 (with it)
    (2, 96, 255, 2, 1, 1), (8, 96, 255, 3, 1, 1), (40, 96, 255, 2, 1, 1), (68, 96, 255, 3, 1, 1),
    (2, 80, 127, 3, 1, 1), (8, 80, 127, 2, 1, 1), (40, 80, 127, 3, 1, 1), (68, 80, 127, 2, 1, 1)])
def test_fast_sweeps_lag34(oracle, H, W, md, iters, fuse, refine):
    """The dedicated CBCA sweeps at the reference's lag (34) and whole 64-disparity chunks: the V
    NORM_SCAN sweep (NsV: iteration 0 without the tiny-dividend test, later iterations with it)
    and the H normalising sweep (HNorm, with and without SolveAll's scale), both views, lines
    long enough for steady tiles and lines shorter than the lag.  The aggregated volume
    (cbca_core, cpp:5585-5666) and the maps must equal the oracle's bit for bit."""
    pair = S.make_pair(H, W, md + 1, 960 + iters * 7 + md)
    cfg = oracle.config(H, W, md, cbca_iters=iters, do_refine=refine)
    lib = _capi.load()
    p = _capi.default_params(md, H, W, cbca_iterations=iters, fuse_norm_scan=fuse, keep_final_volume=1,
                             do_refine=refine)
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        a = {k: np.ascontiguousarray(pair[k]) for k in ("lbgr", "rbgr", "lgray", "rgray")}
        _capi.check(lib, ctx, lib.sm_set_images(ctx, _capi.ptr(a["lbgr"]), _capi.ptr(a["rbgr"]), W * 3,
                                                _capi.ptr(a["lgray"]), _capi.ptr(a["rgray"]), W))
        _capi.check(lib, ctx, lib.sm_cost_calculate(ctx))
        ref = oracle.run_ex(pair, cfg, dumps=("agg", "agg_right") if refine else ("agg",))
        for view in ((0, 1) if refine else (0,)):
            got = np.empty((H, W, md + 1), np.float32)
            _capi.check(lib, ctx, lib.sm_get_volume(ctx, view, _capi.ptr(got)))
            np.testing.assert_array_equal(bits(got), bits(ref["agg" if view == 0 else "agg_right"]), err_msg=f"view {view}")
        _capi.check(lib, ctx, lib.sm_solve_all(ctx, 1, 0.3))
        dp = np.empty((H, W), np.int16)
        _capi.check(lib, ctx, lib.sm_disp_optimize(ctx, _capi.ptr(dp)))
        if refine:
            _capi.check(lib, ctx, lib.sm_refine(ctx, _capi.ptr(dp)))
        np.testing.assert_array_equal(dp, ref["disp"])
    finally:
        lib.sm_destroy(ctx)
    # the batched path fuses SolveAll into the last (H) normalising sweep
    sb = StereoBatch(md, H, W, 2, cbca_iterations=iters, fuse_norm_scan=fuse, do_refine=refine)
    try:
        b = S.make_batch(2, H, W, md + 1, first_index=990 + iters)
        sb.upload(b["lbgr"], b["rbgr"], b["lgray"], b["rgray"])
        got = sb.run(0.3)
        for i in range(2):
            pr = {k: b[k][i] for k in ("lbgr", "rbgr", "lgray", "rgray")}
            np.testing.assert_array_equal(got[i], oracle.run_ex(pr, cfg)["disp"], err_msg=f"pair {i}")
    finally:
        sb.close()
