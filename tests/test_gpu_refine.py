"""GPU parity of the refine() path (Do_refine = 1) against the CPU oracle.

Covers: the right view's CBCA volume (cbca_core LOR = 1, cpp:5598-5622), DP[1] from SGM with the
right image's penalties (leftFirst = false, h:2219-2224), and refine() (cpp:1347-1510): LR check,
region votes, proper interpolation, 3x3 median — all bit-exact / int16-exact.
"""
import numpy as np
import pytest

from mystereomatching_amd import StereoBatch, StereoMatching, SolveAll
from mystereomatching_amd import synthetic as S

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def smooth(p, q=64):
    for k in ("lbgr", "rbgr"):
        p[k] = (p[k] // q * q).astype(np.uint8)
    p["lgray"], p["rgray"] = S.bgr_to_gray(p["lbgr"]), S.bgr_to_gray(p["rbgr"])
    return p


def make(pair, md, paths=4, cost="censusGrad", agg="CBCA", opt="sgm", switches=(True, True, True)):
    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = cost, agg, opt
    StereoMatching.Do_refine = True
    StereoMatching.Do_regionVote, StereoMatching.Do_properIpol, StereoMatching.Do_lastMedianBlur = switches
    try:
        H, W = pair["lgray"].shape
        prm = StereoMatching.Parameters(md, H, W)
        prm.sgm_scanNum = paths
        return StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], None, None, None, None, prm)
    finally:
        StereoMatching.Do_refine = False
        StereoMatching.Do_regionVote = StereoMatching.Do_properIpol = StereoMatching.Do_lastMedianBlur = True


@pytest.mark.parametrize("H,W,md,idx,sm_q,paths", [
    (37, 53, 15, 1, 0, 4), (48, 70, 23, 2, 64, 4), (40, 90, 63, 3, 32, 4),
    (33, 100, 64, 4, 0, 8), (30, 47, 127, 5, 64, 4), (24, 20, 31, 6, 0, 4),   # D > W
])
def test_refine_pipeline_reference_order(oracle, H, W, md, idx, sm_q, paths):
    pair = S.make_pair(H, W, md + 1, 40 + idx)
    if sm_q:
        pair = smooth(pair, sm_q)
    cfg = oracle.config(H, W, md, do_refine=1, sgm_paths=paths)
    ref = oracle.run_ex(pair, cfg, dumps=("agg", "agg_right", "disp_raw", "disp_right"))
    sm = make(pair, md, paths)
    sm.costCalculate()
    vm = sm.vm
    np.testing.assert_array_equal(bits(vm[0]), bits(ref["agg"]))
    np.testing.assert_array_equal(bits(vm[1]), bits(ref["agg_right"]))
    SolveAll([sm], 1, 0.3)
    sm.dispOptimize()
    np.testing.assert_array_equal(sm.DP[0], ref["disp_raw"])
    np.testing.assert_array_equal(sm.DP[1], ref["disp_right"])
    dp = sm.refine()
    np.testing.assert_array_equal(dp, ref["disp"])
    assert (ref["disp"] != ref["disp_raw"]).any()   # refine did something


@pytest.mark.parametrize("switches", [(False, True, True), (True, False, True), (True, True, False), (False, False, False)])
def test_refine_stage_switches(oracle, switches):
    H, W, md = 44, 61, 19
    pair = smooth(S.make_pair(H, W, md + 1, 77), 64)
    cfg = oracle.config(H, W, md, do_refine=1, do_region_vote=int(switches[0]), do_proper_ipol=int(switches[1]),
                        do_last_median=int(switches[2]))
    ref = oracle.run_ex(pair, cfg)
    sm = make(pair, md, switches=switches)
    sm.costCalculate()
    SolveAll([sm], 1, 0.3)
    sm.dispOptimize()
    np.testing.assert_array_equal(sm.refine(), ref["disp"])


def _noisy_map(H, W, D, seed, invalid, occ=False):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, D, size=(H // 6 + 1, W // 6 + 1))
    dp = np.kron(base, np.ones((6, 6), np.int64))[:H, :W]
    dp = np.where(rng.random((H, W)) < invalid, -32 if occ else -1, dp)
    if occ:
        dp = np.where(rng.random((H, W)) < 0.1, -1, dp)
    return dp.astype(np.int16)


@pytest.mark.parametrize("seed,invalid,occ,flat", [(0, 0.1, False, False), (1, 0.4, False, True), (2, 0.6, True, False),
                                                   (3, 0.3, True, True)])
def test_refine_on_given_maps(oracle, seed, invalid, occ, flat):
    """DP[0] / DP[1] overwritten (public members, h:2724) with synthetic maps, then refine()."""
    H, W, md = 52, 83, 15
    pair = S.make_pair(H, W, md + 1, 90 + seed)
    if flat:   # long arms: large vote regions
        pair = smooth(pair, 128)
    cfg = oracle.config(H, W, md, do_refine=1)
    sm = make(pair, md)
    sm.costCalculate()
    SolveAll([sm], 1, 0.3)
    sm.dispOptimize()
    d0 = _noisy_map(H, W, md + 1, seed, invalid, occ)
    d1 = _noisy_map(H, W, md + 1, seed + 50, 0.05)
    d0[:, ::7] = d1[:, ::7]   # some LR-consistent pixels survive the check
    lib, ctx = sm._lib, sm._ctx
    from mystereomatching_amd import _capi
    for view, m in ((0, d0), (1, d1)):
        _capi.check(lib, ctx, lib.sm_set_disp(ctx, view, _capi.ptr(np.ascontiguousarray(m))), "set_disp")
    got = sm.refine()
    aL = oracle.arms(pair["lbgr"], cfg)
    np.testing.assert_array_equal(got, oracle.refine(d0, d1, aL, pair["lbgr"], cfg))
    # and the LR check alone (other stages off)
    cfg2 = oracle.config(H, W, md, do_refine=1, do_region_vote=0, do_proper_ipol=0, do_last_median=0)
    sm2 = make(pair, md, switches=(False, False, False))
    sm2.costCalculate()
    SolveAll([sm2], 1, 0.3)
    sm2.dispOptimize()
    for view, m in ((0, d0), (1, d1)):
        _capi.check(sm2._lib, sm2._ctx, sm2._lib.sm_set_disp(sm2._ctx, view, _capi.ptr(np.ascontiguousarray(m))), "")
    np.testing.assert_array_equal(sm2.refine(), oracle.lr_check(d0, d1, cfg2))


def test_refine_batch_matches_oracle(oracle):
    H, W, md, n = 45, 72, 31, 5
    pairs = [smooth(S.make_pair(H, W, md + 1, 200 + i), 32 if i % 2 else 1) for i in range(n)]
    st = {k: np.stack([p[k] for p in pairs]) for k in ("lbgr", "rbgr", "lgray", "rgray")}
    b = StereoBatch(md, H, W, n, do_refine=1)
    b.upload(st["lbgr"], st["rbgr"], st["lgray"], st["rgray"])
    out = b.run()
    out2 = b.run()
    np.testing.assert_array_equal(out, out2)
    cfg = oracle.config(H, W, md, do_refine=1)
    for i, p in enumerate(pairs):
        np.testing.assert_array_equal(out[i], oracle.run_ex(p, cfg)["disp"], err_msg=f"pair {i}")


def test_refine_errors():
    H, W, md = 20, 30, 7
    pair = S.make_pair(H, W, md + 1, 3)
    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = "censusGrad", "CBCA", "sgm"
    prm = StereoMatching.Parameters(md, H, W)
    sm = StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], None, None, None, None, prm)
    sm.costCalculate()
    SolveAll([sm], 1, 0.3)
    sm.dispOptimize()
    with pytest.raises(Exception, match="do_refine"):
        sm.refine()
    sm2 = make(pair, md)
    sm2.costCalculate()
    with pytest.raises(Exception, match="must follow"):
        sm2.refine()
