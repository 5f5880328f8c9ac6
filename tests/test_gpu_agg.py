"""GPU parity of the alternative aggregators against the CPU restatement, bit for bit.

"GF": guideFilter (stereoMatching.cpp:4492-4516), r = 9, eps = 1e-4, in the shipped build's form
(cv::ximgproc::guidedFilter, cpp:4513, the default) and the MY_GUIDE form (guideFilterCore_matlab,
cpp:4975-5104, with the reference's BoxFilter / CumSum, cpp:5107-5202); its costs can be negative,
so SGM runs its float-minimum variant.  "NL": NL() (cpp:4892-4917),
the MST tree filter of NL/ (spanning trees by Boruvka rounds on the GPU -- the same tree as the
reference's Kruskal -- walked on host threads, filter on the GPU).
PARITY UNPINNED (the oracle restates the reference text; tests/test_oracle_agg.py cross-checks
it against an independent numpy restatement).
"""
import numpy as np
import pytest

from mystereomatching_amd import SolveAll, StereoBatch, StereoMatching, _capi
from mystereomatching_amd import synthetic as S

pytestmark = pytest.mark.gpu

KEYS = ("lbgr", "rbgr", "lgray", "rgray")
AGG = {"GF": 2, "NL": 3}


def _gf_mode():
    """The library's default guideFilter form (sm_params_default): the oracle is configured alike."""
    return _capi.default_params(15, 32, 32).gf_mode


def ocfg(oracle, H, W, md, **kw):
    return oracle.config(H, W, md, gf_mode=_gf_mode(), **kw)


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _agg_volume(pair, H, W, md, agg, cost="censusGrad"):
    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = cost, agg, "sgm"
    try:
        sm = StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], None, None, None, None,
                            StereoMatching.Parameters(md, H, W), device=0)
        sm.costCalculate()
        return sm.vm[0]
    finally:
        StereoMatching.aggregation = "CBCA"
        StereoMatching.costcalculation = "censusGrad"


@pytest.mark.parametrize("agg", ["GF", "NL"])
@pytest.mark.parametrize("H,W,md,idx", [(24, 30, 7, 500), (40, 61, 63, 501), (33, 47, 69, 502), (21, 19, 255, 503)])
def test_aggregated_volume_bits(oracle, agg, H, W, md, idx):
    pair = S.make_pair(H, W, md + 1, idx)
    cfg = ocfg(oracle, H, W, md)
    vm = oracle.cost_volume(pair, cfg)
    want = oracle.guided_filter(vm, pair["lbgr"], cfg) if agg == "GF" else oracle.nl_aggregate(vm, pair["lbgr"], cfg)
    got = _agg_volume(pair, H, W, md, agg)
    np.testing.assert_array_equal(bits(got), bits(want))


@pytest.mark.parametrize("H,W,md,idx", [(3, 3, 4, 560), (3, 90, 15, 561), (90, 3, 15, 562), (4, 257, 63, 563),
                                        (130, 5, 70, 564)])
def test_nl_thin_images(oracle, H, W, md, idx):
    """NL on the thinnest images ctmf allows (3 rows or columns) and long single paths: the GPU
    tree walk (Euler tour ranking, heavy-first preorder, path tables) and both filter kernels
    (block rounds and producer / consumer rounds, partial last chunks) against the restatement."""
    pair = S.make_pair(H, W, md + 1, idx)
    cfg = ocfg(oracle, H, W, md)
    vm = oracle.cost_volume(pair, cfg)
    want = oracle.nl_aggregate(vm, pair["lbgr"], cfg)
    got = _agg_volume(pair, H, W, md, "NL")
    np.testing.assert_array_equal(bits(got), bits(want))


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("H,W,md,idx", [(24, 30, 7, 540), (40, 61, 63, 541), (19, 23, 255, 542), (9, 12, 20, 543),
                                        (11, 9, 64, 544), (33, 70, 130, 545)])
def test_gf_modes_volume_bits(oracle, mode, H, W, md, idx):
    """Both guideFilter builds through the C ABI: gf_mode 0 = ximgproc::guidedFilter (the shipped
    build, sm_gf_cv.hip; images down to 9 x 9, the reflected border's minimum) and 1 = MY_GUIDE
    (sm_gf.hip; 19 x 19 minimum), D up to 256 and ragged, left and right views."""
    import ctypes as C
    if mode == 1 and min(H, W) < 19:
        pytest.skip("MY_GUIDE needs 19 x 19")
    pair = S.make_pair(H, W, md + 1, idx)
    cfg = oracle.config(H, W, md, gf_mode=mode)
    lib = _capi.load()
    p = _capi.default_params(md, H, W, aggregation=2, optimization=0, gf_mode=mode, do_refine=1)
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        a = {k: np.ascontiguousarray(pair[k]) for k in KEYS}
        _capi.check(lib, ctx, lib.sm_set_images(ctx, _capi.ptr(a["lbgr"]), _capi.ptr(a["rbgr"]), W * 3,
                                                _capi.ptr(a["lgray"]), _capi.ptr(a["rgray"]), W))
        _capi.check(lib, ctx, lib.sm_cost_calculate(ctx))
        for view, img in ((0, "lbgr"), (1, "rbgr")):
            got = np.empty((H, W, md + 1), np.float32)
            _capi.check(lib, ctx, lib.sm_get_volume(ctx, view, _capi.ptr(got)))
            want = oracle.guided_filter(oracle.cost_volume(pair, cfg, view=view), pair[img], cfg)
            np.testing.assert_array_equal(bits(got), bits(want))
    finally:
        lib.sm_destroy(ctx)


@pytest.mark.parametrize("agg", ["GF", "NL"])
@pytest.mark.parametrize("H,W,md,paths,cost", [(48, 64, 31, 4, "censusGrad"), (37, 70, 15, 8, "Census"),
                                               (30, 44, 127, 4, "censusGrad"),
                                               (21, 30, 199, 4, "censusGrad"),    # checkpointed SGM pairs (GF: signed)
                                               (19, 26, 159, 8, "censusGrad")])   # + the diagonal pair (4, 6)
def test_batch_maps_match_oracle(oracle, agg, H, W, md, paths, cost):
    n = 3
    batch = S.make_batch(n, H, W, md + 1, first_index=510)
    sb = StereoBatch(md, H, W, n, device=0, aggregation=AGG[agg], sgm_paths=paths, cost_method=cost)
    try:
        sb.upload(*(batch[k] for k in KEYS))
        got = sb.run(0.3)
    finally:
        sb.close()
    cfg = ocfg(oracle, H, W, md, cost=cost, aggregation=AGG[agg], sgm_paths=paths)
    for i in range(n):
        want = oracle.run({k: batch[k][i] for k in KEYS}, cfg)["disp"]
        np.testing.assert_array_equal(got[i], want)


@pytest.mark.parametrize("agg", ["GF", "NL"])
def test_with_refine_both_views(oracle, agg):
    """Do_refine: guideFilter runs on both views (num = 2, cpp:4499) with each view's colours; NL
    aggregates vm[0] only, so in sm_run SolveAll is fused into its output for view 0 and a separate
    pass for view 1."""
    H, W, md = 40, 56, 23
    pair = S.make_pair(H, W, md + 1, 520)
    sb = StereoBatch(md, H, W, 1, device=0, aggregation=AGG[agg], do_refine=1)
    try:
        sb.upload(*(pair[k][None] for k in KEYS))
        got = sb.run(0.3)[0]
    finally:
        sb.close()
    want = oracle.run(pair, ocfg(oracle, H, W, md, aggregation=AGG[agg], do_refine=1))["disp"]
    np.testing.assert_array_equal(got, want)


def test_reference_ordered_api_nl(oracle):
    H, W, md = 36, 50, 31
    pair = S.make_pair(H, W, md + 1, 530)
    StereoMatching.aggregation = "NL"
    try:
        sm = StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], None, None, None, None,
                            StereoMatching.Parameters(md, H, W), device=0)
        sm.costCalculate()
        SolveAll([sm], 1, 0.3)
        got = sm.dispOptimize()
    finally:
        StereoMatching.aggregation = "CBCA"
    np.testing.assert_array_equal(got, oracle.run(pair, ocfg(oracle, H, W, md, aggregation=3))["disp"])


@pytest.mark.parametrize("agg", ["GF", "NL"])
def test_teddy_size_maps(oracle, agg):
    """BASELINE configs[1] shape (450x375, D = 64) with GF / NL in place of CBCA."""
    H, W, md = 375, 450, 63
    pair = S.make_pair(H, W, md + 1, 0)
    sb = StereoBatch(md, H, W, 1, device=0, aggregation=AGG[agg])
    try:
        sb.upload(*(pair[k][None] for k in KEYS))
        got = sb.run(0.3)[0]
    finally:
        sb.close()
    want = oracle.run(pair, ocfg(oracle, H, W, md, aggregation=AGG[agg]))["disp"]
    np.testing.assert_array_equal(got, want)


def test_nl_teddy_batch_all_round_kernels(oracle):
    """Two Teddy-size pairs in one batch: the first up / down rounds then hold >= 64 K (path, chunk)
    units and run the 2-node block kernel, the middle rounds the 4-node one and the long-path
    rounds the producer / consumer workgroups -- all three filter kernels, both maps bit-exact."""
    H, W, md, n = 375, 450, 63, 2
    batch = S.make_batch(n, H, W, md + 1, first_index=20)
    sb = StereoBatch(md, H, W, n, device=0, aggregation=AGG["NL"])
    try:
        sb.upload(*(batch[k] for k in KEYS))
        got = sb.run(0.3)
    finally:
        sb.close()
    cfg = ocfg(oracle, H, W, md, aggregation=AGG["NL"])
    for i in range(n):
        pair = {k: batch[k][i] for k in KEYS}
        np.testing.assert_array_equal(got[i], oracle.run(pair, cfg)["disp"])


@pytest.mark.parametrize("agg", ["GF", "NL"])
@pytest.mark.parametrize("sub_batch,num_streams", [(2, 2), (1, 3), (2, 1)])
def test_sub_batches_and_streams(oracle, agg, sub_batch, num_streams):
    """Groups of pairs on alternating streams (sm_params.sub_batch / num_streams) only reschedule
    sm_run: GF's scratch is per pair, NL's trees, records and staging are shared by the groups and
    reused across runs — the maps of both runs must equal the oracle's."""
    H, W, md, n = 29, 41, 15, 5
    batch = S.make_batch(n, H, W, md + 1, first_index=530)
    sb = StereoBatch(md, H, W, n, device=0, aggregation=AGG[agg], sub_batch=sub_batch, num_streams=num_streams)
    try:
        sb.upload(*(batch[k] for k in KEYS))
        first = sb.run(0.3)
        second = sb.run(0.3)
    finally:
        sb.close()
    cfg = ocfg(oracle, H, W, md, aggregation=AGG[agg])
    for i in range(n):
        np.testing.assert_array_equal(first[i], oracle.run({k: batch[k][i] for k in KEYS}, cfg)["disp"])
    np.testing.assert_array_equal(second, first)


def test_nl_pipelined_calls_and_new_inputs(oracle):
    """NL's front (median, edge weights, spanning trees) runs on its own stream and the host walks
    a call's trees while the GPU still runs the previous call: runs queued back to back without
    downloads, then new images uploaded and run again, must give the oracle's maps for the images
    each run saw."""
    H, W, md, n = 31, 43, 15, 4
    a = S.make_batch(n, H, W, md + 1, first_index=560)
    b = S.make_batch(n, H, W, md + 1, first_index=570)
    sb = StereoBatch(md, H, W, n, device=0, aggregation=AGG["NL"])
    try:
        sb.upload(*(a[k] for k in KEYS))
        for _ in range(3):
            sb.run(0.3, download=False)
        got_a = sb.download()
        sb.upload(*(b[k] for k in KEYS))
        for _ in range(2):
            sb.run(0.3, download=False)
        got_b = sb.download()
    finally:
        sb.close()
    cfg = ocfg(oracle, H, W, md, aggregation=AGG["NL"])
    for i in range(n):
        np.testing.assert_array_equal(got_a[i], oracle.run({k: a[k][i] for k in KEYS}, cfg)["disp"])
        np.testing.assert_array_equal(got_b[i], oracle.run({k: b[k][i] for k in KEYS}, cfg)["disp"])
