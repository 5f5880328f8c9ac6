"""GPU: the two-pass 4-path SGM (sm_sgm2.hip, opt-in through sm_params.sgm_2pass = 1 for D = 64 / 128 /
256: measured slower than the four path sweeps) against the oracle and against the four
path sweeps (sgm_2pass = 0, the default), bit for bit.

Pass A computes the paths r = (+1,0) and (0,+1) (L0, L2), pass B the paths (-1,0) and (0,-1)
(L1, L3), the sum (((0 + L0) + L1) + L2) + L3 and the WTA (sgm / costScan / gen_sgm_vm /
gen_dispFromVm, stereoMatching.cpp:6204-6224, 1983-2056, 3928-3967; updateCost h:2206-2280).
Strips of 8 rows hand the vertical paths to each other through global memory with progress
counters; the shapes below cover one strip, partial last strips, many strips, one- and two-column
tiles, several pairs (the strips of all pairs interleave in the ticket order), the guided filter's
signed costs and the right view of Do_refine.
"""
import numpy as np
import pytest

from mystereomatching_amd import StereoBatch
from mystereomatching_amd import synthetic as S

pytestmark = pytest.mark.gpu

KEYS = ("lbgr", "rbgr", "lgray", "rgray")


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _run(batch, md, H, W, n, **kw):
    kw.setdefault("sgm_2pass", 1)
    sb = StereoBatch(md, H, W, n, device=0, **kw)
    try:
        sb.upload(*(batch[k] for k in KEYS))
        return sb.run(0.3)
    finally:
        sb.close()


@pytest.mark.parametrize("H,W,md,n", [(2, 5, 63, 1), (7, 33, 63, 2), (8, 40, 127, 1), (9, 2, 63, 3), (17, 3, 255, 2),
                                      (40, 57, 63, 3), (65, 31, 255, 1), (24, 70, 127, 2), (100, 23, 63, 2)])
def test_two_pass_maps_match_oracle_and_path_sweeps(oracle, H, W, md, n):
    batch = S.make_batch(n, H, W, md + 1, first_index=600 + H)
    two = _run(batch, md, H, W, n)
    four = _run(batch, md, H, W, n, sgm_2pass=0)
    np.testing.assert_array_equal(two, four)
    cfg = oracle.config(H, W, md)
    for i in range(n):
        np.testing.assert_array_equal(two[i], oracle.run({k: batch[k][i] for k in KEYS}, cfg)["disp"])


@pytest.mark.parametrize("md", [63, 127, 255])
def test_two_pass_summed_volume_bits(oracle, md):
    """keep_final_volume = 1: pass B writes the path sum back into vm (gen_sgm_vm, cpp:2031-2056)."""
    import ctypes as C
    from mystereomatching_amd import _capi
    H, W = 29, 47
    pair = S.make_pair(H, W, md + 1, 640 + md)
    ref = oracle.run(pair, oracle.config(H, W, md), dumps=True)
    lib = _capi.load()
    p = _capi.default_params(md, H, W, keep_final_volume=1)
    p.sgm_2pass = 1
    ctx = C.c_void_p()
    _capi.check(lib, ctx, lib.sm_create(C.byref(ctx), C.byref(p), 0))
    try:
        a = {k: np.ascontiguousarray(pair[k]) for k in KEYS}
        _capi.check(lib, ctx, lib.sm_set_images(ctx, _capi.ptr(a["lbgr"]), _capi.ptr(a["rbgr"]), W * 3,
                                                _capi.ptr(a["lgray"]), _capi.ptr(a["rgray"]), W))
        _capi.check(lib, ctx, lib.sm_cost_calculate(ctx))
        _capi.check(lib, ctx, lib.sm_solve_all(ctx, 1, 0.3))
        dp = np.empty((H, W), np.int16)
        _capi.check(lib, ctx, lib.sm_disp_optimize(ctx, _capi.ptr(dp)))
        vol = np.empty((H, W, md + 1), np.float32)
        _capi.check(lib, ctx, lib.sm_get_volume(ctx, 0, _capi.ptr(vol)))
    finally:
        lib.sm_destroy(ctx)
    np.testing.assert_array_equal(dp, ref["disp"])
    np.testing.assert_array_equal(bits(vol), bits(ref["final"]))


@pytest.mark.parametrize("agg,refine", [(2, 0), (1, 1), (2, 1)])
def test_two_pass_signed_costs_and_right_view(oracle, agg, refine):
    """GF's costs can be negative (float minima, SIGNED instantiation); Do_refine runs both views'
    SGM (the right view with the right image's penalty flags) before refine()."""
    H, W, md, n = 30, 44, 63, 2
    batch = S.make_batch(n, H, W, md + 1, first_index=660 + agg)
    two = _run(batch, md, H, W, n, aggregation=agg, do_refine=refine)
    four = _run(batch, md, H, W, n, aggregation=agg, do_refine=refine, sgm_2pass=0)
    np.testing.assert_array_equal(two, four)
    cfg = oracle.config(H, W, md, aggregation=agg, do_refine=refine)
    for i in range(n):
        np.testing.assert_array_equal(two[i], oracle.run_ex({k: batch[k][i] for k in KEYS}, cfg)["disp"])


def test_two_pass_repeated_runs_deterministic():
    """The strip tickets and progress counters are reset per pass: back-to-back runs without a host
    synchronisation give identical maps."""
    H, W, md, n = 50, 60, 127, 3
    batch = S.make_batch(n, H, W, md + 1, first_index=680)
    sb = StereoBatch(md, H, W, n, device=0, sgm_2pass=1)
    try:
        sb.upload(*(batch[k] for k in KEYS))
        for _ in range(3):
            sb.run(0.3, download=False)
        first = sb.download()
        again = sb.run(0.3)
    finally:
        sb.close()
    np.testing.assert_array_equal(first, again)
