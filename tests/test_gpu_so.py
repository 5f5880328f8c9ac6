"""GPU parity of the scan-line optimiser (optimization == "so", cpp:1091-1105, 6272-6394).

so() replaces SGM + WTA: a left-to-right DP per row with a trace and a backtrack.  Maps (and,
with keep_final_volume, the accumulated volume) bit-exact against the oracle.
"""
import numpy as np
import pytest

from mystereomatching_amd import StereoBatch, StereoMatching, SolveAll
from mystereomatching_amd import synthetic as S

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("H,W,md,idx", [(31, 57, 15, 1), (24, 130, 63, 2), (20, 90, 64, 3), (17, 150, 127, 4),
                                        (13, 300, 255, 5), (9, 70, 99, 6), (5, 3, 9, 7),
                                        (6, 1100, 255, 8), (7, 2100, 63, 9)])
def test_so_reference_order(oracle, H, W, md, idx):
    """Rows whose trace fits in LDS (most) and rows that keep it in global memory (W = 1100 at
    D = 256, W = 2100 at D = 64: four rows' masks exceed 64 KB)."""
    pair = S.make_pair(H, W, md + 1, 500 + idx)
    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = "censusGrad", "CBCA", "so"
    prm = StereoMatching.Parameters(md, H, W)
    sm = StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], None, None, None, None, prm,
                        keep_final_volume=True)
    sm.costCalculate()
    SolveAll([sm], 1, 0.3)
    dp = sm.dispOptimize()
    ref = oracle.run(pair, oracle.config(H, W, md, optimization=2), dumps=True)
    np.testing.assert_array_equal(dp, ref["disp"])
    np.testing.assert_array_equal(bits(sm.vm[0]), bits(ref["final"]))
    StereoMatching.optimization = "sgm"


@pytest.mark.parametrize("cost,agg", [("Census", ""), ("AD", "CBCA"), ("ADCensus", "")])
def test_so_other_costs_batch(oracle, cost, agg):
    H, W, md, n = 26, 71, 31, 3
    pairs = [S.make_pair(H, W, md + 1, 600 + i) for i in range(n)]
    st = {k: np.stack([p[k] for p in pairs]) for k in ("lbgr", "rbgr", "lgray", "rgray")}
    b = StereoBatch(md, H, W, n, optimization="so", cost_method=cost, aggregation=agg or "")
    b.upload(st["lbgr"], st["rbgr"], st["lgray"], st["rgray"])
    out = b.run()
    cfg = oracle.config(H, W, md, cost=cost, optimization=2, aggregation=1 if agg else 0)
    for i, p in enumerate(pairs):
        np.testing.assert_array_equal(out[i], oracle.run(p, cfg)["disp"], err_msg=f"pair {i}")


@pytest.mark.parametrize("cost,H,W,md", [("censusGrad", 29, 83, 31), ("ADCensus", 18, 140, 127)])
def test_so_right_view_without_refine(oracle, cost, H, W, md):
    """so runs on both views whenever Do_LRConsis (num = Do_LRConsis ? 2 : 1, cpp:1093), also
    with Do_refine off: DP[1] = so(vm[1]) on the raw right cost volume (CBCA, cpp:5592, and
    SolveAll, cpp:2178, touch vm[1] only with Do_refine), with the left colours (cpp:1098)."""
    pair = S.make_pair(H, W, md + 1, 700 + md)
    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = cost, "CBCA", "so"
    try:
        prm = StereoMatching.Parameters(md, H, W)
        sm = StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], None, None, None, None, prm)
        sm.costCalculate()
        SolveAll([sm], 1, 0.3)
        sm.dispOptimize()
    finally:
        StereoMatching.optimization = "sgm"
    ref = oracle.run_ex(pair, oracle.config(H, W, md, cost=cost, optimization=2), dumps=("disp_right",))
    np.testing.assert_array_equal(sm.DP[0], ref["disp"])
    np.testing.assert_array_equal(sm.DP[1], ref["disp_right"])
    # the batch path leaves DP[1] in the context too
    b = StereoBatch(md, H, W, 1, optimization="so", cost_method=cost)
    try:
        b.upload(*(pair[k][None] for k in ("lbgr", "rbgr", "lgray", "rgray")))
        np.testing.assert_array_equal(b.run()[0], ref["disp"])
        np.testing.assert_array_equal(b.get_disp(1), ref["disp_right"])
    finally:
        b.close()


def test_so_with_refine(oracle):
    H, W, md = 40, 66, 23
    pair = S.make_pair(H, W, md + 1, 77)
    b = StereoBatch(md, H, W, 1, optimization="so", do_refine=1)
    b.upload(*(pair[k][None] for k in ("lbgr", "rbgr", "lgray", "rgray")))
    out = b.run()
    ref = oracle.run_ex(pair, oracle.config(H, W, md, optimization=2, do_refine=1))["disp"]
    np.testing.assert_array_equal(out[0], ref)
