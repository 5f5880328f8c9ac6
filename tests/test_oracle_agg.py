"""CPU: the oracle's GF (MY_GUIDE) and NL aggregators against the independent numpy restatement
(tests/pyref_agg.py), bit for bit, plus structural checks of the NL tree.  PARITY UNPINNED (the
reference needs OpenCV / ximgproc and ships no fixtures); see oracle/sm_oracle_agg.c."""
import numpy as np
import pytest

import pyref_agg as R
from mystereomatching_amd import synthetic as S


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("H,W,r", [(19, 19, 9), (25, 31, 9), (12, 9, 4), (5, 7, 2)])
def test_box_filter_matches_pyref(oracle, H, W, r):
    img = np.random.default_rng(H * W).random((H, W)).astype(np.float32) * 100
    np.testing.assert_array_equal(bits(oracle.box_filter(img, r)), bits(R.box_filter(img, r)))


@pytest.mark.parametrize("H,W,r", [(19, 19, 9), (25, 31, 9), (12, 9, 4), (5, 7, 2), (3, 4, 9), (1, 6, 2)])
def test_box_filter_cv_matches_pyref(oracle, H, W, r):
    """OpenCV's normalised box filter (BORDER_REFLECT, double running sums), including images smaller
    than the window (multiple reflections)."""
    img = np.random.default_rng(H * W + 7).random((H, W)).astype(np.float32) * 100
    got = oracle.box_filter_cv(img, r)
    np.testing.assert_array_equal(bits(got), bits(R.box_filter_cv(img, r)))
    # against a float64 windowed mean over the reflected image: within a few ulp
    pad = np.pad(img.astype(np.float64), r, mode="symmetric") if min(H, W) >= r else None
    if pad is not None:
        k = 2 * r + 1
        want = np.lib.stride_tricks.sliding_window_view(pad, (k, k)).mean(axis=(2, 3))
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-4)


def test_reflect_border(oracle):
    """borderInterpolate(BORDER_REFLECT): fedcba|abcdefgh|hgfedcb."""
    got = [oracle.load().smo_reflect(p, 8) for p in range(-6, 14)]
    assert got == [5, 4, 3, 2, 1, 0, 0, 1, 2, 3, 4, 5, 6, 7, 7, 6, 5, 4, 3, 2]


@pytest.mark.parametrize("H,W,md,idx", [(24, 30, 7, 402), (19, 40, 11, 403), (12, 10, 5, 404)])
def test_guided_filter_ximgproc_matches_pyref(oracle, H, W, md, idx):
    """gf_mode 0 (the shipped build's ximgproc::guidedFilter) against the numpy twin."""
    pair = S.make_pair(H, W, md + 1, idx)
    cfg = oracle.config(H, W, md, gf_mode=0)
    vm = oracle.cost_volume(pair, cfg)
    got = oracle.guided_filter(vm, pair["lbgr"], cfg)
    np.testing.assert_array_equal(bits(got), bits(R.guided_filter_cv(vm, pair["lbgr"])))
    # an edge-aware local average: constant slices stay (numerically) constant
    flat = np.full_like(vm, 0.75)
    assert np.allclose(oracle.guided_filter(flat, pair["lbgr"], cfg), 0.75, atol=2e-2)


@pytest.mark.parametrize("H,W,md,idx", [(24, 30, 7, 400), (19, 40, 11, 401)])
def test_guided_filter_matches_pyref(oracle, H, W, md, idx):
    pair = S.make_pair(H, W, md + 1, idx)
    cfg = oracle.config(H, W, md, gf_mode=1)
    vm = oracle.cost_volume(pair, cfg)
    got = oracle.guided_filter(vm, pair["lbgr"], cfg)
    want = R.guided_filter(vm, pair["lbgr"])
    np.testing.assert_array_equal(bits(got), bits(want))
    # constant slices stay (numerically) constant: the filter is an edge-aware local average
    flat = np.full_like(vm, 0.75)
    assert np.allclose(oracle.guided_filter(flat, pair["lbgr"], cfg), 0.75, atol=1e-3)


def test_guided_filter_rejects_small_images(oracle):
    cfg = oracle.config(10, 30, 3, gf_mode=1)
    with pytest.raises(ValueError):
        oracle.guided_filter(np.zeros((10, 30, 4), np.float32), np.zeros((10, 30, 3), np.uint8), cfg)


@pytest.mark.parametrize("H,W,idx", [(24, 30, 410), (31, 18, 411)])
def test_nl_tree_matches_pyref(oracle, H, W, idx):
    bgr = S.make_pair(H, W, 8, idx)["lbgr"]
    t = oracle.nl_tree(bgr)
    order, parent, weight, children = R.nl_tree(bgr)
    assert t["order"].tolist() == order
    assert t["parent"].tolist() == parent
    assert t["weight"].tolist() == weight
    for i in range(H * W):
        assert t["child"][i, :t["nchild"][i]].tolist() == children[i]
    # a spanning tree: n - 1 edges, every node reached once, parents precede children in BFS order
    assert t["nchild"].sum() == H * W - 1
    pos = np.empty(H * W, int)
    pos[t["order"]] = np.arange(H * W)
    assert all(pos[t["parent"][i]] < pos[i] for i in range(1, H * W) if i != t["order"][0])


def test_nl_median_clamped(oracle):
    bgr = np.random.default_rng(3).integers(0, 256, (9, 11, 3), dtype=np.uint8)
    pad = np.pad(bgr.astype(np.int32), ((1, 1), (1, 1), (0, 0)), mode="edge")
    win = np.stack([pad[dy:dy + 9, dx:dx + 11] for dy in range(3) for dx in range(3)])
    np.testing.assert_array_equal(oracle.nl_median3(bgr), np.sort(win, axis=0)[4])


@pytest.mark.parametrize("H,W,md,idx", [(24, 30, 7, 420), (20, 33, 15, 421)])
def test_nl_aggregate_matches_pyref(oracle, H, W, md, idx):
    pair = S.make_pair(H, W, md + 1, idx)
    cfg = oracle.config(H, W, md)
    vm = oracle.cost_volume(pair, cfg)
    got = oracle.nl_aggregate(vm, pair["lbgr"], cfg)
    np.testing.assert_array_equal(bits(got), bits(R.nl_aggregate(vm, pair["lbgr"])))
    # normalised by the aggregated ones: a constant volume stays constant
    c = oracle.nl_aggregate(np.full_like(vm, 2.5), pair["lbgr"], cfg)
    assert np.allclose(c, 2.5, rtol=1e-6)


@pytest.mark.parametrize("agg", [2, 3])
def test_pipeline_with_gf_and_nl(oracle, agg):
    H, W, md = 40, 52, 15
    pair = S.make_pair(H, W, md + 1, 430)
    r = oracle.run_ex(pair, oracle.config(H, W, md, aggregation=agg), dumps=("agg",))
    vm = oracle.cost_volume(pair, oracle.config(H, W, md))
    want = oracle.guided_filter(vm, pair["lbgr"], oracle.config(H, W, md)) if agg == 2 else \
        oracle.nl_aggregate(vm, pair["lbgr"], oracle.config(H, W, md))
    np.testing.assert_array_equal(bits(r["agg"]), bits(want))
    assert r["disp"].min() >= -1 and r["disp"].max() <= md
