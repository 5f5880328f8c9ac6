"""GPU maps at the BASELINE configs' own shapes against committed oracle fixtures (bit-exact).

The fixtures (tests/golden/large_*.npz, made by tests/golden/make_large.py in the build container)
hold the CPU restatement's int16 map for a seeded synthetic pair of each shape: full resolution
3000x2000 D = 256 (configs[3]), 1920x1080 D = 256 (configs[4]), Cones-shaped Census + SGM at
D = 60 / 64 (configs[0]), Teddy-shaped Do_refine and "so" (configs[1] variants) and KITTI 8-path
(configs[2]).  Here the same pair is regenerated with synthetic.py (its inputs checked against the
fixture's sha256 first), run through the C-ABI, and the map compared element for element.
Reference: dispOptimize / WTA DP[0] (stereoMatching.cpp:1046-1136, 3928-3967), refine
(cpp:1138-1511), so (cpp:6272-6394).
"""
import glob
import hashlib
import os

import numpy as np
import pytest

from mystereomatching_amd import SolveAll, StereoBatch, StereoMatching
from mystereomatching_amd import synthetic as S

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "large_*.npz")))
KEYS = ("lbgr", "rbgr", "lgray", "rgray")


def _load(path):
    z = np.load(path)
    ov = {k[3:]: int(z[k]) for k in z.files if k.startswith("ov_")}
    return z, ov


def _pair(z):
    H, W, md, idx = int(z["H"]), int(z["W"]), int(z["max_disp"]), int(z["index"])
    pair = S.make_pair(H, W, md + 1, idx)
    for k in KEYS:
        got = hashlib.sha256(np.ascontiguousarray(pair[k]).tobytes()).hexdigest()
        assert got == str(z["sha_" + k]), f"synthetic {k} no longer regenerates the fixture's input"
    return pair, H, W, md


def _diff_msg(got, want):
    bad = np.argwhere(got != want)
    v, u = bad[0]
    return f"{len(bad)} pixels differ; first at (v={v}, u={u}): gpu {got[v, u]} oracle {want[v, u]}"


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[6:-4] for p in FIXTURES])
def test_batch_path_matches_oracle_fixture(path):
    z, ov = _load(path)
    pair, H, W, md = _pair(z)
    sb = StereoBatch(md, H, W, 1, device=0, **ov)
    try:
        sb.upload(*(pair[k][None] for k in KEYS))
        got = sb.run(0.3)[0]
    finally:
        sb.close()
    want = z["disp"]
    assert hashlib.sha256(want.tobytes()).hexdigest() == str(z["sha_disp"])
    assert np.array_equal(got, want), _diff_msg(got, want)


COST_NAMES = {0: "censusGrad", 1: "Census", 2: "ADCensus", 3: "AD"}
OPT_NAMES = {0: "", 1: "sgm", 2: "so"}


@pytest.mark.parametrize("name", ["large_cones_census_sgm_d60", "large_hd1080_d256"])
def test_reference_ordered_api_matches_oracle_fixture(name):
    """The same maps through main_.cpp's call order (ctor, costCalculate, SolveAll, dispOptimize)."""
    path = os.path.join(HERE, "golden", name + ".npz")
    if not os.path.exists(path):
        pytest.skip("fixture not generated")
    z, ov = _load(path)
    pair, H, W, md = _pair(z)
    sel = (StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization)
    StereoMatching.costcalculation = COST_NAMES[ov["cost_method"]]
    StereoMatching.aggregation = "CBCA" if ov["aggregation"] else ""
    StereoMatching.optimization = OPT_NAMES[ov["optimization"]]
    try:
        prm = StereoMatching.Parameters(md, H, W)
        prm.sgm_scanNum = ov["sgm_paths"]
        sm = StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], pair["gt"], None,
                            pair["nonocc"], None, prm, device=0)
        sm.costCalculate()
        SolveAll([sm], 1, 0.3)
        got = sm.dispOptimize()
    finally:
        StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = sel
    want = z["disp"]
    assert np.array_equal(got, want), _diff_msg(got, want)


@pytest.mark.parametrize("name", ["large_fullres_d256", "large_hd1080_d256", "large_teddy_refine_d64"])
def test_fuse_norm_scan_matches_oracle_fixture(name):
    """sm_params.fuse_norm_scan = 1 (CB_NORM_SCAN sweeps) at configs[3] / configs[4] size and with
    Do_refine: the maps must equal the same oracle fixtures as the default sweep sequence."""
    z, ov = _load(os.path.join(HERE, "golden", name + ".npz"))
    pair, H, W, md = _pair(z)
    sb = StereoBatch(md, H, W, 1, device=0, fuse_norm_scan=1, **ov)
    try:
        sb.upload(*(pair[k][None] for k in KEYS))
        got = sb.run(0.3)[0]
    finally:
        sb.close()
    want = z["disp"]
    assert np.array_equal(got, want), _diff_msg(got, want)


BENCH_MAPS = sorted(glob.glob(os.path.join(HERE, "golden", "bench_maps_*.npz")))


@pytest.mark.parametrize("path", BENCH_MAPS, ids=[os.path.basename(p)[11:-4] for p in BENCH_MAPS])
def test_bench_batch_default_schedule_every_pair(path):
    """A bench workload's whole batch (tests/golden/bench_maps_<workload>.npz: the oracle map of
    every pair, made by make_bench_maps.py) through the schedule bench.py times: the default
    (num_streams 0: at these sizes two pair groups pipelined across calls), three back-to-back
    runs with asynchronous map copies into page-locked memory, the last two without anything
    joining the pipeline in between.  Every pair of every call must equal its oracle map."""
    import torch
    z = np.load(path)
    H, W, md, B, paths = (int(z[k]) for k in ("H", "W", "max_disp", "pairs", "sgm_paths"))
    batch = S.make_batch(B, H, W, md + 1)
    for i in range(B):
        for k in KEYS:
            got = hashlib.sha256(np.ascontiguousarray(batch[k][i]).tobytes()).hexdigest()
            assert got == str(z[f"sha_{k}_{i}"]), f"synthetic {k} of pair {i} no longer regenerates the fixture"
    want = z["disp"]
    sb = StereoBatch(md, H, W, B, device=0, sgm_paths=paths)
    try:
        sb.upload(*(batch[k] for k in KEYS))
        outs = [torch.full((B, H, W), -9, dtype=torch.int16, pin_memory=True).numpy() for _ in range(3)]
        for o in outs:
            sb.run(0.3, download=False)
            sb.download_async(o)
        sb.synchronize()
        for c, o in enumerate(outs):
            for i in range(B):
                assert np.array_equal(o[i], want[i]), f"call {c} pair {i}: " + _diff_msg(o[i], want[i])
    finally:
        sb.close()
