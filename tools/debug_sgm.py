"""GPU debugging aid: SGM final volumes per path count vs the oracle, first mismatches printed.

usage (GPU box): python tools/debug_sgm.py [H W max_disp]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mystereomatching_amd import StereoMatching, SolveAll  # noqa: E402
from mystereomatching_amd import synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    H, W, md = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (9, 21, 7)))
    pair = S.make_pair(H, W, md + 1, 5)
    for paths in (1, 2, 3, 4):
        cfg = O.config(H, W, md, sgm_paths=paths)
        ref = O.run(pair, cfg, dumps=True)
        StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = "censusGrad", "CBCA", "sgm"
        prm = StereoMatching.Parameters(md, H, W)
        prm.sgm_scanNum = paths
        sm = StereoMatching(pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"], None, None, None, None, prm,
                            keep_final_volume=True)
        sm.costCalculate()
        agg = sm.vm[0]
        SolveAll([sm], 1, 0.3)
        dp = sm.dispOptimize()
        fin = sm.vm[0]
        ok_agg = np.array_equal(agg.view(np.uint32), ref["agg"].view(np.uint32))
        bad = np.argwhere(fin.view(np.uint32) != ref["final"].view(np.uint32))
        print(f"paths={paths} agg_ok={ok_agg} final_mismatch={len(bad)} disp_mismatch={int((dp != ref['disp']).sum())}")
        for v, u, d in bad[:6]:
            print(f"   (v={v}, u={u}, d={d}) gpu={fin[v, u, d]!r} ref={ref['final'][v, u, d]!r}")


if __name__ == "__main__":
    main()
