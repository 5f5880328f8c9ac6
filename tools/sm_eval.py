#!/usr/bin/env python3
"""Evaluate the GPU pipeline on a Middlebury-layout dataset, the way main_.cpp does (main:26-178).

usage: tools/sm_eval.py ROOT [--objects teddy cones ...] [--refine] [--pyr L] [--device N]

For each object: load (mystereomatching_amd.dataset), Parameters(maxdisp, ...), costCalculate per
pyramid level, SolveAll(PY_LEV, 0.3), dispOptimize [, refine], then calErr over nonocc / all /
disc at t = 1 (errorThreshold, h:225) and t = 2 (BASELINE's bad-2.0).  Prints one JSON line per
object.  No dataset ships with this repository; point ROOT at a local Middlebury copy.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from mystereomatching_amd import SolveAll, StereoMatching, dataset, pyrDown  # noqa: E402
from mystereomatching_amd.evaluate import cal_err_regions  # noqa: E402


def run(sample, refine, levels, device):
    StereoMatching.costcalculation, StereoMatching.aggregation, StereoMatching.optimization = "censusGrad", "CBCA", "sgm"
    StereoMatching.Do_refine = refine
    imgs = sample.pair()
    sms, md, sc = [], sample.max_disp, 1
    t0 = time.perf_counter()
    for _ in range(levels):
        H, W = imgs["lgray"].shape
        prm = StereoMatching.Parameters(md, H, W, 13, 1, 2, 109, 10, "", sc)
        sm = StereoMatching(imgs["lbgr"], imgs["rbgr"], imgs["lgray"], imgs["rgray"], sample.gt, None, None, None,
                            prm, device=device)
        sm.costCalculate()
        sms.append(sm)
        md, sc = md // 2 + 1, sc * 2
        imgs = {k: pyrDown(v, device) for k, v in imgs.items()}
    SolveAll(sms, levels, 0.3)
    dp = sms[0].dispOptimize()
    if refine:
        dp = sms[0].refine()
    return dp, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--objects", nargs="*", default=["teddy", "cones"])
    ap.add_argument("--refine", action="store_true")
    ap.add_argument("--pyr", type=int, default=1)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--dataset", default="MD")
    a = ap.parse_args()
    for obj in a.objects:
        s = dataset.load(a.root, obj, a.dataset)
        dp, t = run(s, a.refine, a.pyr, a.device)
        out = {"object": obj, "H": s.lgray.shape[0], "W": s.lgray.shape[1], "D": s.max_disp + 1,
               "refine": a.refine, "py_lev": a.pyr, "seconds": round(t, 4)}
        if s.gt is not None:
            for t_ in (1.0, 2.0):
                for r, (pbm, rms) in cal_err_regions(dp, s.gt, s.masks, t_).items():
                    out[f"bad{t_:.1f}_{r}"] = round(100 * pbm, 3)
                    if t_ == 1.0:
                        out[f"rms_{r}"] = round(rms, 4)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
