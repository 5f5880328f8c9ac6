"""Generates tests/golden/*.npz from the CPU oracle (oracle/sm_oracle.c).

PARITY UNPINNED: the reference cannot be built or run here and ships no fixtures, so these
vectors are the oracle's output (itself cross-checked against tests/pyref.py).  They freeze the
restatement so that any later change to it, or to the GPU path, shows up as a diff.
Run:  python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from mystereomatching_amd import synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

# (name, H, W, max_disp, pair index, cost, sgm paths, dump volumes)
CASES = [
    ("small_censusgrad", 24, 32, 15, 100, "censusGrad", 4, True),
    ("small_census", 20, 28, 11, 101, "Census", 4, True),
    ("small_adcensus", 22, 30, 13, 102, "ADCensus", 8, True),
    ("small_ad", 18, 26, 9, 103, "AD", 4, True),
    ("mid_censusgrad_d60", 60, 80, 59, 104, "censusGrad", 4, True),
    ("teddy_censusgrad_d64", 375, 450, 63, 0, "censusGrad", 4, False),
]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    out_dir = os.path.dirname(os.path.abspath(__file__))
    for name, H, W, md, idx, cost, paths, dump in CASES:
        p = S.make_pair(H, W, md + 1, idx)
        cfg = O.config(H, W, md, cost=cost, sgm_paths=paths)
        r = O.run(p, cfg, dumps=True)
        rec = dict(H=H, W=W, max_disp=md, index=idx, cost=cost, paths=paths,
                   lbgr=p["lbgr"], rbgr=p["rbgr"], lgray=p["lgray"], rgray=p["rgray"],
                   gt=p["gt"], nonocc=p["nonocc"], disp=r["disp"],
                   sha_cost=sha(r["cost"]), sha_agg=sha(r["agg"]), sha_final=sha(r["final"]))
        if dump:
            rec.update(cost_vol=r["cost"], agg_vol=r["agg"], final_vol=r["final"])
        np.savez_compressed(os.path.join(out_dir, name + ".npz"), **rec)
        print(name, "written")


if __name__ == "__main__":
    main()
