#!/usr/bin/env python3
"""Fold rocprofv3 --pmc counter_collection.csv files (one counter group per pass) into per-kernel
means per dispatch, plus the derived issue ratios used in DESIGN.md §5.

usage: tools/sq_summary.py OUT.json "description of the runs" A.csv [B.csv ...]

Rows are one (dispatch, counter) value each (rocprofv3 already sums the counter's hardware
instances); kernels are keyed by their symbol (template arguments included).
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    out, desc, paths = sys.argv[1], sys.argv[2], sys.argv[3:]
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> per-dispatch values
    for p in paths:
        for r in csv.DictReader(open(p)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["dispatches"] = max(len(v) for v in cs.values())
        w = m.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                      "SQ_WAVE_CYCLES", "SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if c in m:
                    m[c + "_per_wave"] = m[c] / w
        if m.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in m:
                    m[c + "_frac_of_wave_cycles"] = m[c] / m["SQ_WAVE_CYCLES"]
        kernels[k] = m
    json.dump({"source": desc, "files": paths, "kernels": kernels}, open(out, "w"), indent=1, sort_keys=True)
    for k, m in sorted(kernels.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:12]:
        print(f"{k[:60]:60s} " + " ".join(f"{c[3:]}={m[c]:.3g}" for c in sorted(m) if c.endswith("_per_wave")))


if __name__ == "__main__":
    main()
