#!/usr/bin/env python3
"""Attributes per-dispatch rocprofv3 counters of a tools/place_probe.py run to its instances and
prints them beside each instance's per-kernel time (placement spread).

usage: tools/place_counters.py <place_probe json> <out.json> <counter_collection.csv> [...]

In place_probe.py every instance runs one step per round in a fixed order (warm-up first), so
the j-th dispatch of a kernel symbol belongs to instance j % copies; warm-up dispatches
(j < copies) are skipped and the counters are summed per dispatch, medians over the rounds.
"""
import csv
import json
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import profile_name  # noqa: E402


def main():
    meta = json.load(open(sys.argv[1]))
    copies = meta["copies"]
    per = defaultdict(lambda: defaultdict(float))   # (dispatch id) -> counter -> value
    sym_of = {}
    for path in sys.argv[3:]:
        for r in csv.DictReader(open(path)):
            d = (path, int(r["Dispatch_Id"]))
            sym_of[d] = r["Kernel_Name"]
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    # per file: dispatches of each profile name in order -> instance
    out = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))   # name -> inst -> counter -> [v]
    files = sorted({d[0] for d in per})
    for f in files:
        seen, idx = {}, defaultdict(int)
        for d in sorted((d for d in per if d[0] == f), key=lambda d: d[1]):
            name = profile_name(sym_of[d], seen)
            j = idx[name]
            idx[name] += 1
            if j < copies:
                continue   # warm-up
            for c, v in per[d].items():
                out[name][j % copies][c].append(v)
    res = {}
    for name in sorted(out):
        res[name] = {}
        print(name)
        for i in range(copies):
            cs = {c: statistics.median(v) for c, v in sorted(out[name][i].items())}
            ms = meta["median_ms"][i].get(name)
            res[name][i] = {"ms": ms, **cs}
            print(f"  inst {i} ms {ms if ms is None else round(ms, 3)} " +
                  " ".join(f"{c}={v:.4g}" for c, v in cs.items()))
    json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
