#!/usr/bin/env python3
"""Which kernels of the two pipelined pair groups run beside which: reads a rocprofv3
--kernel-trace CSV of tools/pipe_trace.py (or bench.py), keeps the dispatches of the last
`--tail` fraction of the trace, and prints per kernel name its mean duration, the share of its
time another queue was busy, and the other queue's kernels it overlapped (ms per launch).

usage: python tools/pipe_overlap.py <kernel_trace.csv> [--tail 0.6]
"""
import argparse
import collections
import csv
import re


def short(name):
    n = re.sub(r"\(.*$", "", name)
    n = n.replace("void ", "").replace("sm::", "")
    n = re.sub(r"<.*>", "", n)
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--tail", type=float, default=0.6)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    key_q = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key_q], short(r["Kernel_Name"])))
    ks.sort()
    t0, t1 = ks[0][0], max(k[1] for k in ks)
    cut = t1 - a.tail * (t1 - t0)
    ks = [k for k in ks if k[0] >= cut]
    queues = sorted({k[2] for k in ks})
    print(f"{len(ks)} dispatches on queues {queues} over {(ks[-1][1] - ks[0][0]) / 1e6:.2f} ms")
    dur = collections.defaultdict(list)
    busy_other = collections.defaultdict(float)
    pair = collections.defaultdict(lambda: collections.defaultdict(float))
    byq = {q: [k for k in ks if k[2] == q] for q in queues}
    for s, e, q, n in ks:
        dur[(q, n)].append(e - s)
        for q2 in queues:
            if q2 == q:
                continue
            cover = 0
            for s2, e2, _, n2 in byq[q2]:
                if e2 <= s or s2 >= e:
                    continue
                ov = min(e, e2) - max(s, s2)
                cover += ov
                pair[(q, n)][n2] += ov
            busy_other[(q, n)] += min(cover, e - s)
    for (q, n), ds in sorted(dur.items(), key=lambda x: (x[0][0], -sum(x[1]))):
        tot = sum(ds)
        cnt = len(ds)
        others = ", ".join(f"{n2} {v / cnt / 1e6:.2f}" for n2, v in
                           sorted(pair[(q, n)].items(), key=lambda x: -x[1]) if v / tot > 0.03)
        print(f"q{q} {n:18s} x{cnt:3d} {tot / cnt / 1e6:6.3f} ms  beside other queue {100 * busy_other[(q, n)] / tot:5.1f} %  [{others}]")
    # period: the time between consecutive launches of the first kernel name on each queue
    for q in queues:
        first = byq[q][0][3]
        st = [k[0] for k in byq[q] if k[3] == first]
        if len(st) > 2:
            gaps = [(b - a_) / 1e6 for a_, b in zip(st, st[1:])]
            print(f"q{q}: {first} every {sum(gaps) / len(gaps):.2f} ms ({len(gaps)} periods)")
    # the other queue's offset: start of queue B's first kernel relative to queue A's cycle
    if len(queues) == 2:
        qa, qb = queues
        fa = byq[qa][0][3]
        sa = [k[0] for k in byq[qa] if k[3] == fa]
        sb = [k[0] for k in byq[qb] if k[3] == fa]
        offs = []
        for s in sb:
            prev = [x for x in sa if x <= s]
            if prev and len(sa) > 1:
                offs.append((s - prev[-1]) / 1e6)
        if offs:
            print(f"q{qb}'s {fa} starts {sum(offs) / len(offs):.2f} ms after q{qa}'s (mean of {len(offs)})")


if __name__ == "__main__":
    main()
