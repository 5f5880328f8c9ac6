#!/usr/bin/env python3
"""Fold the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of a bench run into per-kernel HBM bytes.

usage: tools/pmc_summary.py <fetch counter_collection.csv> <write counter_collection.csv> <out.json>

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KB; on gfx950 FETCH_SIZE
reports half of the bytes of a wide streaming read, so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE is exact for streaming stores.  Kernel symbols are mapped onto the profile names the
C-ABI uses (sm_capi.cpp); the two middle SGM paths share one symbol and are told apart by
dispatch order.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def profile_name(sym: str, seen: dict) -> str:
    m = re.search(r"k_cbca<(true|false), (\d)[,>]", sym)
    if m:
        h = m.group(1) == "true"
        mode = {"0": "scan", "1": "norm", "2": "norm_scan"}[m.group(2)]
        return f"cbca_{'h' if h else 'v'}_{mode}"
    if "k_cbca_nsv" in sym:
        return "cbca_v_norm_scan"
    if "k_cbca_hn" in sym:
        return "cbca_h_norm"
    m = re.search(r"k_sgm_ck<\d+, (\d+),", sym)
    if m:
        mode = int(m.group(1))  # CK_A = 16, CK_B = 32, CK_MID = 64, SGM_LAST = 2
        if mode & 16:
            seen["ck_a"] = seen.get("ck_a", 0) + 1
            return "sgm_ck_a01" if seen["ck_a"] % 2 == 1 else "sgm_ck_a23"
        if mode & 64:
            return "sgm_ck_b23"
        return "sgm_last_wta" if mode & 2 else "sgm_ck_b01"
    m = re.search(r"k_sgm(?:_rows)?<\d+, (\d+),", sym)
    if m:
        mode = int(m.group(1))  # SGM_FIRST = 1, SGM_LAST = 2, SGM_KEEP = 4
        if mode & 2:
            return "sgm_last_wta"
        if mode & 1:
            seen["mid"] = 0
            return "sgm_path0"
        seen["mid"] = seen.get("mid", 0) + 1
        return f"sgm_path{seen['mid']}"
    if "k_cost" in sym:
        return "cost_volume"
    if "k_prep" in sym or "k_pack_bgr" in sym or "k_pack_arms" in sym:
        return "prep"
    if "k_wta" in sym:
        return "wta"
    if "k_scale" in sym:
        return "solve_all"
    return sym


def load(path: str, counter: str):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    out, seen = [], {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        # a step of "prep" is several dispatches (k_pack_bgr4, k_pack_arms, k_prep, or the split
        # prep's k_prep_h, k_prep_v): count steps by k_prep / k_prep_h only
        k = r["Kernel_Name"]
        step = "k_pack" not in k and "k_prep_v" not in k
        out.append((profile_name(r["Kernel_Name"], seen), float(r["Counter_Value"]) * 1024.0, step))
    return out


def main():
    fetch, write, dst = sys.argv[1:4]
    acc = defaultdict(lambda: {"read": 0.0, "write": 0.0, "n_read": 0, "n_write": 0})
    for name, v, step in load(fetch, "FETCH_SIZE"):
        acc[name]["read"] += 2.0 * v
        acc[name]["n_read"] += step
    for name, v, step in load(write, "WRITE_SIZE"):
        acc[name]["write"] += v
        acc[name]["n_write"] += step
    kernels = {}
    for name, a in acc.items():
        if not a["n_read"] or not a["n_write"] or name.startswith("__"):
            continue
        r, w = a["read"] / a["n_read"], a["write"] / a["n_write"]
        # "prep" sums its three dispatches per step, like the bench's "prep" timer
        kernels[name] = {"hbm_read_bytes_per_launch": r, "hbm_write_bytes_per_launch": w,
                         "hbm_bytes_per_launch": r + w, "steps": a["n_read"]}
    json.dump({"source": [fetch, write],
               "correction": "read = 2 x FETCH_SIZE(KB) x 1024 (gfx950 half-count), write = WRITE_SIZE(KB) x 1024",
               "kernels": kernels}, open(dst, "w"), indent=1)
    for k, v in kernels.items():
        print(f"{k:16s} read {v['hbm_read_bytes_per_launch']/1e6:9.1f} MB  write {v['hbm_write_bytes_per_launch']/1e6:9.1f} MB")


if __name__ == "__main__":
    main()
