#!/usr/bin/env python3
"""Interleaved in-process A/B of library variants (tools/build_variants.sh) on one GPU.

Box clocks drift within a call by more than the effects being measured, so timing variant A in
one process and B in the next compares different clocks.  This loads every variant into one
process (each StereoBatch keeps the library it was created with), then alternates short timed
rounds A, B, C, A, B, C, ... and reports each variant's median per-kernel HIP-event time and
median ms per step over the rounds.

usage: python tools/ab_inproc.py [--workload teddy] [--rounds 8] [--steps 5] v1 v2 ...
       (variant v = tools/abvar/libsm_hip_<v>.so; "base" = the in-tree library; v:ENV=VAL,...
       sets environment variables while that instance is created, v:key=N overrides sm_params)
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="teddy")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--kernels", default="", help="comma-separated profile-name filter")
    ap.add_argument("--agg", default="CBCA", help="aggregation (CBCA, GF, NL)")
    ap.add_argument("--copies", type=int, default=1,
                    help="instances per variant, created interleaved (A B A B ...): device allocations fall into "
                         "fast and slow placements (DESIGN §6), so compare medians over several instances")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import bench
    from mystereomatching_amd import _capi, StereoBatch
    from mystereomatching_amd import synthetic as S

    H, W, md, paths, B, _ = bench.WORKLOADS[a.workload]
    batch = S.make_batch(B, H, W, md + 1)
    sbs = {}
    maps = {}   # each instance's first maps: every variant must reproduce the first one's bits
    if a.copies > 1:
        a.variants = [v for _ in range(a.copies) for v in a.variants]
    names = [f"{v}#{i}" if a.variants.count(v) > 1 else v for i, v in enumerate(a.variants)]
    for spec, key in zip(a.variants, names):
        # spec = lib[:ENV=VAL[,ENV=VAL]]: environment set while this instance is created
        v, _, envs = spec.partition(":")
        params = {}
        for kv in filter(None, envs.split(",")):
            k, _, val = kv.partition("=")
            if k.islower():   # lower-case keys are sm_params overrides (integers)
                params[k] = int(val)
            else:
                os.environ[k] = val
        _capi._lib = None
        if v == "base":
            os.environ.pop("SM_HIP_LIB", None)
        else:
            os.environ["SM_HIP_LIB"] = os.path.join(ROOT, "tools", "abvar", f"libsm_hip_{v}.so")
        sb = StereoBatch(md, H, W, B, sgm_paths=paths, aggregation=a.agg, **params)
        sb.upload(batch["lbgr"], batch["rbgr"], batch["lgray"], batch["rgray"])
        maps[key] = sb.run(0.3)
        sbs[key] = sb
        for kv in filter(None, envs.split(",")):
            if not kv.partition("=")[0].islower():
                os.environ.pop(kv.partition("=")[0], None)
    _capi._lib = None
    import numpy as np
    first = names[0]
    for v in names[1:]:
        same = np.array_equal(maps[v], maps[first])
        print(f"maps {v} == {first}: {'identical' if same else 'DIFFERENT'}", flush=True)
    step_ms = {v: [] for v in names}
    kern = {v: {} for v in names}
    order = list(sbs.items())
    for r in range(a.rounds):
        # each round starts one instance later, so no variant always runs first after the print
        for v, sb in order[r % len(order):] + order[:r % len(order)]:
            sb.profile(True)
            sb.profile_reset()
            sb.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                sb.run(0.3, download=False)
            sb.synchronize()
            step_ms[v].append((time.perf_counter() - t0) * 1e3 / a.steps)
            for name, rec in sb.profile_read().items():
                kern[v].setdefault(name, []).append(rec["total_ms"] / max(1, rec["launches"]))
        print(f"round {r + 1}/{a.rounds} done", flush=True)
    want = [k for k in a.kernels.split(",") if k]
    for v in names:
        ks = " ".join(f"{n}={statistics.median(x):.4f}" for n, x in kern[v].items() if not want or any(w in n for w in want))
        print(f"{v:10s} step={statistics.median(step_ms[v]):.3f} ms  {ks}")
    if a.copies > 1:   # per variant: median over its instances of the per-instance medians
        print("-- medians over instances --")
        for v in dict.fromkeys(a.variants):
            inst = [nm for nm, sp in zip(names, a.variants) if sp == v]
            ks = {}
            for nm in inst:
                for n, x in kern[nm].items():
                    if not want or any(w in n for w in want):
                        ks.setdefault(n, []).append(statistics.median(x))
            st = statistics.median(statistics.median(step_ms[nm]) for nm in inst)
            print(f"{v:10s} step={st:.3f} ms  " + " ".join(f"{n}={statistics.median(x):.4f}" for n, x in ks.items()))


if __name__ == "__main__":
    main()
