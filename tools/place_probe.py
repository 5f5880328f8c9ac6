#!/usr/bin/env python3
"""Per-allocation placement spread: several one-stream instances of the same library
in ONE process, each timed per kernel (HIP events) in interleaved rounds, and run in a fixed
order so that a profiler's per-dispatch counters (rocprofv3 --pmc ...) can be attributed to the
instance: in every round, instance i's 9 kernels are the i-th block of dispatches.  Prints one
line per instance (median per-kernel ms over the rounds, allocation addresses) and writes a JSON
with the dispatch layout for tools/place_counters.py.

usage: python tools/place_probe.py [--copies 6] [--rounds 3] [--workload fullres] [--out file.json]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--workload", default="fullres")
    ap.add_argument("--out", default="")
    ap.add_argument("--trials", default="0",
                    help="sm_params.placement_trials per instance, cycled (e.g. 0,3: alternate off / three sets)")
    a = ap.parse_args()
    import bench
    from mystereomatching_amd import StereoBatch
    from mystereomatching_amd import synthetic as S
    H, W, md, paths, B, _ = bench.WORKLOADS[a.workload]
    batch = S.make_batch(B, H, W, md + 1)
    sbs = []
    trials = [int(x) for x in a.trials.split(",")]
    for i in range(a.copies):
        sb = StereoBatch(md, H, W, B, device=0, sgm_paths=paths, num_streams=1,
                         placement_trials=trials[i % len(trials)])
        sb.upload(batch["lbgr"], batch["rbgr"], batch["lgray"], batch["rgray"])
        sb.run(0.3, download=False)   # warm-up (these dispatches precede the rounds)
        sb.synchronize()
        print(f"instance {i}: placement_trials {trials[i % len(trials)]} -> {sb.placement()}", flush=True)
        sbs.append(sb)
    times = [dict() for _ in sbs]
    for r in range(a.rounds):
        for i, sb in enumerate(sbs):
            sb.profile(True)
            sb.profile_reset()
            sb.run(0.3, download=False)
            sb.synchronize()
            for k, v in sb.profile_read().items():
                times[i].setdefault(k, []).append(v["total_ms"] / max(1, v["launches"]))
            sb.profile(False)
            print(f"round {r} instance {i} " + " ".join(f"{k}={v[-1]:.3f}" for k, v in times[i].items()), flush=True)
    med = [{k: statistics.median(v) for k, v in t.items()} for t in times]
    for i, m in enumerate(med):
        print(f"instance {i} (trials {trials[i % len(trials)]}): step {sum(m.values()):.3f} " +
              " ".join(f"{k}={v:.3f}" for k, v in m.items()))
    if a.out:
        json.dump({"workload": a.workload, "copies": a.copies, "rounds": a.rounds,
                   "kernels_per_step": len(med[0]), "order": "warm-up: one step per instance in order; then rounds x "
                   "instances, one step each", "median_ms": med}, open(a.out, "w"), indent=1)
    for sb in sbs:
        sb.close()


if __name__ == "__main__":
    main()
