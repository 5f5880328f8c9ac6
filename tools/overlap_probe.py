#!/usr/bin/env python3
"""Probe: do two pair pipelines on separate streams overlap usefully when their phases are offset?

Two single-pair contexts (A, B; one stream each) run back-to-back sm_run calls without host
synchronisation, so each context's calls queue on its own stream; B's stream is first delayed by a
spin kernel of `offset` ms, so in steady state B's pipeline runs that far behind A's (B's LDS-bound
CBCA sweeps against A's SGM passes, which use no LDS).  Reported: ms per pair-pair (A call + B
call) against the same two pairs as one two-pair context on one stream and with the default
schedule.  Maps are compared with the one-context maps.  Timing only; not a product path.

usage: python tools/overlap_probe.py [--workload fullres] [--steps 10] [--offsets 0,8,17]
("default" = the two-pair context on num_streams 0: the pipelined groups of sm_run; "piped_d2h" the
same with each step's maps copied to page-locked memory, as bench.py times it)
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="fullres")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--offsets", default="0,8,17")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from mystereomatching_amd import StereoBatch
    from mystereomatching_amd import synthetic as S

    H, W, md, paths, B, _ = bench.WORKLOADS[a.workload]
    batch = S.make_batch(2, H, W, md + 1)
    keys = ("lbgr", "rbgr", "lgray", "rgray")
    one = StereoBatch(md, H, W, 2, sgm_paths=paths, num_streams=1)
    one.upload(*(batch[k] for k in keys))
    want = one.run(0.3)
    ctx = []
    for i in range(2):
        sb = StereoBatch(md, H, W, 1, sgm_paths=paths, num_streams=1)
        sb.upload(*(batch[k][i:i + 1] for k in keys))
        got = sb.run(0.3)
        print(f"pair {i} single-pair context == two-pair context: {bool(np.array_equal(got[0], want[i]))}", flush=True)
        ctx.append(sb)
    streams = [torch.cuda.ExternalStream(int(sb._lib.sm_stream(sb._ctx))) for sb in ctx]

    # spin-kernel cycles per ms on this box
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    torch.cuda._sleep(10_000_000)
    e1.record(s)
    torch.cuda.synchronize()
    cyc_per_ms = 10_000_000 / e0.elapsed_time(e1)

    def time_one(ns):
        one.set_schedule(ns, 0)
        one.run(0.3, download=False)
        one.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            one.run(0.3, download=False)
        one.synchronize()
        return (time.perf_counter() - t) / a.steps * 1e3

    def time_pair(offset_ms):
        for sb in ctx:
            sb.synchronize()
        with torch.cuda.stream(streams[1]):
            if offset_ms > 0:
                torch.cuda._sleep(int(offset_ms * cyc_per_ms))
        t = time.perf_counter()
        for _ in range(a.steps):
            ctx[0].run(0.3, download=False)
            ctx[1].run(0.3, download=False)
        for sb in ctx:
            sb.synchronize()
        return (time.perf_counter() - t) / a.steps * 1e3 - offset_ms / a.steps

    host = torch.empty((2, H, W), dtype=torch.int16, pin_memory=True).numpy()

    def time_pair_seq():
        # the same two single-pair contexts run one after the other (each waits for the other's
        # previous call through events): their one-stream baseline on these allocations
        for sb in ctx:
            sb.synchronize()
        ev = [torch.cuda.Event(), torch.cuda.Event()]
        t = time.perf_counter()
        for _ in range(a.steps):
            for i in range(2):
                ctx[i].run(0.3, download=False)
                ev[i].record(streams[i])
                streams[1 - i].wait_event(ev[i])
        for sb in ctx:
            sb.synchronize()
        return (time.perf_counter() - t) / a.steps * 1e3

    def time_piped(d2h):
        # the two-pair context with the default schedule (pipelined groups), K steps after a sync
        one.set_schedule(0, 0)
        one.run(0.3, download=False)
        one.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            one.run(0.3, download=False)
            if d2h:
                one.download_async(host)
        one.synchronize()
        return (time.perf_counter() - t) / a.steps * 1e3

    offs = [float(x) for x in a.offsets.split(",")]
    res = {"one_stream": [], "default": [], "piped_d2h": [], "pair_seq": []}
    res.update({f"pair_off{o:g}": [] for o in offs})
    for r in range(3):
        res["one_stream"].append(time_one(1))
        res["default"].append(time_one(0))
        res["piped_d2h"].append(time_piped(True))
        res["pair_seq"].append(time_pair_seq())
        for o in offs:
            res[f"pair_off{o:g}"].append(time_pair(o))
        print(f"round {r + 1}: " + "  ".join(f"{k}={v[-1]:.2f}" for k, v in res.items()), flush=True)
    for k, v in res.items():
        print(f"{k:14s} median {sorted(v)[1]:.3f} ms per 2 pairs  {['%.2f' % x for x in v]}")
    for i, sb in enumerate(ctx):
        print(f"pair {i} after the overlapped runs == two-pair context: {bool(np.array_equal(sb.download()[0], want[i]))}")


if __name__ == "__main__":
    main()
