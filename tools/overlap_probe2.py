#!/usr/bin/env python3
"""Probe 2: the pipelined two-pair context (num_streams 0) against two single-pair contexts issued
back to back, with two instances of each (allocation placement differs per instance),
interleaved rounds; ms per two full-resolution pairs.  Timing only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import statistics
    import bench
    from mystereomatching_amd import StereoBatch
    from mystereomatching_amd import synthetic as S
    H, W, md, paths, B, _ = bench.WORKLOADS["fullres"]
    batch = S.make_batch(2, H, W, md + 1)
    keys = ("lbgr", "rbgr", "lgray", "rgray")
    inst = {}
    for r in range(2):
        one = StereoBatch(md, H, W, 2, sgm_paths=paths)
        one.upload(*(batch[k] for k in keys))
        inst[f"one{r}"] = [one]
        two = []
        for i in range(2):
            sb = StereoBatch(md, H, W, 1, sgm_paths=paths, num_streams=1)
            sb.upload(*(batch[k][i:i + 1] for k in keys))
            two.append(sb)
        inst[f"two{r}"] = two
    steps = 20
    res = {k: [] for k in inst}
    seq = {k: [] for k in inst}
    for rnd in range(3):
        for k, sbs in inst.items():
            for sb in sbs:
                sb.run(0.3, download=False)
                sb.synchronize()
            t = time.perf_counter()
            for _ in range(steps):
                for sb in sbs:
                    sb.run(0.3, download=False)
            for sb in sbs:
                sb.synchronize()
            res[k].append((time.perf_counter() - t) / steps * 1e3)
            # the same instance one pair after the other (one stream per context / one stream)
            if len(sbs) == 1:
                sbs[0].set_schedule(1, 0)
            t = time.perf_counter()
            for _ in range(steps):
                for sb in sbs:
                    sb.run(0.3, download=False)
                    sb.synchronize() if len(sbs) > 1 else None
            for sb in sbs:
                sb.synchronize()
            seq[k].append((time.perf_counter() - t) / steps * 1e3)
            if len(sbs) == 1:
                sbs[0].set_schedule(0, 0)
        print(f"round {rnd}: " + "  ".join(f"{k}={res[k][-1]:.2f}/{seq[k][-1]:.2f}" for k in inst), flush=True)
    for k in inst:
        print(f"{k}: concurrent {statistics.median(res[k]):.3f} ms   sequential {statistics.median(seq[k]):.3f} ms")


if __name__ == "__main__":
    main()
