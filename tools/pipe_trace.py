#!/usr/bin/env python3
"""Kernel-trace subject for the pipelined schedule: `one` = one two-pair context on the default
schedule (pipelined groups), `two` = two single-pair contexts issued back to back (no
synchronisation between them).  Six full-resolution steps after a warm-up; run it under
rocprofv3 --kernel-trace and read the overlap of the two pipelines from the trace."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "one"
    import bench
    from mystereomatching_amd import StereoBatch
    from mystereomatching_amd import synthetic as S
    H, W, md, paths, B, _ = bench.WORKLOADS["fullres"]
    batch = S.make_batch(2, H, W, md + 1)
    keys = ("lbgr", "rbgr", "lgray", "rgray")
    if mode == "one":
        sbs = [StereoBatch(md, H, W, 2, sgm_paths=paths)]
        sbs[0].upload(*(batch[k] for k in keys))
    else:
        sbs = []
        for i in range(2):
            sb = StereoBatch(md, H, W, 1, sgm_paths=paths, num_streams=1)
            sb.upload(*(batch[k][i:i + 1] for k in keys))
            sbs.append(sb)
    for sb in sbs:
        sb.run(0.3, download=False)
        sb.synchronize()
    t = time.perf_counter()
    for _ in range(6):
        for sb in sbs:
            sb.run(0.3, download=False)
    for sb in sbs:
        sb.synchronize()
    print(f"{mode}: {(time.perf_counter() - t) / 6 * 1e3:.2f} ms per step")


if __name__ == "__main__":
    main()
