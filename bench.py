"""bench.py — Mdisparities/s of the census+CBCA+SGM+WTA hot path on MI355X.

Contract (driver): python bench.py --gpus N --steps K --warmup W ; for N > 1 launched by
torch.distributed.run, one rank per GPU.  A step = one pass of the whole hot path
(cost volume -> CBCA x2 -> SolveAll -> 4-path SGM -> WTA) over one batch of synthetic pairs
already resident in HBM.  Pairs shard across ranks with no data-path collective (weak scaling:
each rank owns its own batch); RCCL is used only for the barrier and the max-over-ranks time.
With N > 1 the line also carries "e2e_batch": a few steps of the product batching path
(DistributedBatchRunner: rank 0's host batch scattered over RCCL, maps gathered back), timed after
the resident measurement.

Default workload = BASELINE.json configs[3], the largest single-GPU config and the one north_star's
targets are quoted on: Middlebury-2014 full resolution 3000x2000, D = 256, censusGrad + CBCA(2) +
SolveAll + SGM 4-path + WTA, 2 pairs per GPU.  Every map rank 0's timed loop produced is checked
bit-exact against the committed oracle map of that pair (tests/golden/bench_maps_<workload>.npz),
and the one-stream per-kernel pass must reproduce them.  Other configs:
--workload teddy (configs[1], 16 pairs, CPU baseline on whole pairs with map comparison),
kitti (configs[2]), hd (configs[4] per-GPU shard).  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mdisparities/s (W×H×D/s) + Middlebury bad-2.0 %, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

WORKLOADS = {
    # name: (H, W, max_disp, sgm_paths, pairs per GPU, description)
    "teddy": (375, 450, 63, 4, 16, "Middlebury Teddy 450x375 D=64, censusGrad+CBCA(2 it)+SolveAll+SGM 4-path+WTA "
                                   "(BASELINE configs[1], bit-exact path)"),
    "kitti": (375, 1242, 191, 8, 4, "KITTI-2015 1242x375 D=192, censusGrad+CBCA+SGM 8-path+WTA (configs[2])"),
    "fullres": (2000, 3000, 255, 4, 2, "Middlebury-2014 full-res 3000x2000 D=256, censusGrad+CBCA+SGM 4-path+WTA (configs[3])"),
    "hd": (1080, 1920, 255, 4, 8, "1920x1080 D=256 synthetic pairs, censusGrad+CBCA+SGM 4-path+WTA (configs[4] per-GPU shard)"),
}


CPU_FULL_PAIR_MAX = 200_000_000   # disparities per pair the CPU baseline runs whole (KITTI: 89 M)

# oracle fixture of synthetic pair 0 per workload (tests/golden/make_large.py / make_golden.py)
FIXTURE = {"fullres": "large_fullres_d256", "hd": "large_hd1080_d256", "kitti": "large_kitti_8path_d192",
           "teddy": "teddy_censusgrad_d64"}


SGM_RV = (+1, -1, 0, 0, +1, +1, -1, -1)   # direction table, stereoMatching.cpp:6207-6208
SGM_RU = (0, 0, +1, -1, -1, +1, +1, -1)


def kernel_symbol(name, D, paths):
    """The kernel a profile name's launches run (sm_capi.cpp names -> sm_*.hip symbols).  The
    middle SGM paths share one symbol (k_sgm<K, 0, ..>) except the straight vertical ones with
    D % 4 == 0 and D <= 128, which run k_sgm_rows (sm_sgm.hip rows_kv); the right view's SGM
    launches (suffix _r) run the left view's kernels, its CBCA sweeps a separate instantiation.
    The checkpointed SGM pairs' A passes (sgm_ck_a01, sgm_ck_a23) share one symbol too; the
    diagonal pair's (sgm_ck_a46, 8 paths) is its own instantiation."""
    base = name[:-2] if name.endswith("_r") else name
    if base == "sgm_ck_a46":
        return "k_sgm_ck<A,diag>"
    if base.startswith("sgm_ck_a"):
        return "k_sgm_ck<A>"
    if base.startswith("sgm_path"):
        i = int(base[len("sgm_path"):])
        if 0 < i < paths - 1:
            rows = SGM_RV[i] != 0 and SGM_RU[i] == 0 and D % 4 == 0 and D <= 128
            return "k_sgm_rows<mid>" if rows else "k_sgm<mid>"
        return base
    return base if base.startswith("sgm") else name


def fixture_check(workload, refine, opt, maps, batch=None):
    """Compare rank 0's maps -- every pair of the batch, as the TIMED loop left them -- with the
    committed oracle maps of those pairs (tests/golden/bench_maps_<workload>.npz, made by
    tests/golden/make_bench_maps.py; no oracle run here).  The inputs' sha256 are checked first
    when the batch is given, so an RNG drift is not reported as a kernel mismatch.  Falls back to
    the pair-0 fixture (tests/golden/large_*.npz) when a workload has no per-pair file.  A
    mismatch aborts the bench."""
    if refine or opt != "sgm":
        return None
    maps = np.asarray(maps)
    path = os.path.join(ROOT, "tests", "golden", f"bench_maps_{workload}.npz")
    if os.path.exists(path):
        z = np.load(path)
        want = z["disp"]
        n = min(len(maps), len(want))
        if batch is not None:
            import hashlib
            for i in range(n):
                for k in ("lbgr", "rbgr", "lgray", "rgray"):
                    if hashlib.sha256(np.ascontiguousarray(batch[k][i]).tobytes()).hexdigest() != str(z[f"sha_{k}_{i}"]):
                        raise SystemExit(f"bench: synthetic input {k} of pair {i} differs from bench_maps_{workload}.npz")
        per = []
        for i in range(n):
            ok = want[i].shape == maps[i].shape and bool(np.array_equal(want[i], maps[i]))
            if not ok:
                bad = int(np.count_nonzero(want[i] != maps[i])) if want[i].shape == maps[i].shape else -1
                raise SystemExit(f"bench: pair {i} map differs from bench_maps_{workload}.npz ({bad} pixels)")
            per.append({"pair": i, "bit_exact": ok})
        return {"fixture": f"tests/golden/bench_maps_{workload}.npz", "maps": "the timed loop's last step",
                "pairs_checked": n, "bit_exact": all(p["bit_exact"] for p in per), "per_pair": per}
    name = FIXTURE.get(workload)
    path = os.path.join(ROOT, "tests", "golden", f"{name}.npz") if name else None
    if not path or not os.path.exists(path):
        return None
    want = np.load(path)["disp"]
    ok = want.shape == maps[0].shape and bool(np.array_equal(want, maps[0]))
    if not ok:
        raise SystemExit(f"bench: pair 0 map differs from the oracle fixture {name}.npz")
    return {"fixture": f"tests/golden/{name}.npz", "pair": 0, "bit_exact": ok}


def _host_cpu():
    """CPU model and logical CPU count of this host (the CPU baseline's machine)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return f"{model}, {os.cpu_count()} logical CPUs"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="fullres", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="pairs per GPU (0 = workload default)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip per-kernel HIP-event timing")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle-map comparison (timing probes)")
    ap.add_argument("--no-d2h", action="store_true",
                    help="leave the maps in HBM at the end of a step (default: every timed step ends with the "
                         "int16 maps in pinned host memory, SURVEY §8d's `disp_out` ready)")
    ap.add_argument("--sub-batch", type=int, default=0, help="sm_params.sub_batch: run the pairs in groups of k")
    ap.add_argument("--streams", type=int, default=0,
                    help="sm_params.num_streams: 0 = auto (two streams, two groups for CBCA at >= 256 MiB per pair), "
                         "1 = one stream, s = groups alternate over s streams")
    ap.add_argument("--fuse-norm-scan", choices=["auto", "on", "off"], default="auto",
                    help="CBCA: fuse iteration k's normalising sweep with iteration k+1's scan (sm_params.fuse_norm_scan; "
                         "auto = for volumes >= 256 MiB per pair)")
    ap.add_argument("--no-e2e-batch", action="store_true",
                    help="N > 1: skip the DistributedBatchRunner steps reported as e2e_batch next to the resident line")
    ap.add_argument("--e2e", action="store_true",
                    help="time the product multi-GPU path instead of resident batches: rank 0 holds the global "
                         "batch on the host; each step broadcasts the header, scatters the pairs (RCCL), runs "
                         "them and gathers the int16 maps back (mystereomatching_amd.batch.DistributedBatchRunner)")
    ap.add_argument("--e2e-sub-batch", default="0",
                    help="--e2e: the sub-blocks of a rank's pairs (DistributedBatchRunner sub_batch): s pairs each, "
                         "a comma list of sizes, or 0 = auto (batch.sub_sizes)")
    ap.add_argument("--e2e-stream", action="store_true",
                    help="--e2e: time DistributedBatchRunner.run_many over the K batches as one stream (batch k + 1's "
                         "first scatter overlaps batch k's last sub-block; every batch's maps still end in host memory)")
    ap.add_argument("--e2e-input", choices=["pinned", "numpy"], default="pinned",
                    help="--e2e: rank 0's host batch as page-locked torch tensors (batch.pinned_batch) or numpy "
                         "arrays (staged into page-locked buffers by the runner's copy threads)")
    ap.add_argument("--agg", default="CBCA", choices=["CBCA", "GF", "NL"],
                    help='aggregation selector (h:52): "CBCA" (default), "GF" guided filter (cpp:4492-4516, the shipped '
                         'ximgproc::guidedFilter form; sm_params.gf_mode = 1 for MY_GUIDE), '
                         '"NL" non-local MST filter (cpp:4892-4917)')
    ap.add_argument("--opt", default="sgm", choices=["sgm", "so"],
                    help='optimization selector (h:53): "sgm" (default) or "so" scan-line DP (cpp:6272-6394)')
    ap.add_argument("--refine", action="store_true",
                    help="Do_refine = 1 (h:70): both views through CBCA/SolveAll/SGM/WTA, then refine() "
                         "(LR check, 2x region vote, 2x proper interpolation, 3x3 median)")
    return ap.parse_args()


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus and world > 1:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    return world, rank, local


def main():
    args = parse()
    world, rank, local = dist_setup(args.gpus)
    import torch
    # SM_BENCH_BACKEND=gloo rehearses the multi-rank path on a box with fewer GPUs than ranks
    # (ranks share devices round-robin; the driver's runs use RCCL, one rank per GPU)
    backend = os.environ.get("SM_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from mystereomatching_amd import StereoBatch
    from mystereomatching_amd import synthetic as S
    from mystereomatching_amd.evaluate import cal_err

    if args.e2e:
        return run_e2e(args, world, rank, local, dist, backend)

    H, W, md, paths, B0, desc = WORKLOADS[args.workload]
    B = args.batch or B0
    D = md + 1
    # this rank's shard of the global batch: pair indices [rank*B, rank*B + B)
    batch = S.make_batch(B, H, W, D, first_index=rank * B)
    sb = StereoBatch(md, H, W, B, device=local, sgm_paths=paths, do_refine=int(args.refine), optimization=args.opt,
                     aggregation=args.agg, fuse_norm_scan={"auto": -1, "on": 1, "off": 0}[args.fuse_norm_scan], sub_batch=args.sub_batch,
                     num_streams=args.streams)
    if args.agg != "CBCA":
        agg_name = {"GF": "GF (ximgproc::guidedFilter, r 9, eps 1e-4)", "NL": "NL (MST tree filter)"}[args.agg]
        desc = desc.replace("CBCA(2 it)", agg_name, 1).replace("CBCA", agg_name, 1)
    if args.opt == "so":
        desc = desc.replace("SGM 4-path+WTA", "so (scan-line DP)").replace("SGM 8-path+WTA", "so (scan-line DP)")
    if args.refine:
        desc = desc + " + Do_refine (right view CBCA/SGM, LR check, region vote, proper ipol, median)"
    sb.upload(batch["lbgr"], batch["rbgr"], batch["lgray"], batch["rgray"])

    def barrier():
        if dist is not None:
            dist.barrier()

    # A step ends with the maps on the host (t up to "disp_out ready"): the int16 maps
    # of the batch are copied into page-locked host memory on the context's copy stream
    # (sm_download_disp_async), overlapping the next step's cost / aggregation work; the next
    # step's map-writing kernels wait for the copy, and the timed region ends after the last copy.
    host_maps = torch.empty((B, H, W), dtype=torch.int16, pin_memory=True).numpy() if not args.no_d2h else None

    def step():
        sb.run(0.3, download=False)
        if host_maps is not None:
            sb.download_async(host_maps)

    for _ in range(args.warmup):
        step()
    sb.synchronize()

    barrier()
    torch.cuda.synchronize()
    sb.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sb.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the maps the TIMED loop produced (its last step, default schedule): what parity is checked on
    disp = host_maps.copy() if host_maps is not None else sb.download()
    # the first run's volume placement trials (sm_params.placement_trials; in the warm-up)
    place_ms, place_kept = sb.placement()

    # measured HBM ceiling next to the 8 TB/s spec: a dwordx4 copy over a buffer the
    # size of one pair's volume (at least 2 GiB, far past the 256 MB Infinity Cache).  After the
    # timed loop: run right before the warmup it slowed NL's first steps (Teddy x16 6.83 -> 7.32 ms
    # with three warmup steps, profiles/r5t)
    ceiling = None
    if not args.no_profile:
        ceiling = sb.copy_ceiling(max(H * W * D * 4, 2 << 30), reps=5)

    # Schedule A/B on the SAME context (same device allocations, sm_set_schedule): the default
    # schedule and one stream, timed bare in interleaved rounds (order alternating), so the
    # default can be checked against one stream without the per-instance placement spread
    # (DESIGN §6).  Reported beside the contract's timing, never instead of it.
    sched_ab = None
    if not args.no_profile and args.streams != 1 and world == 1:
        sched_ab = {"default": [], "one_stream": []}
        for r in range(3):
            order = (("default", args.streams), ("one_stream", 1))
            for name, ns in (order if r % 2 == 0 else order[::-1]):
                sb.set_schedule(ns, args.sub_batch)
                step()
                sb.synchronize()
                ta = time.perf_counter()
                for _ in range(args.steps):
                    step()
                sb.synchronize()
                sched_ab[name].append(round((time.perf_counter() - ta) / args.steps * 1e3, 4))
        sb.set_schedule(args.streams, args.sub_batch)

    # Per-kernel durations: the same K steps again with a HIP event pair around every kernel on
    # the context stream.  Kept out of the throughput timing above: each event record is a
    # barrier packet on the queue (~0.14 ms per Teddy x16 step), which perturbs the step time
    # but not the kernels' own durations.
    # With more than one stream (num_streams 0 = auto picks two for large CBCA volumes) the
    # timed loop overlaps two groups of pairs, and a kernel's launch then shares the GPU with the
    # other group's kernels; the per-kernel pass runs the same pairs through a one-stream context
    # instead, so each duration (and the roofline below) is the kernel's own.
    profile = not args.no_profile
    kernels, ms_prof = {}, None
    kern_schedule = "one stream: the timed loop's own context" if args.streams == 1 else \
        "one stream (the timed loop's own context switched by sm_set_schedule): each kernel alone; the timed " \
        "loop runs sm_params.num_streams = %d (0 = auto: two pair groups on two streams for CBCA >= 256 MiB " \
        "per pair)" % args.streams
    if profile:
        sbk = sb
        if args.streams != 1:
            sbk.set_schedule(1, args.sub_batch)
            sbk.run(0.3, download=False)
            sbk.synchronize()
        sbk.profile(True)
        sbk.profile_reset()
        tp = time.perf_counter()
        for _ in range(args.steps):
            sbk.run(0.3, download=False)
        sbk.synchronize()
        ms_prof = (time.perf_counter() - tp) / args.steps * 1e3
        kernels = sbk.profile_read()
        sbk.profile(False)
        sbk.set_schedule(args.streams, args.sub_batch)
    parity = fixture_check(args.workload, args.refine or args.agg != "CBCA", args.opt, disp, batch) \
        if rank == 0 and not args.no_parity else None
    if profile and parity is not None:
        # the one-stream per-kernel pass must have produced the same maps
        if not np.array_equal(sb.download(), disp):
            raise SystemExit("bench: the one-stream per-kernel pass's maps differ from the timed loop's")
        parity["one_stream_pass_equal"] = True
    bad2 = float(np.mean([cal_err(disp[i], batch["gt"][i], batch["nonocc"][i], 2.0)[0] for i in range(B)]))
    bad1 = float(np.mean([cal_err(disp[i], batch["gt"][i], batch["nonocc"][i], 1.0)[0] for i in range(B)]))

    elems_per_step = world * B * H * W * D
    value = elems_per_step * args.steps / elapsed / 1e6

    roofline = None
    kern_out = {}
    if kernels:
        tot = sum(k["total_ms"] for k in kernels.values())
        for name, k in kernels.items():
            if k["launches"] == 0:
                continue
            avg = k["total_ms"] / k["launches"]
            gbs = k["bytes_per_launch"] / (avg * 1e-3) / 1e9
            kern_out[name] = {"avg_ms": round(avg, 4), "share": round(k["total_ms"] / tot, 4),
                              "GB_s": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                              "bytes_per_launch": k["bytes_per_launch"]}
        # Dominant kernel = the code object with the largest share of the step, as rocprofv3
        # --stats ranks kernels: profile names whose launches run the same kernel symbol are one
        # group (kernel_symbol); achieved = the group's algorithmic bytes / its HIP-event time.
        groups = {}
        for n in kern_out:
            groups.setdefault(kernel_symbol(n, D, paths), []).append(n)
        tot_by = {g: sum(kernels[n]["total_ms"] for n in ns) for g, ns in groups.items()}
        dom = max(tot_by, key=tot_by.get)
        members = groups[dom]
        launches = sum(kernels[n]["launches"] for n in members)
        gbytes = sum(kernels[n]["bytes_per_launch"] * kernels[n]["launches"] for n in members)
        ach = gbytes / (tot_by[dom] * 1e-3) / 1e9
        traffic = None
        tag = ("_refine" if args.refine else "") + ("_so" if args.opt == "so" else "") + \
            ("" if args.agg == "CBCA" else "_" + args.agg.lower())
        pmc = os.path.join(ROOT, "profiles", f"pmc_{args.workload}{tag}_b{B}.json")
        if os.path.exists(pmc):
            try:
                pk = json.load(open(pmc)).get("kernels", {})
                tr = [pk[n]["hbm_bytes_per_launch"] * kernels[n]["launches"] for n in members]
                traffic = round(sum(tr) / launches, 1)
            except (KeyError, ValueError, TypeError):
                traffic = None
        roofline = {"bound": "hbm", "kernel": dom, "profile_names": members, "achieved": round(ach, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "bytes_per_launch": gbytes / launches}
        if ceiling is not None:
            roofline["copy_ceiling"] = round(ceiling[0], 1)
            roofline["copy_ceiling_median"] = round(ceiling[1], 1)
            roofline["frac_of_ceiling"] = round(ach / ceiling[0], 4)
            roofline["copy_ceiling_how"] = ("sm_copy_ceiling: dwordx4 non-temporal copy of %.2f GB (read + write "
                                            "counted), grids 4K/16K/64K x 5 launches, best sample" % (max(H * W * D * 4, 2 << 30) / 1e9))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        host = _host_cpu()
        if H * W * D <= CPU_FULL_PAIR_MAX:
            cfg = O.config(H, W, md, sgm_paths=paths, do_refine=int(args.refine), optimization=2 if args.opt == "so" else 1,
                           aggregation={"CBCA": 1, "GF": 2, "NL": 3}[args.agg])
            n, t_cpu = 0, 0.0
            while n == 0 or (t_cpu < args.cpu_seconds and n < B):
                pair = {k: batch[k][n] for k in ("lbgr", "rbgr", "lgray", "rgray")}
                t = time.perf_counter()
                r = O.run_ex(pair, cfg)
                t_cpu += time.perf_counter() - t
                if not np.array_equal(r["disp"], disp[n]):
                    raise SystemExit(f"bench: GPU disparity of pair {n} differs from the CPU restatement")
                n += 1
            cpu = {"value": round(n * H * W * D / t_cpu / 1e6, 3), "unit": "Mdisp/s", "cores": 1, "kind": "port",
                   "sample": f"{n} of the {B} bench pairs ({W}x{H} D={D}) through oracle/sm_oracle.c, 1 thread, "
                             f"{t_cpu:.1f} s; GPU maps checked bit-exact against it", "host": host}
        else:
            # a whole pair would take minutes and tens of GB on one core: time the restatement on
            # the first rows of pair 0 as an image of their own (full width, full D; its cost is
            # linear in H*W*D) and report that rate (parity at the full size: the fixture check
            # above and tests/test_gpu_large_fixtures.py).
            hc = max(8, min(H, CPU_FULL_PAIR_MAX // (W * D)))
            pair = {k: np.ascontiguousarray(batch[k][0][:hc]) for k in ("lbgr", "rbgr", "lgray", "rgray")}
            cfg = O.config(hc, W, md, sgm_paths=paths, do_refine=int(args.refine), optimization=2 if args.opt == "so" else 1,
                           aggregation={"CBCA": 1, "GF": 2, "NL": 3}[args.agg])
            t = time.perf_counter()
            r = O.run_ex(pair, cfg)
            t_cpu = time.perf_counter() - t
            # the crop is an image of its own: the GPU runs it too (outside the timed region) and
            # its map must equal the restatement's
            sbc = StereoBatch(md, hc, W, 1, device=local, sgm_paths=paths, do_refine=int(args.refine), optimization=args.opt,
                              aggregation=args.agg, fuse_norm_scan={"auto": -1, "on": 1, "off": 0}[args.fuse_norm_scan],
                              placement_trials=0)
            sbc.upload(pair["lbgr"][None], pair["rbgr"][None], pair["lgray"][None], pair["rgray"][None])
            crop_ok = bool(np.array_equal(sbc.run(0.3)[0], r["disp"]))
            del sbc
            if not crop_ok:
                raise SystemExit(f"bench: GPU disparity of the {W}x{hc} crop differs from the CPU restatement")
            cpu = {"value": round(hc * W * D / t_cpu / 1e6, 3), "unit": "Mdisp/s", "cores": 1, "kind": "port",
                   "sample": f"rows 0-{hc - 1} of bench pair 0 as a {W}x{hc} image (D={D}, {hc * W * D / 1e6:.0f} M "
                             f"disparities) through oracle/sm_oracle.c, 1 thread, {t_cpu:.1f} s; rate extrapolated "
                             f"linearly to the {W}x{H} pairs; the GPU's map of the same crop checked bit-exact against it",
                   "host": host}

    # N > 1: the product batching path as well (configs[4]'s RCCL scatter / gather), timed after
    # the resident-batch line and reported beside it -- never instead of it
    e2e = None
    if world > 1 and not args.no_e2e_batch:
        sb.close()
        e2e = _e2e_batch(args, world, rank, local, dist, backend, batch, H, W, md, paths, B)

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mdisp/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded piecewise-planar pairs, mystereomatching_amd/synthetic.py)",
            "config": {"workload": desc, "H": H, "W": W, "D": D, "pairs_per_gpu": B, "global_batch": B * world,
                       "sgm_paths": paths, "aggregation": args.agg, "optimization": args.opt, "refine": bool(args.refine),
                       "parallelism": f"dp{world} (independent pairs, no data-path collective)",
                       "num_streams": args.streams, "sub_batch": args.sub_batch,
                       "timed_region": "inputs resident in HBM -> maps in HBM (D2H excluded, --no-d2h)" if args.no_d2h
                       else "inputs resident in HBM -> int16 maps in pinned host memory (D2H included, each "
                            "step's copy overlapping the next step's compute; the last copy inside the region)"},
            "bad_2.0_nonocc_pct": round(100 * bad2, 3), "bad_1.0_nonocc_pct": round(100 * bad1, 3),
            "roofline": roofline, "cpu_baseline": cpu, "parity": parity, "kernels": kern_out,
            "ms_per_step_instrumented": None if ms_prof is None else round(ms_prof, 4),
            "kernels_schedule": kern_schedule if profile else None,
        }
        if place_ms:
            out["placement"] = {"how": "sm_params.placement_trials: the first (warm-up) sm_run timed its pipeline on "
                                       "candidate volume sets held at once and kept the fastest (DESIGN §6)",
                                "trial_ms": place_ms, "kept": place_kept}
        if sched_ab is not None:
            out["schedule_ab"] = {
                "how": "same context, sm_set_schedule between rounds; 3 interleaved rounds of K bare steps each",
                "default_num_streams": args.streams, "default_ms": sched_ab["default"],
                "one_stream_ms": sched_ab["one_stream"]}
            out["ms_per_step_one_stream"] = float(np.median(sched_ab["one_stream"]))
            out["ms_per_step_default_ab"] = float(np.median(sched_ab["default"]))
        if cpu:
            out["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        if e2e is not None:
            out["e2e_batch"] = e2e
        print(json.dumps(out))
    sb.close()
    if dist is not None:
        dist.destroy_process_group()


def _e2e_batch(args, world, rank, local, dist, backend, batch, H, W, md, paths, B, steps=3):
    """A few steps of mystereomatching_amd.batch.DistributedBatchRunner: rank 0 holds a global
    batch of B x world pairs on the host (its own B pairs, repeated), broadcasts the header,
    scatters the pairs over RCCL, every rank runs its block, the int16 maps are gathered back.
    Errors are reported in the JSON object, never raised (the resident line stands on its own)."""
    import torch
    from mystereomatching_amd.batch import DistributedBatchRunner, hip_compute_fn
    D = md + 1
    fn = None
    try:
        glob = None
        if rank == 0:   # page-locked host batch (batch.pinned_batch): the runner's copies need no staging
            from mystereomatching_amd.batch import pinned_batch
            glob = pinned_batch(B * world, H, W)
            for k in glob:
                glob[k].numpy()[...] = np.concatenate([batch[k]] * world)
        fn = hip_compute_fn(md, H, W, B, local, sgm_paths=paths)
        runner = DistributedBatchRunner(fn)
        maps = runner.run(glob, md, 0.3)   # warm-up
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # the steps as one stream of batches (run_many: each rank's pipeline stays full across
        # batches; every batch's maps still end in rank 0's host memory)
        maps = runner.run_many([glob] * steps if rank == 0 else None, md, 0.3)
        maps = maps[-1] if maps is not None else None
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        dist.barrier()
        t = torch.tensor([el], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        ok = None
        if rank == 0:
            ok = bool(all(np.array_equal(maps[r * B:(r + 1) * B], maps[:B]) for r in range(world)))
            fx = fixture_check(args.workload, False, "sgm", maps[:B]) if not args.no_parity and args.agg == "CBCA" \
                and args.opt == "sgm" and not args.refine else None
            if fx is not None:
                ok = ok and fx["bit_exact"]
        runner.close()
        return {"value": round(world * B * H * W * D * steps / el / 1e6, 2), "unit": "Mdisp/s",
                "ms_per_step": round(el / steps * 1e3, 4), "steps": steps, "global_batch": world * B,
                "path": f"DistributedBatchRunner.run_many ({backend}), {steps} batches as one stream: header "
                        "broadcast, each rank's pairs scattered from page-locked host memory on rank 0 while the "
                        "previous batch computes, int16 maps gathered to rank 0 host memory while the next one "
                        "computes",
                "maps_ok": ok}
    except Exception as e:   # noqa: BLE001 -- reported, not raised
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    finally:
        if fn is not None:
            fn.close()


def run_e2e(args, world, rank, local, dist, backend):
    """--e2e: DistributedBatchRunner.run timed end to end (host batch on rank 0 -> scatter ->
    compute -> gather -> host maps on rank 0).  value = pairs of the global batch x H x W x D per
    second.  No roofline / CPU baseline here: the resident-batch line is the kernel measurement."""
    import torch
    from mystereomatching_amd import synthetic as S
    from mystereomatching_amd.batch import DistributedBatchRunner, hip_compute_fn, sub_sizes

    H, W, md, paths, B0, desc = WORKLOADS[args.workload]
    B = args.batch or B0
    D = md + 1
    n = B * world
    batch = S.make_batch(n, H, W, D) if rank == 0 else None
    if batch is not None and args.e2e_input == "pinned":
        from mystereomatching_amd.batch import pinned_batch
        pb = pinned_batch(n, H, W)
        for k in pb:
            pb[k].numpy()[...] = batch[k]
        batch = pb
    fn = hip_compute_fn(md, H, W, B, local, sgm_paths=paths)
    sub = [int(x) for x in args.e2e_sub_batch.split(",")] if "," in args.e2e_sub_batch else int(args.e2e_sub_batch)
    runner = DistributedBatchRunner(fn, sub_batch=sub)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        runner.run(batch, md, 0.3)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    maps = None
    if args.e2e_stream:   # one stream of K batches (run_many); the last batch's maps are checked
        maps = runner.run_many([batch] * args.steps if rank == 0 else None, md, 0.3)
        maps = maps[-1] if maps is not None else None
    else:
        for _ in range(args.steps):
            maps = runner.run(batch, md, 0.3)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    parity = None
    if rank == 0 and not args.no_parity:
        parity = fixture_check(args.workload, False, "sgm", maps[:min(n, 64)])
    value = n * H * W * D * args.steps / elapsed / 1e6
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(value, 2), "unit": "Mdisp/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded piecewise-planar pairs, mystereomatching_amd/synthetic.py), host-resident on rank 0",
            "config": {"workload": desc + " -- end to end: broadcast header, scatter pairs, compute, gather maps",
                       "H": H, "W": W, "D": D, "pairs_per_gpu": B, "global_batch": n, "sgm_paths": paths,
                       "parallelism": f"dp{world} via DistributedBatchRunner ({backend})", "e2e": True,
                       "e2e_input": args.e2e_input,
                       "sub_blocks": [B] if args.e2e_stream and sub == 0 else sub_sizes(B, sub),
                       "e2e_stream": bool(args.e2e_stream),
                       "timed_region": ("K batches as one stream (run_many): rank 0 host batches -> maps in rank 0 "
                                        "host memory" if args.e2e_stream else
                                        "rank 0 host batch -> maps in rank 0 host memory, one run() per step")},
            "parity": parity,
        }))
    runner.close()
    fn.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
