"""GPU: device-resident batch entry points and the batch runner's product compute path."""
import contextlib

import numpy as np
import pytest

from mystereomatching_amd import StereoBatch
from mystereomatching_amd import synthetic as S
from mystereomatching_amd.batch import DistributedBatchRunner, hip_compute_fn

pytestmark = pytest.mark.gpu

KEYS = ("lbgr", "rbgr", "lgray", "rgray")


def _oracle_maps(oracle, batch, H, W, md):
    cfg = oracle.config(H, W, md)
    return np.stack([oracle.run({k: batch[k][i] for k in KEYS}, cfg)["disp"] for i in range(batch["lgray"].shape[0])])


def test_device_tensor_upload_download(oracle):
    import torch
    H, W, md, n = 41, 67, 23, 3
    batch = S.make_batch(n, H, W, md + 1, first_index=300)
    sb = StereoBatch(md, H, W, n, device=0)
    try:
        dev = {k: torch.from_numpy(np.ascontiguousarray(batch[k])).cuda() for k in KEYS}
        sb.upload(*(dev[k] for k in KEYS))
        sb.run(0.3, download=False)
        out = torch.full((n, H, W), 7, dtype=torch.int16, device="cuda")
        sb.download(out)
        got = out.cpu().numpy()
        np.testing.assert_array_equal(got, _oracle_maps(oracle, batch, H, W, md))
        # host path gives the same maps
        sb.upload(*(batch[k] for k in KEYS))
        np.testing.assert_array_equal(sb.run(0.3), got)
    finally:
        sb.close()


def test_runner_single_rank_hip(oracle):
    import torch
    H, W, md, n = 30, 52, 15, 4
    batch = S.make_batch(n, H, W, md + 1, first_index=400)
    fn = hip_compute_fn(md, H, W, n, device=0)
    try:
        runner = DistributedBatchRunner(fn, device=torch.device("cuda", 0))
        got = runner.run(batch, max_disp=md, reg_lambda=0.3)
        want = _oracle_maps(oracle, batch, H, W, md)
        np.testing.assert_array_equal(got, want)
        # one process without torch.distributed: the runner keeps the blocks on the GPU by default
        default = DistributedBatchRunner(fn)
        assert default.device.type == "cuda"
        for _ in range(2):
            np.testing.assert_array_equal(default.run(batch, max_disp=md, reg_lambda=0.3), want)
        # a stream of batches through one pipeline (run_many), device and host inputs mixed
        other = S.make_batch(n, H, W, md + 1, first_index=420)
        want2 = _oracle_maps(oracle, other, H, W, md)
        dev = {k: torch.from_numpy(np.ascontiguousarray(other[k])).cuda() for k in KEYS}
        got = DistributedBatchRunner(fn, sub_batch=1).run_many([batch, dev, other, batch], max_disp=md, reg_lambda=0.3)
        for g, w in zip(got, (want, want2, want2, want)):
            np.testing.assert_array_equal(g, w)
    finally:
        fn.close()


@pytest.mark.parametrize("sub_batch,num_streams", [(2, 2), (1, 3), (2, 1)])
def test_multi_stream_sub_batches(oracle, sub_batch, num_streams):
    """sm_params.sub_batch / num_streams only reschedule sm_run: groups of pairs alternate over
    side streams with the stagger / join events; the maps must equal the oracle's."""
    H, W, md, n = 37, 53, 19, 5
    batch = S.make_batch(n, H, W, md + 1, first_index=340)
    sb = StereoBatch(md, H, W, n, device=0, sub_batch=sub_batch, num_streams=num_streams)
    try:
        sb.upload(*(batch[k] for k in KEYS))
        first = sb.run(0.3)
        np.testing.assert_array_equal(first, _oracle_maps(oracle, batch, H, W, md))
        np.testing.assert_array_equal(sb.run(0.3), first)
    finally:
        sb.close()


def test_set_schedule_same_context(oracle):
    """sm_set_schedule switches num_streams / sub_batch between runs of one context (the bench's
    same-allocation schedule A/B): every schedule, including side streams created on first use and
    a return to one stream, gives the oracle's maps; out-of-range schedules are refused."""
    from mystereomatching_amd._capi import SMError
    H, W, md, n = 29, 61, 31, 9
    batch = S.make_batch(n, H, W, md + 1, first_index=560)
    sb = StereoBatch(md, H, W, n, device=0, num_streams=1)
    try:
        sb.upload(*(batch[k] for k in KEYS))
        want = _oracle_maps(oracle, batch, H, W, md)
        for ns, sub in ((1, 0), (0, 0), (3, 2), (1, 0), (2, 4), (0, 0)):
            sb.set_schedule(ns, sub)
            np.testing.assert_array_equal(sb.run(0.3), want, err_msg=f"num_streams {ns} sub_batch {sub}")
        for ns, sub in ((5, 0), (-1, 0), (1, -2)):
            with pytest.raises(SMError):
                sb.set_schedule(ns, sub)
    finally:
        sb.close()


def test_copy_ceiling_runs():
    """sm_copy_ceiling returns a positive best >= median rate below the 8 TB/s spec (x1.1)."""
    sb = StereoBatch(15, 16, 32, 1, device=0)
    try:
        best, med = sb.copy_ceiling(1 << 30, reps=2)
        assert 0 < med <= best < 8800
    finally:
        sb.close()


def test_auto_two_groups(oracle):
    """num_streams 0 (auto) with batch_capacity >= 8, CBCA and 4-path SGM: sm_run splits the 9
    pairs into groups of 5 and 4 on two streams, the second starting after the first's first CBCA
    sweep; the maps must equal the oracle's."""
    H, W, md, n = 29, 61, 31, 9
    batch = S.make_batch(n, H, W, md + 1, first_index=520)
    sb = StereoBatch(md, H, W, n, device=0)
    try:
        sb.upload(*(batch[k] for k in KEYS))
        first = sb.run(0.3)
        np.testing.assert_array_equal(first, _oracle_maps(oracle, batch, H, W, md))
        np.testing.assert_array_equal(sb.run(0.3), first)
    finally:
        sb.close()


def test_pipelined_runs(oracle):
    """num_streams 0 with CBCA + SGM: sm_run returns with its second group still running on the
    side stream (no join), the next run's groups follow their own stream, download_async copies
    each group's maps after that group.  Back-to-back runs with async copies, a run over fewer
    pairs (a different split: joined first), new images uploaded mid-pipeline, DP[0] read mid-
    pipeline: every map must equal the oracle's."""
    import torch
    H, W, md, n = 29, 61, 31, 9
    a = S.make_batch(n, H, W, md + 1, first_index=600)
    b = S.make_batch(n, H, W, md + 1, first_index=620)
    wa, wb = _oracle_maps(oracle, a, H, W, md), _oracle_maps(oracle, b, H, W, md)
    sb = StereoBatch(md, H, W, n, device=0)
    try:
        sb.upload(*(a[k] for k in KEYS))
        outs = [torch.empty((n, H, W), dtype=torch.int16, pin_memory=True).numpy() for _ in range(4)]
        for i in range(4):
            sb.run(0.3, download=False)
            sb.download_async(outs[i])
        sb.synchronize()
        for o in outs:
            np.testing.assert_array_equal(o, wa)
        sb.run(0.3, download=False)   # pipeline live
        np.testing.assert_array_equal(sb.get_disp(0), wa[0])
        sb.n = 7                      # fewer pairs: another split of the groups
        part = sb.run(0.3)
        np.testing.assert_array_equal(part, wa[:7])
        sb.n = n
        sb.run(0.3, download=False)   # live again, then new images
        sb.upload(*(b[k] for k in KEYS))
        for i in range(3):
            sb.run(0.3, download=False)
            sb.download_async(outs[i])
        sb.synchronize()
        for o in outs[:3]:
            np.testing.assert_array_equal(o, wb)
        np.testing.assert_array_equal(sb.run(0.3), wb)
    finally:
        sb.close()


def test_pipelined_d256_kernels(oracle):
    """The bench's timed schedule on the kernels the headline uses: D = 256 with the reference's
    lag, so the V NORM_SCAN sweep is the two-wave k_cbca_nsv2 and 4-path SGM the checkpointed
    k_sgm_ck pairs; batch_capacity 16 and num_streams 0, so sm_run pipelines two groups across
    calls (group 1 left running on the side stream).  Two image sets alternate between calls, so
    a map overwritten while its asynchronous copy still reads it, or a group reading the other
    set's inputs, shows up as a wrong map; then n changes between a download_async and the next
    run (a different group split: the copy-split race of sm_run's map-copy waits), and the one-
    stream schedule is switched in mid-pipeline.  Every map is compared with the oracle's."""
    import torch
    H, W, md, n, cap = 72, 96, 255, 8, 16
    sets = [S.make_batch(cap, H, W, md + 1, first_index=700 + 40 * s) for s in range(2)]
    want = [_oracle_maps(oracle, b, H, W, md) for b in sets]
    sb = StereoBatch(md, H, W, cap, device=0)
    try:
        # the kernels this shape reaches (one-stream pass with per-kernel events)
        sb.upload(*(sets[0][k] for k in KEYS))
        sb.set_schedule(1, 0)
        sb.profile(True)
        sb.profile_reset()
        sb.n = n
        np.testing.assert_array_equal(sb.run(0.3), want[0][:n])
        names = set(sb.profile_read())
        sb.profile(False)
        assert {"cbca_v_norm_scan", "sgm_ck_a01", "sgm_ck_b01", "sgm_ck_a23", "sgm_last_wta"} <= names, names
        sb.set_schedule(0, 0)
        outs = [torch.full((cap, H, W), -7, dtype=torch.int16, pin_memory=True).numpy() for _ in range(6)]
        # back-to-back pipelined calls, the image set alternating every call (upload joins)
        for i in range(6):
            s = i % 2
            sb.upload(*(sets[s][k] for k in KEYS))
            sb.n = n
            sb.run(0.3, download=False)
            sb.download_async(outs[i][:n])
        sb.synchronize()
        for i in range(6):
            np.testing.assert_array_equal(outs[i][:n], want[i % 2][:n], err_msg=f"call {i}")
        # the same set, no upload in between: the steady pipelined state the bench times
        sb.upload(*(sets[1][k] for k in KEYS))
        sb.n = n
        for i in range(4):
            sb.run(0.3, download=False)
            sb.download_async(outs[i][:n])
        sb.synchronize()
        for i in range(4):
            np.testing.assert_array_equal(outs[i][:n], want[1][:n], err_msg=f"steady call {i}")
        # n = 10 (groups 5 + 5), async copy, then n = 16 (groups 8 + 8) on the other set: the new
        # group 0 writes pairs 5-7, which the previous call's SECOND copy reads
        sb.upload(*(sets[0][k] for k in KEYS))
        sb.n = 10
        sb.run(0.3, download=False)
        sb.download_async(outs[0][:10])
        sb.upload(*(sets[1][k] for k in KEYS))
        sb.n = cap
        sb.run(0.3, download=False)
        sb.download_async(outs[1])
        sb.synchronize()
        np.testing.assert_array_equal(outs[0][:10], want[0][:10])
        np.testing.assert_array_equal(outs[1], want[1])
        # one stream switched in while the pipeline is live, then back
        sb.run(0.3, download=False)
        sb.set_schedule(1, 0)
        np.testing.assert_array_equal(sb.run(0.3), want[1])
        sb.set_schedule(0, 0)
        np.testing.assert_array_equal(sb.run(0.3), want[1])
    finally:
        sb.close()


@pytest.mark.parametrize("n,caps", [(5, (3, 3)), (4, (2, 2, 2)), (1, (1, 1))])
def test_run_batch_multi_contexts(oracle, n, caps):
    """sm_run_batch_multi over several contexts on device 0 (one host thread each): contiguous
    blocks of ceil(n / nctx) pairs, maps returned in pair order, equal to the oracle's."""
    from mystereomatching_amd import run_batch_multi
    H, W, md = 33, 47, 15
    batch = S.make_batch(n, H, W, md + 1, first_index=360)
    sbs = [StereoBatch(md, H, W, c, device=0) for c in caps]
    try:
        got = run_batch_multi(sbs, *(batch[k] for k in KEYS))
        np.testing.assert_array_equal(got, _oracle_maps(oracle, batch, H, W, md))
    finally:
        for sb in sbs:
            sb.close()


def test_runner_numpy_fn_gets_host_arrays(oracle):
    """A compute function without a `device` attribute (numpy-based) gets host arrays even in a
    process with a GPU; hip_compute_fn's blocks stay on its own device."""
    H, W, md, n = 20, 28, 11, 3
    batch = S.make_batch(n, H, W, md + 1, first_index=420)
    seen = []

    def fn(block, lam):
        seen.append(type(block["lgray"]))
        return _oracle_maps(oracle, block, H, W, md)

    got = DistributedBatchRunner(fn).run(batch, max_disp=md, reg_lambda=0.3)
    assert seen and all(t is np.ndarray for t in seen)
    np.testing.assert_array_equal(got, _oracle_maps(oracle, batch, H, W, md))


@contextlib.contextmanager
def _rccl_world_one():
    """An initialised `nccl` (RCCL) process group of size 1 on device 0 (127.0.0.1 rendezvous)."""
    import socket
    import torch
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        yield
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sub_batch,inp", [(0, "numpy"), (1, "pinned"), (2, "numpy"), (2, "device")])
def test_runner_rccl_world_one(oracle, sub_batch, inp):
    """DistributedBatchRunner over an initialised `nccl` (RCCL) process group of size 1: header
    broadcast, scatter and gather run as RCCL collectives on device tensors, as on the 8-GPU node
    (configs[4]), in sub-blocks (scatter k + 1 and gather k - 1 in flight around compute k) from
    numpy, page-locked or device inputs; the maps must equal the oracle's."""
    import torch
    from mystereomatching_amd.batch import pinned_batch
    H, W, md, n = 30, 52, 15, 5
    batch = S.make_batch(n, H, W, md + 1, first_index=440)
    src = batch
    if inp == "pinned":
        src = pinned_batch(n, H, W)
        for k in KEYS:
            src[k].numpy()[...] = batch[k]
    elif inp == "device":
        src = {k: torch.from_numpy(np.ascontiguousarray(batch[k])).cuda() for k in KEYS}
    with _rccl_world_one():
        fn = hip_compute_fn(md, H, W, n, device=0)
        try:
            runner = DistributedBatchRunner(fn, sub_batch=sub_batch)
            assert runner.collective and runner.device.type == "cuda"
            want = _oracle_maps(oracle, batch, H, W, md)
            for _ in range(3):
                np.testing.assert_array_equal(runner.run(src, max_disp=md, reg_lambda=0.3), want)
            runner.close()
        finally:
            fn.close()


@pytest.mark.parametrize("sub_batch", [1, 3])
def test_runner_single_process_sub_blocks(oracle, sub_batch):
    """No process group, device compute: sub-block k + 1's inputs are copied on the copy stream
    while sub-block k computes and its maps copied out after; maps in order, runs repeatable."""
    H, W, md, n = 30, 52, 15, 7
    batch = S.make_batch(n, H, W, md + 1, first_index=480)
    fn = hip_compute_fn(md, H, W, n, device=0)
    try:
        runner = DistributedBatchRunner(fn, sub_batch=sub_batch)
        want = _oracle_maps(oracle, batch, H, W, md)
        for _ in range(2):
            np.testing.assert_array_equal(runner.run(batch, max_disp=md, reg_lambda=0.3), want)
        runner.close()
    finally:
        fn.close()


def test_runner_rccl_hd1080_rank_shard():
    """configs[4] on one rank: one rank's share of the 64-pair batch (8 synthetic pairs of
    1920 x 1080, D = 256) through DistributedBatchRunner over RCCL (broadcast, scatter of the
    images as device tensors, the whole hot path per pair, gather of the int16 maps), i.e.
    main_.cpp:135-163 per pair.  Pair 0 must equal the oracle fixture large_hd1080_d256 bit for
    bit, and all 8 maps must equal a plain StereoBatch.run of the same pairs."""
    import hashlib
    import os
    H, W, md, n = 1080, 1920, 255, 8
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "large_hd1080_d256.npz"))
    assert (int(z["H"]), int(z["W"]), int(z["max_disp"]), int(z["index"])) == (H, W, md, 0)
    batch = S.make_batch(n, H, W, md + 1, first_index=0)
    for k in KEYS:
        assert hashlib.sha256(np.ascontiguousarray(batch[k][0]).tobytes()).hexdigest() == str(z["sha_" + k])
    with _rccl_world_one():
        fn = hip_compute_fn(md, H, W, n, device=0)
        try:
            runner = DistributedBatchRunner(fn)
            assert runner.collective and runner.device.type == "cuda"
            got = runner.run(batch, max_disp=md, reg_lambda=0.3)
        finally:
            fn.close()
    assert got.shape == (n, H, W)
    np.testing.assert_array_equal(got[0], z["disp"])
    sb = StereoBatch(md, H, W, n, device=0)
    try:
        sb.upload(*(batch[k] for k in KEYS))
        np.testing.assert_array_equal(got, sb.run(0.3))
    finally:
        sb.close()


def test_async_map_download_overlaps_next_run(oracle):
    """sm_download_disp_async: the copy of run k's maps (copy stream) must not see run k+1's maps
    -- run k+1's map-writing kernels wait for it -- and must be complete after synchronize()."""
    import torch
    H, W, md, n = 29, 61, 19, 3
    a = S.make_batch(n, H, W, md + 1, first_index=460)
    b = S.make_batch(n, H, W, md + 1, first_index=470)
    sb = StereoBatch(md, H, W, n, device=0)
    try:
        bufs = [torch.empty((n, H, W), dtype=torch.int16, pin_memory=True).numpy() for _ in range(2)]
        for rnd in range(2):
            for i, bt in enumerate((a, b)):
                sb.upload(*(bt[k] for k in KEYS))
                sb.run(0.3, download=False)
                sb.download_async(bufs[i])
            sb.synchronize()
            np.testing.assert_array_equal(bufs[0], _oracle_maps(oracle, a, H, W, md), err_msg=f"round {rnd}, batch a")
            np.testing.assert_array_equal(bufs[1], _oracle_maps(oracle, b, H, W, md), err_msg=f"round {rnd}, batch b")
    finally:
        sb.close()


def test_placement_trials_keep_maps(oracle):
    """sm_params.placement_trials: the first sm_run times its pipeline on k candidate volume sets
    (held at once) and keeps the fastest; the maps of that and every later run equal the oracle's,
    the trial times are reported, and contexts without trials report none."""
    H, W, md, n = 40, 72, 255, 3
    batch = S.make_batch(n, H, W, md + 1, first_index=760)
    want = _oracle_maps(oracle, batch, H, W, md)
    for k in (3, 2, 0):
        sb = StereoBatch(md, H, W, n, device=0, placement_trials=k)
        try:
            sb.upload(*(batch[key] for key in KEYS))
            np.testing.assert_array_equal(sb.run(0.3), want, err_msg=f"trials {k}, first run")
            np.testing.assert_array_equal(sb.run(0.3), want, err_msg=f"trials {k}, second run")
            ms, kept = sb.placement()
            if k:
                assert len(ms) == k and 0 <= kept < k and all(t > 0 for t in ms), (ms, kept)
                assert ms[kept] == min(ms)
            else:
                assert (ms, kept) == ([], -1)
        finally:
            sb.close()


def test_async_upload_stream(oracle):
    """sm_upload_batch_async + sm_run + sm_download_disp_async back to back, no host wait and no
    join in between (the batch runner's asynchronous form): the next call's inputs are copied in
    behind the previous call's pair groups on their own streams.  Two image sets alternate (a copy
    racing a group that still reads its pairs would mix them), download_wait(1) releases the
    previous call's maps mid-stream, then a call with fewer pairs (another group split: joined)
    and a synchronous upload.  Every map equals the oracle's."""
    import torch
    H, W, md, n = 72, 96, 255, 8
    sets = [S.make_batch(n, H, W, md + 1, first_index=840 + 20 * s) for s in range(2)]
    want = [_oracle_maps(oracle, b, H, W, md) for b in sets]
    dev = [{k: torch.from_numpy(np.ascontiguousarray(b[k])).cuda() for k in KEYS} for b in sets]
    torch.cuda.synchronize()
    sb = StereoBatch(md, H, W, n, device=0)
    try:
        outs = [torch.full((n, H, W), -5, dtype=torch.int16, pin_memory=True).numpy() for _ in range(6)]
        for i in range(6):
            sb.upload_async(*(dev[i % 2][k] for k in KEYS))
            sb.run(0.3, download=False)
            sb.download_async(outs[i])
            if i >= 1:
                sb.download_wait(1)
                np.testing.assert_array_equal(outs[i - 1], want[(i - 1) % 2], err_msg=f"call {i - 1}")
            sb.upload_wait()
        sb.download_wait(0)
        np.testing.assert_array_equal(outs[5], want[1])
        sub = {k: dev[0][k][:5] for k in KEYS}
        sb.upload_async(*(sub[k] for k in KEYS))
        np.testing.assert_array_equal(sb.run(0.3), want[0][:5])
        sb.upload(*(sets[1][k] for k in KEYS))
        np.testing.assert_array_equal(sb.run(0.3), want[1])
    finally:
        sb.close()
