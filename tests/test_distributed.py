"""World-size-2 gloo tests of the batch sharding path (CPU; the oracle stands in for the GPU
compute only as test infrastructure — the product path uses hip_compute_fn)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from mystereomatching_amd.batch import DistributedBatchRunner, shard_bounds

H, W, MD = 20, 28, 11


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_fn():
    from oracle import oracle as O
    cfg = O.config(H, W, MD)

    def run(block, lam):
        return np.stack([O.run({k: block[k][i] for k in block}, cfg)["disp"] for i in range(block["lgray"].shape[0])])
    return run


def _worker(rank, world, port, n, out_path, sub_batch=0, tensor_in=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mystereomatching_amd import synthetic as S
        import torch
        runner = DistributedBatchRunner(_oracle_fn(), sub_batch=sub_batch)
        batch = S.make_batch(n, H, W, MD + 1, first_index=50) if rank == 0 else None
        if batch is not None and tensor_in:
            batch = {k: torch.from_numpy(np.ascontiguousarray(batch[k])) for k in ("lbgr", "rbgr", "lgray", "rgray")}
        disp = runner.run(batch, max_disp=MD, reg_lambda=0.3)
        disp2 = runner.run(batch, max_disp=MD, reg_lambda=0.3)   # reused staging buffers
        if rank == 0:
            np.testing.assert_array_equal(disp2, disp)
        runner.close()
        if rank == 0:
            np.save(out_path, disp)
        else:
            assert disp is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [4, 3, 1])
def test_two_rank_scatter_gather_matches_single(tmp_path, n):
    out = str(tmp_path / "disp.npy")
    mp.spawn(_worker, args=(2, _free_port(), n, out), nprocs=2, join=True)
    got = np.load(out)
    from mystereomatching_amd import synthetic as S
    batch = S.make_batch(n, H, W, MD + 1, first_index=50)
    ref = _oracle_fn()({k: batch[k] for k in ("lbgr", "rbgr", "lgray", "rgray")}, 0.3)
    assert got.shape == (n, H, W)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("n,sub_batch,tensor_in", [(7, 1, False), (7, 3, False), (5, 2, True), (8, 0, False),
                                                    (11, (1, 3), False)])
def test_two_rank_sub_blocks(tmp_path, n, sub_batch, tensor_in):
    """Sub-blocks of s pairs per rank (scatter k + 1 and gather k - 1 in flight around compute k):
    ragged blocks, a last sub-block shorter than s, torch inputs, the auto size; maps in order."""
    out = str(tmp_path / "disp.npy")
    mp.spawn(_worker, args=(2, _free_port(), n, out, sub_batch, tensor_in), nprocs=2, join=True)
    got = np.load(out)
    from mystereomatching_amd import synthetic as S
    batch = S.make_batch(n, H, W, MD + 1, first_index=50)
    ref = _oracle_fn()({k: batch[k] for k in ("lbgr", "rbgr", "lgray", "rgray")}, 0.3)
    np.testing.assert_array_equal(got, ref)


def _stream_worker(rank, world, port, n, out_path, sub_batch):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mystereomatching_amd import synthetic as S
        runner = DistributedBatchRunner(_oracle_fn(), sub_batch=sub_batch)
        bs = [S.make_batch(n, H, W, MD + 1, first_index=200 + 10 * i) for i in range(3)] if rank == 0 else None
        got = runner.run_many(bs, max_disp=MD, reg_lambda=0.3)
        runner.close()
        if rank == 0:
            np.save(out_path, np.stack(got))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,sub_batch", [(5, 2), (4, 0), (3, 1)])
def test_two_rank_stream_of_batches(tmp_path, n, sub_batch):
    """run_many: three different batches as one stream of sub-blocks (batch b + 1's first scatter
    while batch b's last block computes); every batch's maps in order, equal to the oracle's."""
    out = str(tmp_path / "disp.npy")
    mp.spawn(_stream_worker, args=(2, _free_port(), n, out, sub_batch), nprocs=2, join=True)
    got = np.load(out)
    from mystereomatching_amd import synthetic as S
    for i in range(3):
        b = S.make_batch(n, H, W, MD + 1, first_index=200 + 10 * i)
        ref = _oracle_fn()({k: b[k] for k in ("lbgr", "rbgr", "lgray", "rgray")}, 0.3)
        np.testing.assert_array_equal(got[i], ref, err_msg=f"batch {i}")


def test_single_process_sub_blocks():
    """No process group: the runner pipelines rank 0's own sub-blocks (host compute function)."""
    from mystereomatching_amd import synthetic as S
    n = 5
    batch = S.make_batch(n, H, W, MD + 1, first_index=90)
    ref = _oracle_fn()({k: batch[k] for k in ("lbgr", "rbgr", "lgray", "rgray")}, 0.3)
    for sb in (0, 1, 2, 5):
        r = DistributedBatchRunner(_oracle_fn(), sub_batch=sb)
        np.testing.assert_array_equal(r.run(batch, max_disp=MD, reg_lambda=0.3), ref)
        # a stream: the same batch twice and a shuffled copy, one pipeline
        perm = [3, 0, 4, 1, 2]
        shuf = {k: v[perm] for k, v in batch.items()}
        got = r.run_many([batch, shuf, batch], max_disp=MD, reg_lambda=0.3)
        np.testing.assert_array_equal(got[0], ref)
        np.testing.assert_array_equal(got[1], ref[perm])
        np.testing.assert_array_equal(got[2], ref)
        r.close()
    with pytest.raises(ValueError):
        DistributedBatchRunner(_oracle_fn()).run_many([batch, {k: v[:3] for k, v in batch.items()}], max_disp=MD)


def test_capacity_exceeded_is_refused_at_the_header():
    """More pairs per rank than 32 sub-blocks of the compute function's capacity cannot be
    scheduled: run() refuses at the header instead of failing inside the compute call; a batch
    that fits runs as capacity-sized blocks."""
    from mystereomatching_amd import synthetic as S
    calls = []

    def fn(block, lam):
        calls.append(block["lgray"].shape[0])
        return np.zeros(block["lgray"].shape, np.int16)
    fn.capacity = 1
    r = DistributedBatchRunner(fn, sub_batch=0)
    big = {k: np.zeros((33,) + v.shape[1:], v.dtype) for k, v in S.make_batch(1, H, W, MD + 1).items()}
    with pytest.raises(ValueError, match="capacity"):
        r.run(big, max_disp=MD, reg_lambda=0.3)
    assert calls == []
    ok = {k: v[:5] for k, v in big.items()}
    assert r.run(ok, max_disp=MD, reg_lambda=0.3).shape == (5, H, W)
    assert calls == [1] * 5
    r.close()


def test_sub_sizes():
    from mystereomatching_amd.batch import sub_sizes
    assert [sub_sizes(p) for p in (0, 1, 2, 3, 4, 8, 9, 16)] == \
        [[], [1], [1, 1], [1, 1, 1], [1, 3], [1, 7], [1, 8], [2, 14]]
    for p in range(0, 40):
        for sb in (0, 1, 3, 7, [2, 4], (1, 6, 1), [50]):
            z = sub_sizes(p, sb)
            assert sum(z) == p and all(q > 0 for q in z)
    assert sub_sizes(8, 3) == [3, 3, 2] and sub_sizes(8, [1, 6]) == [1, 6, 1]


def test_shard_bounds_cover_exactly_once():
    for n in range(0, 20):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi, per = shard_bounds(n, world, r)
                assert hi - lo <= per
                seen += list(range(lo, hi))
            assert seen == list(range(n))
