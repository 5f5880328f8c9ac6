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


def _worker(rank, world, port, n, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mystereomatching_amd import synthetic as S
        runner = DistributedBatchRunner(_oracle_fn())
        batch = S.make_batch(n, H, W, MD + 1, first_index=50) if rank == 0 else None
        disp = runner.run(batch, max_disp=MD, reg_lambda=0.3)
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


def test_shard_bounds_cover_exactly_once():
    for n in range(0, 20):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi, per = shard_bounds(n, world, r)
                assert hi - lo <= per
                seen += list(range(lo, hi))
            assert seen == list(range(n))
