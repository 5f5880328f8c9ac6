"""Multi-GPU batch runner: independent stereo pairs sharded across ranks.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on ROCm, "gloo" on CPU
for tests).  Rank 0 owns the global batch.  Per call:

  1. broadcast the run parameters (shape, disparity range, SolveAll lambda)        ~ 100 B
  2. scatter the pairs: contiguous blocks of ceil(n / world) pairs, zero-padded     BGR + gray
  3. every rank runs the whole hot path on its block (one set of batched launches)
  4. gather the int16 disparity maps back to rank 0 and drop the padding

There is no collective inside the per-pair computation (a pair never spans GPUs: CBCA prefix
sums and SGM paths run along whole rows and columns); the scatter/gather is the
only data exchange and is ~12 MB per 1080p pair, negligible next to the compute.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

KEYS = ("lbgr", "rbgr", "lgray", "rgray")


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous block of pair indices owned by `rank` (the last blocks may be short or empty)."""
    per = (n + world - 1) // world
    lo = min(rank * per, n)
    return lo, min(lo + per, n), per


def hip_compute_fn(max_disp: int, rows: int, cols: int, capacity: int, device: int, **overrides) -> Callable:
    """The product compute path: a StereoBatch on this rank's GPU."""
    from .stereo_matching import StereoBatch, _is_device_tensor

    sb = StereoBatch(max_disp, rows, cols, capacity, device=device, **overrides)

    def run(block: dict, reg_lambda: float):
        # device tensors (RCCL scatter output) go in and out device-to-device; no host round trip
        sb.upload(block["lbgr"], block["rbgr"], block["lgray"], block["rgray"])
        sb.run(reg_lambda, download=False)
        if _is_device_tensor(block["lgray"]):
            import torch
            out = torch.empty(tuple(block["lgray"].shape), dtype=torch.int16, device=block["lgray"].device)
            return sb.download(out)
        return sb.download()

    run.close = sb.close  # type: ignore[attr-defined]
    # the runner may hand this function device tensors on its own GPU (no host round trip)
    run.device = torch.device("cuda", device)  # type: ignore[attr-defined]
    return run


class DistributedBatchRunner:
    def __init__(self, compute_fn: Callable[[dict, float], np.ndarray], device: Optional[torch.device] = None,
                 group=None):
        self.compute_fn = compute_fn
        self.group = group
        # with a process group the collectives run even at world size 1 (RCCL on the device
        # tensors, as on 8 ranks); without one the block is rank 0's own copy
        self.collective = dist.is_initialized()
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        backend = dist.get_backend(group) if dist.is_initialized() else None
        # Blocks live on a GPU only for a compute function that takes device tensors (it says so
        # with a `device` attribute, as hip_compute_fn does) and then on that function's device:
        # RCCL needs device tensors, and a single process keeps the blocks on its GPU (one
        # host-to-device copy in, one device-to-host copy out).  Any other function (numpy-based,
        # e.g. a CPU reference) gets host arrays, as it does over gloo.
        fn_dev = getattr(compute_fn, "device", None)
        if device is not None:
            self.device = device
        elif fn_dev is not None and (backend == "nccl" or backend is None):
            self.device = torch.device(fn_dev)
        elif backend == "nccl":
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.device = torch.device("cpu")

    def _bcast_header(self, header: Optional[list]) -> list:
        t = torch.zeros(6, dtype=torch.float64, device=self.device)
        if self.rank == 0:
            t[:] = torch.tensor(header, dtype=torch.float64)
        if self.collective:
            dist.broadcast(t, 0, group=self.group)
        return t.tolist()

    def run(self, batch: Optional[dict], max_disp: int = 0, reg_lambda: float = 0.3) -> Optional[np.ndarray]:
        """batch (rank 0 only): dict of stacked arrays lbgr/rbgr [n,H,W,3], lgray/rgray [n,H,W].
        Returns the [n,H,W] int16 maps on rank 0, None elsewhere."""
        header = None
        if self.rank == 0:
            n, H, W = batch["lgray"].shape
            header = [n, H, W, max_disp, reg_lambda, 0]
        n, H, W, max_disp, reg_lambda, _ = self._bcast_header(header)
        n, H, W, max_disp = int(n), int(H), int(W), int(max_disp)
        _, _, per = shard_bounds(n, self.world, self.rank)
        # scatter the pairs
        block = {}
        for k in KEYS:
            shape = (per, H, W, 3) if "bgr" in k else (per, H, W)
            recv = torch.empty(shape, dtype=torch.uint8, device=self.device)
            chunks = None
            if self.rank == 0:
                src = torch.from_numpy(np.ascontiguousarray(batch[k]))
                pad = per * self.world - n
                if pad:
                    src = torch.cat([src, torch.zeros((pad,) + src.shape[1:], dtype=torch.uint8)])
                chunks = [c.contiguous().to(self.device) for c in src.split(per)]
            if self.collective:
                dist.scatter(recv, chunks, src=0, group=self.group)
            else:
                recv = chunks[0]   # one rank: the block is rank 0's own copy
            block[k] = recv
        lo, hi, _ = shard_bounds(n, self.world, self.rank)
        mine = hi - lo
        out = torch.zeros((per, H, W), dtype=torch.int16, device=self.device)
        if mine > 0:
            mine_block = {k: v[:mine] for k, v in block.items()}
            if self.device.type == "cpu" or getattr(self.compute_fn, "device", None) is None:
                mine_block = {k: v.cpu().numpy() for k, v in mine_block.items()}
            res = self.compute_fn(mine_block, reg_lambda)
            out[:mine] = res if isinstance(res, torch.Tensor) else torch.from_numpy(res).to(self.device)
        # gather the disparity maps to rank 0 (moved as bytes: gloo has no int16 collectives)
        raw = out.view(torch.uint8)
        if not self.collective:
            return out[:n].cpu().numpy()
        gl = [torch.empty_like(raw) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(raw, gl, dst=0, group=self.group)
        if self.rank != 0:
            return None
        return torch.cat(gl).view(torch.int16)[:n].cpu().numpy()
