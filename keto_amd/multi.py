"""Multi-GPU check batches: one process per GPU, every rank holding the whole (replicated) snapshot.

The check path shards by request: requests are independent, so a batch is split into contiguous
per-rank shards, each rank runs its shard through its own GPU's engine, and the decisions are
gathered with one all-gather (RCCL over xGMI on GPUs, gloo in the CPU tests).  There is no
exchange inside the traversal.  SURVEY.md section 8(e), "replicated mode"; the reference itself
serves each check on one goroutine against one database (internal/check/handler.go:108-184).
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of n requests for `rank` of `world` (sizes differ by at most 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class ShardedChecker:
    """Runs `local_check(requests) -> uint8 decisions` on this rank's shard of every batch and
    all-gathers the decisions, so every rank returns the decisions of the whole batch.

    local_check is the rank's engine (keto_amd.Snapshot.check_batch_ids on its GPU); `device` is
    where the gather buffers live ("cuda:<local rank>" with the nccl backend, "cpu" with gloo)."""

    def __init__(self, local_check: Callable[[np.ndarray], np.ndarray], group=None, device: str = "cpu"):
        import torch.distributed as dist
        self.local_check = local_check
        self.group = group
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def __call__(self, requests: np.ndarray) -> np.ndarray:
        import torch
        import torch.distributed as dist
        n = len(requests)
        lo, hi = shard_bounds(n, self.rank, self.world)
        mine = np.asarray(self.local_check(requests[lo:hi]), dtype=np.uint8)
        if len(mine) != hi - lo:
            raise RuntimeError(f"local engine returned {len(mine)} decisions for {hi - lo} requests")
        # equal-size all-gather: pad every shard to the largest one
        width = shard_bounds(n, 0, self.world)[1]
        buf = torch.zeros(width, dtype=torch.uint8, device=self.device)
        if hi > lo:
            buf[: hi - lo] = torch.from_numpy(mine).to(self.device)
        out = torch.empty(width * self.world, dtype=torch.uint8, device=self.device)
        dist.all_gather_into_tensor(out, buf, group=self.group)
        out = out.cpu().numpy()
        res = np.empty(n, dtype=np.uint8)
        for r in range(self.world):
            a, b = shard_bounds(n, r, self.world)
            res[a:b] = out[r * width: r * width + (b - a)]
        return res
