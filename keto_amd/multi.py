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


class PartitionedChecker:
    """Edge-partitioned mode, for graphs larger than one GPU (keto_snapshot_upload_part).

    Every part holds the rows that some subject set points at; the root rows (rows no subject set
    points at -- in an ACL graph the documents, which are most rows) are split by
    hash(namespace_id, object) over the parts.  A check below its top-level row only visits rows
    every part holds, so the only exchange is routing: one all-to-all sends each request to the
    owner of its top-level row (requests on shared rows stay where they are), the owner runs its
    engine, and a second all-to-all returns the decisions.  Both go over RCCL (xGMI) with the nccl
    backend.  The reference's DFS cannot be cut into level-synchronous frontier exchanges without
    changing its answers, so the partitioning keeps every traversal on one GPU.

    owner(rows) -> int32 part per row id (-1 = held by every part), e.g. Snapshot.row_owner;
    local_check(requests) -> uint8 decisions for the requests routed to this rank."""

    def __init__(self, owner: Callable[[np.ndarray], np.ndarray], local_check: Callable[[np.ndarray], np.ndarray],
                 group=None, device: str = "cpu"):
        import torch.distributed as dist
        self.owner = owner
        self.local_check = local_check
        self.group = group
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.last_routed = 0            # requests this rank received in the last call

    def __call__(self, requests: np.ndarray) -> np.ndarray:
        import torch
        import torch.distributed as dist
        n = len(requests)
        own = np.asarray(self.owner(requests["row"]), dtype=np.int64)
        dest = np.where(own < 0, self.rank, own)
        order = np.argsort(dest, kind="stable")
        send = np.ascontiguousarray(requests[order])
        counts = np.bincount(dest, minlength=self.world).astype(np.int64)
        c_out = torch.from_numpy(counts).to(self.device)
        c_in = torch.empty(self.world, dtype=torch.int64, device=self.device)
        dist.all_to_all_single(c_in, c_out, group=self.group)
        in_counts = c_in.cpu().numpy()
        item = requests.dtype.itemsize
        sb = torch.from_numpy(send.view(np.uint8).copy()).to(self.device)
        rb = torch.empty(int(in_counts.sum()) * item, dtype=torch.uint8, device=self.device)
        dist.all_to_all_single(rb, sb, output_split_sizes=(in_counts * item).tolist(),
                               input_split_sizes=(counts * item).tolist(), group=self.group)
        mine = np.frombuffer(rb.cpu().numpy().tobytes(), dtype=requests.dtype)
        self.last_routed = len(mine)
        dec = np.asarray(self.local_check(mine), dtype=np.uint8)
        if len(dec) != len(mine):
            raise RuntimeError(f"local engine returned {len(dec)} decisions for {len(mine)} requests")
        db = torch.from_numpy(dec.copy()).to(self.device)
        back = torch.empty(n, dtype=torch.uint8, device=self.device)
        dist.all_to_all_single(back, db, output_split_sizes=counts.tolist(),
                               input_split_sizes=in_counts.tolist(), group=self.group)
        res = np.empty(n, dtype=np.uint8)
        res[order] = back.cpu().numpy()
        return res


def route_device(d_reqs, owner_dev, rank: int, world: int, group=None):
    """Device-side routing of a partitioned check batch (all tensors on this rank's GPU).

    d_reqs: int32 [n, 4] keto_check_ids naming rows by row id; owner_dev: int16 [n_rows] owner part
    per row (-1 = every part).  The grouping by destination is the engine's stable counting sort
    (keto_route_rows_device, repo:keto_amd/csrc/route.hip); the exchange is one RCCL all-to-all.
    Returns (received requests [m, 4], state) where `state` carries what send_back() needs to
    return the m decisions to their origins."""
    import torch
    import torch.distributed as dist
    from . import capi
    if owner_dev.dtype != torch.int16 or not owner_dev.is_contiguous():
        raise ValueError("owner_dev must be a contiguous int16 tensor (keto_row_owner output)")
    d_reqs = d_reqs.contiguous()
    n = len(d_reqs)
    stream = torch.cuda.current_stream(d_reqs.device).cuda_stream
    wb = capi.route_work_bytes(n, world)
    work = torch.empty(max(wb, 1), dtype=torch.uint8, device=d_reqs.device)
    send = torch.empty_like(d_reqs)
    order = torch.empty(max(n, 1), dtype=torch.int32, device=d_reqs.device)
    cs = capi.route_rows_device(d_reqs.data_ptr(), n, owner_dev.data_ptr(), len(owner_dev), rank, world,
                                work.data_ptr(), wb, send.data_ptr(), order.data_ptr(), stream)
    if world == 1:
        return send, (order, cs, cs)
    counts = torch.tensor(cs, dtype=torch.int64, device=d_reqs.device)
    in_counts = torch.empty_like(counts)
    dist.all_to_all_single(in_counts, counts, group=group)
    ics = in_counts.cpu().tolist()
    recv = torch.empty((sum(ics), 4), dtype=d_reqs.dtype, device=d_reqs.device)
    dist.all_to_all_single(recv, send, output_split_sizes=ics, input_split_sizes=cs, group=group)
    return recv, (order, cs, ics)


def send_back(decisions, state, out, world: int, group=None):
    """Return the decisions of route_device()'s received requests to their origins, in the
    origin's order, into `out` (uint8 [n] on the device; keto_unroute_device)."""
    import torch
    import torch.distributed as dist
    from . import capi
    order, cs, ics = state
    if world == 1:
        back = decisions
    else:
        back = torch.empty(sum(cs), dtype=torch.uint8, device=decisions.device)
        dist.all_to_all_single(back, decisions.contiguous(), output_split_sizes=cs, input_split_sizes=ics, group=group)
    capi.unroute_device(back.data_ptr(), order.data_ptr(), sum(cs), out.data_ptr(),
                        torch.cuda.current_stream(out.device).cuda_stream)
