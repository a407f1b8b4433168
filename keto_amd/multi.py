"""Multi-GPU check and expand batches: one process per GPU, every rank holding the whole (replicated)
snapshot, or a part of an edge-partitioned one.

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


# ---------------------------------------------------------------------------------------------
# Expand across GPUs ("roots split across GPUs").  A batch of BuildTree roots
# (internal/expand/engine.go:33-102) is as independent as a batch of checks: every tree is built by
# one DFS with its own visited map.  Trees travel as the engine's arena: per root a status and a
# pre-order node list (keto_tree_node: subject = bit31 | row id, or a string id; info = leaf bit |
# child count).  Row and string ids are the host snapshot's, the same on every rank (every part is
# uploaded from the same build), so a tree expanded on one GPU reads the same on any other.

_TREE_NODE = np.dtype([("subject", "<u4"), ("info", "<u4")])


def _pack_trees(status, offsets, nodes):
    """(status int32 [n], offsets int64 [n+1], nodes uint32 [m, 2]) -> one int64 header per root
    (status << 40 | node count) and the uint32 node words."""
    status = np.asarray(status, dtype=np.int64)
    counts = np.diff(np.asarray(offsets, dtype=np.int64))
    return status << 40 | counts, np.ascontiguousarray(nodes, dtype=np.uint32).reshape(-1)


def _unpack_trees(head, words):
    status = (head >> 40).astype(np.int32)
    counts = head & ((1 << 40) - 1)
    offsets = np.zeros(len(head) + 1, dtype=np.int64)
    np.cumsum(counts, out=offsets[1:])
    return status, offsets, words.reshape(-1, 2)


class ShardedExpander:
    """Replicated snapshot: each rank expands its contiguous shard of the roots on its own GPU
    (local_expand(roots, depths) -> (status, offsets, nodes), e.g. Snapshot.expand_batch_ids), and
    the trees are all-gathered so every rank returns the whole batch's trees, in root order."""

    def __init__(self, local_expand, group=None, device: str = "cpu"):
        import torch.distributed as dist
        self.local_expand = local_expand
        self.group = group
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def _gather(self, arr: np.ndarray, width: int):
        import torch
        import torch.distributed as dist
        buf = torch.zeros(width, dtype=torch.int64 if arr.dtype == np.int64 else torch.int32, device=self.device)
        if len(arr):
            buf[: len(arr)] = torch.from_numpy(arr.view(np.int32) if arr.dtype == np.uint32 else arr).to(self.device)
        out = torch.empty(width * self.world, dtype=buf.dtype, device=self.device)
        dist.all_gather_into_tensor(out, buf, group=self.group)
        return out.cpu().numpy()

    def __call__(self, roots: np.ndarray, depths: np.ndarray):
        import torch
        import torch.distributed as dist
        n = len(roots)
        lo, hi = shard_bounds(n, self.rank, self.world)
        st, off, nd = self.local_expand(roots[lo:hi], depths[lo:hi])
        if len(st) != hi - lo:
            raise RuntimeError(f"local engine returned {len(st)} trees for {hi - lo} roots")
        head, words = _pack_trees(st, off, nd)
        sizes = torch.tensor([len(words)], dtype=torch.int64, device=self.device)
        all_sizes = torch.empty(self.world, dtype=torch.int64, device=self.device)
        dist.all_gather_into_tensor(all_sizes, sizes, group=self.group)
        all_sizes = all_sizes.cpu().tolist()
        hw = shard_bounds(n, 0, self.world)[1]
        heads = self._gather(head, hw)
        ww = max(1, max(all_sizes))
        wordss = self._gather(words, ww).view(np.uint32)
        h_all, w_all = [], []
        for r in range(self.world):
            a, b = shard_bounds(n, r, self.world)
            h_all.append(heads[r * hw: r * hw + (b - a)])
            w_all.append(wordss[r * ww: r * ww + all_sizes[r]])
        return _unpack_trees(np.concatenate(h_all) if h_all else np.zeros(0, np.int64),
                             np.concatenate(w_all) if w_all else np.zeros(0, np.uint32))


class PartitionedExpander:
    """Edge-partitioned snapshot (KETO_PART_SHARED): a tree below its root only visits subject-set
    targets, which every part holds, so each root is expanded on the part that owns its row (root rows
    by hash(namespace_id, object); other rows and subject-id roots where they are) and the trees come
    back with one all-to-all.  roots: keto_expand_batch_ids form (bit31 | row id for subject sets).
    owner(rows) -> int32 part per row id (-1 = every part), e.g. Snapshot.row_owner."""

    def __init__(self, owner, local_expand, group=None, device: str = "cpu"):
        import torch.distributed as dist
        self.owner = owner
        self.local_expand = local_expand
        self.group = group
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.last_routed = 0

    def _a2a(self, send: np.ndarray, sc, rc, dtype):
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(np.ascontiguousarray(send).view(dtype)).to(self.device)
        out = torch.empty(int(sum(rc)), dtype=t.dtype, device=self.device)
        dist.all_to_all_single(out, t, output_split_sizes=[int(x) for x in rc],
                               input_split_sizes=[int(x) for x in sc], group=self.group)
        return out.cpu().numpy()

    def __call__(self, roots: np.ndarray, depths: np.ndarray):
        import torch
        import torch.distributed as dist
        roots = np.ascontiguousarray(roots, dtype=np.uint32)
        depths = np.ascontiguousarray(depths, dtype=np.int32)
        n = len(roots)
        is_set = (roots >> 31).astype(bool)
        dest = np.full(n, self.rank, dtype=np.int64)
        if is_set.any():
            own = np.asarray(self.owner(roots[is_set] & np.uint32(0x7FFFFFFF)), dtype=np.int64)
            dest[is_set] = np.where(own < 0, self.rank, own)
        order = np.argsort(dest, kind="stable")
        counts = np.bincount(dest, minlength=self.world).astype(np.int64)
        c_in = torch.empty(self.world, dtype=torch.int64, device=self.device)
        dist.all_to_all_single(c_in, torch.from_numpy(counts).to(self.device), group=self.group)
        in_counts = c_in.cpu().numpy()
        req = np.empty(n, dtype=[("root", "<u4"), ("depth", "<i4")])
        req["root"], req["depth"] = roots, depths
        mine = self._a2a(req[order].view(np.int64), counts, in_counts, np.int64).view(req.dtype)
        self.last_routed = len(mine)
        st, off, nd = self.local_expand(mine["root"].copy(), mine["depth"].copy())
        head, words = _pack_trees(st, off, nd)
        # per source rank: its roots' headers, then their node words
        src_bounds = _prefix(in_counts)
        w_counts = [int(off[src_bounds[r + 1]] - off[src_bounds[r]]) * 2 for r in range(self.world)]
        w_in = torch.empty(self.world, dtype=torch.int64, device=self.device)
        dist.all_to_all_single(w_in, torch.tensor(w_counts, dtype=torch.int64, device=self.device), group=self.group)
        back_heads = self._a2a(head, in_counts, counts, np.int64)
        back_words = self._a2a(words.view(np.int32), w_counts, w_in.cpu().tolist(), np.int32).view(np.uint32)
        st_b, off_b, nd_b = _unpack_trees(back_heads, back_words)
        # back in the caller's root order
        res_counts = np.empty(n, dtype=np.int64)
        res_status = np.empty(n, dtype=np.int32)
        res_counts[order] = np.diff(off_b)
        res_status[order] = st_b
        offsets = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(res_counts, out=offsets[1:])
        nodes = np.empty((int(offsets[-1]), 2), dtype=np.uint32)
        for j, i in enumerate(order):
            nodes[offsets[i]:offsets[i + 1]] = nd_b[off_b[j]:off_b[j + 1]]
        return res_status, offsets, nodes


def _a2a(out, inp, out_splits=None, in_splits=None, group=None, comm_device=None):
    """all_to_all_single, staged through comm_device when the backend cannot use the tensors' own
    device (gloo with GPU tensors: the rehearsal of a multi-rank run on a smaller box)."""
    import torch.distributed as dist
    if comm_device is None or str(comm_device) == str(inp.device):
        dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits, group=group)
        return
    o = out.new_empty(out.shape, device=comm_device)
    dist.all_to_all_single(o, inp.to(comm_device), output_split_sizes=out_splits, input_split_sizes=in_splits,
                           group=group)
    out.copy_(o)


def route_device(d_reqs, owner_dev, rank: int, world: int, group=None, comm_device=None):
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
    _a2a(in_counts, counts, group=group, comm_device=comm_device)
    ics = in_counts.cpu().tolist()
    recv = torch.empty((sum(ics), 4), dtype=d_reqs.dtype, device=d_reqs.device)
    _a2a(recv, send, ics, cs, group, comm_device)
    return recv, (order, cs, ics)


def send_back(decisions, state, out, world: int, group=None, comm_device=None):
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
        _a2a(back, decisions.contiguous(), cs, ics, group, comm_device)
    capi.unroute_device(back.data_ptr(), order.data_ptr(), sum(cs), out.data_ptr(),
                        torch.cuda.current_stream(out.device).cuda_stream)


# ---------------------------------------------------------------------------------------------
# Migrating partition (KETO_PART_MIGRATE): every row on one part, searches migrate between parts.
#
# The reference's DFS (internal/check/engine.go:36-114) marks nodes on first encounter in SQL
# order, so it cannot be split into level-synchronous frontier exchanges without changing answers
# (SURVEY.md H1).  Each search runs on the part that owns the row it is in and moves, as one
# continuation record (its frames and visited map), when it crosses to a row another part owns
# (repo:keto_amd/csrc/migrate.hip).  A round = every part continues the searches it received, then
# one all-to-all delivers the records they emitted.  Closure filters (the exact pruning of
# DESIGN.md) are closed across parts the same way before the first batch.

def _prefix(xs):
    out = [0]
    for x in xs:
        out.append(out[-1] + int(x))
    return out


class SnapshotMigEngine:
    """The mig_* calls of one migrating part (keto_amd.capi.Snapshot) on its GPU, with the library's
    output copied into torch tensors for the exchange layer."""

    def __init__(self, snap, device="cuda:0"):
        self.snap = snap
        self.device = device

    def _stream(self):
        import torch
        return torch.cuda.current_stream(self.device).cuda_stream

    def begin(self, routed, decisions, global_max_depth):
        return self.snap.mig_begin(routed.data_ptr(), len(routed), decisions.data_ptr(), global_max_depth,
                                   self._stream())

    def round(self, buf, off, in_records, in_units):
        return self.snap.mig_round(buf.data_ptr(), off.data_ptr(), in_records, in_units, self._stream())

    def fetch(self, out):
        """(records as uint8 [16 * units], unit offsets as int32 [records]) of a begin/round output."""
        import torch
        from . import capi
        units, recs = sum(out["units"]), sum(out["records"])
        buf = torch.empty(units * 16, dtype=torch.uint8, device=self.device)
        off = torch.empty(recs, dtype=torch.int32, device=self.device)
        st = self._stream()
        if units:
            capi.device_copy(buf.data_ptr(), out["d_records"], units * 16, st)
        if recs:
            capi.device_copy(off.data_ptr(), out["d_offsets"], recs * 4, st)
        return buf, off


def mig_check(engine, routed, global_max_depth=5, group=None, device="cuda:0", max_rounds=1 << 20,
              comm_device=None):
    """Decisions (uint8 [len(routed)] on `device`) of the row-id requests routed to this rank, all
    owned by its part, on a migrating partition with one rank per part.  Every rank calls this
    collectively.  engine: SnapshotMigEngine (or an object with the same begin/round/fetch);
    comm_device: where the collectives run when the backend cannot use `device` (gloo).
    Returns (decisions, rounds)."""
    import torch
    import torch.distributed as dist
    dec = torch.full((len(routed),), 255, dtype=torch.uint8, device=device)
    if not dist.is_initialized():                      # one part, no process group: a local loop
        dl, rounds = mig_check_loopback([engine], [routed], global_max_depth, device, max_rounds)
        dec.copy_(dl[0])
        return dec, rounds
    world = dist.get_world_size(group)
    out = engine.begin(routed, dec, global_max_depth)
    rounds = 0
    while True:
        mine = sum(out["records"])
        tot = torch.tensor([mine], dtype=torch.int64, device=comm_device or device)
        dist.all_reduce(tot, group=group)
        if int(tot.item()) == 0:
            return dec, rounds
        if rounds >= max_rounds:
            raise RuntimeError(f"migrating check did not finish in {max_rounds} rounds")
        buf, off = engine.fetch(out)
        units, recs = out["units"][:world], out["records"][:world]
        cnt = torch.tensor([[u, r] for u, r in zip(units, recs)], dtype=torch.int64, device=device).reshape(-1)
        in_cnt = torch.empty_like(cnt)
        _a2a(in_cnt, cnt, group=group, comm_device=comm_device)
        ic = in_cnt.reshape(world, 2).cpu().tolist()
        in_units, in_recs = [c[0] for c in ic], [c[1] for c in ic]
        rbuf = torch.empty(sum(in_units) * 16, dtype=torch.uint8, device=device)
        _a2a(rbuf, buf, [u * 16 for u in in_units], [u * 16 for u in units], group, comm_device)
        roff = torch.empty(sum(in_recs), dtype=torch.int32, device=device)
        _a2a(roff, off, in_recs, recs, group, comm_device)
        out = engine.round(rbuf, roff, in_recs, in_units)
        rounds += 1


def mig_check_loopback(engines, routed, global_max_depth=5, device="cuda:0", max_rounds=1 << 20):
    """mig_check for every part in one process (all parts on one GPU, the exchange by copies):
    SURVEY.md section 4's "test partitioning on one device before RCCL".  routed[p]: the requests
    owned by part p.  Returns (decisions per part, rounds)."""
    import torch
    P = len(engines)
    dec = [torch.full((len(r),), 255, dtype=torch.uint8, device=device) for r in routed]
    outs = [engines[p].begin(routed[p], dec[p], global_max_depth) for p in range(P)]
    rounds = 0
    while sum(sum(o["records"]) for o in outs):
        if rounds >= max_rounds:
            raise RuntimeError(f"migrating check did not finish in {max_rounds} rounds")
        inbox = [[None] * P for _ in range(P)]
        for s in range(P):
            buf, off = engines[s].fetch(outs[s])
            ub, rb = _prefix(outs[s]["units"][:P]), _prefix(outs[s]["records"][:P])
            for q in range(P):
                inbox[q][s] = (buf[ub[q] * 16: ub[q + 1] * 16], off[rb[q]: rb[q + 1]])
        for q in range(P):
            rbuf = torch.cat([inbox[q][s][0] for s in range(P)])
            roff = torch.cat([inbox[q][s][1] for s in range(P)])
            in_units = [len(inbox[q][s][0]) // 16 for s in range(P)]
            in_recs = [len(inbox[q][s][1]) for s in range(P)]
            outs[q] = engines[q].round(rbuf, roff, in_recs, in_units)
        rounds += 1
    return dec, rounds


def close_filters_loopback(parts, max_rounds=256):
    """Closure-filter exchange of a migrating partition whose parts all live in this process:
    rounds of (every part asks each stub's owner for its filter, then ORs the answers in and
    re-closes) until a round changes nothing anywhere.  Returns the number of rounds."""
    from .capi import FILTER_WORDS
    P = len(parts)
    stubs = [p.part_stubs() for p in parts]
    owners = [parts[0].row_owner(s, P) for s in stubs]
    changed, rounds = 1, 0
    while changed and rounds < max_rounds:
        answers = []
        for i in range(P):
            f = np.zeros((len(stubs[i]), FILTER_WORDS), dtype=np.uint32)
            for q in range(P):
                sel = owners[i] == q
                if sel.any():
                    f[sel] = parts[q].part_filters(stubs[i][sel])
            answers.append(f)
        changed = sum(parts[i].part_close(stubs[i], answers[i]) for i in range(P))
        rounds += 1
    for p in parts:
        p.part_closure_done(changed == 0)
    return rounds


def close_filters_dist(snap, group=None, device="cpu", max_rounds=256):
    """close_filters_loopback with one rank per part: the stub lists go to their owners once (one
    all-to-all), then every round returns the owners' filters with one all-to-all and ends with an
    all-reduce of the changes.  Every rank calls this collectively.  Returns the number of rounds."""
    import torch
    import torch.distributed as dist
    from .capi import FILTER_WORDS
    world = dist.get_world_size(group)
    stubs = snap.part_stubs()
    own = np.asarray(snap.row_owner(stubs, world), dtype=np.int64)
    order = np.argsort(own, kind="stable")
    stubs = np.ascontiguousarray(stubs[order])
    counts = np.bincount(own, minlength=world).astype(np.int64)
    c_in = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_to_all_single(c_in, torch.from_numpy(counts).to(device), group=group)
    in_counts = c_in.cpu().numpy()
    asked_t = torch.empty(int(in_counts.sum()), dtype=torch.int32, device=device)
    dist.all_to_all_single(asked_t, torch.from_numpy(stubs.view(np.int32)).to(device),
                           output_split_sizes=in_counts.tolist(), input_split_sizes=counts.tolist(), group=group)
    asked = asked_t.cpu().numpy().view(np.uint32)
    changed, rounds = 1, 0
    while changed and rounds < max_rounds:
        ans = snap.part_filters(asked)
        got = torch.empty((len(stubs), FILTER_WORDS), dtype=torch.int32, device=device)
        dist.all_to_all_single(got, torch.from_numpy(ans.view(np.int32)).to(device),
                               output_split_sizes=counts.tolist(), input_split_sizes=in_counts.tolist(), group=group)
        ch = snap.part_close(stubs, got.cpu().numpy().view(np.uint32))
        tot = torch.tensor([ch], dtype=torch.int64, device=device)
        dist.all_reduce(tot, group=group)
        changed = int(tot.item())
        rounds += 1
    snap.part_closure_done(changed == 0)
    return rounds
