"""The N > 1 path on CPU: world_size-2 gloo process groups run keto_amd.multi.ShardedChecker with the
C oracle as each rank's local engine (the GPU engine takes its place on the box), and the gathered
decisions must equal a single-process run over the whole batch.  Also covers the shard bounds and
bench.py's max-over-ranks timing reduction."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_exactly():
    from keto_amd.multi import shard_bounds
    for n in (0, 1, 7, 8, 1000, 1001):
        for world in (1, 2, 3, 8):
            got = [shard_bounds(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(got[r][1] == got[r + 1][0] for r in range(world - 1))
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def _worker(rank, world, port, q_bytes, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from keto_amd.multi import ShardedChecker
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 8192), threads=2)
    q = np.frombuffer(q_bytes, dtype=g.queries(1, seed=0).dtype)

    def local(part):
        if len(part) == 0:
            return np.zeros(0, dtype=np.uint8)
        tab = g.oracle_table(part, 5)
        return tab.check_batch_reqs(g.oracle_requests(tab, part), 5, threads=1)

    res = ShardedChecker(local)(q)
    # bench.py's timing reduction: max over ranks
    t = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        np.save(out_path, res)
        assert float(t.item()) == 0.5 + world - 1
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [999, 2048])
def test_sharded_checker_gloo_world2(tmp_path, n):
    import torch.multiprocessing as mp
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 8192), threads=2)
    q = g.queries(n, seed=21, depth=5)
    tab = g.oracle_table(q, 5)
    want = tab.check_batch_reqs(g.oracle_requests(tab, q), 5, threads=2)
    out = str(tmp_path / "res.npy")
    mp.start_processes(_worker, args=(2, _free_port(), q.tobytes(), out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    assert got.shape == want.shape and (got == want).all()
    assert 0.05 < want.mean() < 0.95


def _part_worker(rank, world, port, q_bytes, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from keto_amd.multi import PartitionedChecker
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 8192), threads=2)
    host = g.host_snapshot()                       # row owners come from the C-ABI (no device)
    q = np.frombuffer(q_bytes, dtype=g.queries(1, seed=0).dtype)
    seen = []

    def local(part):
        own = host.row_owner(part["row"], world)
        assert ((own == rank) | (own < 0)).all(), "a request reached a part that does not own its row"
        seen.append(int((own == rank).sum()))
        if len(part) == 0:
            return np.zeros(0, dtype=np.uint8)
        tab = g.oracle_table(part, 5)
        return tab.check_batch_reqs(g.oracle_requests(tab, part), 5, threads=1)

    lo, hi = (0, len(q) // 2) if rank == 0 else (len(q) // 2, len(q))
    res = PartitionedChecker(lambda rows: host.row_owner(rows, world), local)(q[lo:hi])
    np.save(out_path + f".{rank}.npy", res)
    np.save(out_path + f".{rank}.seen.npy", np.array(seen))
    dist.destroy_process_group()


def test_partitioned_routing_gloo_world2(tmp_path):
    """Requests whose top-level row is a root row travel to the part that owns it and come back in
    order; the decisions equal a single-process oracle run."""
    import torch.multiprocessing as mp
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 8192), threads=2)
    q = g.queries(3000, seed=31, depth=5)
    host = g.host_snapshot()
    own = host.row_owner(q["row"], 2)
    assert (own >= 0).mean() > 0.9                # the docs:d#view rows of the requests are root rows
    assert 0.3 < (own == 0).mean() < 0.7
    tab = g.oracle_table(q, 5)
    want = tab.check_batch_reqs(g.oracle_requests(tab, q), 5, threads=2)
    out = str(tmp_path / "res")
    mp.start_processes(_part_worker, args=(2, _free_port(), q.tobytes(), out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.concatenate([np.load(out + ".0.npy"), np.load(out + ".1.npy")])
    assert (got == want).all()
    routed = int(np.load(out + ".0.seen.npy").sum() + np.load(out + ".1.seen.npy").sum())
    assert routed == int((own >= 0).sum())


# ---- migrating partition: the exchange loop of keto_amd.multi.mig_check over gloo, driving a
# Python restatement of the migrating DFS (the GPU engine's protocol, repo:keto_amd/csrc/migrate.hip)
# over the synthetic CSR graph, checked against the C oracle.  Every row has an owner part; a search
# that enters a row or pops to a frame another part owns travels as a record (head, frames, visited
# map) in 16-B units.

class _PyMigEngine:
    """begin / round / fetch of SnapshotMigEngine, on the CPU, for the synthetic graphs (no
    visit-key collisions, subject-id requests): the ordered DFS of internal/check/engine.go:36-123
    with a visited map per top-level tuple, cut at part crossings."""
    ENTER, RESUME, DECISION = 0, 1, 2

    def __init__(self, g, rank, world):
        self.ptr, self.edges, self.rank, self.world = g.row_ptr, g.edges, rank, world
        self.n_sets = None

    def owner(self, r):
        return int((r * 2654435761) >> 7) % self.world

    def _sets(self, r):
        lo, hi = int(self.ptr[r]), int(self.ptr[r + 1])
        e = self.edges[lo:hi]
        k = int(np.searchsorted(~(e >> 31).astype(bool), True)) if len(e) else 0   # sets come first
        return lo, k, e[k:]

    def _run(self, st, out):
        idx, origin, T = st["idx"], st["origin"], st["T"]
        frames, vis = st["frames"], st["vis"]
        cur, enter = None, st.get("enter")
        if st["kind"] == self.RESUME:
            cur = frames.pop()
        while True:
            if enter is not None:
                r, k, fl = enter
                enter = None
                lo, n_sets, ids = self._sets(r)
                if T in set(ids.tolist()):
                    return self._decide(idx, origin, 1, out)
                if cur is not None and cur[2] > 0:
                    frames.append(cur)
                cur = [r, lo, n_sets, k, fl]
                continue
            if cur is None or cur[2] == 0:
                if not frames:
                    return self._decide(idx, origin, 0, out)
                if self.owner(frames[-1][0]) != self.rank:
                    return out.append((self.owner(frames[-1][0]), dict(st, kind=self.RESUME, frames=frames, vis=vis)))
                cur = frames.pop()
                continue
            e = int(self.edges[cur[1]])
            cur[1] += 1
            cur[2] -= 1
            c = e & 0x7FFFFFFF
            if cur[4]:                                   # top-level tuple: a fresh map
                vis = []
            if c in vis:
                continue
            vis.append(c)
            if cur[3] < 2:
                continue
            if self.owner(c) != self.rank:
                if cur[2] > 0:
                    frames.append(cur)
                return out.append((self.owner(c), dict(st, kind=self.ENTER, enter=(c, cur[3] - 1, 0), frames=frames,
                                                       vis=vis)))
            enter = (c, cur[3] - 1, 0)

    def _decide(self, idx, origin, v, out):
        if origin == self.rank:
            self.dec[idx] = v
        else:
            out.append((origin, dict(kind=self.DECISION, idx=idx, origin=origin, v=v)))

    @staticmethod
    def _pack(st):
        """A state as int32 16-B units: head, frames (5 words padded to 8), visited ids."""
        fr = st.get("frames", [])
        vis = st.get("vis", [])
        en = st.get("enter") or (0, 0, 0)
        head = [st["kind"], st["idx"], st["origin"], st.get("T", 0), st.get("v", 0), en[0], en[1], en[2],
                len(fr), len(vis), 0, 0]
        words = head + [w for f in fr for w in (list(f) + [0, 0, 0])] + list(vis)
        words += [0] * (-len(words) % 4)
        return np.array(words, dtype=np.int32)

    @staticmethod
    def _unpack(w):
        kind, idx, origin, T, v, e0, e1, e2, nf, nv = (int(x) for x in w[:10])
        fr = [list(int(y) for y in w[12 + 8 * i: 12 + 8 * i + 5]) for i in range(nf)]
        vis = [int(x) for x in w[12 + 8 * nf: 12 + 8 * nf + nv]]
        return dict(kind=kind, idx=idx, origin=origin, T=T, v=v, enter=(e0, e1, e2), frames=fr, vis=vis)

    def _emit(self, out):
        import torch
        by = [[] for _ in range(self.world)]
        for dest, st in out:
            by[dest].append(self._pack(st))
        units, recs, chunks, offs = [], [], [], []
        for d in range(self.world):
            u = 0
            for a in by[d]:
                offs.append(u)
                chunks.append(a)
                u += len(a) // 4
            units.append(u)
            recs.append(len(by[d]))
        self._buf = torch.from_numpy(np.concatenate(chunks).view(np.uint8).copy() if chunks else np.zeros(0, np.uint8))
        self._off = torch.tensor(offs, dtype=torch.int32)
        return {"units": units, "records": recs}

    def begin(self, routed, decisions, global_max_depth):
        self.dec = decisions
        out = []
        for i, (row, target, flags, d) in enumerate(routed.tolist()):
            d = global_max_depth if d <= 0 or d > global_max_depth else d
            assert self.owner(row) == self.rank
            self._run(dict(kind=self.ENTER, idx=i, origin=self.rank, T=target, enter=(row, d, 1), frames=[],
                           vis=[]), out)
        return self._emit(out)

    def round(self, buf, off, in_records, in_units):
        w = buf.numpy().view(np.int32)
        offs = off.numpy()
        out, j, base = [], 0, 0
        for s in range(self.world):
            for _ in range(in_records[s]):
                st = self._unpack(w[(base + int(offs[j])) * 4:])
                j += 1
                if st["kind"] == self.DECISION:
                    self.dec[st["idx"]] = st["v"]
                else:
                    self._run(st, out)
            base += in_units[s]
        return self._emit(out)

    def fetch(self, out):
        return self._buf, self._off


def _mig_worker(rank, world, port, q_bytes, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from keto_amd.multi import mig_check
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 8192), threads=2)
    q = np.frombuffer(q_bytes, dtype=g.queries(1, seed=0).dtype)
    eng = _PyMigEngine(g, rank, world)
    own = np.array([eng.owner(int(r)) for r in q["row"]])
    mine = q[own == rank]
    routed = torch.from_numpy(np.ascontiguousarray(mine).view(np.int32).reshape(-1, 4).copy())
    dec, rounds = mig_check(eng, routed, 5, device="cpu")
    np.save(out_path + f".{rank}.npy", dec.numpy())
    np.save(out_path + f".{rank}.rounds.npy", np.array([rounds]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_migrating_dfs_gloo(tmp_path, world):
    """keto_amd.multi.mig_check over gloo: searches cross parts as records and every decision
    equals the C oracle's on the whole graph."""
    import torch.multiprocessing as mp
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 8192), threads=2)
    q = g.queries(300, seed=41 + world, depth=5)
    tab = g.oracle_table(q, 5)
    want = tab.check_batch_reqs(g.oracle_requests(tab, q), 5, threads=2)
    out = str(tmp_path / "mig")
    mp.start_processes(_mig_worker, args=(world, _free_port(), q.tobytes(), out), nprocs=world, join=True,
                       start_method="spawn")
    eng = _PyMigEngine(g, 0, world)
    own = np.array([eng.owner(int(r)) for r in q["row"]])
    got = np.full(len(q), 255, dtype=np.uint8)
    for r in range(world):
        got[own == r] = np.load(out + f".{r}.npy")
    assert (got == want).all(), f"{int((got != want).sum())} mismatches"
    assert int(np.load(out + ".0.rounds.npy")[0]) >= 2          # searches crossed parts
    assert 0.05 < want.mean() < 0.95


# ---- expand across ranks: ShardedExpander (replicated) and PartitionedExpander (shared-rows
# partition), with the C oracle's BuildTree as each rank's local engine, against a single-process run

def _oracle_arena(g, roots, depths, gmd=5):
    """keto_expand_batch_ids' (status, offsets, nodes) from the C oracle (oracle/keto_oracle.c
    ora_expand): set subjects as bit31 | row id, ids as string ids."""
    from tests.test_gpu_synth import _oracle_expand_nodes
    rows = (roots & np.uint32(0x7FFFFFFF)).astype(np.uint32)
    q = np.zeros(len(rows), dtype=[("row", "<u4"), ("target", "<u4"), ("flags", "<u4"), ("max_depth", "<i4")])
    q["row"] = rows
    status = np.zeros(len(roots), dtype=np.int32)
    offsets = np.zeros(len(roots) + 1, dtype=np.int64)
    nodes = []
    if len(roots):
        tab = g.oracle_table(q, gmd)
        key = {(int(a), int(b), int(c)): r for r, (a, b, c) in enumerate(zip(g.row_ns, g.row_obj, g.row_rel))}
        for i, (row, d) in enumerate(zip(rows, depths)):
            if not roots[i] >> 31:                      # a SubjectID root is a leaf (engine.go:97-101)
                nodes.append((int(roots[i]), 0x80000000))
                offsets[i + 1] = len(nodes)
                continue
            r, tree = _oracle_expand_nodes(g, tab, int(row), int(d), gmd)
            status[i] = 0 if r == 1 else 1
            for leaf, is_set, sid, name, obj, rel, nc in tree:
                subj = (0x80000000 | key[(name - 0xFFFF0000, obj, rel)]) if is_set else sid
                nodes.append((subj, (0x80000000 if leaf else 0) | nc))
            offsets[i + 1] = len(nodes)
    return status, offsets, np.array(nodes, dtype=np.uint32).reshape(-1, 2)


def _expand_worker(rank, world, port, roots_b, depths_b, mode, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from keto_amd.multi import PartitionedExpander, ShardedExpander
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 8192), threads=2)
    roots = np.frombuffer(roots_b, dtype=np.uint32)
    depths = np.frombuffer(depths_b, dtype=np.int32)
    if mode == "sharded":
        st, off, nd = ShardedExpander(lambda r, d: _oracle_arena(g, r, d))(roots, depths)
    else:
        host = g.host_snapshot()
        seen = []

        def local(r, d):
            sets = (r >> 31).astype(bool)
            own = host.row_owner(r[sets] & np.uint32(0x7FFFFFFF), world)
            assert ((own == rank) | (own < 0)).all(), "a root reached a part that does not own its row"
            seen.append(int((own == rank).sum()))
            return _oracle_arena(g, r, d)

        half = len(roots) // 2
        lo, hi = (0, half) if rank == 0 else (half, len(roots))
        ex = PartitionedExpander(lambda rows: host.row_owner(rows, world), local)
        st, off, nd = ex(roots[lo:hi], depths[lo:hi])
        np.save(out_path + f".{rank}.seen.npy", np.array(seen))
    np.save(out_path + f".{rank}.st.npy", st)
    np.save(out_path + f".{rank}.off.npy", off)
    np.save(out_path + f".{rank}.nd.npy", nd)
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["sharded", "partitioned"])
def test_expanders_gloo_world2(tmp_path, mode):
    """Trees of roots split across two ranks (replicated) or routed to the part owning their row
    (shared-rows partition) come back in root order, equal to one process expanding them all."""
    import torch.multiprocessing as mp
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 8192), threads=2)
    rng = np.random.default_rng(3)
    n = 301
    roots = rng.integers(0, g.n_rows, size=n).astype(np.uint32) | np.uint32(0x80000000)
    roots[::17] = rng.integers(0, 1000, size=len(roots[::17])).astype(np.uint32)     # subject-id roots
    depths = rng.integers(0, 6, size=n).astype(np.int32)
    want = _oracle_arena(g, roots, depths)
    out = str(tmp_path / "res")
    mp.start_processes(_expand_worker, args=(2, _free_port(), roots.tobytes(), depths.tobytes(), mode, out),
                       nprocs=2, join=True, start_method="spawn")
    if mode == "sharded":
        for r in range(2):              # every rank holds the whole batch
            st, off, nd = (np.load(out + f".{r}.{k}.npy") for k in ("st", "off", "nd"))
            assert (st == want[0]).all() and (off == want[1]).all() and (nd == want[2]).all()
    else:
        parts = [tuple(np.load(out + f".{r}.{k}.npy") for k in ("st", "off", "nd")) for r in range(2)]
        st = np.concatenate([p[0] for p in parts])
        assert (st == want[0]).all()
        for i in range(n):
            p, j = (0, i) if i < n // 2 else (1, i - n // 2)
            off, nd = parts[p][1], parts[p][2]
            assert (nd[off[j]:off[j + 1]] == want[2][want[1][i]:want[1][i + 1]]).all(), i
        host = g.host_snapshot()
        own = host.row_owner(roots[roots >> 31 == 1] & np.uint32(0x7FFFFFFF), 2)
        routed = int(np.load(out + ".0.seen.npy").sum() + np.load(out + ".1.seen.npy").sum())
        assert routed == int((own >= 0).sum()) and routed > 0
