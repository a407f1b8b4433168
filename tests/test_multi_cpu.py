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
