"""BASELINE configs #3 and #5 at their full sizes, in the driver's -m gpu run (they were bench-only
parity before): the nested-groups graph of 100,000,000 tuples (chains up to 32, cycles, seed 3),
1,000,000 checks at global max-depth 32 with request depths 5 / 16 / 32, the first 20,000 compared
with the C oracle; and 100,000 expand roots on the same graph at max-depth 5, 5,000 trees compared
node for node (pre-order, child order included)."""
import numpy as np
import pytest

from tests.test_gpu_synth import _oracle_expand_nodes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nested_100m():
    from tools import synth
    g = synth.SynthGraph(dict(synth.NESTED_100M), threads=16, kind="nested", chain=32)
    snap = g.snapshot(device=0)
    yield g, snap
    snap.close()
    g.close()


def test_config3_full_scale_matches_oracle(nested_100m):
    g, snap = nested_100m
    assert g.n_edges == 100_000_000
    q = g.queries_nested(1_000_000, seed=3, depths=(5, 16, 32), threads=16)
    gpu = snap.check_batch_ids(snap.with_handles(q), 32)
    _, n = snap.last_timing()
    assert (gpu <= 1).all(), "a request was left undecided"
    k = 20_000
    tab = g.oracle_table(q[:k], 32)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q[:k]), 32, threads=16)
    assert (gpu[:k] == ref).all(), f"{int((gpu[:k] != ref).sum())} mismatches of {k} (tiers {n})"
    assert 0.2 < gpu.mean() < 0.8


def test_config5_full_scale_matches_oracle(nested_100m):
    g, snap = nested_100m
    rng = np.random.default_rng(5)
    n = 100_000
    rows = rng.integers(0, g.n_rows, size=n).astype(np.uint32)
    depths = np.zeros(n, dtype=np.int32)                      # request depth 0 -> global max-depth 5
    status, offs, nodes = snap.expand_batch_ids(rows | np.uint32(0x80000000), depths, 5)
    assert len(status) == n and (status <= 1).all()
    k = 5_000
    q = np.zeros(k, dtype=[("row", "<u4"), ("target", "<u4"), ("flags", "<u4"), ("max_depth", "<i4")])
    q["row"] = rows[:k]
    tab = g.oracle_table(q, 5)
    n_nodes = 0
    for i in range(k):
        r, want = _oracle_expand_nodes(g, tab, int(rows[i]), 5, 5)
        if r == 0:
            assert status[i] == 1, i
            continue
        assert r == 1 and status[i] == 0, i
        have = []
        for subj, info in nodes[offs[i]:offs[i + 1]]:
            leaf, nc = int(info >> 31), int(info & 0x7FFFFFFF)
            if subj >> 31:
                t = int(subj & 0x7FFFFFFF)
                have.append((leaf, 1, 0, 0xFFFF0000 + int(g.row_ns[t]), int(g.row_obj[t]), int(g.row_rel[t]), nc))
            else:
                have.append((leaf, 0, int(subj), 0, 0, 0, nc))
        n_nodes += len(have)
        assert have == want, f"root row {rows[i]}"
    assert n_nodes > 50_000
