"""Streamed host batches (keto_check_batch_pairs from pinned memory, engine.hip check_streamed): one
tier-0 launch takes the batch's chunks as the copy stream lands them and turns row ids into handles
itself.  Decisions must equal the device-resident handle form (keto_check_batch_ids) and the C
oracle -- with subject-set and unknown subjects, NO_ROW requests, odd batch sizes, chunks of 2^16,
requests pushed up to tiers 1 and 2 (the handle form of those is made after tier 0), a lost chunk
mark (the kernel gives up waiting and the chunked pipeline decides the batch), and another part's
root rows (an error, as in the pipeline)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def graph():
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 1024), threads=16)
    snap = g.snapshot(device=0)
    yield g, snap
    snap.close()
    g.close()


def _requests(g, n, seed, depth):
    q = g.queries(n, seed=seed, depth=5)
    rng = np.random.default_rng(seed)
    sets = rng.random(n) < 0.2
    q["target"][sets] = rng.integers(0, g.n_rows, size=int(sets.sum()))
    q["flags"][sets] = 1
    q["target"][rng.random(n) < 0.01] = 0xFFFFFFFF
    q["row"][rng.random(n) < 0.01] = 0xFFFFFFFF
    q["max_depth"] = depth
    return q


def _want(snap, q):
    from keto_amd.capi import CHECK_IDS_DTYPE
    h = np.array(q, dtype=CHECK_IDS_DTYPE, copy=True)
    ok = q["row"] != 0xFFFFFFFF
    h["row"][ok] = snap.row_handles(q["row"][ok])
    s = (q["flags"] & 1) != 0
    t = s & (q["target"] != 0xFFFFFFFF)
    h["target"][t] = snap.row_handles(q["target"][t])
    return snap.check_batch_ids(h, 5)


def _streamed(snap, q, depth):
    from keto_amd.capi import HostBuffer, pairs_of
    p = pairs_of(q)
    hq, ho = HostBuffer(len(q), p.dtype), HostBuffer(len(q), np.uint8)
    hq.array[:] = p
    out = snap.check_batch_pairs(hq.array, depth, 5, out=ho.array).copy()
    return out, snap.last_timing_full()


@pytest.mark.parametrize("n,depth,t0cap", [(300_001, 0, 0), (262_144, 3, 0), (65_537, 5, 0), (200_003, 0, 32)])
def test_streamed_matches_handle_form(graph, monkeypatch, n, depth, t0cap):
    g, snap = graph
    monkeypatch.setenv("KETO_STREAM_MIN", "1")
    monkeypatch.setenv("KETO_STREAM_CHUNK_LOG2", "16")
    monkeypatch.setenv("KETO_CHUNK", "1000000")
    if t0cap:
        monkeypatch.setenv("KETO_TEST_T0_CAP", str(t0cap))
    q = _requests(g, n, seed=n % 97, depth=depth)
    out, t = _streamed(snap, q, depth)
    assert t["chunks"] == -(-n // 65536), t                         # the streamed path ran
    assert t["streamed"] == 1 and t["stream_stalls"] == 0 and t["stream_fallbacks"] == 0, t
    want = _want(snap, q)
    assert (out == want).all(), f"{int((out != want).sum())} mismatches of {n}"
    ids = ((q["flags"] & 1) == 0) & (q["row"] != 0xFFFFFFFF)
    tab = g.oracle_table(q[ids][:50_000], 5)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q[ids][:50_000]), 5, threads=16)
    assert (out[ids][:50_000] == ref).all()
    assert 0.05 < out.mean() < 0.95


def test_lost_chunk_mark_falls_back(graph, monkeypatch):
    """The last chunk's mark never comes: lanes give up after KETO_STREAM_WAIT_MS, and the chunked
    pipeline decides the whole batch instead."""
    g, snap = graph
    monkeypatch.setenv("KETO_STREAM_MIN", "1")
    monkeypatch.setenv("KETO_STREAM_CHUNK_LOG2", "16")
    monkeypatch.setenv("KETO_STREAM_WAIT_MS", "50")
    monkeypatch.setenv("KETO_STREAM_TEST_DROP", "1")
    monkeypatch.setenv("KETO_CHUNK", "1000000")
    q = _requests(g, 150_000, seed=7, depth=0)
    out, t = _streamed(snap, q, 0)
    assert t["chunks"] == 1, t                                       # the pipeline's one chunk
    assert t["streamed"] == 0 and t["stream_fallbacks"] == 1 and t["stream_stalls"] >= 1, t   # counted
    assert (out == _want(snap, q)).all()


def test_default_geometry_never_stalls(graph, monkeypatch):
    """The default streamed geometry (chunks of 2^20 pairs, 7/8 of the lanes, 1 s waits) on a batch of
    several chunks: one streamed launch, no lane's chunk wait hits the limit, no fallback."""
    g, snap = graph
    monkeypatch.setenv("KETO_STREAM_MIN", "1")
    q = _requests(g, 3 * (1 << 20) + 17, seed=11, depth=0)
    for _ in range(3):
        out, t = _streamed(snap, q, 0)
        assert t["streamed"] == 1 and t["stream_stalls"] == 0 and t["stream_fallbacks"] == 0, t
    assert (out == _want(snap, q)).all()


def test_streamed_rejects_foreign_root_rows(graph, monkeypatch):
    import keto_amd
    g, _ = graph
    monkeypatch.setenv("KETO_STREAM_MIN", "1")
    monkeypatch.setenv("KETO_STREAM_CHUNK_LOG2", "16")
    part = g.snapshot_part(0, 2, 0)
    q = g.queries(100_000, seed=5, depth=5)
    q["max_depth"] = 0
    own = part.row_owner(q["row"], 2)
    assert (own == 1).any()
    with pytest.raises(keto_amd.KetoError, match="another part"):
        _streamed(part, q, 0)
    mine = q[own != 1]
    out, t = _streamed(part, mine, 0)
    assert t["chunks"] == -(-len(mine) // 65536)
    tab = g.oracle_table(mine, 5)
    assert (out == tab.check_batch_reqs(g.oracle_requests(tab, mine), 5, threads=16)).all()
    part.close()
