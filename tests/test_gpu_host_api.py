"""Host-buffer entry points and per-request statuses of the C-ABI, on the GPU, against the C oracle:

* keto_check_batch_rows / keto_check_batch_ids run as a pipeline of chunks (H2D of the next chunk
  and D2H of the previous one overlapped with the check); chunk sizes from one request per chunk
  to the whole batch, pinned (keto_host_alloc) and pageable caller buffers;
* concurrent calls from several threads on one snapshot (device-resident row-id batches share the
  translation buffer: each must get its own decisions);
* a request that exceeds the final tier's limits is KETO_UNDECIDED on its own, the rest of the batch
  is decided (the reference decides every check independently, internal/check/engine.go:116-123).
"""
import os
import threading

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


def _oracle(g, q, gmd):
    tab = g.oracle_table(q, gmd)
    return tab.check_batch_reqs(g.oracle_requests(tab, q), gmd, threads=16)


@pytest.mark.parametrize("chunk,pinned,first", [(1000, False, 0), (1000, True, 0), (4096, True, 0), (1, False, 0),
                                                (0, False, 0), (1000, True, 300), (4096, False, 5000)])
def test_rows_pipeline_matches_oracle(graph, monkeypatch, chunk, pinned, first):
    """The pipelined host path (chunks of KETO_CHUNK after a first chunk of KETO_CHUNK_FIRST)
    decides like the oracle and reports its chunk count."""
    from keto_amd.capi import CHECK_IDS_DTYPE, HostBuffer
    g, snap = graph
    n = 10_007 if chunk != 1 else 700
    q = g.queries(n, seed=chunk + 3, depth=5)
    if chunk:
        monkeypatch.setenv("KETO_CHUNK", str(chunk))
    if first:
        monkeypatch.setenv("KETO_CHUNK_FIRST", str(first))
    if pinned:
        hq, ho = HostBuffer(n, CHECK_IDS_DTYPE), HostBuffer(n, np.uint8)
        hq.array[:] = q
        out = snap.check_batch_rows(hq.array, 5, out=ho.array).copy()
    else:
        out = snap.check_batch_rows(q, 5)
    t = snap.last_timing_full()
    c = max(chunk, 256) if chunk else 4 << 20
    c0 = min(c, max(first, 256)) if first else c
    want_chunks = 1 + -(-(n - min(n, c0)) // c)
    assert t["chunks"] == want_chunks and t["requests"][0] == n, t
    ref = _oracle(g, q, 5)
    assert (out == ref).all(), f"{int((out != ref).sum())} mismatches of {n}"
    # the handle form through keto_check_batch_ids (same pipeline) agrees
    assert (snap.check_batch_ids(snap.with_handles(q), 5) == ref).all()


def test_rows_pipeline_rejects_foreign_root_rows(graph):
    """A partitioned snapshot fails a host row-id batch that names another part's root row, like
    the device form does."""
    import keto_amd
    g, _ = graph
    part = g.snapshot_part(0, 2, 0)
    q = g.queries(2000, seed=5, depth=5)
    own = part.row_owner(q["row"], 2)
    assert (own == 1).any()
    with pytest.raises(keto_amd.KetoError, match="another part"):
        part.check_batch_rows(q, 5)
    mine = q[own != 1]
    ref = _oracle(g, mine, 5)
    assert (part.check_batch_rows(mine, 5) == ref).all()
    part.close()


def test_concurrent_device_row_batches(graph):
    """Threads issuing keto_check_batch_rows_device on one snapshot with different batches (the
    shared translation buffer is held from translation through the check)."""
    import torch
    g, snap = graph
    batches = [g.queries(20_000 + 3000 * i, seed=40 + i, depth=5) for i in range(4)]
    want = [snap.check_batch_ids(snap.with_handles(b), 5) for b in batches]
    errs, got = [], [None] * len(batches)

    def run(i):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            d = torch.from_numpy(batches[i].view(np.int32).reshape(-1, 4).copy()).to("cuda:0")
            out = torch.empty(len(batches[i]), dtype=torch.uint8, device="cuda:0")
            for _ in range(5):
                with torch.cuda.stream(s):
                    snap.check_batch_rows_device(d.data_ptr(), len(batches[i]), out.data_ptr(), 5, s.cuda_stream)
                s.synchronize()
                r = out.cpu().numpy()
                if not (r == want[i]).all():
                    errs.append((i, int((r != want[i]).sum())))
            got[i] = r
        except Exception as e:        # surfaced below
            errs.append((i, repr(e)))

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(batches))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs


@pytest.fixture(scope="module")
def nested():
    from tools import synth
    g = synth.SynthGraph(dict(n_docs=0, n_folders=0, n_groups=1 << 14, n_users=1 << 14, target_edges=0, seed=3),
                         threads=16, kind="nested", chain=32)
    snap = g.snapshot(device=0)
    yield g, snap
    snap.close()
    g.close()


@pytest.mark.parametrize("chunk", [0, 1000])
def test_final_tier_overflow_is_per_request(nested, monkeypatch, chunk):
    """Tiny tier-0/1 tables without the borrowing pool push deep requests to tier 2, and a tier-2
    stack of 3 frames (KETO_TEST_T2_FRAMES) leaves the deepest of them undecided: those requests
    come back KETO_UNDECIDED (keto_check_batch: status KETO_CHECK_UNDECIDED, allowed 0) and every
    other decision of the batch equals the oracle's.  The host pipeline stashes each chunk's tier-1
    overflows and decides them after the last chunk (chunks of 1000: the stash spans 6 chunks)."""
    from keto_amd.capi import UNDECIDED
    g, snap = nested
    for k, v in {"KETO_T0_CAP": "256", "KETO_T1_CAP": "1024", "KETO_NO_POOL": "1", "KETO_TEST_T2_FRAMES": "3"}.items():
        monkeypatch.setenv(k, v)
    if chunk:
        monkeypatch.setenv("KETO_CHUNK", str(chunk))
    q = g.queries_nested(6000, seed=91, depths=(16, 32, 0, 40))
    out = snap.check_batch_ids(snap.with_handles(q), 40)
    t = snap.last_timing_full()
    und = out == UNDECIDED
    assert und.sum() == t["undecided"] > 0, (int(und.sum()), t)
    assert und.mean() < 0.5 and t["requests"][2] >= t["undecided"], t
    ref = _oracle(g, q, 40)
    assert (out[~und] == ref[~und]).all(), f"{int((out[~und] != ref[~und]).sum())} mismatches"


@pytest.mark.parametrize("chunk,depth", [(1000, 0), (0, 3), (300, 5)])
def test_pairs_pipeline_matches_oracle(graph, monkeypatch, chunk, depth):
    """keto_check_batch_pairs (8-B requests, one request depth per batch): subject ids, subject-set
    subjects (bit 31) and unknown subjects, against the oracle at that request depth."""
    from keto_amd.capi import CHECK_IDS_DTYPE, pairs_of
    g, snap = graph
    q = g.queries(9_001, seed=60 + depth, depth=5)
    rng = np.random.default_rng(depth)
    sets = rng.random(len(q)) < 0.2                              # some subject-set requests
    q["target"][sets] = rng.integers(0, g.n_rows, size=int(sets.sum()))
    q["flags"][sets] = 1
    q["target"][rng.random(len(q)) < 0.01] = 0xFFFFFFFF
    q["max_depth"] = depth
    if chunk:
        monkeypatch.setenv("KETO_CHUNK", str(chunk))
    out = snap.check_batch_pairs(pairs_of(q), depth, 5)
    h = np.array(q, dtype=CHECK_IDS_DTYPE, copy=True)
    h["row"] = snap.row_handles(q["row"])
    s = (q["flags"] & 1) != 0
    t = s & (q["target"] != 0xFFFFFFFF)
    h["target"][t] = snap.row_handles(q["target"][t])
    want = snap.check_batch_ids(h, 5)
    assert (out == want).all(), f"{int((out != want).sum())} mismatches of {len(q)}"
    ids = ~s
    ref = _oracle(g, q[ids], 5)
    assert (out[ids] == ref).all()
    assert out.mean() > 0.05
