"""Migrating partition (KETO_PART_MIGRATE) on one GPU with P logical parts and a loopback exchange
(test partitioning on one device before RCCL).

Every row lives on exactly one part (hash(namespace id, object)); a check's DFS moves between parts
as continuation records (repo:keto_amd/csrc/migrate.hip, keto_amd/multi.py).  The decisions must
equal the replicated snapshot's (itself pinned to the oracle) and, on the quirk-heavy random graphs,
the SQL oracle's (oracle/oracle_sql.py: internal/check/engine.go:36-123 over the reference's SQL).
"""
import numpy as np
import pytest

from keto_amd.capi import PART_MIGRATE

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _parts_from_csr(g, n_parts, hot_bytes=0):
    from keto_amd.capi import Snapshot
    parts = []
    for p in range(n_parts):
        s = Snapshot.from_csr(g.namespaces, g.row_ns, g.row_obj, g.row_rel, g.row_ptr, g.edges, device=-1)
        parts.append(s.upload_part(p, n_parts, 0, mode=PART_MIGRATE, hot_bytes=hot_bytes))
    return parts


def _route(parts, q):
    """Row-id requests -> per-part tensors of the requests each part owns, and their positions."""
    import torch
    P = len(parts)
    own = parts[0].row_owner(q["row"], P)
    own[own < 0] = 0                                            # KETO_NO_ROW: decided anywhere
    routed, where = [], []
    for p in range(P):
        sel = np.nonzero(own == p)[0]
        where.append(sel)
        routed.append(torch.from_numpy(np.ascontiguousarray(q[sel]).view(np.int32).reshape(-1, 4).copy()).to(DEV))
    return routed, where


def _mig_decide(parts, q, gmd):
    from keto_amd.multi import SnapshotMigEngine, close_filters_loopback, mig_check_loopback
    if not all(getattr(p, "_closed", False) for p in parts):
        close_filters_loopback(parts)
        for p in parts:
            p._closed = True
    routed, where = _route(parts, q)
    dec, rounds = mig_check_loopback([SnapshotMigEngine(p, DEV) for p in parts], routed, gmd, DEV)
    out = np.full(len(q), 255, dtype=np.uint8)
    for p in range(len(parts)):
        out[where[p]] = dec[p].cpu().numpy()
    return out, rounds


@pytest.mark.parametrize("n_parts,hot_bytes", [(1, 0), (2, 0), (3, 0), (5, 0), (2, 1 << 20), (3, 4 << 20), (4, 1 << 30)])
def test_powerlaw_parts_match_replicated(n_parts, hot_bytes):
    """hot_bytes > 0: the hottest rows replicated on every part (1 GiB: every set target, no stubs)."""
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 512), threads=16)
    full = g.snapshot(device=0)
    parts = _parts_from_csr(g, n_parts, hot_bytes)
    q = g.queries(60000, seed=140 + n_parts, depth=5)
    rng = np.random.default_rng(n_parts)
    q["max_depth"] = rng.integers(-1, 7, size=len(q))
    for gmd in (5, 3):
        want = full.check_batch_ids(full.with_handles(q), gmd)
        got, rounds = _mig_decide(parts, q, gmd)
        assert (got == want).all(), f"gmd {gmd}: {int((got != want).sum())} mismatches"
        if n_parts > 1 and hot_bytes < (1 << 30):
            assert rounds >= 2                                    # searches did cross parts
        if hot_bytes >= (1 << 30):
            assert rounds == 0 and all(len(p.part_stubs()) == 0 for p in parts)
    if n_parts > 1:
        st = [p.stats()["device_bytes"] for p in parts]
        assert max(st) < full.stats()["device_bytes"]


def test_nested_groups_deep_parts_match_replicated():
    """Config #3's graph at small scale: chains up to 32 deep with cycles, depth 32 -- long
    searches, big visited maps (the big-lane tier) and many crossings per search."""
    from tools import synth
    g = synth.SynthGraph(dict(n_docs=0, n_folders=0, n_groups=1 << 14, n_users=1 << 14, target_edges=0, seed=3),
                         threads=16, kind="nested", chain=32)
    full = g.snapshot(device=0)
    parts = _parts_from_csr(g, 3, hot_bytes=64 << 10)
    q = g.queries_nested(6000, seed=5, depths=(5, 16, 32, 0, 40))
    for gmd in (32, 40):
        want = full.check_batch_ids(full.with_handles(q), gmd)
        got, rounds = _mig_decide(parts, q, gmd)
        assert (got == want).all(), f"gmd {gmd}: {int((got != want).sum())} mismatches"
        assert rounds >= 2


def test_unexchanged_filters_still_exact():
    """A part whose filter exchange gave up (all-ones filters, no pruning) answers exactly too."""
    from keto_amd.multi import SnapshotMigEngine, mig_check_loopback
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 1024), threads=16)
    full = g.snapshot(device=0)
    parts = _parts_from_csr(g, 2)
    for p in parts:
        p.part_closure_done(False)
    q = g.queries(20000, seed=9, depth=5)
    want = full.check_batch_ids(full.with_handles(q), 5)
    routed, where = _route(parts, q)
    dec, _ = mig_check_loopback([SnapshotMigEngine(p, DEV) for p in parts], routed, 5, DEV)
    got = np.full(len(q), 255, dtype=np.uint8)
    for p in range(2):
        got[where[p]] = dec[p].cpu().numpy()
    assert (got == want).all()


def test_filter_exchange_gives_owner_filters():
    """After the exchange every stub carries exactly its owner's closure filter."""
    from keto_amd.multi import close_filters_loopback
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 1024), threads=16)
    parts = _parts_from_csr(g, 3)
    rounds = close_filters_loopback(parts)
    assert rounds >= 1
    for i, p in enumerate(parts):
        stubs = p.part_stubs()
        assert len(stubs)
        own = p.row_owner(stubs, 3)
        assert (own != i).all()
        for q in range(3):
            sel = stubs[own == q][:500]
            if len(sel):
                assert (p.part_filters(sel) == parts[q].part_filters(sel)).all()


def test_migrating_part_refuses_other_entry_points():
    from keto_amd.capi import KetoError, Snapshot
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 4096), threads=16)
    s = Snapshot.from_csr(g.namespaces, g.row_ns, g.row_obj, g.row_rel, g.row_ptr, g.edges, device=-1)
    part = s.upload_part(0, 2, 0, mode=PART_MIGRATE)
    q = g.queries(100, seed=1, depth=5)
    with pytest.raises(KetoError):
        part.check_batch_ids(part.with_handles(q[part.row_owner(q["row"], 2) == 0]), 5)
    import torch
    d = torch.zeros((4, 4), dtype=torch.int32, device=DEV)
    out = torch.zeros(4, dtype=torch.uint8, device=DEV)
    with pytest.raises(KetoError):                                 # the filter exchange is not done
        part.mig_begin(d.data_ptr(), 4, out.data_ptr(), 5)
    part.part_closure_done(False)
    other = q[part.row_owner(q["row"], 2) == 1][:4]
    d2 = torch.from_numpy(np.ascontiguousarray(other).view(np.int32).reshape(-1, 4).copy()).to(DEV)
    with pytest.raises(KetoError):                                 # rows another part owns
        part.mig_begin(d2.data_ptr(), len(other), out.data_ptr(), 5)


def _row_ids_of(full, ids):
    """keto_resolve_checks output (handles) -> row-id form, or None for requests with no row id
    (batch-local wildcard rows)."""
    n_rows = full.stats()["n_rows"]
    h = full.row_handles(np.arange(n_rows, dtype=np.uint32))
    inv = {int(x): r for r, x in enumerate(h) if x != 0xFFFFFFFF}
    out = ids.copy()
    ok = np.ones(len(ids), dtype=bool)
    for i, x in enumerate(ids):
        if x["row"] != 0xFFFFFFFF:
            r = inv.get(int(x["row"]))
            if r is None:
                ok[i] = False
                continue
            out[i]["row"] = r
        if x["flags"] & 1 and x["target"] != 0xFFFFFFFF:
            r = inv.get(int(x["target"]))
            if r is None:
                ok[i] = False
                continue
            out[i]["target"] = r
    return out, ok


@pytest.mark.parametrize("seed", range(60))
def test_random_graphs_match_oracle(seed):
    """Quirk-heavy random graphs (cycles, duplicates, wildcard sets, poisoned pages, visit-key
    collisions, page sizes 1..100) on 2-4 migrating parts against the SQL oracle."""
    import keto_amd
    from keto_amd.capi import KetoError
    from oracle.oracle_sql import CheckEngine
    from tests.engine_util import rows_from_tuples, subj
    from tests.randgraph import random_checks, random_store
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=seed % 5 == 4)
    rows = rows_from_tuples(ns, tuples, raw)
    full = keto_amd.Snapshot.build(ns, rows, page_size=ps, device=0)
    n_parts = 2 + seed % 3
    hot = [0, 256, 4096][seed % 3 if seed % 2 else 0]
    parts = [keto_amd.Snapshot.build(ns, rows, page_size=ps, device=-1).upload_part(p, n_parts, 0, mode=PART_MIGRATE,
                                                                                    hot_bytes=hot)
             for p in range(n_parts)]
    checks = random_checks(seed, alph, k=40)
    for gmd in sorted({c[2] for c in checks}):
        grp = []
        for t, d, g in checks:
            if g != gmd:
                continue
            try:                         # wildcard queries no stored set uses: batch-local rows, no row id
                full.resolve_checks([(t.namespace, t.object, t.relation, subj(t.subject), d)])
            except KetoError:
                continue
            grp.append((t, d, g))
        if not grp:
            continue
        ids, status = full.resolve_checks([(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in grp])
        rid, ok = _row_ids_of(full, ids)
        ok &= status == 0
        if not ok.any():
            continue
        sel = np.nonzero(ok)[0]
        got, _ = _mig_decide(parts, rid[sel], gmd)
        for k, i in enumerate(sel):
            t, d, _ = grp[i]
            assert bool(got[k]) == CheckEngine(store, gmd).subject_is_allowed(t, d), (seed, t, d, gmd)


def test_tiny_record_pool_reruns_exact(monkeypatch):
    """A record pool far too small for a round (KETO_MIG_POOL_UNITS): the records that do not fit
    are re-run from their input records once the pool has grown, and every decision stays exact."""
    from tools import synth
    monkeypatch.setenv("KETO_MIG_POOL_UNITS", "64")
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 1024), threads=16)
    full = g.snapshot(device=0)
    parts = _parts_from_csr(g, 3)
    q = g.queries(30000, seed=12, depth=5)
    want = full.check_batch_ids(full.with_handles(q), 5)
    got, rounds = _mig_decide(parts, q, 5)
    assert rounds >= 2
    assert (got == want).all(), f"{int((got != want).sum())} mismatches"
