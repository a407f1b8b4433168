"""Arenas past 32 GiB (snapshot.hpp SEG_SHIFT): subject-set targets keep handles below 2^31, root rows
lie above, in arena segments 2 and 3.  KETO_TEST_ROOT_BASE lays a small graph out that way (the
roots from just below 3 x 2^32 words on, a ~48 GiB arena on the device whose gap is never built on
the host); KETO_TEST_TGT_RESERVE shrinks the reserve for targets later writes add, so that a write
overflows it and the snapshot lays its arena out afresh inside keto_snapshot_apply.

Wide arenas (past 64 GiB, snapshot.hpp hword; round 6): the roots past word 2^33 take handles in
units of 32, 64 or 128 B, and tier 0 keeps a root's segment (any of up to 18) in a register
(check_wave_kernel_wide).  The same tests run on a wide layout at ~80 GiB (32-B units, roots in
segments 4 and 5), at ~100 GiB (64-B units, segments 6 and 7) and at 48 GiB forced to 128-B units
(KETO_TEST_ROOT_G), each a real device allocation of that size.

Every decision and tree is compared with the oracle (or with the same graph in an ordinary layout):
checks at max-depth 5 (tier 0), 9 (the 8-frame tier 0), 16 and 32 (top-level items, the reachability
pretest -- whose index holds target handles only, below 2^31 in every layout -- and check_kernel), subject-set requests naming root rows (handles past 2^31, never
allowed: no tuple has them as subject), expand trees rooted at high rows, the streamed pair form, and
writes interleaved with checks and expands against the SQL oracle."""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT_BASE = 3 * (1 << 32) - (1 << 16)        # words: roots straddle segments 2 and 3
# layout -> (KETO_TEST_ROOT_BASE in words, KETO_TEST_ROOT_G or None, root unit g, root segments)
LAYOUTS = {
    "split48": (ROOT_BASE, None, 0, (2, 3)),
    "wide48_g3": (ROOT_BASE, 3, 3, (2, 3)),
    "wide80": ((1 << 34) + (1 << 32) - (1 << 16), None, 1, (4, 5)),
    "wide100": ((7 << 32) - (1 << 16), None, 2, (6, 7)),
}


def _env(layout):
    base, force_g, _, _ = LAYOUTS[layout]
    env = {"KETO_TEST_ROOT_BASE": str(base)}
    if force_g is not None:
        env["KETO_TEST_ROOT_G"] = str(force_g)
    return env


def hword(h, g):
    h = np.asarray(h, dtype=np.uint64)
    return np.where(h < (1 << 31), h * np.uint64(4), np.uint64(1 << 33) + ((h - np.uint64(1 << 31)) << np.uint64(2 + g)))


@pytest.fixture(scope="module")
def graph():
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 4096), threads=16)
    plain = g.snapshot(device=0)
    yield g, plain
    plain.close()
    g.close()


@pytest.fixture(scope="module", params=list(LAYOUTS))
def split(request, graph):
    g, plain = graph
    env = _env(request.param)
    os.environ.update(env)
    try:
        snap = g.snapshot(device=0)
    finally:
        for k in env:
            del os.environ[k]
    snap.layout = request.param
    yield g, snap, plain
    snap.close()


def test_split_layout_places_roots_high(split):
    g, snap, _ = split
    _, _, rg, segs = LAYOUTS[snap.layout]
    h = snap.row_handles(np.arange(g.n_rows, dtype=np.uint32)).astype(np.int64)
    assert (h < (1 << 31)).any()                               # the targets
    assert (h >= (1 << 31)).mean() > 0.5                       # the roots
    seg = hword(h[h >= (1 << 31)], rg) >> np.uint64(32)
    assert set(np.unique(seg).tolist()) == set(segs)           # both segments
    if rg:
        assert snap.stats()["device_bytes"] > (LAYOUTS[snap.layout][0] * 4)


@pytest.mark.parametrize("gmd", [5, 9, 16, 32])
def test_split_checks_match_oracle(split, gmd):
    g, snap, _ = split
    q = g.queries(20000, seed=700 + gmd, depth=gmd)
    gpu = snap.check_batch_ids(snap.with_handles(q), gmd)
    tab = g.oracle_table(q, gmd)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), gmd, threads=16)
    assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)}"
    assert 0.05 < gpu.mean() < 0.95


def test_split_subject_set_requests_equal_plain_layout(split):
    """Subject-set requests whose target is any row -- root rows included, whose handles do not fit
    an edge -- decide like the same graph in the ordinary layout (rows by row id, both forms)."""
    from keto_amd.capi import pairs_of
    g, snap, plain = split
    q = g.queries(30000, seed=71, depth=5)
    rng = np.random.default_rng(71)
    sets = rng.random(len(q)) < 0.5
    q["target"][sets] = rng.integers(0, g.n_rows, size=int(sets.sum()))
    q["flags"][sets] = 1
    want = plain.check_batch_rows(q, 5)
    assert (snap.check_batch_rows(q, 5) == want).all()
    q["max_depth"] = 0
    assert (snap.check_batch_pairs(pairs_of(q), 0, 5) == plain.check_batch_pairs(pairs_of(q), 0, 5)).all()


def test_split_streamed_pairs_equal_plain_layout(split, monkeypatch):
    from keto_amd.capi import HostBuffer, pairs_of
    g, snap, plain = split
    monkeypatch.setenv("KETO_STREAM_MIN", "1")
    monkeypatch.setenv("KETO_STREAM_CHUNK_LOG2", "16")
    q = g.queries(200_000, seed=72, depth=5)
    q["max_depth"] = 0
    p = pairs_of(q)
    hq, ho = HostBuffer(len(q), p.dtype), HostBuffer(len(q), np.uint8)
    hq.array[:] = p
    got = snap.check_batch_pairs(hq.array, 0, 5, out=ho.array).copy()
    assert snap.last_timing_full()["chunks"] == -(-len(q) // 65536)
    assert (got == plain.check_batch_pairs(p, 0, 5)).all()


def test_split_expand_matches_oracle(split):
    from tests.test_gpu_synth import _expand_matches_oracle
    g, snap, _ = split
    _expand_matches_oracle(g, snap)


def test_split_expand_trees_equal_plain_layout(split):
    g, snap, plain = split
    rng = np.random.default_rng(8)
    rows = rng.integers(0, g.n_rows, size=4000).astype(np.uint32) | np.uint32(0x80000000)
    depths = rng.integers(0, 6, size=4000).astype(np.int32)
    a = snap.expand_batch_ids(rows, depths, 5)
    b = plain.expand_batch_ids(rows, depths, 5)
    for x, y in zip(a, b):
        assert (np.asarray(x) == np.asarray(y)).all()


# (the wide layouts' seeds are fewer: each build allocates their full arena; wide48_g3 seed 9 is the
# moved-target case below)
@pytest.mark.parametrize("layout,seed", [("split48", s) for s in range(10)] + [("wide48_g3", s) for s in (5, 7, 9)] +
                         [("wide80", s) for s in (0, 4, 8)])
def test_split_writes_interleaved_with_checks(layout, seed, monkeypatch):
    """Writes on a split layout whose target reserve holds a few rows: new targets fill it, then a
    write lays the arena out afresh (no KETO_E_REBUILD reaches the caller); every check and tree
    after every write equals the SQL oracle's.  On a wide layout a target a write moves keeps its
    content in the target reserve (tier 0 holds only the top row's segment): wide48_g3 seed 9 read
    a moved target in a root segment through the top row's before that."""
    import keto_amd
    from oracle.oracle_sql import CheckEngine, ExpandEngine, NotFoundError, SQLStore
    from tests.engine_util import rows_from_tuples, subj
    from tests.randgraph import random_checks, random_expands, random_graph
    from tests.test_gpu_lifecycle import _random_write, _row
    for k, v in _env(layout).items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("KETO_TEST_TGT_RESERVE", "256")
    ns, tuples, raw, ps, alph = random_graph(seed + 900, wide=seed % 3 == 2, allow_poison=False,
                                             allow_collisions=seed % 2 == 0)
    names, objs, rels, users = alph
    names = [n for n in names if n]
    if not names:
        pytest.skip("only a namespace named ''")
    store = SQLStore(ns, tuples, page_size=ps)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), page_size=ps, device=0)
    rng = random.Random(seed)
    for step in range(8):
        ins = [_random_write(rng, names, objs, rels, users) for _ in range(rng.randint(1, 12))]
        cur = store.tuples()
        dels = [rng.choice(cur) for _ in range(rng.randint(0, 3))] if cur else []
        v0 = snap.version()
        assert snap.apply([_row(ns, t) for t in ins], [_row(ns, t) for t in dels]) == v0 + 1
        for t in ins:
            store.insert(t)
        for t in dels:
            store.delete(t)
        checks = random_checks(seed * 13 + step, (names, objs + ["new1", "new7", "a0"], rels + ["q"],
                                                  users + ["w001", "a"]), k=40)
        for gm in sorted({c[2] for c in checks}):
            grp = [c for c in checks if c[2] == gm]
            allowed, _ = snap.check_batch([(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in grp], gm)
            for (t, d, _), a in zip(grp, allowed):
                assert bool(a) == CheckEngine(store, gm).subject_is_allowed(t, d), (seed, step, t, d, gm)
        exps = random_expands(seed * 7 + step, (names, objs + ["new3"], rels + ["q"], users), k=8)
        for gm in sorted({e[2] for e in exps}):
            grp = [e for e in exps if e[2] == gm]
            got = snap.expand_batch([(subj(s), d) for s, d, _ in grp], gm)
            for (s, d, _), (st, js) in zip(grp, got):
                try:
                    tr = ExpandEngine(store, gm).build_tree(s, d)
                    want = ("tree", tr.to_json()) if tr is not None else ("nil", None)
                except NotFoundError:
                    want = ("error", None)
                assert ({0: "tree", 1: "nil", 2: "error"}[st], js) == want, (seed, step, s, d, gm)
    snap.close()


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("seed", range(4100, 4103))
def test_wide_shared_parts_routed(P, seed, monkeypatch):
    """Shared-rows parts whose arenas are wide (32 GiB, 128-B root units), P ranks of the local
    transport on the one GPU: each rank's named batch is routed to the parts owning its rows and
    checked on their wide arenas; every decision equals the replicated snapshot's and the SQL
    oracle's (internal/check/engine.go:36-123)."""
    import keto_amd
    from keto_amd.capi import PART_SHARED
    from oracle.oracle_sql import CheckEngine
    from tests.test_gpu_comm import _local_comms, _ok, _ranks, _reqs
    from tests.engine_util import rows_from_tuples
    from tests.randgraph import random_store
    monkeypatch.setenv("KETO_COMM_TIMEOUT_MS", "60000")
    store, ns, tuples, raw, ps, alph = random_store(seed)
    rows = rows_from_tuples(ns, tuples, raw)
    full = keto_amd.Snapshot.build(ns, rows, page_size=ps, device=0)
    reqs, checks = _reqs(seed, alph)
    g = 5
    want, want_st = full.check_batch(reqs, g)
    for (t, d, _), a in zip(checks, want):
        assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, t, d)
    # roots from just past word 2^33 in 128-B units: ~32 GiB per part (the module's wide100 arena may
    # still be held)
    monkeypatch.setenv("KETO_TEST_ROOT_BASE", str((1 << 33) + (1 << 20)))
    monkeypatch.setenv("KETO_TEST_ROOT_G", "3")
    parts = [keto_amd.Snapshot.build(ns, rows, page_size=ps, device=-1).upload_part(r, P, 0, mode=PART_SHARED)
             for r in range(P)]
    comms = _local_comms(P)
    mine = [list(range(r, len(reqs), P)) for r in range(P)]
    res = _ok(_ranks(P, lambda r: comms[r].check_batch_routed(parts[r], [reqs[i] for i in mine[r]], g)))
    for r, (got, st) in enumerate(res):
        for k, i in enumerate(mine[r]):
            assert got[k] == want[i] and st[k] == want_st[i], (seed, P, r, reqs[i])
    for c in comms:
        c.close()
    for p in parts:
        p.close()
    full.close()


@pytest.mark.parametrize("layout,seed", [("wide48_g3", s) for s in range(4600, 4604)] + [("wide80", 4604)])
def test_wide_packed_and_device_proto(layout, seed, monkeypatch):
    """The Go shim's calls on a wide arena: packed string batches resolved on the GPU (the in-flight
    path that enqueues tier 0 alone on its own stream, check_wave_kernel_wide), named batches, and
    expand trees with their SubjectTree bytes encoded on the device -- each equal to the same graph
    in the narrow layout and to the SQL oracle (internal/check/engine.go:36-123,
    internal/expand/engine.go:33-102)."""
    import keto_amd
    from keto_amd.capi import pack_requests
    from oracle.oracle_sql import CheckEngine
    from tests.engine_util import rows_from_tuples, subj
    from tests.randgraph import random_expands, random_store
    from tests.test_gpu_comm import _reqs
    store, ns, tuples, raw, ps, alph = random_store(seed)
    rows = rows_from_tuples(ns, tuples, raw)
    plain = keto_amd.Snapshot.build(ns, rows, page_size=ps, device=0)
    for k, v in _env(layout).items():
        monkeypatch.setenv(k, v)
    wide = keto_amd.Snapshot.build(ns, rows, page_size=ps, device=0)
    reqs, checks = _reqs(seed, alph)
    for g in (3, 5, 12):
        want, want_st = plain.check_batch(reqs, g)
        got, st = wide.check_batch(reqs, g)
        assert (got == want).all() and (st == want_st).all(), (seed, g)
        blob, pk = pack_requests(reqs)
        got_p, st_p = wide.check_batch_packed(blob, pk, g)
        assert (got_p == want).all() and (st_p == want_st).all(), (seed, g)
        if g == 5:
            for (t, d, _), a in zip(checks, got):
                assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, t, d)
    exps = random_expands(seed, alph, k=24)
    er = [(subj(s), d) for s, d, _ in exps]
    a, pa = plain.expand_batch(er, 5, proto_all="host")
    b, pb = wide.expand_batch(er, 5, proto_all="device")
    assert [x[:2] for x in a] == [x[:2] for x in b]
    assert pa == pb
    wide.close()
    plain.close()


@pytest.mark.parametrize("seed", range(4700, 4703))
def test_wide_after_writes_clone_and_persist(seed, monkeypatch, tmp_path):
    """A wide snapshot (32 GiB, 128-B root units) after writes, then cloned and saved / loaded (both
    lay the arena out afresh, wide again): every copy decides and expands like the narrow snapshot at
    the same version and like the SQL oracle."""
    import keto_amd
    from oracle.oracle_sql import CheckEngine, SQLStore
    from tests.engine_util import rows_from_tuples, subj
    from tests.randgraph import random_expands, random_graph
    from tests.test_gpu_comm import _reqs
    from tests.test_gpu_lifecycle import _random_write, _row
    ns, tuples, raw, ps, alph = random_graph(seed, allow_poison=False, allow_collisions=seed % 2 == 0)
    names, objs, rels, users = alph
    names = [n for n in names if n]
    if not names:
        pytest.skip("only a namespace named ''")
    store = SQLStore(ns, tuples, page_size=ps)
    plain = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), page_size=ps, device=0)
    # roots from just past word 2^33 in 128-B units: three ~32 GiB copies (the module's wide100 arena
    # may still be held)
    monkeypatch.setenv("KETO_TEST_ROOT_BASE", str((1 << 33) + (1 << 20)))
    monkeypatch.setenv("KETO_TEST_ROOT_G", "3")
    wide = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), page_size=ps, device=0)
    rng = random.Random(seed)
    for _ in range(4):
        ins = [_random_write(rng, names, objs, rels, users) for _ in range(rng.randint(1, 10))]
        cur = store.tuples()
        dels = [rng.choice(cur) for _ in range(rng.randint(0, 2))] if cur else []
        for snap in (plain, wide):
            snap.apply([_row(ns, t) for t in ins], [_row(ns, t) for t in dels])
        for t in ins:
            store.insert(t)
        for t in dels:
            store.delete(t)
    clone = wide.clone(0)
    path = str(tmp_path / "wide.snap")
    wide.save(path, tag=seed)
    loaded, tag = keto_amd.Snapshot.load(path, device=0)
    assert tag == seed
    reqs, checks = _reqs(seed, (names, objs, rels, users))
    want, want_st = plain.check_batch(reqs, 5)
    for (t, d, _), a in zip(checks, want):
        assert bool(a) == CheckEngine(store, 5).subject_is_allowed(t, d), (seed, t, d)
    exps = random_expands(seed, (names, objs, rels, users), k=16)
    er = [(subj(s), d) for s, d, _ in exps]
    want_t = [x[:2] for x in plain.expand_batch(er, 5)]
    for name, snap in (("wide", wide), ("clone", clone), ("loaded", loaded)):
        got, st = snap.check_batch(reqs, 5)
        assert (got == want).all() and (st == want_st).all(), (seed, name)
        assert [x[:2] for x in snap.expand_batch(er, 5)] == want_t, (seed, name)
    h = loaded.row_handles(np.arange(loaded.stats()["n_rows"], dtype=np.uint32)).astype(np.int64)
    assert (h >= (1 << 31)).any()                              # laid out wide again
    for snap in (loaded, clone, wide, plain):
        snap.close()
