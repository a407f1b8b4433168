"""Deep batches (global max-depth > 9) through top-level items and the hop-bounded reachability
pretest (keto_amd/csrc/reach.hip): every request split into one item per top-level subject set (a
fresh visited map each, internal/check/engine.go:47-48), items with no row holding the subject within
their hop budget dropped, the rest checked and OR-ed back.  Decisions must equal the oracle's with
the split on or off, the pretest on or off, pretest bounds so small that most searches give up
(and keep their items), one-request grabs or contiguous runs, and tiny visited tables that push
items up the tiers; on quirk-heavy random graphs (collisions, wildcard sets, poisoned pages, overlay
rows) against the SQL oracle; and across writes, which rebuild the index."""
import random

import pytest

from oracle.oracle_sql import CheckEngine, RelationTuple, SQLStore, SubjectID, SubjectSet
from tests.engine_util import rows_from_tuples, subj
from tests.randgraph import random_checks, random_graph, random_store

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nested():
    from tools import synth
    g = synth.SynthGraph(dict(n_docs=0, n_folders=0, n_groups=1 << 15, n_users=1 << 15, target_edges=0, seed=3),
                         threads=16, kind="nested", chain=32)
    snap = g.snapshot(device=0)
    yield g, snap
    g.close()


ENVS = {
    "default": {},
    "pretest_all": {"KETO_REACH_MIN_DEPTH": "2"},
    "no_items": {"KETO_ITEMS": "0"},
    "no_pretest": {"KETO_REACH_PRETEST": "0"},
    "tiny_bounds": {"KETO_REACH_WORK": "40", "KETO_REACH_MIN_DEPTH": "2"},
    "lane_pretest": {"KETO_REACH_PRETEST": "1", "KETO_REACH_CAP": "64", "KETO_REACH_WORK": "200"},
    "lane_pretest_few_lanes": {"KETO_REACH_PRETEST": "1", "KETO_REACH_LANES": "256"},
    "small_wave_tables": {"KETO_REACH_WAVE_SLOTS": "2048", "KETO_REACH_MIN_DEPTH": "2"},
    "runs": {"KETO_T0_NEXT": "0", "KETO_REACH_MIN_DEPTH": "2"},
    "tiny_tables": {"KETO_T0_CAP": "256", "KETO_T1_CAP": "1024"},
}


@pytest.mark.parametrize("gmd", [12, 32, 40])
@pytest.mark.parametrize("env", list(ENVS))
def test_nested_items_match_oracle(nested, monkeypatch, env, gmd):
    g, snap = nested
    for k, v in ENVS[env].items():
        monkeypatch.setenv(k, v)
    q = g.queries_nested(12000, seed=300 + gmd, depths=(5, 16, 32, 0, -1, 40, 2, 1))
    gpu = snap.check_batch_ids(snap.with_handles(q), gmd)
    t = snap.last_timing_full()
    tab = g.oracle_table(q, gmd)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), gmd, threads=16)
    assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)} ({env}, gmd {gmd}, {t})"
    if env == "no_items":
        assert t["items"] == 0
    else:
        assert t["items"] > 0, t
        if env in ("pretest_all", "runs", "lane_pretest_few_lanes", "small_wave_tables") or (env == "default" and gmd > 12):
            assert t["items_kept"] < t["items"], t       # the pretest dropped items it proved false


def test_nested_items_host_pipeline(nested, monkeypatch):
    """keto_check_batch_ids (host buffers, pipelined chunks): a deep chunk is decided whole through
    the items path; small chunks make several."""
    g, snap = nested
    monkeypatch.setenv("KETO_CHUNK", "3000")
    q = g.queries_nested(10000, seed=91, depths=(16, 32, 40, 0))
    gpu = snap.check_batch_ids(snap.with_handles(q), 32)
    t = snap.last_timing_full()
    tab = g.oracle_table(q, 32)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), 32, threads=16)
    assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches"
    assert t["chunks"] >= 3 and t["items"] > 0, t


def test_nested_items_steps(nested):
    """keto_check_steps_device through the items path: a request's steps are its longest item's."""
    import numpy as np
    import torch
    g, snap = nested
    q = g.queries_nested(4000, seed=5, depths=(16, 32))
    qd = snap.with_handles(q)
    d_q = torch.from_numpy(qd.view(np.uint8)).to("cuda:0")
    d_out = torch.empty(len(q), dtype=torch.uint8, device="cuda:0")
    d_steps = torch.zeros(len(q), dtype=torch.int32, device="cuda:0")
    snap.check_steps_device(d_q.data_ptr(), len(q), d_out.data_ptr(), d_steps.data_ptr(), 32)
    torch.cuda.synchronize()
    gpu = d_out.cpu().numpy()
    tab = g.oracle_table(q, 32)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), 32, threads=16)
    assert (gpu == ref).all()
    steps = d_steps.cpu().numpy()
    assert steps.max() > 0


@pytest.mark.parametrize("seed,wide", [(s, False) for s in range(3000, 3080)] + [(s, True) for s in range(3500, 3520)])
def test_random_graphs_deep_match_oracle(seed, wide, monkeypatch):
    """Quirk-heavy random graphs (cycles, duplicates, wildcard sets, poisoned pages, visit-key
    collisions, overlay rows of wildcard requests) at global max-depths 10 and 13, every item
    pretested."""
    import keto_amd
    monkeypatch.setenv("KETO_REACH_MIN_DEPTH", "2")
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=wide)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples, raw), page_size=ps, device=0)
    rng = random.Random(seed)
    checks = random_checks(seed, alph, k=40)
    for g in (10, 13):
        reqs = [(t, rng.choice([0, 1, 2, 3, 5, 9, 11, 14, -1])) for t, _, _ in checks]
        allowed, _ = snap.check_batch([(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d in reqs], g)
        for (t, d), a in zip(reqs, allowed):
            assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, t, d, g)
    snap.close()


def _write(rng, names, objs, rels, users):
    o = rng.choice(objs + [f"new{rng.randrange(20)}"])
    r = rng.choice(rels)
    if rng.random() < 0.5:
        sub = SubjectID(rng.choice(users + [f"w{rng.randrange(50):03d}"]))
    else:
        sub = SubjectSet(rng.choice(names), rng.choice(objs + [f"new{rng.randrange(20)}"]), rng.choice(rels))
    return RelationTuple(rng.choice(names), o, r, sub)


@pytest.mark.parametrize("seed", range(16))
def test_writes_then_deep_checks(seed, monkeypatch):
    """Writes bump the snapshot version; the next deep batch rebuilds the reverse / postings index,
    so new subject-set edges and ids are seen by the pretest (a stale index would drop items)."""
    import keto_amd
    monkeypatch.setenv("KETO_REACH_MIN_DEPTH", "2")
    ns, tuples, raw, ps, alph = random_graph(seed + 700, allow_wildcards=False, allow_poison=False,
                                             allow_collisions=seed % 3 == 0)
    names, objs, rels, users = alph
    names = [n for n in names if n]
    if not names:
        pytest.skip("only a namespace named ''")
    store = SQLStore(ns, tuples, page_size=ps)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), page_size=ps, device=0)
    rng = random.Random(seed)
    for step in range(6):
        ins = [_write(rng, names, objs, rels, users) for _ in range(rng.randint(1, 10))]
        cur = store.tuples()
        dels = [rng.choice(cur) for _ in range(rng.randint(0, 3))] if cur else []
        v0 = snap.version()
        try:
            snap.apply([rows_from_tuples(ns, [t])[0] for t in ins], [rows_from_tuples(ns, [t])[0] for t in dels])
        except keto_amd.KetoError as e:
            assert "-6" in str(e), e
        for t in ins:
            store.insert(t)
        for t in dels:
            store.delete(t)
        if snap.version() == v0:
            snap.close()
            snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, store.tuples()), page_size=ps, device=0)
        checks = random_checks(seed * 13 + step, (names, objs + ["new1", "new7"], rels, users + ["w001", "w013"]), k=40)
        reqs = [(t, rng.choice([0, 2, 4, 9, 12, -1])) for t, _, _ in checks]
        allowed, _ = snap.check_batch([(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d in reqs], 12)
        for (t, d), a in zip(reqs, allowed):
            assert bool(a) == CheckEngine(store, 12).subject_is_allowed(t, d), (seed, step, t, d)
    snap.close()
