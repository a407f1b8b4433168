"""The product's builder (keto_snapshot_build) beyond toy sizes, on the GPU.

* config #2 at full size: the 10,000,000-tuple Drive-like graph emitted as string rows in a random
  commit order and built by keto_snapshot_build (parallel interning / ORDER BY / collision classes)
  decides 1,000,000 string requests (keto_check_batch, in-library resolution) exactly like the
  keto_snapshot_from_csr snapshot of the same graph;
* visit-key collisions and stored wildcard sets injected into a 150k-tuple graph: the built
  snapshot's decisions equal the C oracle's over the same table (ordered by SQLite itself).
"""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_drive_10m_string_build_matches_csr():
    from tools import synth
    g = synth.SynthGraph(dict(synth.DRIVE_10M), threads=16, kind="drive")
    st = g.string_tuples(seed=11)
    try:
        snap, t_build = g.snapshot_from_strings(st, device=0)
        ref = g.snapshot(device=0)
        q = g.queries(1_000_000, seed=2, depth=5)
        got, status = snap.check_batch_reqs(g.string_requests(st, q), len(q), 5)
        want = ref.check_batch_rows(q, 5)
        assert (status == 0).all()
        assert (got == want).all(), f"{int((got != want).sum())} mismatches of {len(q)}"
        assert snap.stats()["n_tuples"] == 10_000_000
        snap.close()
        ref.close()
    finally:
        g.free_strings(st)
        g.close()


@pytest.mark.parametrize("par", [True, False])
def test_injected_collisions_and_wildcards_match_oracle(monkeypatch, par):
    from oracle.oracle_c import OracleTable
    from oracle.oracle_sql import RelationTuple, SQLStore, SubjectID, SubjectSet
    from tools import synth
    import keto_amd
    from tests.engine_util import rows_from_tuples
    if par:
        monkeypatch.setenv("KETO_BUILD_PAR_MIN", "1")
    g = synth.SynthGraph(synth.scaled(synth.DRIVE_10M, 1 / 64), threads=16, kind="drive")
    names = dict(g.namespaces)
    rel = g.relation_names()
    hx = lambda v: f"{int(v):08x}"
    tuples = []
    for r in range(g.n_rows):
        ns, o, rl = names[int(g.row_ns[r])], hx(g.row_obj[r]), rel[int(g.row_rel[r])]
        for e in g.edges[g.row_ptr[r]:g.row_ptr[r + 1]]:
            e = int(e)
            if e & 0x80000000:
                t = e & 0x7FFFFFFF
                tuples.append(RelationTuple(ns, o, rl, SubjectSet(names[int(g.row_ns[t])], hx(g.row_obj[t]),
                                                                    rel[int(g.row_rel[t])])))
            else:
                tuples.append(RelationTuple(ns, o, rl, SubjectID(f"u{e:08x}")))
    rng = random.Random(3)
    n_groups, n_folders = g.params["n_groups"], g.params["n_folders"]
    for _ in range(300):        # subject ids whose text is a group's String(): collision classes
        tuples.append(RelationTuple("folders", hx(rng.randrange(n_folders)), "view",
                                    SubjectID(f"groups:{hx(rng.randrange(n_groups))}#member")))
    for _ in range(60):         # stored subject sets with an empty relation: materialized wildcard rows
        tuples.append(RelationTuple("folders", hx(rng.randrange(n_folders)), "view",
                                    SubjectSet("groups", hx(rng.randrange(min(64, n_groups))), "")))
    rng.shuffle(tuples)
    ns = list(g.namespaces)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), device=0)
    s = snap.stats()
    assert s["n_collision_keys"] > 100 and s["n_wildcard_rows"] > 10 and s["n_seq_rows"] > 100, s
    tab = OracleTable.from_store(SQLStore(ns, tuples))
    users = sorted({t.subject.id for t in tuples if isinstance(t.subject, SubjectID)})
    reqs = []
    for _ in range(20000):
        f = rng.randrange(g.params["n_docs"])
        sub = SubjectID(rng.choice(users)) if rng.random() < 0.9 else \
            SubjectSet("groups", hx(rng.randrange(n_groups)), "member")
        reqs.append((RelationTuple("files", hx(f), "view", sub), rng.choice([0, 3, 5])))
    from tests.engine_util import subj
    got, _ = snap.check_batch([(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d in reqs], 5)
    want = tab.check_batch_reqs([tab.check_req(t, d) for t, d in reqs], 5, threads=16)
    assert (got == want).all(), f"{int((got != want).sum())} mismatches of {len(reqs)}"
    assert got.sum() > 100 and got.mean() < 0.98
    g.close()
