"""Snapshot lifecycle on the GPU (keto_snapshot_apply): write transactions interleaved with check
and expand batches, every decision and tree compared with the SQL oracle after each write
(oracle_sql.SQLStore insert / delete = InsertRelationTuple / DeleteRelationTuples,
internal/persistence/sql/relationtuples.go:128-149,200-223).

The writes exercise the delta path: rows rewritten in place, rows that outgrow their place (a
forward at the identity handle), rows that get an id table, root rows that become subject-set
targets (a new identity with a closure filter), new rows, new strings that sort between the build's,
duplicate inserts and deletes of every equal tuple, wildcard (empty-field) subject sets and the rows
their materialized wildcard rows match.  Writes the delta path refuses (KETO_E_REBUILD: a poisoned
row) leave the snapshot unchanged and are followed by a rebuild, as a caller would do."""
import random

import pytest

from oracle.oracle_sql import (CheckEngine, ExpandEngine, NotFoundError, RelationTuple, SQLStore, SubjectID,
                               SubjectSet)
from tests.engine_util import rows_from_tuples, subj
from tests.randgraph import random_checks, random_expands, random_graph

pytestmark = pytest.mark.gpu


def _row(ns_ids, t):
    return rows_from_tuples(ns_ids, [t])[0]


def _random_write(rng, names, objs, rels, users, set_names=None, wild=0.0):
    o = rng.choice(objs + [f"new{rng.randrange(40)}", "a0", "Z", "b#c"])
    r = rng.choice(rels + ["q"])
    if rng.random() < 0.55:
        sub = SubjectID(rng.choice(users + [f"w{rng.randrange(200):03d}", "a", "zz"]))
    else:
        so = rng.choice(objs + [f"new{rng.randrange(40)}"])
        sr = rng.choice(rels + ["q"])
        if rng.random() < wild:                       # a wildcard subject set: an empty field
            so, sr = rng.choice([("", sr), (so, ""), ("", "")])
        sub = SubjectSet(rng.choice(set_names or names), so, sr)
    return RelationTuple(rng.choice(names), o, r, sub)


@pytest.mark.parametrize("seed", range(40))
def test_writes_interleaved_with_checks(seed):
    import keto_amd
    wide = seed % 4 == 3
    ns, tuples, raw, ps, alph = random_graph(seed + 500, wide=wide, allow_wildcards=seed % 5 == 0,
                                             allow_poison=False, allow_collisions=seed % 3 == 0)
    names, objs, rels, users = alph
    set_names = list(names)                           # a namespace named "": wildcard subject sets
    names = [n for n in names if n]
    if not names:
        pytest.skip("only a namespace named ''")
    wild = 0.15 if seed % 2 == 0 else 0.0
    store = SQLStore(ns, tuples, page_size=ps)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), page_size=ps, device=0)
    rng = random.Random(seed)
    applied = rebuilt = 0
    for step in range(10):
        cur = store.tuples()
        ins = [_random_write(rng, names, objs, rels, users, set_names, wild) for _ in range(rng.randint(1, 30 if wide else 8))]
        dels = [rng.choice(cur) for _ in range(rng.randint(0, 4))] if cur else []
        dels += [_random_write(rng, names, objs, rels, users, set_names, wild) for _ in range(rng.randint(0, 2))]
        v0 = snap.version()
        try:
            v = snap.apply([_row(ns, t) for t in ins], [_row(ns, t) for t in dels])
            assert v == v0 + 1
            applied += 1
        except keto_amd.KetoError as e:
            assert "-6" in str(e), e                   # KETO_E_REBUILD only
            assert snap.version() == v0
            rebuilt += 1
        for t in ins:
            store.insert(t)
        for t in dels:
            store.delete(t)
        if snap.version() == v0:                       # refused: rebuild from the table
            snap.close()
            snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, store.tuples()), page_size=ps, device=0)
        checks = random_checks(seed * 31 + step, (names, objs + ["new1", "new7", "a0"], rels + ["q"],
                                                  users + ["w001", "a"]), k=40)
        for g in sorted({c[2] for c in checks}):
            grp = [c for c in checks if c[2] == g]
            allowed, _ = snap.check_batch([(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in grp], g)
            for (t, d, _), a in zip(grp, allowed):
                assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, step, t, d, g)
        exps = random_expands(seed * 17 + step, (names, objs + ["new3"], rels + ["q"], users), k=10)
        for g in sorted({e[2] for e in exps}):
            grp = [e for e in exps if e[2] == g]
            got = snap.expand_batch([(subj(s), d) for s, d, _ in grp], g)
            for (s, d, _), (st, js) in zip(grp, got):
                try:
                    tr = ExpandEngine(store, g).build_tree(s, d)
                    want = ("tree", tr.to_json()) if tr is not None else ("nil", None)
                except NotFoundError:
                    want = ("error", None)
                have = {0: "tree", 1: "nil", 2: "error"}[st]
                assert (have, js) == want, (seed, step, s, d, g)
    assert applied == 10 and rebuilt == 0         # no poisoned rows: every write takes the delta path
    snap.close()


def test_large_row_growth_and_new_targets():
    """One hub row grown from 2 to 3,000 ids over several writes (in place, then relocated with an
    id table, then relocated again), a root row turned into a subject-set target (identity move), and
    checks through both after every write."""
    import keto_amd
    ns = [(1, "n")]
    base = [RelationTuple("n", "doc", "view", SubjectSet("n", "hub", "member")),
            RelationTuple("n", "hub", "member", SubjectID("u0001")),
            RelationTuple("n", "hub", "member", SubjectID("u0002")),
            RelationTuple("n", "root", "view", SubjectID("r1"))]
    store = SQLStore(ns, base)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, base), device=0)
    rng = random.Random(1)
    for step, k in enumerate((1, 5, 40, 400, 2600)):
        ins = [RelationTuple("n", "hub", "member", SubjectID(f"u{rng.randrange(10000):04d}")) for _ in range(k)]
        if step == 2:
            ins.append(RelationTuple("n", "hub", "member", SubjectSet("n", "root", "view")))     # root -> target
        snap.apply([_row(ns, t) for t in ins])
        for t in ins:
            store.insert(t)
        reqs = [("n", "doc", "view", ("id", f"u{i:04d}"), 0) for i in range(0, 10000, 7)]
        reqs += [("n", "doc", "view", ("id", "r1"), 0), ("n", "doc", "view", ("id", "r1"), 2),
                 ("n", "root", "view", ("id", "r1"), 0), ("n", "hub", "member", ("id", "r1"), 0)]
        allowed, _ = snap.check_batch(reqs, 5)
        eng = CheckEngine(store, 5)
        for (n_, o, r, u, d), a in zip(reqs, allowed):
            assert bool(a) == eng.subject_is_allowed(RelationTuple(n_, o, r, SubjectID(u[1])), d), (step, o, u, d)
        (st, js), = snap.expand_batch([(("set", "n", "doc", "view"), 0)], 5)
        assert js == ExpandEngine(store, 5).build_tree(SubjectSet("n", "doc", "view"), 0).to_json()
    assert snap.version() == 5


def test_collisions_applied_without_rebuild():
    """Writes that create Subject.String() collisions (graph_utils.go:13-35 keys) go through the delta
    path: a subject id equal to an existing set's String() (the DF3 shape), a new row whose String()
    equals an existing subject id, and two rows with one String() ("a#b"#"c" vs "a"#"b#c").  Each is
    applied (version + 1, no KETO_E_REBUILD), and every check and expand then equals the SQL oracle."""
    import keto_amd
    ns = [(1, "n")]
    base = [RelationTuple("n", "root", "r", SubjectSet("n", "p", "r")),
            RelationTuple("n", "p", "r", SubjectSet("n", "q", "r")),
            RelationTuple("n", "q", "r", SubjectSet("n", "g", "m")),
            RelationTuple("n", "g", "m", SubjectID("u")),
            RelationTuple("n", "h", "m", SubjectID("n:x#y")),          # an id that looks like a set
            RelationTuple("n", "doc", "v", SubjectSet("n", "h", "m")),
            RelationTuple("n", "a#b", "c", SubjectID("w")),
            RelationTuple("n", "top", "v", SubjectSet("n", "a#b", "c"))]
    store = SQLStore(ns, base)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, base), device=0)
    writes = [
        # DF3: n:a#r holds the id "n:g#m", checked before the set n:g#m under n:p#r
        [RelationTuple("n", "a", "r", SubjectID("n:g#m")), RelationTuple("n", "p", "r", SubjectSet("n", "a", "r"))],
        # a new row n:x#y collides with the subject id "n:x#y"
        [RelationTuple("n", "x", "y", SubjectID("u2")), RelationTuple("n", "doc", "v", SubjectSet("n", "x", "y"))],
        # a new row n:a#b#c (object "a", relation "b#c") collides with the row n:a#b#c (object "a#b")
        [RelationTuple("n", "a", "b#c", SubjectID("w2")), RelationTuple("n", "top", "v", SubjectSet("n", "a", "b#c"))],
        # more edges to classed subjects, and a delete
        [RelationTuple("n", "root", "r", SubjectID("n:x#y")), RelationTuple("n", "q", "r", SubjectSet("n", "x", "y"))],
    ]
    objs = ["root", "p", "q", "g", "h", "doc", "a#b", "top", "a", "x"]
    rels = ["r", "m", "v", "c", "y", "b#c"]
    users = ["u", "u2", "w", "w2", "n:g#m", "n:x#y", "nobody"]
    for step, ins in enumerate(writes):
        dels = [base[3]] if step == 3 else []
        v0 = snap.version()
        v = snap.apply([_row(ns, t) for t in ins], [_row(ns, t) for t in dels])
        assert v == v0 + 1, step
        for t in ins:
            store.insert(t)
        for t in dels:
            store.delete(t)
        assert snap.stats()["n_collision_keys"] >= min(step + 1, 3)
        reqs = [("n", o, r, ("id", u), d) for o in objs for r in rels for u in users for d in (0, 2, 3)]
        reqs += [("n", o, r, ("set", "n", so, sr), 0) for o in objs for r in rels for so, sr in
                 (("g", "m"), ("x", "y"), ("a#b", "c"), ("a", "b#c"))]
        for g in (3, 5):
            allowed, _ = snap.check_batch(reqs, g)
            for (n_, o, r, u, d), a in zip(reqs, allowed):
                sub = SubjectID(u[1]) if u[0] == "id" else SubjectSet(*u[1:])
                assert bool(a) == CheckEngine(store, g).subject_is_allowed(RelationTuple(n_, o, r, sub), d), \
                    (step, g, o, r, u, d)
            exps = [(("set", "n", o, r), d) for o in objs for r in rels for d in (0, 3)]
            for ((s_, d), (st, js)) in zip(exps, snap.expand_batch(exps, g)):
                try:
                    tr = ExpandEngine(store, g).build_tree(SubjectSet(*s_[1:]), d)
                    want = ("tree", tr.to_json()) if tr is not None else ("nil", None)
                except NotFoundError:
                    want = ("error", None)
                assert ({0: "tree", 1: "nil", 2: "error"}[st], js) == want, (step, g, s_, d)
    snap.close()


def test_wildcard_sets_applied_without_rebuild():
    """Writes through stored wildcard subject sets (a field left empty: the set's query returns every
    row it matches, relationtuples.go:178-198): new wildcard sets with an empty object, an empty
    relation, both, and in the namespace named ""; then writes to, and deletes from, the rows those
    sets match, new matching rows whose strings sort between the build's, and a delete of a wildcard
    set itself.  Each write is applied (version + 1), and every check and expand equals the oracle."""
    import keto_amd
    ns = [(1, "n"), (2, "m"), (3, "")]
    base = [RelationTuple("n", "doc", "view", SubjectSet("n", "team", "member")),
            RelationTuple("n", "team", "member", SubjectID("u1")),
            RelationTuple("n", "team", "owner", SubjectID("u2")),
            RelationTuple("n", "crew", "member", SubjectID("u3")),
            RelationTuple("m", "team", "member", SubjectID("u4")),
            RelationTuple("n", "all", "view", SubjectSet("n", "", "member")),      # a stored wildcard set
            RelationTuple("n", "page", "view", SubjectID("u5"))]
    store = SQLStore(ns, base, page_size=2)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, base), page_size=2, device=0)
    writes = [
        ([RelationTuple("n", "crew", "member", SubjectID("u6"))], []),              # a row n:*#member matches
        ([RelationTuple("n", "any", "view", SubjectSet("n", "team", "")),           # new wildcard sets
          RelationTuple("n", "every", "view", SubjectSet("n", "", "")),
          RelationTuple("m", "x", "view", SubjectSet("", "team", "member"))], []),
        ([RelationTuple("n", "bbb", "member", SubjectID("u7")),                     # a new row between the build's
          RelationTuple("m", "team", "member", SubjectSet("n", "bbb", "member")),
          RelationTuple("n", "team", "admin", SubjectID("u8"))], [base[1]]),
        ([RelationTuple("n", "team", "member", SubjectSet("n", "", "owner"))], [base[3]]),
        ([], [RelationTuple("n", "all", "view", SubjectSet("n", "", "member"))]),    # a wildcard set deleted
        ([RelationTuple("n", "all", "view", SubjectSet("n", "", "member")),
          RelationTuple("n", "crew", "member", SubjectID("u9"))], []),
    ]
    objs = ["doc", "team", "crew", "all", "page", "any", "every", "x", "bbb"]
    rels = ["view", "member", "owner", "admin"]
    users = [f"u{i}" for i in range(1, 11)]
    n_wild0 = snap.stats()["n_wildcard_rows"]
    for step, (ins, dels) in enumerate(writes):
        v0 = snap.version()
        assert snap.apply([_row(ns, t) for t in ins], [_row(ns, t) for t in dels]) == v0 + 1, step
        for t in ins:
            store.insert(t)
        for t in dels:
            store.delete(t)
        reqs = [(n_, o, r, ("id", u), d) for n_ in ("n", "m") for o in objs + [""] for r in rels + [""]
                for u in users for d in (0, 2)]
        reqs += [("n", o, "view", ("set", "n", "team", "member"), 0) for o in objs]
        for g in (3, 5):
            allowed, _ = snap.check_batch(reqs, g)
            for (n_, o, r, u, d), a in zip(reqs, allowed):
                sub = SubjectID(u[1]) if u[0] == "id" else SubjectSet(*u[1:])
                assert bool(a) == CheckEngine(store, g).subject_is_allowed(RelationTuple(n_, o, r, sub), d), \
                    (step, g, n_, o, r, u, d)
            exps = [(("set", n_, o, r), d) for n_ in ("n", "m") for o in objs for r in rels for d in (0, 3)]
            exps += [(("set", "n", "", "member"), 0), (("set", "", "team", "member"), 0)]
            for ((s_, d), (st, js)) in zip(exps, snap.expand_batch(exps, g)):
                try:
                    tr = ExpandEngine(store, g).build_tree(SubjectSet(*s_[1:]), d)
                    want = ("tree", tr.to_json()) if tr is not None else ("nil", None)
                except NotFoundError:
                    want = ("error", None)
                assert ({0: "tree", 1: "nil", 2: "error"}[st], js) == want, (step, g, s_, d)
    assert snap.stats()["n_wildcard_rows"] == n_wild0 + 4
    snap.close()
