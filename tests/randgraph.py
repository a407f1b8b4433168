"""Seeded random relation-tuple graphs that exercise every quirk of the reference engines:
cycles, duplicates, sets before ids, namespace-id ordering, visit-key collisions (an id whose
text equals a set's String(), '#' inside objects), wildcard (empty-field) subject sets,
poisoned pages (subject-set namespace ids missing from the config) and small page sizes."""
import random

from oracle.oracle_sql import RelationTuple, SQLStore, SubjectID, SubjectSet


def random_graph(seed, n_tuples=None, page_size=None, allow_wildcards=True, allow_poison=True,
                 allow_collisions=True, wide=False):
    rng = random.Random(seed)
    n_ns = rng.randint(1, 3)
    ids = rng.sample([0, 1, 2, 5, 7, 10], n_ns)
    names = rng.sample(["n", "m", "docs", "grp"], n_ns)
    if allow_wildcards and rng.random() < 0.15:
        names[rng.randrange(n_ns)] = ""          # a namespace literally named "" (engine_test.go:223-225)
    namespaces = list(zip(ids, names))
    objs = ["a", "b", "c", "d", "a#b", "B", "é"][: rng.randint(2, 7)]
    rels = ["r", "s", "b#c", "t"][: rng.randint(1, 4)]
    users = ["u", "v", "w", "U"][: rng.randint(1, 4)]
    if wide:  # few rows with long, byte-ordered subject-id regions (binary-search paths)
        objs = objs[:2]
        users = [f"u{i:03d}" for i in rng.sample(range(1000), 80)]
    if allow_collisions:
        # an id whose text equals a set's String() (SURVEY A.Q4 / DF3)
        for _ in range(rng.randint(0, 2)):
            ns = rng.choice(names)
            users.append(f"{ns}:{rng.choice(objs)}#{rng.choice(rels)}")
    n = n_tuples if n_tuples is not None else (rng.randint(100, 400) if wide else rng.randint(0, 40))
    tuples, raw = [], []
    for _ in range(n):
        ns = rng.choice(names)
        o, r = rng.choice(objs), rng.choice(rels)
        if rng.random() < (0.85 if wide else 0.45):
            sub = SubjectID(rng.choice(users))
        else:
            so, sr = rng.choice(objs), rng.choice(rels)
            if allow_wildcards and rng.random() < 0.07:
                so = ""
            if allow_wildcards and rng.random() < 0.07:
                sr = ""
            sub = SubjectSet(rng.choice(names), so, sr)
        tuples.append(RelationTuple(ns, o, r, sub))
    nsid = dict((n_, i) for i, n_ in namespaces)
    if allow_poison and rng.random() < 0.15:
        for _ in range(rng.randint(1, 2)):
            # subject set pointing at a namespace id that is not configured (A.Q8)
            raw.append((nsid[rng.choice(names)], rng.choice(objs), rng.choice(rels), None, 99,
                        rng.choice(objs), rng.choice(rels)))
    ps = page_size if page_size is not None else rng.choice([1, 2, 3, 100])
    return namespaces, tuples, raw, ps, (names, objs, rels, users)


def random_store(seed, **kw):
    namespaces, tuples, raw, ps, alph = random_graph(seed, **kw)
    # interleave raw rows at random positions by inserting them after the tuples (commit order)
    store = SQLStore(namespaces, tuples, page_size=ps, raw_rows=raw)
    return store, namespaces, tuples, raw, ps, alph


def random_checks(seed, alph, k=12):
    rng = random.Random(seed * 7919 + 1)
    names, objs, rels, users = alph
    out = []
    for _ in range(k):
        ns = rng.choice(names + (["unknown-ns"] if rng.random() < 0.05 else []))
        o = rng.choice(objs + ([""] if rng.random() < 0.05 else []))
        r = rng.choice(rels + ([""] if rng.random() < 0.05 else []))
        if rng.random() < 0.7:
            sub = SubjectID(rng.choice(users))
        else:
            sub = SubjectSet(rng.choice(names), rng.choice(objs), rng.choice(rels))
        out.append((RelationTuple(ns, o, r, sub), rng.choice([0, 1, 2, 3, 4, 5, 7]), rng.choice([1, 2, 3, 5, 6])))
    return out


def random_expands(seed, alph, k=6):
    rng = random.Random(seed * 104729 + 3)
    names, objs, rels, users = alph
    out = []
    for _ in range(k):
        if rng.random() < 0.1:
            sub = SubjectID(rng.choice(users))
        else:
            sub = SubjectSet(rng.choice(names), rng.choice(objs + ([""] if rng.random() < 0.05 else [])),
                             rng.choice(rels))
        out.append((sub, rng.choice([0, 1, 2, 3, 4, 6]), rng.choice([1, 2, 3, 5])))
    return out


def poisoned_wildcard_case(seed):
    """A random graph with 1-3 failing tuples (subject sets of a namespace id the config lacks),
    page sizes 1-5, and wildcard queries over every (namespace, relation) and (namespace, object)
    pair of its alphabet at depths 1-7, subject ids and sets, plus random checks.  Returns
    (store, namespaces, tuples, raw, page size, request tuples, [(RelationTuple, depth)])."""
    rng = random.Random(seed * 31 + 7)
    ns, tuples, raw, _, alph = random_graph(seed, n_tuples=rng.randint(20, 60), allow_poison=False)
    names, objs, rels, users = alph
    nsid = dict((n_, i) for i, n_ in ns)
    for _ in range(rng.randint(1, 3)):
        raw.append((nsid[rng.choice(names)], rng.choice(objs), rng.choice(rels), None, 99, rng.choice(objs),
                    rng.choice(rels)))
    ps = rng.choice([1, 2, 3, 5])
    store = SQLStore(ns, tuples, page_size=ps, raw_rows=raw)
    checks = []
    for n_ in names:
        for o, r in [("", r) for r in rels] + [(o, "") for o in objs]:
            for _ in range(2):
                if rng.random() < 0.6:
                    sub = SubjectID(rng.choice(users))
                else:
                    sub = SubjectSet(rng.choice(names), rng.choice(objs), rng.choice(rels))
                checks.append((RelationTuple(n_, o, r, sub), rng.choice([1, 2, 3, 5, 7])))
    checks += [(t, d) for t, d, _ in random_checks(seed, alph, k=24)]
    reqs = [(t.namespace, t.object, t.relation, _subj(t.subject), d) for t, d in checks]
    return store, ns, tuples, raw, ps, reqs, checks


def _subj(s):
    return ("id", s.id) if isinstance(s, SubjectID) else ("set", s.namespace, s.object, s.relation)
