"""The two facts the deep-batch path (keto_amd/csrc/reach.hip) stands on, checked on the SQL oracle
(the reference's recursion over its own SQL, oracle/oracle_sql.py) over quirk-heavy random graphs:

1. A check is the OR over its top-level tuples, each searched with a fresh visited map that holds
   only that tuple's subject (internal/check/engine.go:47-48: the shadowed ctx), in the pages before
   the first page that fails (relationtuples.go:43-80 -> engine.go:99-101 returns false there).
2. A check can only be allowed if some row holding the requested subject id lies within
   max-depth - 1 subject-set hops of the request's row (engine.go:54, :88-91).

The GPU tests (tests/test_gpu_items.py) compare the engine with the oracle; these pin the reasoning
itself, with wildcard rows, visit-key collisions and poisoned pages included."""
import pytest

from oracle.oracle_sql import CheckEngine, NotFoundError, SubjectID, SubjectSet, _Ctx, check_and_add_visited
from tests.randgraph import random_checks, random_store


def _pages(store, query):
    """Every tuple a query returns, page by page, up to the first page that fails."""
    out, prev = [], ""
    while True:
        try:
            rels, nxt = store.get_relation_tuples(*query, token=prev)
        except NotFoundError:
            return out, True
        out.extend(rels)
        if nxt == "":
            return out, False
        prev = nxt


def _items_decision(store, g, t, d):
    eng = CheckEngine(store, g)
    if d <= 0 or g < d:
        d = g
    rels, _ = _pages(store, (t.namespace, t.object, t.relation))
    for sr in rels:
        if t.subject.equals(sr.subject):
            return True
        if isinstance(sr.subject, SubjectSet):
            ctx, _ = check_and_add_visited(_Ctx(), sr.subject)       # the item's fresh map: its set
            s = sr.subject
            if eng._check_one_indirection_further(ctx, t, (s.namespace, s.object, s.relation), d - 1):
                return True
    return False


def _within(store, t, hops):
    """Is some query holding the subject id within `hops` subject-set hops of the request's?"""
    seen = set()
    frontier = [(t.namespace, t.object, t.relation)]
    for level in range(hops + 1):
        nxt = []
        for q in frontier:
            if q in seen:
                continue
            seen.add(q)
            rels, _ = _pages(store, q)
            for sr in rels:
                if isinstance(sr.subject, SubjectID) and sr.subject.equals(t.subject):
                    return True
                if isinstance(sr.subject, SubjectSet):
                    nxt.append((sr.subject.namespace, sr.subject.object, sr.subject.relation))
        frontier = nxt
    return False


@pytest.mark.parametrize("seed", range(120))
def test_items_and_hop_bound_on_the_oracle(seed):
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=seed % 5 == 4)
    checks = random_checks(seed + 17, alph, k=30)
    for t, d, g in checks:
        g = max(g, 3) + seed % 9                          # deep enough for long paths and cycles
        want = CheckEngine(store, g).subject_is_allowed(t, d)
        assert _items_decision(store, g, t, d) == want, (seed, t, d, g)
        if isinstance(t.subject, SubjectID) and want:
            dd = g if (d <= 0 or g < d) else d
            assert _within(store, t, dd - 1), (seed, t, d, g)
