"""Overflow paths of the tier-0 check kernel, against the SQL oracle:

* a hub row with hundreds of subject sets: its edges come in block by block (P_EDGE), and one
  top-level tuple's visited map grows past registers + LDS (HBM spill) and past the tier-0 table
  (the request moves to tier 1);
* cycles back into the hub, so revisits are cut by the visited map;
* id rows big enough to get bucketed id tables and saturated bloom filters;
* every global max-depth from 1 to 7, so both tier-0 instances (4 and 8 saved frames) and the
  request-depth clamp run.
"""
import random

import pytest

from oracle.oracle_sql import CheckEngine, RelationTuple, SQLStore, SubjectID, SubjectSet
from tests.engine_util import rows_from_tuples, subj

pytestmark = pytest.mark.gpu


def _graph(fan=150, seed=7):
    rng = random.Random(seed)
    t = [RelationTuple("n", "root", "r", SubjectSet("n", "hub", "r"))]
    for i in range(fan):
        t.append(RelationTuple("n", "hub", "r", SubjectSet("n", f"x{i:04d}", "r")))
    for i in range(fan):
        t.append(RelationTuple("n", f"x{i:04d}", "r", SubjectSet("n", f"y{i:04d}", "r")))
        if rng.random() < 0.2:
            t.append(RelationTuple("n", f"x{i:04d}", "r", SubjectSet("n", "hub", "r")))      # cycle
        for k in range(rng.choice([0, 1, 3, 9, 40])):                                    # id rows of all sizes
            t.append(RelationTuple("n", f"y{i:04d}", "r", SubjectID(f"u{rng.randrange(2000):05d}")))
        if rng.random() < 0.1:
            t.append(RelationTuple("n", f"y{i:04d}", "r", SubjectSet("n", f"x{rng.randrange(fan):04d}", "r")))
    rng.shuffle(t)                                                                       # commit order
    return [(1, "n")], t


def test_hub_overflow_matches_oracle():
    import keto_amd
    ns, tuples = _graph()
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), device=0)
    store = SQLStore(ns, tuples)
    rng = random.Random(3)
    moved = 0
    for gmd in range(1, 8):
        reqs = []
        for _ in range(50):
            obj = rng.choice(["root", "hub", f"x{rng.randrange(150):04d}"])
            if rng.random() < 0.8:
                sub = SubjectID(f"u{rng.randrange(2000):05d}")
            else:
                sub = SubjectSet("n", f"y{rng.randrange(150):04d}", "r")
            reqs.append((RelationTuple("n", obj, "r", sub), rng.choice([0, 1, 2, 3, 5, 8])))
        allowed, _ = snap.check_batch([(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d in reqs], gmd)
        moved += snap.last_timing()[1][1]                     # requests that overflowed tier 0
        eng = CheckEngine(store, gmd)
        want = [eng.subject_is_allowed(t, d) for t, d in reqs]
        bad = [(t, d) for (t, d), a, w in zip(reqs, allowed, want) if bool(a) != w]
        assert not bad, (gmd, bad[:5])
        if gmd >= 4:
            assert any(want) and not all(want)
    assert moved > 0, "no request exercised the tier-0 -> tier-1 overflow path"
