"""One server process, several snapshot replicas (keto_snapshot_clone): the in-process multi-GPU
mode of the drop-in (integration/go/internal/driver/registry_gpu.go EnableGPU over several devices;
on this one-GPU box every replica lives on device 0).  Batches are dealt among the replicas, every
write transaction is applied to each (keto_snapshot_apply), and every decision and tree is compared
with the SQL oracle after each write (internal/check/engine.go:36-123,
internal/expand/engine.go:33-102, internal/persistence/sql/relationtuples.go:128-149,200-223).
Clones taken after writes start from the source's current version."""
import random
import threading

import pytest

from oracle.oracle_sql import CheckEngine, ExpandEngine, NotFoundError, SQLStore
from tests.engine_util import rows_from_tuples, subj
from tests.randgraph import random_checks, random_expands, random_graph
from tests.test_gpu_lifecycle import _random_write, _row

pytestmark = pytest.mark.gpu


def _want_tree(store, s, d, g):
    try:
        tr = ExpandEngine(store, g).build_tree(s, d)
        return ("tree", tr.to_json()) if tr is not None else ("nil", None)
    except NotFoundError:
        return ("error", None)


@pytest.mark.parametrize("seed", range(24))
def test_replicas_follow_writes(seed):
    import keto_amd
    ns, tuples, raw, ps, alph = random_graph(seed + 900, wide=seed % 4 == 3, allow_wildcards=seed % 3 == 0,
                                             allow_poison=False, allow_collisions=seed % 2 == 0)
    names, objs, rels, users = alph
    set_names = list(names)
    names = [n for n in names if n]
    if not names:
        pytest.skip("only a namespace named ''")
    store = SQLStore(ns, tuples, page_size=ps)
    first = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), page_size=ps, device=0)
    reps = [first, first.clone(0)]
    rng = random.Random(seed)
    for step in range(8):
        cur = store.tuples()
        ins = [_random_write(rng, names, objs, rels, users, set_names, 0.1) for _ in range(rng.randint(1, 8))]
        dels = [rng.choice(cur) for _ in range(rng.randint(0, 3))] if cur else []
        for r in reps:                                   # the write reaches every replica
            r.apply([_row(ns, t) for t in ins], [_row(ns, t) for t in dels])
        for t in ins:
            store.insert(t)
        for t in dels:
            store.delete(t)
        assert len({r.version() for r in reps}) == 1
        if step == 3:
            reps.append(reps[0].clone(0))                # a replica joining after writes
        checks = random_checks(seed * 37 + step, (names, objs + ["new1", "a0"], rels + ["q"], users + ["w001"]), k=48)
        for g in sorted({c[2] for c in checks}):
            grp = [c for c in checks if c[2] == g]
            # dealt round-robin, each replica's share checked concurrently from its own thread
            shares = [grp[k::len(reps)] for k in range(len(reps))]
            out = [None] * len(reps)

            def run(k):
                out[k] = reps[k].check_batch([(t.namespace, t.object, t.relation, subj(t.subject), d)
                                              for t, d, _ in shares[k]], g)[0]

            ts = [threading.Thread(target=run, args=(k,)) for k in range(len(reps))]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            for k, share in enumerate(shares):
                for (t, d, _), a in zip(share, out[k]):
                    assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, step, k, t, d, g)
        exps = random_expands(seed * 19 + step, (names, objs + ["new3"], rels + ["q"], users), k=8)
        for g in sorted({e[2] for e in exps}):
            grp = [e for e in exps if e[2] == g]
            for k, r in enumerate(reps):
                got = r.expand_batch([(subj(s), d) for s, d, _ in grp], g)
                for (s, d, _), (st, js) in zip(grp, got):
                    have = {0: "tree", 1: "nil", 2: "error"}[st]
                    assert (have, js) == _want_tree(store, s, d, g), (seed, step, k, s, d, g)
    for r in reps:
        r.close()


def test_clone_refuses_parts():
    import keto_amd
    ns = [(1, "n")]
    rows = [(1, "a", "r", "u")]
    part = keto_amd.Snapshot.build(ns, rows, device=-1).upload_part(0, 2, 0)
    with pytest.raises(keto_amd.KetoError):
        part.clone(0)
    part.close()
