"""Parity of the MI355X engine (through the C-ABI) with the oracle.

* golden: every check / expand vector transcribed from the reference's tests and docs
  (tests/golden/reference_cases.json) -- expand trees compared exactly (child order included).
* random: quirk-heavy random graphs (cycles, duplicates, wildcard sets, poisoned pages, visit-key
  collisions, page sizes 1..100) against the SQL-level oracle, decisions bit-exact and expand
  trees exact.
"""
import pytest

from oracle.oracle_sql import (CheckEngine, ExpandEngine, NotFoundError, SQLStore, subject_from_json,
                               tuple_from_json)
from tests.engine_util import rows_from_tuples, subj
from tests.golden_util import case_namespaces, case_tuples, load_cases
from tests.randgraph import random_checks, random_expands, random_store

pytestmark = pytest.mark.gpu


def _snapshot(namespaces, rows, page_size):
    import keto_amd
    return keto_amd.Snapshot.build(namespaces, rows, page_size=page_size, device=0)


@pytest.mark.parametrize("case", load_cases(), ids=lambda c: c["name"])
def test_golden_on_gpu(case):
    from keto_amd.capi import EXPAND_NIL, EXPAND_NOT_FOUND, EXPAND_TREE
    ns = case_namespaces(case)
    snap = _snapshot(ns, rows_from_tuples(ns, case_tuples(case)), case.get("page_size", 100))
    for chk in case.get("checks", []):
        t = tuple_from_json(chk["tuple"])
        allowed, _ = snap.check_batch([(t.namespace, t.object, t.relation, subj(t.subject), chk["max_depth"])],
                                      chk["global_max_depth"])
        assert bool(allowed[0]) == chk["expected"], chk
    for ex in case.get("expands", []):
        (st, js), = snap.expand_batch([(subj(subject_from_json(ex["subject"])), ex["max_depth"])],
                                      ex["global_max_depth"])
        if ex.get("expected_error"):
            assert st == EXPAND_NOT_FOUND
        elif ex["expected"] is None:
            assert st == EXPAND_NIL
        else:
            assert st == EXPAND_TREE and js == ex["expected"]


@pytest.mark.parametrize("seed,wide", [(s, False) for s in range(300)] + [(s, True) for s in range(1000, 1060)])
def test_random_graphs_match_oracle(seed, wide):
    from keto_amd.capi import EXPAND_NIL, EXPAND_NOT_FOUND, EXPAND_TREE
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=wide)
    snap = _snapshot(ns, rows_from_tuples(ns, tuples, raw), ps)
    checks = random_checks(seed, alph, k=24)
    # the engine takes one global max-depth per batch: group by it
    for g in sorted({c[2] for c in checks}):
        grp = [c for c in checks if c[2] == g]
        allowed, _ = snap.check_batch([(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in grp], g)
        for (t, d, _), a in zip(grp, allowed):
            assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, t, d, g)
    exps = random_expands(seed, alph, k=12)
    for g in sorted({e[2] for e in exps}):
        grp = [e for e in exps if e[2] == g]
        got = snap.expand_batch([(subj(s), d) for s, d, _ in grp], g)
        for (s, d, _), (st, js) in zip(grp, got):
            try:
                t = ExpandEngine(store, g).build_tree(s, d)
                want = ("tree", t.to_json()) if t is not None else ("nil", None)
            except NotFoundError:
                want = ("error", None)
            have = {EXPAND_TREE: "tree", EXPAND_NIL: "nil", EXPAND_NOT_FOUND: "error"}[st]
            assert (have, js) == want, (seed, s, d, g)


STAGE_ENVS = {
    "two_pass": {"KETO_EXPAND_STAGE": "0"},
    "tiny_regions": {"KETO_EXPAND_STAGE": "3"},                    # most trees go on in overflow chunks
    "shared_regions": {"KETO_EXPAND_STAGE": "40", "KETO_SLOTS": "256"},   # many roots per lane's region
    "default_few_slots": {"KETO_SLOTS": "256"},                   # lanes' run queues fill: runs copied in place
    "inline_runs": {"KETO_EXPAND_RUN_INLINE": "32"},
    # trees past their region go on in overflow chunks: most trees in two pieces, the rest spill
    "split_chunks": {"KETO_EXPAND_STAGE": "3", "KETO_EXPAND_OVF_CHUNK": "40"},
    # the chunk pool runs out (4 chunks), with many roots per lane's region
    "split_pool_full": {"KETO_EXPAND_STAGE": "8", "KETO_SLOTS": "256", "KETO_EXPAND_OVF_CHUNK": "64",
                        "KETO_EXPAND_OVF_NODES": "256"},
    # no overflow chunks: every tree past its region goes to the second pass
    "no_chunks": {"KETO_EXPAND_STAGE": "5", "KETO_EXPAND_OVF_NODES": "0"},
}


@pytest.mark.parametrize("env", sorted(STAGE_ENVS))
@pytest.mark.parametrize("seed", range(3300, 3330))
def test_expand_staging_modes_match_oracle(monkeypatch, env, seed):
    """The one-pass expand (trees staged in per-lane regions while counted, then gathered to their
    offsets; a tree past its region goes on in an overflow chunk and is copied in two pieces; trees
    that fit neither filled by a second pass) in every regime: the two-pass form, regions so small
    that most trees spill, many roots sharing one lane's region, the default regions with few lanes
    (whose id-run queues fill up), short id runs copied in place, most trees in two pieces, a chunk
    pool that runs out, and no chunks.  Trees
    equal the oracle's, child order included."""
    from keto_amd.capi import EXPAND_NIL, EXPAND_NOT_FOUND, EXPAND_TREE
    for k, v in STAGE_ENVS[env].items():
        monkeypatch.setenv(k, v)
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=seed % 3 == 0)
    snap = _snapshot(ns, rows_from_tuples(ns, tuples, raw), ps)
    exps = random_expands(seed, alph, k=600)
    for g in sorted({e[2] for e in exps}):
        grp = [e for e in exps if e[2] == g]
        got = snap.expand_batch([(subj(s), d) for s, d, _ in grp], g)
        want_cache = {}
        for (s, d, _), (st, js) in zip(grp, got):
            key = (repr(s), d)
            if key not in want_cache:
                try:
                    t = ExpandEngine(store, g).build_tree(s, d)
                    want_cache[key] = ("tree", t.to_json()) if t is not None else ("nil", None)
                except NotFoundError:
                    want_cache[key] = ("error", None)
            have = {EXPAND_TREE: "tree", EXPAND_NIL: "nil", EXPAND_NOT_FOUND: "error"}[st]
            assert (have, js) == want_cache[key], (env, seed, s, d, g)


@pytest.mark.parametrize("seed", range(2100, 2160))
def test_random_expand_proto_device_equals_host(seed):
    """keto_tree_proto_all_device on quirk-heavy random graphs (wildcard roots answered by batch-local
    rows, subject ids the snapshot does not know, empty fields, unknown namespaces, collisions): the
    host encoder's bytes, tree by tree."""
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=seed % 3 == 0)
    snap = _snapshot(ns, rows_from_tuples(ns, tuples, raw), ps)
    exps = random_expands(seed, alph, k=24)
    for g in sorted({e[2] for e in exps}):
        grp = [(subj(s), d) for s, d, gg in exps if gg == g]
        _, host = snap.expand_batch(grp, g, proto_all="host")
        _, dev = snap.expand_batch(grp, g, proto_all="device")
        assert host == dev, (seed, g)


@pytest.mark.parametrize("seed", range(2200, 2240))
def test_random_expand_json_all_equals_per_tree(seed):
    """keto_tree_json_all (every tree's JSON on host threads) gives keto_tree_json's text for each
    tree, "null" for nil trees and "" for error roots, on quirk-heavy random graphs."""
    import json
    from keto_amd.capi import EXPAND_NIL, EXPAND_TREE
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=seed % 3 == 0)
    snap = _snapshot(ns, rows_from_tuples(ns, tuples, raw), ps)
    exps = random_expands(seed, alph, k=24)
    for g in sorted({e[2] for e in exps}):
        grp = [(subj(s), d) for s, d, gg in exps if gg == g]
        got, texts = snap.expand_batch(grp, g, json_all=True)
        for (st, js), txt in zip(got, texts):
            if st == EXPAND_TREE:
                assert json.loads(txt) == js, (seed, g)
            elif st == EXPAND_NIL:
                assert txt == "null"
            else:
                assert txt == ""


def test_deep_chain_tree_json():
    """A 2,500-level tree (a chain of nested groups expanded with max-depth 3000): the JSON encoders
    are iterative, so a tree as deep as the max-depth allows encodes without exhausting the host
    stack; the text equals the chain's expected JSON."""
    import sys
    from keto_amd.capi import EXPAND_TREE
    from oracle.oracle_sql import RelationTuple, SubjectID, SubjectSet
    k = 2500
    ns = [(1, "n")]
    tuples = [RelationTuple("n", f"g{i}", "m", SubjectSet("n", f"g{i + 1}", "m")) for i in range(k - 1)]
    tuples.append(RelationTuple("n", f"g{k - 1}", "m", SubjectID("user")))
    snap = _snapshot(ns, rows_from_tuples(ns, tuples), 100)
    want = '{"type":"leaf","subject_id":"user"}'
    for i in reversed(range(k)):
        want = ('{"type":"union","children":[' + want +
                '],"subject_set":{"namespace":"n","object":"g%d","relation":"m"}}' % i)
    old = sys.getrecursionlimit()
    sys.setrecursionlimit(max(old, 4 * k + 1000))   # expand_batch parses the per-tree text
    try:
        got, texts = snap.expand_batch([(("set", "n", "g0", "m"), 3000)], 3000, json_all=True)
    finally:
        sys.setrecursionlimit(old)
    assert got[0][0] == EXPAND_TREE
    assert texts[0] == want
    # the protobuf encoders on the same tree: per tree, all trees on host threads, and on the GPU
    sys.setrecursionlimit(max(old, 4 * k + 1000))
    try:
        (st, _, pb), = snap.expand_batch([(("set", "n", "g0", "m"), 3000)], 3000, want_proto=True)
        _, host = snap.expand_batch([(("set", "n", "g0", "m"), 3000)], 3000, proto_all="host")
        _, dev = snap.expand_batch([(("set", "n", "g0", "m"), 3000)], 3000, proto_all="device")
    finally:
        sys.setrecursionlimit(old)
    assert st == EXPAND_TREE and len(pb) > 0
    assert host[0] == pb and dev[0] == pb


@pytest.mark.parametrize("seed", range(2000, 2060))
def test_random_expand_proto_matches_oracle(seed):
    """keto_tree_proto = proto.Marshal(Tree.ToProto()) of the oracle's tree (internal/expand/tree.go:165-188),
    byte for byte, on quirk-heavy random graphs (empty fields, collisions, duplicates, cycles)."""
    from keto_amd.capi import EXPAND_TREE
    from tests.proto_util import tree_json_to_proto
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=seed % 3 == 0)
    snap = _snapshot(ns, rows_from_tuples(ns, tuples, raw), ps)
    exps = random_expands(seed, alph, k=16)
    for g in sorted({e[2] for e in exps}):
        grp = [e for e in exps if e[2] == g]
        got = snap.expand_batch([(subj(s), d) for s, d, _ in grp], g, want_proto=True)
        for (s, d, _), (st, js, pb) in zip(grp, got):
            if st == EXPAND_TREE:
                assert pb == tree_json_to_proto(js), (seed, s, d, g)
                try:
                    t = ExpandEngine(store, g).build_tree(s, d)
                except NotFoundError:
                    t = None
                assert t is not None and pb == tree_json_to_proto(t.to_json())
            else:
                assert pb in (None, b""), (seed, st, pb)


@pytest.mark.parametrize("seed", range(2300, 2340))
def test_random_expand_via_fields_matches_json(seed):
    """Trees rebuilt from keto_tree_nodes + keto_subject_fields (how the Go shim builds expand.Tree
    values, integration/go/internal/gpu/gpu.go) equal keto_tree_json's trees, on quirk-heavy random
    graphs (batch-local wildcard roots, unknown subject ids, empty fields, collisions)."""
    from keto_amd.capi import EXPAND_TREE
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=seed % 3 == 0)
    snap = _snapshot(ns, rows_from_tuples(ns, tuples, raw), ps)
    exps = random_expands(seed, alph, k=16)
    for g in sorted({e[2] for e in exps}):
        grp = [(subj(s), d) for s, d, gg in exps if gg == g]
        for st, js, tf in snap.expand_batch(grp, g, via_fields=True):
            assert (st == EXPAND_TREE) == (tf is not None)
            assert tf == js, (seed, g)


@pytest.mark.parametrize("env", [{}, {"KETO_EXPAND_BIG_CAP": "7"}, {"KETO_EXPAND_BIG_CAP": "64"},
                                 {"KETO_EXPAND_STAGE": "0"}, {"KETO_SLOTS": "256"}],
                         ids=["default", "big_cap_7", "big_cap_64", "two_pass", "few_slots"])
def test_expand_many_big_runs(monkeypatch, env):
    """Trees too big for a staging region (20 subject sets of 1,025-1,044 ids each: every set's id
    run is longer than BIG_RUN and takes 2 pieces) go through the second pass, whose shared queue of
    big-run pieces fills up when it is small: a run whose pieces do not all fit is copied in place
    and no queue slot is left unwritten.  The trees are written out here and compared whole
    (internal/expand/engine.go:33-102: sets before ids, both in ORDER BY order)."""
    from keto_amd.capi import EXPAND_TREE
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    roots, sets = 16, 20
    ns = [(1, "n")]
    rows, want = [], []
    for i in range(roots):
        kids = []
        for j in range(sets):
            c = f"c{i:02d}_{j:02d}"
            rows.append((1, f"r{i:02d}", "m", None, 1, c, "m"))
            ids = [f"u{(i * 7919 + j * 104729 + k) % 1000003:07d}" for k in range(1025 + j)]
            ids = sorted(set(ids))
            for u in ids:
                rows.append((1, c, "m", u))
            kids.append({"type": "union", "subject_set": {"namespace": "n", "object": c, "relation": "m"},
                         "children": [{"type": "leaf", "subject_id": u} for u in ids]})
        want.append({"type": "union", "subject_set": {"namespace": "n", "object": f"r{i:02d}", "relation": "m"},
                     "children": kids})
    snap = _snapshot(ns, rows, 100)
    got = snap.expand_batch([(("set", "n", f"r{i:02d}", "m"), 0) for i in range(roots)] * 3, 5)
    for k, (st, js) in enumerate(got):
        assert st == EXPAND_TREE
        assert js == want[k % roots], (env, k)
