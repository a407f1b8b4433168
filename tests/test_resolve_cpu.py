"""String-form request resolution (keto_resolve_checks, resolve.cpp) on host-only snapshots: the
hashed string / row indexes and the staged resolver give every request exactly the ids the id path
gives it (row handle, subject string id), on the power-law generator's graph with its string table,
plus unknown strings, unknown namespaces, empty fields and subject-set subjects through the general
path (whereQuery semantics, internal/persistence/sql/relationtuples.go:178-198)."""
import numpy as np
import pytest

from keto_amd.capi import CHECK_IDS_DTYPE


@pytest.fixture(scope="module")
def unified_graph():
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 4096), threads=4)
    u = g.unified(threads=4)
    snap = g.snapshot_unified(u, device=-1)
    yield g, u, snap
    snap.close()
    u.free()
    g.close()


@pytest.mark.parametrize("threads", ["1", "4"])
def test_string_path_equals_id_path(unified_graph, monkeypatch, threads):
    monkeypatch.setenv("KETO_BUILD_THREADS", threads)
    g, u, snap = unified_graph
    q = g.queries(200_000, seed=11, depth=5, threads=4)
    reqs = g.string_requests(u.names, q, threads=4)
    got, st = snap.resolve_checks_reqs(reqs, len(q))
    want = snap.with_handles(u.to_device_targets(q))
    assert (st == 0).all()
    assert (got == want).all()


def test_unknown_and_general_forms(unified_graph):
    g, u, snap = unified_graph
    ns = dict(g.namespaces)
    obj = f"{int(g.row_obj[0]):08x}"
    rel = g.relation_names()[int(g.row_rel[0])]
    nsn = ns[int(g.row_ns[0])]
    reqs = [(nsn, obj, rel, ("id", "u00000000"), 0),          # fast path
            (nsn, obj, rel, ("id", "nobody"), 3),              # unknown subject string
            (nsn, "zzzzzzzz", rel, ("id", "u00000000"), 0),    # unknown object: no row
            ("nope", obj, rel, ("id", "u00000000"), 0),        # unknown namespace
            (nsn, obj, rel, ("set", nsn, obj, rel), 0)]        # subject set: general path
    out, st = snap.resolve_checks(reqs)
    h = snap.row_handles(np.array([0], dtype=np.uint32))[0]
    assert out[0]["row"] == h and out[0]["target"] == u.user_base and st[0] == 0
    assert out[1]["row"] == h and out[1]["target"] == 0xFFFFFFFF and out[1]["max_depth"] == 3
    assert out[2]["row"] == 0xFFFFFFFF and st[2] == 0
    assert out[3]["row"] == 0xFFFFFFFF and st[3] == 1       # KETO_CHECK_UNKNOWN_NAMESPACE
    assert out[4]["row"] == h and out[4]["target"] == h and out[4]["flags"] == 1
    assert out.dtype == CHECK_IDS_DTYPE
