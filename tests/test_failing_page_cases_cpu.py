"""The cases tests/test_gpu_comm.py::test_local_migrating_wildcard_over_failing_pages drives through a
migrating partition, counted on the SQL oracle (no GPU): wildcard queries whose ORDER BY sequence
holds a failing tuple (a subject set of a namespace id the config lacks), so the query's page loop
stops at that page (relationtuples.go:64-71,250-277; internal/check/engine.go:98-100), and among them
the queries whose failing page starts inside a row -- the row is read only in part, which is what the
per-tuple requests of comm.cpp's routed_check answer."""
from oracle.oracle_sql import _NID, _ORDER
from tests.randgraph import poisoned_wildcard_case

SEEDS = range(4500, 4516)       # the GPU test's seeds


def _cut(store, t):
    """(failing tuple found, the failing page starts inside a row) for query t."""
    where, args = ["nid = ?"], [_NID]
    if t.namespace != "":
        where.append("namespace_id = ?")
        args.append(store.nm.by_name(t.namespace)[0])
    if t.object != "":
        where.append("object = ?")
        args.append(t.object)
    if t.relation != "":
        where.append("relation = ?")
        args.append(t.relation)
    rows = store.conn.execute(
        f"SELECT namespace_id, object, relation, subject_set_namespace_id, subject_id FROM keto_relation_tuples "
        f"WHERE {' AND '.join(where)} ORDER BY {_ORDER}", args).fetchall()
    for k, r in enumerate(rows):
        if r[4] is None and _unknown(store, r[3]):
            L = k // store.page_size * store.page_size
            return True, 0 < L < len(rows) and rows[L - 1][:3] == rows[L][:3]
    return False, False


def _unknown(store, nid):
    try:
        store.nm.by_id(nid)
        return False
    except Exception:          # noqa: BLE001 -- NotFoundError
        return True


def test_failing_page_wildcard_cases_are_covered():
    cut = inside = 0
    for seed in SEEDS:
        store, ns, tuples, raw, ps, reqs, checks = poisoned_wildcard_case(seed)
        for t, _ in checks:
            if t.object != "" and t.relation != "":
                continue
            c, i = _cut(store, t)
            cut += c
            inside += i
    assert cut >= 100 and inside >= 50, (cut, inside)     # 132 and 66 at these seeds
