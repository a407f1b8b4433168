"""ref-sql CPU baseline on many cores -- TEST / BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).

The reference check engine's recursion issuing its own SQL (oracle/oracle_sql.py: SELECT ... WHERE
... ORDER BY ... LIMIT 100 OFFSET plus the page count, per expanded node) against SQLite, with one
worker process per core, each with its own in-memory copy of one database image (copied from a
file on tmpfs; the reference's DSN is an in-memory SQLite, internal/driver/config/provider.go:41).  Run as a separate process by bench.py, so the workers
fork from a process that never touched the GPU:

  python -m oracle.sql_bench --db /dev/shm/x.sqlite --requests reqs.json --workers 16 --gmd 5

prints one JSON line {checks_per_s, workers, decisions, ...}.
"""
import argparse
import json
import multiprocessing as mp
import os
import sqlite3
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle.oracle_sql import CheckEngine, Namespaces, RelationTuple, SQLStore, SubjectID, SubjectSet  # noqa: E402


def open_store(db, namespaces, page_size):
    """The worker's own in-memory copy of the database image (SQLite backup API)."""
    st = SQLStore.__new__(SQLStore)
    st.nm = Namespaces(namespaces)
    st.page_size = page_size
    src = sqlite3.connect(f"file:{db}?mode=ro&immutable=1", uri=True)
    st.conn = sqlite3.connect(":memory:")
    src.backup(st.conn)
    src.close()
    st._seq = 0
    st.requested_pages = []
    return st


def _work(args):
    db, namespaces, reqs, gmd, t_start = args
    st = open_store(db, namespaces, 100)
    eng = CheckEngine(st, gmd)
    while time.time() < t_start:          # start together
        time.sleep(0.001)
    t0 = time.perf_counter()
    # a request's subject: a subject id (string) or a subject set [namespace, object, relation]
    out = [int(eng.subject_is_allowed(RelationTuple(ns, o, r, SubjectID(s) if isinstance(s, str) else SubjectSet(*s)), d))
           for ns, o, r, s, d in reqs]
    st.requested_pages = []
    return out, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--db", required=True)
    ap.add_argument("--requests", required=True)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--gmd", type=int, default=5)
    a = ap.parse_args()
    spec = json.load(open(a.requests))
    namespaces = [tuple(x) for x in spec["namespaces"]]
    reqs = [tuple(x) for x in spec["requests"]]
    w = max(1, min(a.workers, len(reqs)))
    parts = [reqs[i::w] for i in range(w)]
    t_start = time.time() + 1.0
    with mp.get_context("fork").Pool(w) as pool:
        res = pool.map(_work, [(a.db, namespaces, p, a.gmd, t_start) for p in parts])
    dec = [0] * len(reqs)
    for i, (out, _) in enumerate(res):
        dec[i::w] = out
    wall = max(t for _, t in res)
    print(json.dumps({"checks_per_s": round(len(reqs) / wall, 1), "workers": w, "requests": len(reqs),
                      "slowest_worker_s": round(wall, 3), "decisions": dec}), flush=True)


if __name__ == "__main__":
    main()
