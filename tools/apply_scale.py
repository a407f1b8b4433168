"""keto_snapshot_apply on a snapshot built from 10M string tuples (tooling): the latency of one
TransactRelationTuples of K tuples, K = 1, 100, 10,000, and that the snapshot still decides
exactly: 1,000,000 string requests that no write touches keep their decisions, every inserted
files:d#view@<new user> is allowed right after its insert and denied again after its delete.
Subject-set inserts (files:d#view@(folders:f#view)) are timed too; their decisions are covered by
tests/test_gpu_lifecycle.py against the SQL oracle.

  python tools/apply_scale.py [--graph drive10m]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(msg):
    print(f"[apply_scale {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from tools import synth
    g = synth.SynthGraph(dict(synth.DRIVE_10M), threads=a.threads, kind="drive")
    st = g.string_tuples(seed=11, threads=a.threads)
    snap, t_build = g.snapshot_from_strings(st, device=0)
    log(f"built {g.n_edges} tuples in {t_build:.1f} s")
    q = g.queries(1_000_000, seed=2, depth=5, threads=a.threads)
    reqs = g.string_requests(st, q, threads=a.threads)
    before, _ = snap.check_batch_reqs(reqs, len(q), 5)
    hx = lambda v: f"{int(v):08x}"
    files_view = np.flatnonzero((g.row_ns == 1) & (g.row_rel == 2))
    folders_view = np.flatnonzero((g.row_ns == 2) & (g.row_rel == 2))
    rng = np.random.default_rng(5)
    out = {"graph": "drive10m (config #2, built from string tuples)", "tuples": int(g.n_edges), "build_s": round(t_build, 2),
           "runs": []}
    serial = 0
    for k in (1, 100, 10_000):
        rows = rng.choice(files_view, size=k, replace=False)
        ins = [(1, hx(g.row_obj[r]), "view", f"unew{serial + i:08x}") for i, r in enumerate(rows)]
        serial += k
        t0 = time.perf_counter()
        v = snap.apply(inserts=ins)
        t_ins = time.perf_counter() - t0
        new = [("files", t[1], "view", ("id", t[3]), 0) for t in ins]
        got_new, _ = snap.check_batch(new, 5)
        after, _ = snap.check_batch_reqs(reqs, len(q), 5)
        unchanged = int((after == before).sum())
        t0 = time.perf_counter()
        snap.apply(deletes=ins)
        t_del = time.perf_counter() - t0
        gone, _ = snap.check_batch(new, 5)
        # subject-set edges: files -> random folders (timed; decisions: test_gpu_lifecycle.py)
        sets = [(1, hx(g.row_obj[r]), "view", None, 2, hx(g.row_obj[f]), "view")
                for r, f in zip(rng.choice(files_view, size=k, replace=False), rng.choice(folders_view, size=k))]
        t0 = time.perf_counter()
        snap.apply(inserts=sets)
        t_set = time.perf_counter() - t0
        t0 = time.perf_counter()
        snap.apply(deletes=sets)
        t_set_del = time.perf_counter() - t0
        back, _ = snap.check_batch_reqs(reqs, len(q), 5)
        r = {"k": k, "insert_ms": round(t_ins * 1e3, 1), "delete_ms": round(t_del * 1e3, 1),
             "set_insert_ms": round(t_set * 1e3, 1), "set_delete_ms": round(t_set_del * 1e3, 1),
             "inserted_allowed": int(np.sum(got_new)), "deleted_denied": int(k - np.sum(gone)),
             "untouched_requests_unchanged": unchanged, "decisions_restored_after_set_round_trip": int((back == before).sum()),
             "version": int(snap.version())}
        log(json.dumps(r))
        out["runs"].append(r)
    out["requests"] = len(q)
    print(json.dumps(out), flush=True)
    snap.close()
    g.free_strings(st)


if __name__ == "__main__":
    main()
