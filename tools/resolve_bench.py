"""Host-side timing of string-form request resolution (keto_resolve_checks: names -> device form)
on the power-law graph with its string table, and a check that the string path resolves every
request exactly like the id path (row handle and subject string id).  Runs without a GPU.

    python tools/resolve_bench.py --scale 0.05 --n 4000000
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.05)
    ap.add_argument("--n", type=int, default=4_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--groups", default="16", help="KETO_RESOLVE_GROUP values to time (comma-separated)")
    a = ap.parse_args()
    os.environ["KETO_BUILD_THREADS"] = str(a.threads)
    from tools import synth
    t0 = time.perf_counter()
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, a.scale), threads=a.threads)
    u = g.unified(threads=a.threads)
    snap = g.snapshot_unified(u, device=-1)
    t_build = time.perf_counter() - t0
    q = g.queries(a.n, seed=1000, depth=5, threads=a.threads)
    reqs = g.string_requests(u.names, q, threads=a.threads)
    want = snap.with_handles(u.to_device_targets(q))
    t0 = time.perf_counter()
    snap.resolve_checks_reqs(reqs, 1)                       # builds the indexes
    t_index = time.perf_counter() - t0
    per_group = {}
    bad = 0
    for grp in a.groups.split(","):
        os.environ["KETO_RESOLVE_GROUP"] = grp
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            got, st = snap.resolve_checks_reqs(reqs, len(q))
            ts.append(time.perf_counter() - t0)
        bad += int((got != want).sum()) + int((st != 0).sum())
        best = min(ts)
        per_group[grp] = {"resolve_ms": round(best * 1e3, 2), "requests_per_s": round(a.n / best, 1)}
    print(json.dumps({"tuples": int(g.n_edges), "rows": int(g.n_rows), "strings": int(u.n_strings), "requests": a.n,
                      "threads": a.threads, "build_s": round(t_build, 2), "index_s": round(t_index, 2),
                      "by_group": per_group, "mismatches_vs_id_path": bad}))


if __name__ == "__main__":
    main()
