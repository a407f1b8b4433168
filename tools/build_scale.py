"""The product's snapshot builder (keto_snapshot_build: sharded interning, parallel ORDER BY sort,
collision classes, layout, upload) at BASELINE scale, timed, and checked against the bulk CSR loader.

For each graph the generator's CSR is emitted as keto_relation_tuples rows with strings in a
seeded random commit order (tools/synth.cpp synth_emit_strings), built with keto_snapshot_build,
and 1,000,000 string requests (keto_check_batch: in-library resolution) are compared with the same
requests on the keto_snapshot_from_csr snapshot (row-id form).  One JSON line per graph.

  python tools/build_scale.py [--graphs drive10m,nested100m] [--threads 16]
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
    print(f"[build_scale {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def peak_rss_gb():
    import resource
    return round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 1)   # KiB -> GB


def run(name, g, q, gmd, threads):
    log(f"{name}: {g.n_edges} tuples; emitting string rows")
    t0 = time.perf_counter()
    st = g.string_tuples(seed=11, threads=threads)
    t_emit = time.perf_counter() - t0
    log(f"{name}: keto_snapshot_build (host + upload)")
    rss0 = peak_rss_gb()
    os.environ["KETO_BUILD_TRACE"] = "1"
    snap, t_build = g.snapshot_from_strings(st, device=0)
    del os.environ["KETO_BUILD_TRACE"]
    rss1 = peak_rss_gb()
    stats = snap.stats()
    log(f"{name}: built in {t_build:.1f} s; from_csr snapshot")
    t0 = time.perf_counter()
    ref_snap = g.snapshot(device=0)
    t_csr = time.perf_counter() - t0
    log(f"{name}: {len(q)} requests: strings on the built snapshot vs row ids on the CSR snapshot")
    reqs = g.string_requests(st, q, threads=threads)
    t0 = time.perf_counter()
    got, status = snap.check_batch_reqs(reqs, len(q), gmd)
    t_str = time.perf_counter() - t0
    want = ref_snap.check_batch_rows(q, gmd)
    mism = int((got != want).sum())
    snap.close()
    ref_snap.close()
    g.free_strings(st)
    return {"graph": name, "tuples": int(g.n_edges), "rows": int(stats["n_rows"]), "strings": int(stats["n_strings"]),
            "build_threads": int(os.environ.get("KETO_BUILD_THREADS", "0") or 0) or "default (<= 16)",
            "emit_s": round(t_emit, 2), "keto_snapshot_build_s": round(t_build, 2),
            "from_csr_s": round(t_csr, 2), "device_bytes": int(stats["device_bytes"]),
            "string_requests": len(q), "string_batch_s": round(t_str, 3),
            "string_checks_per_s": round(len(q) / t_str, 1), "allowed_fraction": round(float(got.mean()), 4),
            "mismatches_vs_from_csr": mism, "unknown_namespace_status": int((status == 1).sum()),
            "peak_rss_gb_before_build": rss0, "peak_rss_gb_after_build": rss1,
            "what_rss": "process peak RSS (graph CSR + string rows + the builder's working set)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", default="drive10m,nested100m")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--requests", type=int, default=1_000_000)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from tools import synth
    for name in a.graphs.split(","):
        if name == "drive10m":
            g = synth.SynthGraph(dict(synth.DRIVE_10M), threads=a.threads, kind="drive")
            q = g.queries(a.requests, seed=2, depth=5, threads=a.threads)
            r = run(name, g, q, 5, a.threads)
        elif name == "nested100m":
            g = synth.SynthGraph(dict(synth.NESTED_100M), threads=a.threads, kind="nested", chain=32)
            q = g.queries_nested(a.requests, seed=3, depths=(5, 16, 32), threads=a.threads)
            r = run(name, g, q, 32, a.threads)
        elif name.startswith("powerlaw") and name.endswith("m"):
            # powerlaw100m, powerlaw500m, powerlaw1000m: the bench graph at that many tuples
            scale = int(name[len("powerlaw"):-1]) / 1000.0
            g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, scale) if scale != 1.0 else dict(synth.POWERLAW_1B),
                                 threads=a.threads)
            q = g.queries(a.requests, seed=4, depth=5, threads=a.threads)
            r = run(name, g, q, 5, a.threads)
        else:
            raise SystemExit(f"unknown graph {name}")
        g.close()
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
