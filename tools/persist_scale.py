"""Persisted snapshots at BASELINE scale (keto_snapshot_save / keto_snapshot_load, persist.cpp): the
restart cost of a GPU server that loads its snapshot from a file instead of rebuilding it from the
table (keto_snapshot_build of the 1B-tuple graph: 170.8 s and 231.8 GB peak RSS,
profiles/r03bs_build_1b.log).

The generator's graph is loaded with its string table (keto_snapshot_from_csr, strings included, as
bench.py's string leg does), saved, loaded back onto the GPU, and 1,048,576 string requests and the
same requests in row-id form are compared between the two snapshots.  The file goes to --dir
(default $TMPDIR or /tmp) and is deleted afterwards; the second read comes from the page cache
unless the file is bigger than free memory (this box does not let a user drop caches), so the cold
rate is the first load's.  One JSON line.

  python tools/persist_scale.py [--scale 1.0] [--dir /tmp]
"""
import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(msg):
    print(f"[persist_scale {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def peak_rss_gb():
    import resource
    return round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR") or "/tmp")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    from keto_amd.capi import Snapshot
    from tools import synth
    log(f"generating the power-law graph at scale {a.scale}")
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, a.scale), threads=a.threads)
    u = g.unified(threads=a.threads)
    t0 = time.perf_counter()
    snap = g.snapshot_unified(u, device=a.device)
    t_csr = time.perf_counter() - t0
    st = snap.stats()
    path = os.path.join(a.dir, f"keto_persist_{os.getpid()}.keto")
    free = shutil.disk_usage(a.dir).free
    log(f"from_csr + upload {t_csr:.1f} s; {st['n_edges']} edges, {st['n_strings']} strings; "
        f"{free / 1e9:.1f} GB free in {a.dir}")
    t0 = time.perf_counter()
    snap.save(path, tag=42)
    t_save = time.perf_counter() - t0
    size = os.path.getsize(path)
    log(f"saved {size / 1e9:.2f} GB in {t_save:.1f} s")
    loads = []
    got = None
    for k in range(2):
        if got is not None:
            got.close()
        t0 = time.perf_counter()
        got, tag = Snapshot.load(path, device=a.device)
        loads.append(round(time.perf_counter() - t0, 2))
        log(f"load {k + 1}: {loads[-1]:.1f} s (host tables + layout + upload), tag {tag}")
    q = g.queries(1 << 20, seed=21, depth=5, threads=a.threads)
    want = snap.check_batch_ids(snap.with_handles(q), 5)
    have = got.check_batch_ids(got.with_handles(q), 5)
    reqs = g.string_requests(u.names, q, threads=a.threads)
    sw, _ = snap.check_batch_reqs(reqs, len(q), 5)
    sh, _ = got.check_batch_reqs(reqs, len(q), 5)
    os.unlink(path)
    out = {"tool": "persist_scale", "scale": a.scale, "tuples": int(st["n_tuples"]), "rows": int(st["n_rows"]),
           "strings": int(st["n_strings"]), "file_gb": round(size / 1e9, 2), "save_s": round(t_save, 2),
           "save_GB_per_s": round(size / 1e9 / t_save, 2), "load_s": loads,
           "from_csr_upload_s": round(t_csr, 2), "stats_equal": got.stats() == st, "tag": tag,
           "checks": len(q), "mismatches_ids": int((np.asarray(want) != np.asarray(have)).sum()),
           "mismatches_strings": int((sw != sh).sum()), "peak_rss_gb": peak_rss_gb(),
           "build_threads": int(os.environ.get("KETO_BUILD_THREADS", "16"))}
    print(json.dumps(out), flush=True)
    got.close()
    snap.close()
    u.free()
    g.close()


if __name__ == "__main__":
    main()
