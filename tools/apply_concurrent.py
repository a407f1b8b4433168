"""Writes concurrent with reads (tooling): one thread runs keto_check_batch on 1,000,000 string
requests back to back while another applies TransactRelationTuples of K tuples (keto_snapshot_apply)
every `--gap-ms`, on config #2's snapshot built from its 10M string tuples.  Reports the check
batches' latency with and without the writer, the writes' latency under read load, and that the
untouched requests keep their decisions throughout.  keto_snapshot_apply stages a transaction under
the snapshot's shared lock (batches keep running) and commits it under the exclusive one, so a write
waits for the running batch only to commit, and the next batch waits only for the commit.

  python tools/apply_concurrent.py [--k 100] [--gap-ms 20] [--seconds 5]
  python tools/apply_concurrent.py --graph powerlaw1b --packed [--requests 1000000] [--readers 4]

--graph powerlaw1b: the headline graph (config #4, 1B tuples) with its string table (the bench's
string_form snapshot, keto_snapshot_from_csr + strings); writes add and remove direct
docs:<object>#view@<new user> tuples.  KETO_APPLY_TRACE=1 prints each write's device phases.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(xs, p):
    return round(float(np.percentile(np.asarray(xs) * 1e3, p)), 2) if xs else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--gap-ms", type=float, default=20.0)
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--packed", action="store_true",
                    help="reads through keto_check_batch_packed (GPU resolution, the Go batcher's call)")
    ap.add_argument("--graph", choices=["drive10m", "powerlaw1b"], default="drive10m")
    ap.add_argument("--requests", type=int, default=1_000_000)
    ap.add_argument("--new-rows", action="store_true",
                    help="each write's tuples name new objects: every write adds K rows (and strings)")
    ap.add_argument("--readers", type=int, default=1,
                    help="reader threads running batches side by side (the snapshot lock is writer-preferring: "
                         "a waiting write holds new batches back, so readers cannot starve it)")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from tools import synth
    t0 = time.perf_counter()
    if a.graph == "drive10m":
        g = synth.SynthGraph(dict(synth.DRIVE_10M), threads=a.threads, kind="drive")
        st = g.string_tuples(seed=11, threads=a.threads)
        snap, t_build = g.snapshot_from_strings(st, device=0)
        doc_ns, label = 1, "drive10m (config #2, built from string tuples)"
    else:
        g = synth.SynthGraph(dict(synth.POWERLAW_1B), threads=a.threads)
        st = g.unified(threads=a.threads)
        snap = g.snapshot_unified(st, device=0)
        st = st.names
        doc_ns, label = 1, "powerlaw1b (config #4, 1B tuples, snapshot with its string table)"
    t_setup = time.perf_counter() - t0
    print(f"[apply] {a.graph}: {g.n_edges} tuples ready in {t_setup:.1f} s", file=sys.stderr, flush=True)
    q = g.queries(a.requests, seed=2, depth=5, threads=a.threads)
    reqs = g.string_requests(st, q, threads=a.threads)
    if a.packed:
        blob, packed, used = g.pack_requests(reqs, len(q), threads=a.threads)

        def batch():
            return snap.check_batch_packed(blob.array[:used], packed.array, 5, n=len(q))[0]
    else:
        def batch():
            return snap.check_batch_reqs(reqs, len(q), 5)[0]
    before = batch().copy()
    hx = lambda v: f"{int(v):08x}"
    files_view = np.flatnonzero((g.row_ns == doc_ns) & (g.row_rel == g.relation_names().index("view")))
    rng = np.random.default_rng(7)

    def reads(seconds, lat, bad):
        t_end = time.perf_counter() + seconds
        while time.perf_counter() < t_end:
            t0 = time.perf_counter()
            out = batch()
            lat.append(time.perf_counter() - t0)
            bad.append(int((out != before).sum()))

    def read_threads(seconds, lat, bad):
        """Runs the readers for `seconds`; returns the checks per second of all of them together."""
        ts = [threading.Thread(target=reads, args=(seconds, lat, bad)) for _ in range(a.readers)]
        n0 = len(lat)
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return round((len(lat) - n0) * len(q) / (time.perf_counter() - t0), 1)

    quiet, quiet_bad = [], []
    rate_quiet = read_threads(a.seconds / 2, quiet, quiet_bad)
    stop = threading.Event()
    wlat, serial = [], [0]

    def writer():
        while not stop.is_set():
            rows = rng.choice(files_view, size=a.k, replace=False)
            ins = [(doc_ns, f"nw{serial[0] + i:08x}" if a.new_rows else hx(g.row_obj[r]), "view",
                    f"uw{serial[0] + i:08x}") for i, r in enumerate(rows)]
            serial[0] += a.k
            t0 = time.perf_counter()
            snap.apply(inserts=ins)
            snap.apply(deletes=ins)                      # back to the same table: reads stay comparable
            wlat.append((time.perf_counter() - t0) / 2)
            time.sleep(a.gap_ms / 1e3)

    loaded, loaded_bad = [], []
    w = threading.Thread(target=writer)
    w.start()
    rate_loaded = read_threads(a.seconds, loaded, loaded_bad)
    stop.set()
    w.join()
    out = {"graph": label, "tuples": int(g.n_edges), "setup_s": round(t_setup, 1),
           "reads": "keto_check_batch_packed (GPU resolution)" if a.packed else "keto_check_batch (host resolution)",
           "requests_per_batch": len(q), "reader_threads": a.readers, "write_tuples": a.k, "writes_add_rows": a.new_rows, "write_gap_ms": a.gap_ms,
           "batch_ms_quiet": {"p50": pct(quiet, 50), "p99": pct(quiet, 99), "n": len(quiet)},
           "batch_ms_with_writes": {"p50": pct(loaded, 50), "p99": pct(loaded, 99), "n": len(loaded)},
           "checks_per_s_quiet": rate_quiet, "checks_per_s_with_writes": rate_loaded,
           "packed_slots": os.environ.get("KETO_PACKED_SLOTS", "2 (default)") if a.packed else None,
           "write_ms_under_reads": {"p50": pct(wlat, 50), "p99": pct(wlat, 99), "n": len(wlat)},
           "writes_per_s": round(2 * len(wlat) / a.seconds, 1),
           "untouched_decisions_changed": int(sum(quiet_bad) + sum(loaded_bad)), "version": int(snap.version())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
