#!/usr/bin/env python3
"""Migrating partition through the product path on one GPU: P parts, each a rank (thread) of the
in-process transport (keto_comm_init_local), one batch of packed string requests per rank through
keto_check_batch_routed_packed (each rank its slice; searches travel between parts as continuation
records, repo:keto_amd/csrc/migrate.hip).  Unlike tools/bench_migrate.py (parts one after another,
a Python loopback), the ranks run side by side as the Go Partition runs them.  Prints one JSON line
per (P, hot MB): the batch wall time, the replicated snapshot's keto_check_batch_packed time on the
same batch, and parity.

  python tools/bench_migrate_local.py --scale 0.125 --parts 1 2 4 8 --batch 4194304 --hot-mb 300
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


def log(msg):
    print(f"[bench_migrate_local {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def ranks(P, fn):
    res = [None] * P

    def run(r):
        try:
            res[r] = (True, fn(r))
        except Exception as e:          # noqa: BLE001
            res[r] = (False, e)

    ts = [threading.Thread(target=run, args=(r,)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a rank is still waiting"
    bad = [(r, v) for r, (ok, v) in enumerate(res) if not ok]
    assert not bad, bad
    return [v for _, v in res]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.125)
    ap.add_argument("--parts", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--batch", type=int, default=4 << 20)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--hot-mb", type=float, nargs="+", default=[300.0])
    a = ap.parse_args()
    import ctypes as C
    import torch
    torch.cuda.init()
    from keto_amd.capi import PART_MIGRATE, Comm, KCheckReq, Snapshot
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, a.scale), threads=16)
    u = g.unified(threads=16)
    log(f"{g.n_edges} tuples, {g.n_rows} rows")
    q = g.queries(a.batch, seed=2024, depth=a.depth, threads=16)
    arr = g.string_requests(u.names, q, threads=16)
    full = g.snapshot_unified(u, device=0)
    blob, packed, used = g.pack_requests(arr, a.batch)
    want = full.check_batch_packed(blob.array[:used], packed.array, a.depth, n=a.batch)[0].copy()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        full.check_batch_packed(blob.array[:used], packed.array, a.depth, n=a.batch)
    rep_ms = (time.perf_counter() - t0) / a.steps * 1e3
    del blob, packed
    full.close()

    def sl(lo, hi):
        return (KCheckReq * max(1, hi - lo)).from_address(C.addressof(arr) + lo * C.sizeof(KCheckReq))

    for P, hot in [(P, h) for P in a.parts for h in (a.hot_mb if P > 1 else [0.0])]:
        t0 = time.perf_counter()
        parts = ranks(P, lambda r: Snapshot.from_csr(g.namespaces, g.row_ns, u.row_obj, u.row_rel, g.row_ptr, u.edges,
                                                     kstrs=(u.strs, u.n_strings), device=-1)
                      .upload_part(r, P, 0, mode=PART_MIGRATE, hot_bytes=int(hot * 1e6)))
        t_up = time.perf_counter() - t0
        cid = os.urandom(32)
        comms = [Comm(cid, P, r, 0, local=True) for r in range(P)]
        t0 = time.perf_counter()
        ranks(P, lambda r: comms[r].close_filters(parts[r]))
        t_close = time.perf_counter() - t0
        bounds = [(r * a.batch // P, (r + 1) * a.batch // P) for r in range(P)]
        packs = [g.pack_requests(sl(lo, hi), hi - lo) for lo, hi in bounds]

        def batch():
            return ranks(P, lambda r: comms[r].check_batch_routed_packed(
                parts[r], packs[r][0].array[:packs[r][2]], packs[r][1].array, a.depth, n=bounds[r][1] - bounds[r][0]))

        res = batch()                                    # warm-up: indexes, workspaces
        got = np.concatenate([x for x, _ in res])
        times = []
        for _ in range(a.steps):
            t0 = time.perf_counter()
            batch()
            times.append(time.perf_counter() - t0)
        ms = float(np.median(times)) * 1e3
        line = {"what": "migrating partition, local transport ranks on one MI355X (keto_check_batch_routed_packed)",
                "parts": P, "hot_mb": hot, "tuples": int(g.n_edges), "batch": a.batch, "max_depth": a.depth,
                "ms_per_batch": round(ms, 2), "ms_min": round(min(times) * 1e3, 2),
                "checks_per_s": round(a.batch / (ms * 1e-3), 1),
                "replicated_packed_ms": round(rep_ms, 2), "x_replicated": round(ms / rep_ms, 2),
                "part_gib": [round(p.stats()["device_bytes"] / 2**30, 3) for p in parts],
                "upload_s": round(t_up, 1), "filter_exchange_s": round(t_close, 2),
                "mismatches_vs_replicated": int((got != want).sum())}
        print(json.dumps(line), flush=True)
        for c in comms:
            c.close()
        for p in parts:
            p.close()
        del packs


if __name__ == "__main__":
    main()
