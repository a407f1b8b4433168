#!/usr/bin/env python3
"""Migrating partition (KETO_PART_MIGRATE) measured on one GPU with P logical parts and a loopback
exchange: every row on one part, checks that move between parts as continuation records
(repo:keto_amd/csrc/migrate.hip, keto_amd/multi.py).  Prints one JSON line per part count with
the batch time, the rounds and records exchanged, per-part arena bytes, and parity against the
replicated snapshot on the same batch.

The exchange here is device-to-device copies on one GPU; on a node each round is one RCCL
all-to-all (keto_amd.multi.mig_check), so the per-round record bytes are reported for pricing it
over xGMI.

  python tools/bench_migrate.py --scale 0.125 --parts 1 2 4 --batch 4194304
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
    print(f"[bench_migrate {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.125)
    ap.add_argument("--parts", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--batch", type=int, default=4 << 20)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--hot-mb", type=float, nargs="+", default=[0.0],
                    help="replicated hot rows per part (MB of arena; keto_snapshot_upload_part_migrate)")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from keto_amd.capi import PART_MIGRATE, Snapshot
    from keto_amd.multi import SnapshotMigEngine, close_filters_loopback
    from tools import synth
    dev = "cuda:0"
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, a.scale), threads=a.threads)
    log(f"{g.n_edges} tuples, {g.n_rows} rows")
    q = g.queries(a.batch, seed=2024, depth=a.depth, threads=a.threads)
    full = g.snapshot(device=0)
    qd = torch.from_numpy(full.with_handles(q).view(np.uint8)).to(dev)
    d_out = torch.empty(a.batch, dtype=torch.uint8, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    full.check_batch_device(qd.data_ptr(), a.batch, d_out.data_ptr(), a.depth, sp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        full.check_batch_device(qd.data_ptr(), a.batch, d_out.data_ptr(), a.depth, sp)
    torch.cuda.synchronize()
    rep_ms = (time.perf_counter() - t0) / a.steps * 1e3
    want = d_out.cpu().numpy()
    full_bytes = full.stats()["device_bytes"]
    del full, qd
    for P, hot_mb in [(P, h) for P in a.parts for h in (a.hot_mb if P > 1 else [0.0])]:
        log(f"P = {P}, hot {hot_mb} MB: building and uploading {P} parts")
        t0 = time.perf_counter()
        parts = []
        for p in range(P):
            s = Snapshot.from_csr(g.namespaces, g.row_ns, g.row_obj, g.row_rel, g.row_ptr, g.edges, device=-1)
            parts.append(s.upload_part(p, P, 0, mode=PART_MIGRATE, hot_bytes=int(hot_mb * 1e6)))
        t_up = time.perf_counter() - t0
        t0 = time.perf_counter()
        crounds = close_filters_loopback(parts)
        t_close = time.perf_counter() - t0
        own = parts[0].row_owner(q["row"], P)
        own[own < 0] = 0
        where = [np.nonzero(own == p)[0] for p in range(P)]
        routed = [torch.from_numpy(np.ascontiguousarray(q[w]).view(np.int32).reshape(-1, 4).copy()).to(dev) for w in where]
        engines = [SnapshotMigEngine(p, dev) for p in parts]

        def batch():
            dec = [torch.empty(len(r), dtype=torch.uint8, device=dev) for r in routed]
            outs = [engines[p].begin(routed[p], dec[p], a.depth) for p in range(P)]
            per_round = []
            while sum(sum(o["records"]) for o in outs):
                recs = sum(sum(o["records"]) for o in outs)
                units = sum(sum(o["units"]) for o in outs)
                per_round.append((recs, units * 16))
                inbox = [[None] * P for _ in range(P)]
                for s in range(P):
                    buf, off = engines[s].fetch(outs[s])
                    ub = np.concatenate([[0], np.cumsum(outs[s]["units"][:P])])
                    rb = np.concatenate([[0], np.cumsum(outs[s]["records"][:P])])
                    for t in range(P):
                        inbox[t][s] = (buf[ub[t] * 16: ub[t + 1] * 16], off[rb[t]: rb[t + 1]])
                for t in range(P):
                    outs[t] = engines[t].round(torch.cat([inbox[t][s][0] for s in range(P)]),
                                               torch.cat([inbox[t][s][1] for s in range(P)]),
                                               [len(inbox[t][s][1]) for s in range(P)],
                                               [len(inbox[t][s][0]) // 16 for s in range(P)])
            return dec, per_round

        dec, per_round = batch()                                   # warm-up (workspaces)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            dec, per_round = batch()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        got = np.full(a.batch, 255, dtype=np.uint8)
        for p in range(P):
            got[where[p]] = dec[p].cpu().numpy()
        line = {"what": "migrating partition, loopback on one MI355X", "parts": P, "hot_mb": hot_mb,
                "tuples": int(g.n_edges),
                "rows": int(g.n_rows), "batch": a.batch, "max_depth": a.depth,
                "ms_per_batch": round(ms, 2), "checks_per_s": round(a.batch / (ms * 1e-3), 1),
                "replicated_ms_per_batch": round(rep_ms, 3),
                "rounds": len(per_round), "records_per_round": [r for r, _ in per_round],
                "record_bytes_per_round": [b for _, b in per_round],
                "part_device_bytes": [p.stats()["device_bytes"] for p in parts], "replicated_device_bytes": full_bytes,
                "stubs": [int(len(p.part_stubs())) for p in parts],
                "filter_exchange_rounds": crounds, "filter_exchange_s": round(t_close, 2),
                "upload_s": round(t_up, 1),
                "mismatches_vs_replicated": int((got != want).sum())}
        print(json.dumps(line), flush=True)
        del parts, engines, routed


if __name__ == "__main__":
    main()
