"""End-to-end (host buffers, pipelined chunks) sweep on the 1B graph (tooling): builds the bench
graph once, then times keto_check_batch_pairs over pinned host buffers for each setting of the
chunking / tier-0 run environment, checking every setting decides like the first.

  python tools/e2e_sweep.py [--scale 1.0] [--reps 5] --settings "KETO_CHUNK=4194304;KETO_CHUNK=2097152,KETO_T0_DYN_FORCE=1"
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--batch", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--settings", default="")
    a = ap.parse_args()
    import torch
    from keto_amd.capi import CHECK_PAIR_DTYPE, HostBuffer, pairs_of
    from tools import synth
    torch.cuda.set_device(0)
    params = synth.scaled(synth.POWERLAW_1B, a.scale) if a.scale != 1.0 else dict(synth.POWERLAW_1B)
    g = synth.SynthGraph(params)
    q = g.queries(a.batch, seed=1000, depth=a.depth)
    snap = g.snapshot(device=0)
    hq, ho = HostBuffer(len(q), CHECK_PAIR_DTYPE), HostBuffer(len(q), np.uint8)
    hq.array[:] = pairs_of(q)
    ref = None
    keys = set()
    for tok in a.settings.split(";"):
        env = dict(kv.split("=") for kv in tok.split(",") if kv)
        for k in keys - set(env):
            os.environ.pop(k, None)
        os.environ.update(env)
        keys |= set(env)
        snap.check_batch_pairs(hq.array, a.depth, a.depth, out=ho.array)      # warm-up
        ts, walls, tiers = [], [], []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            snap.check_batch_pairs(hq.array, a.depth, a.depth, out=ho.array)
            ts.append((time.perf_counter() - t0) * 1e3)
            t = snap.last_timing_full()
            walls.append(t["wall_ms"])
            tiers.append(t["tier_ms"][0])
        out = ho.array.copy()
        if ref is None:
            ref = out
        print(json.dumps({"env": env, "ms": round(float(np.median(ts)), 3), "checks_per_s": round(len(q) / np.median(ts) * 1e3),
                          "tier0_ms_sum": round(float(np.median(tiers)), 3), "chunks": t["chunks"],
                          "mismatch_vs_first": int((out != ref).sum())}), flush=True)


if __name__ == "__main__":
    main()
