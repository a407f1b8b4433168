"""Tier-0 kernel variant sweep on one graph (tooling): builds the bench graph once, then times every
KETO_T0 variant on the same resident batch, checks that all variants agree bit for bit, and prints
the work / line-touch counters of each.

  python tools/tune.py [--scale 1.0] [--batch 16777216] [--depth 5] [--variants 0,1,2,3] [--reps 3]
  (a variant may carry a dynamic run size, static share and heads per XCD: --variants 0:0,0:16:4:8
  sets KETO_T0_DYN, KETO_T0_DYN_STATIC, KETO_T0_HEADS)
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
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--nested", action="store_true", help="config #3 nested-groups graph instead")
    a = ap.parse_args()
    import torch
    from tools import synth
    torch.cuda.set_device(0)
    if a.nested:
        g = synth.SynthGraph(synth.scaled(synth.NESTED_100M, a.scale) if a.scale != 1 else dict(synth.NESTED_100M),
                             kind="nested")
        q = g.queries_nested(a.batch, seed=77)
    else:
        params = synth.scaled(synth.POWERLAW_1B, a.scale) if a.scale != 1.0 else dict(synth.POWERLAW_1B)
        g = synth.SynthGraph(params)
        q = g.queries(a.batch, seed=1000, depth=a.depth)
    snap = g.snapshot(device=0)
    qd = snap.with_handles(q)
    d_q = torch.from_numpy(qd.view(np.uint8)).to("cuda:0")
    d_out = torch.empty(a.batch, dtype=torch.uint8, device="cuda:0")
    sp = torch.cuda.current_stream().cuda_stream
    ref = None
    print(f"graph: {g.n_edges} tuples, {g.n_rows} rows", flush=True)
    for tok in a.variants.split(","):
        # "variant[:run size[:static eighths[:heads per XCD[:walk cap]]]]" (KETO_T0_DYN,
        # KETO_T0_DYN_STATIC, KETO_T0_HEADS, KETO_T0_WALK; run size 0 = static runs; empty = default)
        v, dyn, st, hd, wc = (tok.split(":") + ["", "", "", ""])[:5]
        v = int(v)
        os.environ["KETO_T0"] = str(v)
        for k, x in (("KETO_T0_DYN", dyn), ("KETO_T0_DYN_STATIC", st), ("KETO_T0_HEADS", hd), ("KETO_T0_WALK", wc)):
            if x:
                os.environ[k] = x
            else:
                os.environ.pop(k, None)            # the engine's default
        snap.check_batch_device(d_q.data_ptr(), a.batch, d_out.data_ptr(), a.depth, sp)
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            snap.check_batch_device(d_q.data_ptr(), a.batch, d_out.data_ptr(), a.depth, sp)
            torch.cuda.synchronize()
            t, n = snap.last_timing()
            ms.append(t[0] + t[1] + t[2])
        out = d_out.cpu().numpy()
        if ref is None:
            ref = out.copy()
        mism = int((out != ref).sum())
        w = snap.check_work_device(d_q.data_ptr(), a.batch, d_out.data_ptr(), a.depth)
        per = {k: round(x / a.batch, 3) for k, x in zip(
            ("rows", "set_edges", "id_words", "vprobes", "vinserts", "items", "L_req", "L_hdr", "L_edge",
             "L_idtab", "L_idsearch", "push", "pop", "leaf", "leaf_miss", "pruned"), w[:16])}
        best = min(ms)
        print(json.dumps({"variant": tok, "mean_ms": round(sum(ms) / len(ms), 3), "ms": [round(x, 3) for x in ms], "checks_per_s": round(a.batch / best * 1e3),
                          "overflow": int(n[1]), "mismatch_vs_first": mism, "work": per}), flush=True)


if __name__ == "__main__":
    main()
