"""Config #3's longest serial chain on its own: where does a deep search's step go?

Builds the nested-groups graph (100M tuples), finds the requests with the longest searches among
1M requests at depths 5/16/32 (keto_check_steps_device: loop iterations per request, summed over its
items and tiers), then times batches holding only the top-k of them.  A lone request's batch time is
its longest item's chain, so time / steps is the cost of one dependent iteration of check_kernel on
an otherwise idle chip.  Run under rocprofv3 --pmc to split that cost into instructions and waits
(--only-single skips everything but the timed single-request batches).

  python tools/dev/chain_probe.py [--scale 1.0] [--top 4] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def log(msg):
    print(f"[chain {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--requests", type=int, default=1_000_000)
    ap.add_argument("--top", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--batch-only", action="store_true", help="only time the whole batch (env sweeps)")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from tools import synth
    params = dict(synth.NESTED_100M) if a.scale == 1.0 else synth.scaled(synth.NESTED_100M, a.scale)
    g = synth.SynthGraph(params, threads=a.threads, kind="nested", chain=32)
    log(f"{g.n_edges} tuples; snapshot")
    snap = g.snapshot(device=0)
    q = g.queries_nested(a.requests, seed=3, depths=(5, 16, 32), threads=a.threads)
    qd = snap.with_handles(q)
    d_q = torch.from_numpy(qd.view(np.uint8)).to("cuda:0")
    d_out = torch.empty(len(q), dtype=torch.uint8, device="cuda:0")
    d_steps = torch.zeros(len(q), dtype=torch.int32, device="cuda:0")
    if a.batch_only:
        sp = torch.cuda.current_stream().cuda_stream
        best, full = 1e9, None
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            snap.check_batch_device(d_q.data_ptr(), len(q), d_out.data_ptr(), 32, sp)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            if ms < best:
                best, full = ms, snap.last_timing_full()
        print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("KETO_")}, "wall_ms": round(best, 3),
                          "tier_ms": [round(x, 3) for x in full["tier_ms"]], "items_ms": round(full["items_ms"], 3),
                          "items": full["items"], "kept": full["items_kept"],
                          "allowed": round(float(d_out.float().mean().item()), 5)}), flush=True)
        return
    snap.check_steps_device(d_q.data_ptr(), len(q), d_out.data_ptr(), d_steps.data_ptr(), 32)
    torch.cuda.synchronize()
    steps = d_steps.cpu().numpy().astype(np.int64)
    order = np.argsort(steps)[::-1]
    sp = torch.cuda.current_stream().cuda_stream
    res = {"tuples": int(g.n_edges), "requests": len(q), "single": []}
    for rank in range(a.top):
        i = int(order[rank])
        one = torch.from_numpy(qd[i:i + 1].copy().view(np.uint8)).to("cuda:0")
        o1 = torch.empty(1, dtype=torch.uint8, device="cuda:0")
        times = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            snap.check_batch_device(one.data_ptr(), 1, o1.data_ptr(), 32, sp)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        full = snap.last_timing_full()
        best = min(times)
        deep_ms = full["tier_ms"][0]
        res["single"].append({"request": i, "max_depth": int(q["max_depth"][i]), "steps": int(steps[i]),
                              "allowed": int(o1.item()), "wall_ms": [round(t, 3) for t in times],
                              "tier_ms": [round(x, 3) for x in full["tier_ms"]], "items_ms": round(full["items_ms"], 3),
                              "items": full["items"], "items_kept": full["items_kept"],
                              "us_per_step_tier0": round(deep_ms * 1e3 / max(1, int(steps[i])), 3),
                              "us_per_step_wall": round(best * 1e3 / max(1, int(steps[i])), 3)})
        log(json.dumps(res["single"][-1]))
    # the whole batch, and the batch without its longest searches: how much of the batch is the chain
    for drop in (0, 16, 256):
        keep = np.sort(order[drop:])
        sub = torch.from_numpy(qd[keep].copy().view(np.uint8)).to("cuda:0")
        o = torch.empty(len(keep), dtype=torch.uint8, device="cuda:0")
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            snap.check_batch_device(sub.data_ptr(), len(keep), o.data_ptr(), 32, sp)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e3)
        full = snap.last_timing_full()
        res[f"batch_without_top_{drop}"] = {"wall_ms": round(best, 3), "tier_ms": [round(x, 3) for x in full["tier_ms"]],
                                            "items_ms": round(full["items_ms"], 3),
                                            "longest_steps_left": int(steps[order[drop]])}
        log(json.dumps(res[f"batch_without_top_{drop}"]))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
