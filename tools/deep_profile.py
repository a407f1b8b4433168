"""Config #3 (nested groups, 100M tuples, depth <= 32, cycles): where the deep check kernel's time
goes.  Prints one JSON line: the kernel time per tier, and the histogram of per-request loop
iterations (keto_check_steps_device: the serial chain each request's DFS walks), overall and per
request depth, with the share of requests and of iterations in the longest searches.

  python tools/deep_profile.py [--requests 1000000] [--threads 16]
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
    print(f"[deep {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def hist(steps):
    edges = [1, 2, 4, 8, 16, 64, 256, 1024, 4096, 16384, 65536, 1 << 18, 1 << 20, 1 << 32]
    h = np.histogram(steps, bins=edges)[0]
    return {f"[{edges[i]},{edges[i + 1]})": int(h[i]) for i in range(len(h)) if h[i]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--scale", type=float, default=1.0)
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
    sp = torch.cuda.current_stream().cuda_stream
    snap.check_batch_device(d_q.data_ptr(), len(q), d_out.data_ptr(), 32, sp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    snap.check_batch_device(d_q.data_ptr(), len(q), d_out.data_ptr(), 32, sp)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms, cnt = snap.last_timing()
    full = snap.last_timing_full()
    out = d_out.cpu().numpy()
    log("instrumented pass (per-request steps)")
    snap.check_steps_device(d_q.data_ptr(), len(q), d_out.data_ptr(), d_steps.data_ptr(), 32)
    torch.cuda.synchronize()
    steps = d_steps.cpu().numpy().astype(np.int64)
    assert (d_out.cpu().numpy() == out).all()
    order = np.sort(steps)[::-1]
    tot = int(steps.sum())
    line = {"config": "#3 nested groups (chains <= 32, cycles), global max-depth 32", "tuples": int(g.n_edges),
            "requests": len(q), "wall_ms": round(wall * 1e3, 3), "tier_ms": [round(x, 3) for x in ms],
            "tier_requests": [int(x) for x in cnt], "kernel": snap.check_kernel_name(32),
            "items": {"ms": round(full["items_ms"], 3), "work_requests": full["items"], "kept": full["items_kept"],
                      "env": {k: v for k, v in os.environ.items() if k.startswith("KETO_")}},
            "steps": {"total": tot, "mean": round(float(steps.mean()), 2), "p50": int(np.percentile(steps, 50)),
                      "p99": int(np.percentile(steps, 99)), "p999": int(np.percentile(steps, 99.9)),
                      "max": int(order[0]), "top10": [int(x) for x in order[:10]],
                      "share_of_steps_in_top_100_requests": round(float(order[:100].sum()) / max(1, tot), 4),
                      "share_of_steps_in_top_1pct": round(float(order[:len(q) // 100].sum()) / max(1, tot), 4),
                      "histogram": hist(steps)},
            "by_request_depth": {}}
    for d in (5, 16, 32):
        m = q["max_depth"] == d
        s = steps[m]
        line["by_request_depth"][str(d)] = {"requests": int(m.sum()), "mean": round(float(s.mean()), 2),
                                            "p99": int(np.percentile(s, 99)), "max": int(s.max()),
                                            "allowed": round(float(out[m].mean()), 4)}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
