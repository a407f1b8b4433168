"""Shape of config #5's trees (100k roots on the #3 graph, max-depth 5), for sizing a wave-style
expand: per tree the set nodes (one DFS step each: a visited test and, when new, a header load),
the union nodes (rows opened) and the leaf ids (copied in runs).  The lane-per-tree kernel's time is
set by the longest serial chain, so the tail of `steps` matters, not the mean.

    python tools/dev/expand_shape.py [--roots 100000] [--threads 16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--roots", type=int, default=100_000)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    from tools import synth
    t0 = time.time()
    g = synth.SynthGraph(dict(synth.NESTED_100M), threads=a.threads, kind="nested", chain=32)
    snap = g.snapshot(device=0)
    print(f"graph + upload {time.time() - t0:.1f} s", flush=True)
    rng = np.random.default_rng(5)                 # the roots bench_configs.config5 uses
    rows = rng.integers(0, g.n_rows, size=a.roots).astype(np.uint32)
    roots = rows | np.uint32(0x80000000)
    depths = np.zeros(a.roots, dtype=np.int32)
    status, offs, nodes = snap.expand_batch_ids(roots, depths, 5)
    subj, info = nodes[:, 0], nodes[:, 1]
    is_set = (subj >> 31).astype(np.int64)
    is_union = ((info >> 31) == 0).astype(np.int64)
    cs = np.concatenate([[0], np.cumsum(is_set)])
    cu = np.concatenate([[0], np.cumsum(is_union)])
    o = offs.astype(np.int64)
    sets = cs[o[1:]] - cs[o[:-1]]
    unions = cu[o[1:]] - cu[o[:-1]]
    total = o[1:] - o[:-1]
    steps = sets + unions
    pct = [50, 90, 99, 99.9, 100]

    def dist(x):
        return {str(p): float(np.percentile(x, p)) for p in pct} | {"mean": float(x.mean()), "sum": int(x.sum())}

    top = np.argsort(steps)[-10:][::-1]
    out = {"roots": a.roots, "status": {str(k): int(v) for k, v in zip(*np.unique(status, return_counts=True))},
           "nodes": dist(total), "set_nodes": dist(sets), "unions": dist(unions), "steps": dist(steps),
           "steps_hist_log2": np.bincount(np.log2(np.maximum(steps, 1)).astype(int)).tolist(),
           "top10": [{"root": int(rows[i]), "steps": int(steps[i]), "nodes": int(total[i]),
                      "unions": int(unions[i])} for i in top]}
    # the steps of the trees above each threshold (work a wave-per-tree kernel would take over)
    for th in (64, 256, 1024):
        m = steps > th
        out[f"over_{th}"] = {"trees": int(m.sum()), "steps": int(steps[m].sum())}
    for _ in range(3):
        snap.expand_batch_ids(roots, depths, 5)
    ms, _ = snap.last_timing()
    out["kernel_ms"] = round(float(sum(ms)), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
