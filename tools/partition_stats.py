"""Edge-partitioned mode on the 1B-tuple graph (BASELINE config #4): the arena every part would
hold for P = 1, 2, 4, 8 (keto_snapshot_part_stats on a host-only snapshot; no GPU), the share of
it in rows every part keeps (rows some subject set points at: folders, groups), and the root rows
(documents) split by hash(namespace id, object).  One JSON line.

  python tools/partition_stats.py [--scale 1.0] [--threads 16]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--parts", default="1,2,4,8")
    a = ap.parse_args()
    from tools import synth
    params = dict(synth.POWERLAW_1B) if a.scale == 1.0 else synth.scaled(synth.POWERLAW_1B, a.scale)
    t0 = time.time()
    g = synth.SynthGraph(params, threads=a.threads)
    s = g.host_snapshot()
    out = {"graph": "powerlaw-acl (BASELINE config #4)", "tuples": int(g.n_edges), "rows": int(g.n_rows),
           "build_s": round(time.time() - t0, 1), "parts": {}}
    for P in [int(x) for x in a.parts.split(",")]:
        per = [s.part_stats(p, P) for p in range(P)]
        mx = max(per, key=lambda x: x["arena_bytes"])
        out["parts"][str(P)] = {
            "max_part_arena_GiB": round(mx["arena_bytes"] / 2**30, 3),
            "mean_part_arena_GiB": round(sum(x["arena_bytes"] for x in per) / P / 2**30, 3),
            "shared_GiB": round(mx["shared_bytes"] / 2**30, 3),
            "shared_fraction_of_part": round(mx["shared_bytes"] / mx["arena_bytes"], 4),
            "rows_per_part_max": max(x["rows"] for x in per), "shared_rows": per[0]["shared_rows"],
            "root_rows_per_part": [x["root_rows"] for x in per]}
    full = out["parts"].get("1")
    if full:
        for P, v in out["parts"].items():
            v["saving_vs_replicated"] = round(1 - v["max_part_arena_GiB"] / full["max_part_arena_GiB"], 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
