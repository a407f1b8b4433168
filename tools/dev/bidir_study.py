"""Dev study: how many config #3 requests a hop-bounded reachability test decides (false), and the
reference-DFS work left for the others.  See tools/dev/bidir_study.c.

  python tools/dev/bidir_study.py [--scale 1.0] [--requests 100000] [--threads 8]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "tools", "dev", "bidir_study.c")
LIB = os.path.join(ROOT, "tools", "dev", "libbidir_study.so")

RES = np.dtype([("dfs_steps", "<u8"), ("dfs_rows", "<u4"), ("allowed", "u1"), ("within", "u1"),
                ("bidir_work", "<u4"), ("par_steps", "<u8"), ("par_nocancel", "<u8"), ("worst_item", "<u8"),
                ("worst_hit", "u1"), ("par_work", "<u8"), ("n_items", "<u4"), ("n_items_within", "<u4")], align=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--requests", type=int, default=100_000)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--cap", type=int, default=1 << 26)
    a = ap.parse_args()
    subprocess.check_call(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", "-o", LIB, SRC])
    lib = C.CDLL(LIB)
    from tools import synth
    params = dict(synth.NESTED_100M) if a.scale == 1.0 else synth.scaled(synth.NESTED_100M, a.scale)
    g = synth.SynthGraph(params, threads=a.threads, kind="nested", chain=32)
    q = g.queries_nested(a.requests, seed=3, depths=(5, 16, 32), threads=a.threads)
    rc = lib.bs_init(C.c_uint64(g.n_rows), g.row_ptr.ctypes.data_as(C.c_void_p), g.edges.ctypes.data_as(C.c_void_p),
                     C.c_uint32(params["n_users"]))
    assert rc == 0
    lib.bs_cap(C.c_uint32(a.cap))
    out = np.zeros(len(q), dtype=RES)
    lib.bs_run(q.ctypes.data_as(C.c_void_p), C.c_uint64(len(q)), C.c_int(32), out.ctypes.data_as(C.c_void_p),
               C.c_int(a.threads))
    st = out["dfs_steps"].astype(np.int64)
    al = out["allowed"].astype(bool)
    wi = out["within"].astype(bool)
    assert not (al & ~wi).any(), "an allowed request without a path within D-1 hops"
    keep = wi
    line = {"scale": a.scale, "rows": int(g.n_rows), "edges": int(g.n_edges), "requests": len(q),
            "allowed": float(al.mean()), "within": float(wi.mean()),
            "dfs_steps_total": int(st.sum()), "dfs_steps_max": int(st.max()),
            "dfs_steps_kept_total": int(st[keep].sum()), "dfs_steps_kept_max": int(st[keep].max()) if keep.any() else 0,
            "bidir_work_total": int(out["bidir_work"].astype(np.int64).sum()),
            "bidir_work_max": int(out["bidir_work"].max()),
            "within_but_false": int((wi & ~al).sum())}
    for d in (5, 16, 32):
        m = q["max_depth"] == d
        line[f"d{d}"] = {"allowed": float(al[m].mean()), "within": float(wi[m].mean()),
                         "dfs_steps_total": int(st[m].sum()), "dfs_steps_kept_total": int(st[m & keep].sum()),
                         "dfs_steps_kept_max": int(st[m & keep].max()) if (m & keep).any() else 0,
                         "dfs_p99": int(np.percentile(st[m], 99)),
                         "kept_p99": int(np.percentile(st[m & keep], 99)) if (m & keep).any() else 0,
                         "bidir_p99": int(np.percentile(out["bidir_work"][m], 99)),
                         "bidir_max": int(out["bidir_work"][m].max())}
    ps = out["par_steps"].astype(np.int64)
    line["par_steps_max"] = int(ps.max())
    line["par_steps_p99"] = int(np.percentile(ps, 99))
    line["par_steps_p999"] = int(np.percentile(ps, 99.9))
    line["par_work_total"] = int(out["par_work"].astype(np.int64).sum())
    line["par_top20"] = sorted(ps.tolist())[::-1][:20]
    pn = out["par_nocancel"].astype(np.int64)
    line["nocancel_max"] = int(pn.max())
    line["nocancel_p999"] = int(np.percentile(pn, 99.9))
    ti = np.argsort(out["worst_item"])[::-1][:20]
    line["worst_items_top20"] = [[int(out["worst_item"][i]), int(out["worst_hit"][i]), int(al[i])] for i in ti]
    top = np.argsort(st)[::-1][:20]
    line["top20"] = [[int(st[i]), int(al[i]), int(wi[i]), int(q["max_depth"][i]), int(out["dfs_rows"][i])] for i in top]
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
