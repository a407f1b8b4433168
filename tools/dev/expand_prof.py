"""Config #5 expand (100k roots on the nested-groups 100M graph, max-depth 5) repeated, for kernel
traces and PMC passes: python tools/dev/expand_prof.py [--reps N] [--roots N]  (KETO_EXPAND_TRACE=1
prints the phase times).  Dev tooling, not part of the product."""
import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--roots", type=int, default=100_000)
    ap.add_argument("--check", type=int, default=0, help="trees compared with the C oracle")
    ap.add_argument("--scale", type=int, default=0, help="the graph at 1/2^k size (same degrees): footprint study")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from tools import synth
    t0 = time.time()
    prm = dict(synth.NESTED_100M)
    for k in ("n_groups", "n_users", "target_edges"):
        prm[k] >>= a.scale
    g = synth.SynthGraph(prm, threads=16, kind="nested", chain=32)
    snap = g.snapshot(device=0)
    print(f"graph + upload {time.time() - t0:.1f} s", flush=True)
    rng = np.random.default_rng(5)
    rows = rng.integers(0, g.n_rows, size=a.roots).astype(np.uint32)
    roots = rows | np.uint32(0x80000000)
    depths = np.zeros(a.roots, dtype=np.int32)
    lib = snap.lib
    walls, kms = [], []
    for _ in range(a.reps):
        ar = C.c_void_p()
        t = time.perf_counter()
        assert lib.keto_expand_batch_ids(snap.h, roots.ctypes.data_as(C.c_void_p), depths.ctypes.data_as(C.c_void_p),
                                         C.c_uint32(a.roots), C.c_int32(5), C.byref(ar)) == 0
        walls.append((time.perf_counter() - t) * 1e3)
        kms.append(snap.last_timing()[0][0])
        lib.keto_tree_arena_free(ar)
    print(f"wall ms {np.round(walls, 3).tolist()}", flush=True)
    print(f"tier0+copies ms {np.round(kms, 3).tolist()}", flush=True)
    if a.check:
        from tests.test_gpu_config4_full import ORA_NODE  # noqa: F401 (dtype of the oracle's nodes)
        from tests.test_gpu_synth import _oracle_expand_nodes
        k = a.check
        status, offs, nodes = snap.expand_batch_ids(roots[:k], depths[:k], 5)
        q = np.zeros(k, dtype=[("row", "<u4"), ("target", "<u4"), ("flags", "<u4"), ("max_depth", "<i4")])
        q["row"] = rows[:k]
        tab = g.oracle_table(q, 5)
        bad = 0
        for i in range(k):
            r, want = _oracle_expand_nodes(g, tab, int(rows[i]), 5, 5)
            have = []
            for subj, info in nodes[offs[i]:offs[i + 1]]:
                leaf, nc = int(info >> 31), int(info & 0x7FFFFFFF)
                if subj >> 31:
                    t_ = int(subj & 0x7FFFFFFF)
                    have.append((leaf, 1, 0, 0xFFFF0000 + int(g.row_ns[t_]), int(g.row_obj[t_]), int(g.row_rel[t_]), nc))
                else:
                    have.append((leaf, 0, int(subj), 0, 0, 0, nc))
            bad += (r == 1) != (status[i] == 0) or (r == 1 and have != want)
        print(f"checked {k} trees: {bad} different", flush=True)
    snap.close()
    g.close()


if __name__ == "__main__":
    main()
