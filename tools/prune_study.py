"""Study: how many row visits of the reference DFS a per-row *closure* bloom filter would prune.

Pruning a subject set C whose reachable closure cannot contain the requested id keeps every answer
(the nodes it leaves unmarked are all inside closure(C), which never reaches the target), so the
question is only how often a B-bit filter of closure ids rejects.  Runs on the synthetic power-law
graph at reduced scale; prints header visits per check with and without pruning.

    python tools/prune_study.py --scale 0.015625 --queries 4000
"""
import argparse
import sys
import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools import synth  # noqa: E402

SET = np.uint32(0x80000000)


def hash_bits(ids, nbits, k, seed=0):
    """[n, W] u64 words with k bits set per id."""
    W = (nbits + 63) // 64
    out = np.zeros((len(ids), W), dtype=np.uint64)
    x = ids.astype(np.uint64)
    rows = np.arange(len(ids))
    for j in range(k):
        h = (x * np.uint64(0x9E3779B97F4A7C15 + 2 * j + 1 + 2 * 1000003 * seed)) & np.uint64(0xFFFFFFFFFFFFFFFF)
        h = (h >> np.uint64(40)) % np.uint64(nbits)
        np.bitwise_or.at(out, (rows, (h >> np.uint64(6)).astype(np.int64)), np.uint64(1) << (h & np.uint64(63)))
    return out


def closure_blooms(g, nbits, k, iters=64, seed=0):
    R = g.n_rows
    ptr = g.row_ptr.astype(np.int64)
    e = g.edges
    is_set = (e & SET) != 0
    row_of_edge = np.repeat(np.arange(R, dtype=np.int64), np.diff(ptr))
    own = np.zeros((R, (nbits + 63) // 64), dtype=np.uint64)
    ib = hash_bits(e[~is_set], nbits, k, seed)
    np.bitwise_or.at(own, row_of_edge[~is_set], ib)
    src = row_of_edge[is_set]
    dst = (e[is_set] & np.uint32(0x7FFFFFFF)).astype(np.int64)
    order = np.argsort(src, kind="stable")
    src, dst = src[order], dst[order]
    bl = own.copy()
    starts = np.flatnonzero(np.r_[True, src[1:] != src[:-1]]) if len(src) else np.zeros(0, dtype=np.int64)
    rows_with = src[starts] if len(src) else np.zeros(0, dtype=np.int64)
    for it in range(iters):
        child = bl[dst]
        red = np.bitwise_or.reduceat(child, starts, axis=0) if len(src) else child
        new = bl.copy()
        new[rows_with] |= red
        if (new == bl).all():
            print(f"  closure converged after {it} iterations", flush=True)
            break
        bl = new
    return own, bl


def dfs(g, row, target, depth, bloom, tbits, stats, top_prune=True, ext=None):
    """Reference check for one top-level row (engine.go:36-123), counting row visits."""
    ptr, e = g.row_ptr, g.edges
    visited = set()

    def further(r, rest):
        if rest <= 0:
            return False
        stats["hdr"] += 1
        if bloom is not None and (top_prune or rest < depth) and ((bloom[r] & tbits) != tbits).any():
            stats["pruned"] += 1
            return False
        if ext is not None and (top_prune or rest < depth) and ext[2][r]:
            stats["ext"] += 1                     # second line: the row's large filter
            if ((ext[0][r] & ext[1]) != ext[1]).any():
                stats["pruned2"] += 1
                return False
        stats["lines"] += 1 + max(0, (int(ptr[r + 1] - ptr[r]) - 4 + 31) // 32)
        for x in e[ptr[r]:ptr[r + 1]]:
            x = int(x)
            if x in visited:
                continue
            visited.add(x)
            if x == target:
                return True
            if x & 0x80000000:
                if further(x & 0x7FFFFFFF, rest - 1):
                    return True
        return False

    return further(row, depth)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1 / 64)
    ap.add_argument("--queries", type=int, default=4000)
    ap.add_argument("--bits", type=int, nargs="*", default=[51, 64])
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--no-top", action="store_true", help="prune only below the top-level row")
    ap.add_argument("--second", type=int, default=0, help="bits of a second, larger filter (0 = none)")
    ap.add_argument("--tau", type=float, nargs="*", default=[0.5],
                    help="rows whose first filter is fuller than this get the second one")
    a = ap.parse_args()
    sys.setrecursionlimit(10000)
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, a.scale), threads=8)
    print(f"rows {g.n_rows} edges {g.n_edges} set edges {g.n_set_edges}", flush=True)
    q = g.queries(a.queries, seed=7, depth=5)
    base = dict(hdr=0, pruned=0, lines=0)
    ans0 = [dfs(g, int(r["row"]), int(r["target"]), 5, None, 0, base) for r in q]
    n = len(q)
    print(f"no pruning: {base['hdr'] / n:.2f} row visits/check, {base['lines'] / n:.2f} row lines/check, "
          f"allowed {np.mean(ans0):.3f}", flush=True)
    for nb in a.bits:
        own, bl = closure_blooms(g, nb, a.k)
        fill = np.unpackbits(bl[:200000].view(np.uint8), axis=1).sum(axis=1) / nb
        tb = hash_bits(q["target"], nb, a.k)
        st = dict(hdr=0, pruned=0, lines=0)
        ans = [dfs(g, int(r["row"]), int(r["target"]), 5, bl, t, st, not a.no_top) for r, t in zip(q, tb)]
        assert ans == ans0, "pruning changed an answer"
        print(f"closure bloom {nb} bits k={a.k}: fill mean {fill.mean():.2f}; {st['hdr'] / n:.2f} row visits/check "
              f"({st['pruned'] / n:.2f} pruned), {st['lines'] / n:.2f} row lines/check", flush=True)
        if a.second:
            _, bl2 = closure_blooms(g, a.second, 1, seed=1)
            tb2 = hash_bits(q["target"], a.second, 1, seed=1)
            fill_all = np.unpackbits(bl.view(np.uint8), axis=1).sum(axis=1) / nb
            for tau in a.tau:
                has = fill_all > tau
                st2 = dict(hdr=0, pruned=0, lines=0, ext=0, pruned2=0)
                ans2 = [dfs(g, int(r["row"]), int(r["target"]), 5, bl, t, st2, not a.no_top, (bl2, t2, has))
                        for r, t, t2 in zip(q, tb, tb2)]
                assert ans2 == ans0, "two-level pruning changed an answer"
                print(f"  + {a.second}-bit second filter on rows fuller than {tau} ({has.mean():.3f} of rows): "
                      f"{st2['hdr'] / n:.2f} visits + {st2['ext'] / n:.2f} second-filter loads "
                      f"({st2['pruned2'] / n:.2f} pruned by it), {st2['lines'] / n:.2f} row lines/check", flush=True)


if __name__ == "__main__":
    main()
