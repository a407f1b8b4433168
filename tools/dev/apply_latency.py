"""Latency of keto_snapshot_apply on a large string-built snapshot (delta.cpp collision
scan): a write of new subject ids on existing rows, a write of a new row nothing points at, a write
whose subject-id string is an existing row's Subject.String() (a new collision class: every row's
edges are scanned for the classed values), and a write of a new subject set.  The snapshot holds its
exclusive lock for each call, so this is how long checks wait behind it.

    python tools/dev/apply_latency.py --scale 0.0625 [--device -1]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1 / 16)
    ap.add_argument("--device", type=int, default=-1, help="-1: host-only snapshot (the host half of apply)")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, a.scale), threads=a.threads)
    st = g.string_tuples(seed=5, threads=a.threads)
    t0 = time.perf_counter()
    snap, build_s = g.snapshot_from_strings(st, device=a.device)
    print(f"scale {a.scale}: {st.n} tuples, {g.n_rows} rows, build {build_s:.1f} s "
          f"(device {a.device})", flush=True)
    names = dict(g.namespaces)
    rels = g.relation_names()
    ns_ids = {n: i for i, n in g.namespaces}
    row_names = []
    for r in range(0, g.n_rows, max(1, g.n_rows // 1000)):
        row_names.append((int(g.row_ns[r]), f"{int(g.row_obj[r]):08x}", rels[int(g.row_rel[r])]))
    k = 0

    def timed(label, ins):
        nonlocal k
        ts = []
        for _ in range(a.reps):
            t = time.perf_counter()
            snap.apply(ins(), [])
            ts.append((time.perf_counter() - t) * 1e3)
            k += 1
        print(f"  {label:<52} " + " ".join(f"{x:8.1f}" for x in ts) + " ms", flush=True)

    def ids():
        return [(ns, obj, rel, f"lat-u{k}-{i}") for i, (ns, obj, rel) in enumerate(row_names[:100])]

    def new_root():
        ns, obj, rel = row_names[0]
        return [(ns, f"lat-obj-{k}", rel, "u00000001")]

    def collision():
        ns, obj, rel = row_names[(k * 7) % len(row_names)]
        other = row_names[(k * 7 + 3) % len(row_names)]
        return [(other[0], other[1], other[2], f"{names[ns]}:{obj}#{rel}")]   # an id equal to a row's String()

    def new_set():
        ns, obj, rel = row_names[(k * 5) % len(row_names)]
        other = row_names[(k * 5 + 11) % len(row_names)]
        return [(other[0], other[1], other[2], None, ns, obj, rel)]

    print("  write                                                 ms per call", flush=True)
    timed("100 new subject ids on existing rows", ids)
    timed("a new root row", new_root)
    timed("a subject id equal to a row's String() (collision)", collision)
    timed("a new subject set on an existing row", new_set)
    snap.close()
    g.close()
    del ns_ids, t0


if __name__ == "__main__":
    main()
