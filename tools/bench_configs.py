"""BASELINE.json configs #1, #2, #3 and #5 on one MI355X (config #4 is bench.py's headline line).

Each config prints one JSON line: GPU throughput with inputs resident in HBM (tier timings from the
engine's HIP events), the bit-exactness of a sample against the oracle, and the CPU reference
restatement timed on the same sample and host cores.

  #1 cat-videos: the reference's contrib/cat-videos-example tuples (7), 10,000 seeded checks;
     CPU: the SQL-level restatement of the reference engine over in-memory SQLite (ref-sql) and
     the C restatement; GPU: the same 10,000 checks.
  #2 Drive-like: SURVEY.md 8(d)'s files / folder-forest (fan-out 8, depth <= 6) / Zipf(1.1) groups
     generator at exactly 10,000,000 tuples (seed 2), 1,000,000 files:d#view@u checks (half along
     real paths), max-depth 5.
  #3 nested groups: chains of up to 32 nested groups with back-edges (cycles), 100M tuples,
     1,000,000 checks with request depths {5, 16, 32}, global max-depth 32.
  #5 expand: 100,000 roots sampled from #3's rows, global max-depth 5; trees/s for count + fill
     passes, the roofline of both passes' kernels (SURVEY 8(d) B_expand), every tree encoded as an
     acl.SubjectTree protobuf (keto_tree_proto_all), and 5,000 trees compared node by node
     (pre-order, child order included) with the oracle.

  python tools/bench_configs.py [--configs 1,2,3,5] [--threads 16]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(msg):
    print(f"[configs {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def timed_checks(snap, qd, n, gmd, reps=3):
    import torch
    d_q = torch.from_numpy(qd.view(np.uint8)).to("cuda:0")
    d_out = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    sp = torch.cuda.current_stream().cuda_stream
    snap.check_batch_device(d_q.data_ptr(), n, d_out.data_ptr(), gmd, sp)   # warm-up: workspaces, code objects
    torch.cuda.synchronize()
    timed_checks.index_ms = round(snap.last_timing_full()["index_ms"], 1)
    best, tiers = None, None
    for r in range(reps):
        log(f"  timed run {r + 1}/{reps} of {n} checks")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        snap.check_batch_device(d_q.data_ptr(), n, d_out.data_ptr(), gmd, sp)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ms, cnt = snap.last_timing()
        full = snap.last_timing_full()
        if best is None or dt < best:
            best, tiers = dt, (ms, cnt)
            timed_checks.items = {"items_ms": round(full["items_ms"], 3), "work_requests": full["items"],
                                  "kept": full["items_kept"], "index_ms_first_batch": timed_checks.index_ms}
    return best, tiers, d_out.cpu().numpy()


timed_checks.items = None
timed_checks.index_ms = 0


def config1(a):
    from keto_amd.capi import Snapshot
    from oracle.oracle_sql import CheckEngine, RelationTuple, SQLStore, SubjectID, SubjectSet
    from tests.engine_util import rows_from_tuples
    from tests.golden_util import case_namespaces, case_tuples, load_cases
    case = next(c for c in load_cases() if c["name"] == "contrib/cat-videos-example")
    ns = case_namespaces(case)
    tuples = case_tuples(case)
    rng = np.random.default_rng(1)
    users = [("id", "*"), ("id", "cat lady"), ("id", "dog guy"), ("set", "videos", "/cats", "owner")]
    objs = ["/cats", "/cats/1.mp4", "/cats/2.mp4"]
    rels = ["owner", "view"]
    reqs = [("videos", objs[rng.integers(3)], rels[rng.integers(2)], users[rng.integers(4)], int(rng.integers(4)))
            for _ in range(10_000)]
    store = SQLStore(ns, tuples)
    eng = CheckEngine(store, 5)
    t0 = time.perf_counter()
    ref = []
    for (n_, o, r, u, d) in reqs:
        sub = SubjectID(u[1]) if u[0] == "id" else SubjectSet(*u[1:])
        ref.append(eng.subject_is_allowed(RelationTuple(n_, o, r, sub), d))
    t_sql = time.perf_counter() - t0
    # the same requests with one worker process per core (oracle/sql_bench.py, as bench.py's ref_sql)
    import json as _json
    import subprocess
    import tempfile
    fd, db = tempfile.mkstemp(prefix="keto_c1_", suffix=".sqlite", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    os.close(fd)
    fd, rq = tempfile.mkstemp(prefix="keto_c1_", suffix=".json")
    os.close(fd)
    try:
        dst = __import__("sqlite3").connect(db)
        store.conn.commit()                   # a pending write transaction stalls the backup
        store.conn.backup(dst)
        dst.close()
        _json.dump({"namespaces": ns, "requests": [(n_, o, r, u[1] if u[0] == "id" else list(u[1:]), d)
                                                  for n_, o, r, u, d in reqs]}, open(rq, "w"))
        pr = subprocess.run([sys.executable, "-m", "oracle.sql_bench", "--db", db, "--requests", rq, "--workers",
                             str(a.threads), "--gmd", "5"], capture_output=True, text=True, cwd=ROOT, timeout=600)
        if pr.returncode != 0:
            raise RuntimeError(pr.stderr[-2000:])
        par = _json.loads(pr.stdout.strip().splitlines()[-1])
    finally:
        for f in (db, rq):
            try:
                os.remove(f)
            except OSError:
                pass
    par_mism = int(sum(int(x) != int(y) for x, y in zip(par["decisions"], ref)))
    snap = Snapshot.build(ns, rows_from_tuples(ns, tuples), device=0)
    t0 = time.perf_counter()
    allowed, _ = snap.check_batch(reqs, 5)
    t_gpu = time.perf_counter() - t0
    mism = int(sum(bool(x) != y for x, y in zip(allowed, ref)))
    return {"config": "#1 cat-videos", "tuples": len(tuples), "checks": len(reqs),
            "ref_sql": {"checks_per_s": round(len(reqs) / t_sql, 1), "cores": 1,
                        "what": "oracle/oracle_sql.py: the reference engine's recursion issuing its SQL "
                                "(ORDER BY, LIMIT 100 OFFSET, page count) against in-memory SQLite"},
            "ref_sql_parallel": {"checks_per_s": par["checks_per_s"], "cores": par["workers"],
                                 "mismatches_vs_serial": par_mism,
                                 "what": "the same, one worker process per core (oracle/sql_bench.py), each with its "
                                         "own in-memory copy of the database"},
            "gpu_host_api": {"checks_per_s": round(len(reqs) / t_gpu, 1),
                             "what": "keto_check_batch with string requests (resolution + H2D + kernel + D2H)"},
            "mismatches": mism}


WORK_KEYS = ("rows", "set_edges", "id_words", "vprobes", "vinserts", "items", "L_req", "L_hdr", "L_edge",
             "L_idtab", "L_idsearch", "push", "pop", "leaf", "leaf_miss", "pruned")


def work_counters(snap, qd, n, gmd):
    """Per-check traversal counters of the same batch (instrumented kernels, all tiers)."""
    import torch
    d_q = torch.from_numpy(qd.view(np.uint8)).to("cuda:0")
    d_out = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    w = snap.check_work_device(d_q.data_ptr(), n, d_out.data_ptr(), gmd)
    return {k: round(v / n, 3) for k, v in zip(WORK_KEYS, w)}


HBM_PEAK_GBS = 8000.0


def roofline(tab, reqs, gmd, n_price, n, kernel_ms, threads):
    """SURVEY.md 8(d) roofline of the tier-0 kernel: B_check(q) = 14 + sum over the BFS rows
    (8 + 4 deg) from the oracle's BFS-count mode on the first n_price requests, scaled to the n of
    the launch, over the kernel's HIP-event time."""
    from oracle.oracle_c import OracleTable
    t0 = time.perf_counter()
    bq = tab.bfs_bytes_reqs(OracleTable.prefix(reqs, n_price), gmd, threads=threads)
    per = float(bq.mean())
    ach = per * n / (kernel_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "kernel_ms": round(kernel_ms, 4),
            "alg_bytes_per_check": round(per, 1),
            "alg_bytes_sample": f"B_check over the first {n_price} requests ({time.perf_counter() - t0:.1f} s)"}


def checks_config(a, name, g, q, gmd, sample, reps=3, price=20000):
    log(f"{name}: {g.n_edges} tuples; snapshot")
    snap = g.snapshot(device=0)
    qd = snap.with_handles(q)
    n = len(q)
    dt, (ms, cnt), out = timed_checks(snap, qd, n, gmd, reps)
    work = work_counters(snap, qd, n, gmd) if a.work else None
    if a.no_parity:
        return {"config": name, "tuples": int(g.n_edges), "rows": int(g.n_rows), "checks": n,
                "gpu": {"checks_per_s": round(n / dt, 1), "wall_ms": round(dt * 1e3, 3),
                        "tier_ms": [round(x, 3) for x in ms], "tier_requests": [int(x) for x in cnt]},
                "work": work}
    s = q[:sample]
    log(f"{name}: oracle table over {sample} requests")
    tab = g.oracle_table(s, gmd)
    reqs = g.oracle_requests(tab, s)
    t0 = time.perf_counter()
    ref = tab.check_batch_reqs(reqs, gmd, threads=a.threads)
    t_cpu = time.perf_counter() - t0
    items = timed_checks.items if timed_checks.items and timed_checks.items["work_requests"] else None
    # deep batches: the batch's device time (items split + pretest, then the work requests' tiers)
    roof = roofline(tab, reqs, gmd, min(price, sample), n, sum(ms) + items["items_ms"] if items else ms[0], a.threads)
    roof["kernel"] = snap.check_kernel_name(gmd)
    if items:
        roof["kernel"] = "reach split + pretest, then " + roof["kernel"] + " tiers over the kept work requests"
    return {"config": name, "roofline": roof, "tuples": int(g.n_edges), "rows": int(g.n_rows), "checks": n, "global_max_depth": gmd,
            "gpu": {"checks_per_s": round(n / dt, 1), "wall_ms": round(dt * 1e3, 3),
                    "tier_ms": [round(x, 3) for x in ms], "tier_requests": [int(x) for x in cnt],
                    "kernel": snap.check_kernel_name(gmd), "items": items},
            "work": work,
            "allowed_fraction": round(float(out.mean()), 4),
            "parity": {"sample": sample, "mismatches": int((ref != out[:sample]).sum())},
            "cpu_port": {"checks_per_s": round(sample / t_cpu, 1), "cores": a.threads,
                         "what": f"oracle/keto_oracle.c over the {tab.t.n} tuples the sample can reach"}}


def config2(a):
    from tools import synth
    g = synth.SynthGraph(dict(synth.DRIVE_10M), threads=a.threads, kind="drive")
    q = g.queries(1_000_000, seed=2, depth=5, threads=a.threads)
    return checks_config(a, "#2 Drive-like (files / 8-ary folder forest depth <= 6 / Zipf(1.1) groups, 10M tuples)",
                         g, q, 5, 200_000)


def config3(a):
    from tools import synth
    g = synth.SynthGraph(dict(synth.NESTED_100M), threads=a.threads, kind="nested", chain=32)
    q = g.queries_nested(1_000_000, seed=3, depths=(5, 16, 32), threads=a.threads)
    return checks_config(a, "#3 nested groups (chains <= 32, cycles)", g, q, 32, 20_000, reps=a.reps3, price=2000), g


def expand_bytes(g, tree):
    """SURVEY.md 8(d) B_expand of one tree: 12 + sum over the rows it expands (8 + 4 deg) + 9 per
    tree node.  A set node is an expanded row when it has children or is an empty row.  `tree` is
    the engine's node list of a tree found identical to the oracle's: (subject, info) with set
    subjects as bit31 | row id."""
    deg = np.diff(g.row_ptr)
    b = 12 + 9 * len(tree)
    for subj, info in tree:
        if not (int(subj) >> 31):
            continue
        r = int(subj) & 0x7FFFFFFF
        leaf, nc = int(info) >> 31, int(info) & 0x7FFFFFFF
        if nc > 0 or (leaf and deg[r] == 0):
            b += 8 + 4 * int(deg[r])
    return b


def config5(a, g=None):
    from tools import synth
    from keto_amd.capi import load
    if g is None:
        g = synth.SynthGraph(dict(synth.NESTED_100M), threads=a.threads, kind="nested", chain=32)
    snap = g.snapshot(device=0)
    rng = np.random.default_rng(5)
    n = 100_000
    rows = rng.integers(0, g.n_rows, size=n).astype(np.uint32)
    roots = rows | np.uint32(0x80000000)
    depths = np.zeros(n, dtype=np.int32)          # request depth 0 -> global max-depth 5
    lib = load()
    best, kern = None, None
    for _ in range(3):
        arena = C.c_void_p()
        t0 = time.perf_counter()
        rc = lib.keto_expand_batch_ids(snap.h, roots.ctypes.data_as(C.c_void_p), depths.ctypes.data_as(C.c_void_p),
                                       C.c_uint32(n), C.c_int32(5), C.byref(arena))
        dt = time.perf_counter() - t0
        assert rc == 0
        lib.keto_tree_arena_free(arena)
        ms, _ = snap.last_timing()
        if best is None or dt < best:
            best, kern = dt, sum(ms)
    # every tree as a SubjectTree proto (keto_tree_proto_all, host threads)
    _st, poffs, blob, _te, t_proto = snap.expand_batch_ids_proto(roots, depths, 5)
    # the same on the GPU (keto_tree_proto_all_device: strings resident on the device), best of 3,
    # byte-compared with the host encoder's buffer
    t_dev, dev_equal = None, None
    for _ in range(3):
        _sd, doffs, dblob, _td, t = snap.expand_batch_ids_proto(roots, depths, 5, device=True)
        dev_equal = dblob == blob and bool((doffs == poffs).all())
        t_dev = t if t_dev is None else min(t_dev, t)
    # the device encoder writing into a pinned caller buffer (keto_host_alloc): one DMA, best of 3
    from keto_amd.capi import HostBuffer
    t_pin, pin_equal = None, None
    arena = C.c_void_p()
    assert lib.keto_expand_batch_ids(snap.h, roots.ctypes.data_as(C.c_void_p), depths.ctypes.data_as(C.c_void_p),
                                     C.c_uint32(n), C.c_int32(5), C.byref(arena)) == 0
    try:
        poffs2 = np.zeros(n + 1, dtype=np.uint64)
        hb = HostBuffer(max(1, len(blob)), np.uint8)
        for _ in range(3):
            t0 = time.perf_counter()
            assert lib.keto_tree_proto_all_device(snap.h, arena, None, C.c_uint64(0),
                                                  poffs2.ctypes.data_as(C.c_void_p)) == len(blob)
            got = lib.keto_tree_proto_all_device(snap.h, arena, hb.array.ctypes.data_as(C.c_void_p),
                                                 C.c_uint64(len(blob)), poffs2.ctypes.data_as(C.c_void_p))
            t = time.perf_counter() - t0
            assert got == len(blob)
            t_pin = t if t_pin is None else min(t_pin, t)
        pin_equal = hb.array[:len(blob)].tobytes() == blob and bool((poffs2 == poffs).all())
        del hb
    finally:
        lib.keto_tree_arena_free(arena)
    # every tree as JSON (keto_tree_json_all, host threads: the REST Expand bodies), best of 3
    t_json, json_bytes = None, 0
    arena = C.c_void_p()
    assert lib.keto_expand_batch_ids(snap.h, roots.ctypes.data_as(C.c_void_p), depths.ctypes.data_as(C.c_void_p),
                                     C.c_uint32(n), C.c_int32(5), C.byref(arena)) == 0
    try:
        joffs = np.zeros(n + 1, dtype=np.uint64)
        for _ in range(3):
            t0 = time.perf_counter()
            json_bytes = lib.keto_tree_json_all(snap.h, arena, None, C.c_uint64(0), joffs.ctypes.data_as(C.c_void_p))
            assert json_bytes >= 0
            jbuf = np.empty(max(1, json_bytes), dtype=np.uint8)
            got = lib.keto_tree_json_all(snap.h, arena, jbuf.ctypes.data_as(C.c_void_p), C.c_uint64(json_bytes),
                                         joffs.ctypes.data_as(C.c_void_p))
            t = time.perf_counter() - t0
            assert got == json_bytes
            t_json = t if t_json is None else min(t_json, t)
    finally:
        lib.keto_tree_arena_free(arena)
    # node-by-node comparison of a sample of trees with the oracle (pre-order, child order included)
    from tests.test_gpu_synth import _oracle_expand_nodes
    k = a.expand_sample
    status, offs, nodes = snap.expand_batch_ids(roots[:k], depths[:k], 5)
    q = np.zeros(k, dtype=[("row", "<u4"), ("target", "<u4"), ("flags", "<u4"), ("max_depth", "<i4")])
    q["row"] = rows[:k]
    tab = g.oracle_table(q, 5)
    bad = 0
    n_nodes = 0
    bytes_ = []
    for i in range(k):
        r, want = _oracle_expand_nodes(g, tab, int(rows[i]), 5, 5)
        if r == 0:
            bad += int(status[i] != 1)
            bytes_.append(12 + 8)
            continue
        have = []
        for subj, info in nodes[offs[i]:offs[i + 1]]:
            leaf, nc = int(info >> 31), int(info & 0x7FFFFFFF)
            if subj >> 31:
                t = int(subj & 0x7FFFFFFF)
                have.append((leaf, 1, 0, 0xFFFF0000 + int(g.row_ns[t]), int(g.row_obj[t]), int(g.row_rel[t]), nc))
            else:
                have.append((leaf, 0, int(subj), 0, 0, 0, nc))
        n_nodes += len(have)
        bad += int(have != want or status[i] != 0)
        if have == want:
            bytes_.append(expand_bytes(g, nodes[offs[i]:offs[i + 1]]))
    per = float(np.mean(bytes_))
    ach = per * n / (kern * 1e-3) / 1e9
    return {"config": "#5 expand (100k roots on the #3 graph, max-depth 5)", "tuples": int(g.n_edges), "roots": n,
            "gpu": {"trees_per_s": round(n / best, 1), "wall_ms": round(best * 1e3, 3),
                    "kernel_ms": round(kern, 3),
                    "what": "keto_expand_batch_ids: H2D roots, one pass (trees counted and staged in per-lane "
                            "regions, a tree past its region in an overflow chunk), id-run copies, host scan, gather "
                            "to offsets with set handles -> row ids on the way (split trees piece by piece), a "
                            "second pass only for trees that fit neither, D2H tree arena; kernel_ms = the passes' "
                            "tier kernels, the id-run copies, the gather and the piece copies (HIP events)"},
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 4), "kernel_ms": round(kern, 3),
                         "alg_bytes_per_root": round(per, 1),
                         "alg_bytes_sample": f"SURVEY 8(d) B_expand over the first {k} roots' trees (those equal "
                                             "to the oracle's)"},
            "proto": {"trees_per_s": round(n / t_proto, 1), "bytes": len(blob), "encode_ms": round(t_proto * 1e3, 3),
                      "MB_per_s": round(len(blob) / t_proto / 1e6, 1),
                      "what": "keto_tree_proto_all: every tree of the arena as acl.SubjectTree protobuf, 16 host threads (sizing + filling call)"},
            "proto_device": {"trees_per_s": round(n / t_dev, 1), "encode_ms": round(t_dev * 1e3, 3),
                             "MB_per_s": round(len(blob) / t_dev / 1e6, 1), "bytes_equal_host": dev_equal,
                             "what": "keto_tree_proto_all_device: the same bytes encoded on the GPU (node upload, "
                                     "sizes, scan, write, D2H into pageable numpy memory via pinned bounce chunks; device "
                                     "buffers kept across calls), sizing + filling call"},
            "proto_device_pinned": {"trees_per_s": round(n / t_pin, 1), "encode_ms": round(t_pin * 1e3, 3),
                                    "bytes_equal_host": pin_equal,
                                    "what": "keto_tree_proto_all_device into a pinned caller buffer (keto_host_alloc), sizing + "
                                            "filling call"},
            "json": {"trees_per_s": round(n / t_json, 1), "bytes": int(json_bytes), "encode_ms": round(t_json * 1e3, 3),
                     "MB_per_s": round(json_bytes / t_json / 1e6, 1),
                     "what": "keto_tree_json_all: every tree as Tree.MarshalJSON text, 16 host threads (sizing + "
                             "filling call)"},
            "parity": {"sample_trees": k, "sample_nodes": n_nodes, "mismatched_trees": bad}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3,5")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--work", action="store_true", help="add per-check traversal counters (instrumented run)")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle legs (tuning sweeps)")
    ap.add_argument("--expand-sample", type=int, default=5000, help="config #5 trees compared with the oracle")
    ap.add_argument("--reps3", type=int, default=1, help="config #3 timed batches (the best is reported)")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    want = set(a.configs.split(","))
    g3 = None
    if "1" in want:
        log("config #1")
        print(json.dumps(config1(a)), flush=True)
    if "2" in want:
        log("config #2")
        print(json.dumps(config2(a)), flush=True)
    if "3" in want:
        log("config #3")
        r, g3 = config3(a)
        print(json.dumps(r), flush=True)
    if "5" in want:
        log("config #5")
        print(json.dumps(config5(a, g3)), flush=True)


if __name__ == "__main__":
    main()
