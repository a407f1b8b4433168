#!/usr/bin/env python3
"""Headline benchmark: batched Keto checks on the 1B-tuple power-law ACL graph at max-depth 5.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1 the driver starts one
rank per GPU with torch.distributed.run.  A step = one keto_check_batch_device call over a
resident batch of synthetic docs:d#view@u requests (16M per GPU by default).  The path shards by
request with no data-path collective: every rank holds the whole snapshot (the 1B-tuple arena is
17.2 GiB of a 288 GB HBM3E) and checks its own batch ("weak" scaling).  Rank 0 prints one JSON line.

Extras on the same line:
  roofline      SURVEY.md 8(d) algorithmic bytes of the dominant kernel (the tier-0 check kernel)
                per launch -- B_check(q) = 14 + sum over the BFS rows (8 + 4 deg), priced by the
                oracle's BFS-count mode on a 1 % sample of the batch and scaled -- divided by the
                kernel's average HIP-event duration over the timed steps (events recorded on the
                launch stream); peak = 8 TB/s HBM3E.  `traffic` = HBM bytes per launch from the
                committed rocprofv3 PMC passes of this same engine build (profiles/*_traffic.json);
                `traversal_bytes_per_launch` = what the kernel's own traversal requests.
  end_to_end    SURVEY.md 8(d) t_batch: host entry to decisions on the host (pinned 8-B row-id
                requests -> H2D -> translation -> check -> D2H, chunks pipelined by the library),
                and its frac; the 16-B row-id form alongside.
  cpu_baseline  the C restatement of the reference engine (oracle/keto_oracle.c) on the box's host
                cores over a bounded sample of the same requests; its decisions are also compared
                with the GPU's for that sample ("parity").
  ref_sql       the reference recursion issuing its own SQL against in-memory SQLite, one worker
                process per core, over the first 10,000 requests (compared with the GPU too).
  string_form   (N = 1) the same batch as named requests, packed as the Go shim packs them (every
                request's strings in one pinned blob + 24-B records) through keto_check_batch_packed,
                which the Go shim's CheckBatch calls: resolution on the GPU, then the check; the
                128-B keto_check_req form through keto_check_batch (resolution on host threads)
                alongside as host_resolution.  The snapshot then carries the graph's string table
                (tools/synth.py unified()).
Host cores: --threads defaults to the CPUs this job may use (tools/hostcpu.py: affinity mask,
cgroup quota, the harness's OMP_NUM_THREADS share), recorded with every CPU leg.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _engine_build_id():
    import importlib.util
    spec = importlib.util.spec_from_file_location("_keto_build", os.path.join(ROOT, "keto_amd", "build.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.engine_build_id()


def pmc_traffic(kernel_name, workload):
    """Per-launch HBM bytes of the dominant kernel from the committed rocprofv3 PMC passes
    (profiles/*_traffic.json, written by tools/traffic.py from tools/gpu_round.sh), used only when
    they were measured on this engine.hip, built with these flags, and this workload; else None."""
    import glob
    sha = _engine_build_id()
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        try:
            j = json.load(open(p))
        except (OSError, ValueError):
            continue
        if j.get("engine_sha256") == sha and j.get("kernel") in kernel_name and j.get("workload") == workload:
            return j["traffic_bytes"], os.path.relpath(p, ROOT)
    return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=16 * 1024 * 1024, help="checks per GPU per step")
    ap.add_argument("--scale", type=float, default=1.0, help="graph scale (1.0 = 1B tuples)")
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--threads", type=int, default=None,
                    help="host threads (generator, resolution, cpu baseline); default: the usable host CPUs")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="requests in the cpu_baseline sample")
    ap.add_argument("--sql-sample", type=int, default=10_000, help="requests in the ref_sql (SQLite) sample")
    ap.add_argument("--bytes-sample", type=float, default=0.01,
                    help="fraction of the batch priced in the oracle's BFS-count mode (roofline bytes)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--partitioned", action="store_true",
                    help="edge-partitioned snapshot (root rows split by hash(ns, object)); each step routes the "
                         "batch to the owners with RCCL all-to-all, checks, and returns the decisions")
    ap.add_argument("--part-mode", choices=["shared", "migrate"], default="shared",
                    help="--partitioned layout: shared = set targets on every part; migrate = every row on one part, "
                         "searches move between parts as records (keto_mig_*), one all-to-all per round")
    ap.add_argument("--hot-mb", type=float, default=0.0, help="--part-mode migrate: replicated hot rows per part (MB)")
    ap.add_argument("--check-parity", action="store_true",
                    help="partitioned runs: every rank also checks its batch on a replicated snapshot and the "
                         "mismatches are summed over ranks (small scales: needs the whole graph on each GPU)")
    ap.add_argument("--no-work", action="store_true", help="skip the roofline / cpu_baseline legs (profiling runs)")
    ap.add_argument("--e2e-steps", type=int, default=5,
                    help="batches timed end to end through the host API (keto_check_batch_rows, pinned buffers); 0 = skip")
    ap.add_argument("--e2e-only", action="store_true", help="time only the end-to-end leg (profiling runs)")
    ap.add_argument("--string-steps", type=int, default=3,
                    help="N = 1: batches timed through keto_check_batch with named requests (0 = skip)")
    a = ap.parse_args()
    from tools.hostcpu import host_cores
    a.host = host_cores()
    if a.threads is None:
        a.threads = a.host["usable"]
    os.environ.setdefault("KETO_BUILD_THREADS", str(a.threads))     # the library's host thread pools
    return a


def sql_leg(g, q, a, gpu_out):
    """ref-sql: oracle/oracle_sql.py (the reference check engine's recursion issuing its SELECT ...
    ORDER BY ... LIMIT 100 OFFSET and page count per node) over the tuples the sample reaches, in
    SQLite, with a.threads worker processes (oracle/sql_bench.py, started as a child process)."""
    import subprocess
    import tempfile
    k = min(a.sql_sample, len(q))
    log(f"ref_sql over {k} requests (SQLite, {a.threads} worker processes)")
    t0 = time.perf_counter()
    stab = g.oracle_table(q[:k], a.depth)
    store = g.sql_store(stab)
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else None
    fd, db = tempfile.mkstemp(prefix="keto_refsql_", suffix=".sqlite", dir=shm)
    os.close(fd)
    fd, rq = tempfile.mkstemp(prefix="keto_refsql_", suffix=".json")
    os.close(fd)
    try:
        dst = __import__("sqlite3").connect(db)
        store.conn.commit()                   # a pending write transaction stalls the backup
        store.conn.backup(dst)
        dst.close()
        store.conn.close()
        reqs = [(t.namespace, t.object, t.relation, t.subject.id, d) for t, d in g.sql_requests(q[:k])]
        json.dump({"namespaces": g.namespaces, "requests": reqs}, open(rq, "w"))
        t_setup = time.perf_counter() - t0
        r = subprocess.run([sys.executable, "-m", "oracle.sql_bench", "--db", db, "--requests", rq, "--workers",
                            str(a.threads), "--gmd", str(a.depth)], capture_output=True, text=True, cwd=ROOT,
                           timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f"oracle.sql_bench failed: {r.stderr[-2000:]}")
        res = json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        for f in (db, rq):
            try:
                os.remove(f)
            except OSError:
                pass
    dec = np.array(res["decisions"], dtype=np.uint8)
    return {"value": res["checks_per_s"], "unit": "checks/s", "cores": res["workers"],
            "mismatches_vs_gpu": int((dec != gpu_out[:k]).sum()),
            "host": {**a.host, "workers_used": res["workers"]},
            "sample": f"first {k} requests; oracle/oracle_sql.py (the reference check engine's recursion issuing "
                      f"its SELECT ... ORDER BY ... LIMIT 100 OFFSET and page count per node) over the {stab.t.n} "
                      f"tuples they reach, in-memory SQLite copies of one image in each of {res['workers']} "
                      f"worker processes (setup {t_setup:.1f} s, slowest worker {res['slowest_worker_s']:.2f} s)"}


def end_to_end(snap, q, a, d_out):
    """SURVEY.md 8(d) t_batch: host entry to decisions on the host, for the same batch through
    keto_check_batch_rows -- requests by row id in pinned host memory (keto_host_alloc), H2D,
    row id -> handle translation on the device, the check, D2H, pipelined in chunks."""
    from keto_amd.capi import CHECK_IDS_DTYPE, CHECK_PAIR_DTYPE, HostBuffer, pairs_of
    n = len(q)
    if not (q["max_depth"] == q["max_depth"][0]).all():
        raise ValueError("the pair form needs one request depth per batch")
    legs = {}
    outs = []
    for form, dt, size in (("pairs", CHECK_PAIR_DTYPE, 8), ("rows", CHECK_IDS_DTYPE, 16)):
        hq, ho = HostBuffer(n, dt), HostBuffer(n, np.uint8)
        hq.array[:] = pairs_of(q) if form == "pairs" else q
        if form == "pairs":
            call = lambda: snap.check_batch_pairs(hq.array, int(q["max_depth"][0]), a.depth, out=ho.array)
        else:
            call = lambda: snap.check_batch_rows(hq.array, a.depth, out=ho.array)
        log(f"end-to-end leg ({form}): {a.e2e_steps} batches of {n} through the host API (pinned buffers)")
        call()                                                     # warm-up (slots, staging)
        ts, walls, tiers = [], [], []
        streamed = stalls = fallbacks = 0
        for _ in range(a.e2e_steps):
            t0 = time.perf_counter()
            call()
            ts.append(time.perf_counter() - t0)
            t = snap.last_timing_full()
            walls.append(t["wall_ms"])
            tiers.append(t["tier_ms"][0])
            streamed += t["streamed"]
            stalls += t["stream_stalls"]
            fallbacks += t["stream_fallbacks"]
        ms = float(np.median(ts)) * 1e3
        pcie = n * (size + 1)
        legs[form] = {"value": round(n / (ms * 1e-3), 1), "unit": "checks/s", "ms_per_batch": round(ms, 3),
                      "library_wall_ms": round(float(np.median(walls)), 3),
                      "tier0_ms_sum": round(float(np.median(tiers)), 3), "chunks": t["chunks"],
                      "request_bytes": size, "pcie_bytes_per_batch": pcie,
                      "pcie_GBps": round(pcie / (ms * 1e-3) / 1e9, 1),
                      # over the timed batches: decided by the one streamed launch; lanes whose chunk
                      # wait hit KETO_STREAM_WAIT_MS; batches that fell back to the chunked pipeline
                      "streamed_batches": streamed, "stream_wait_timeouts": stalls, "stream_fallbacks": fallbacks}
        outs.append(ho.array.copy())
    best = legs["pairs"]
    return {**best, "form": "keto_check_batch_pairs (8-B row-id requests, batch depth)", "rows_form": legs["rows"],
            "what": "host entry to decisions on the host: requests by row id in pinned host memory -> H2D -> "
                    "device row-id translation -> check -> 1-B decisions D2H, chunks pipelined over copy / compute "
                    "streams; median of the timed batches", "_out": outs}


def string_form(g, u, snap, q, a):
    """keto_check_batch on the batch as named requests (strings in C memory, built by the
    generator from the same request ids): resolution on host threads, then the device pipeline."""
    n = len(q)
    log(f"string-form leg: {a.string_steps} batches of {n} named requests through keto_check_batch")
    t0 = time.perf_counter()
    reqs = g.string_requests(u.names, q, threads=a.threads)
    t_make = time.perf_counter() - t0
    t0 = time.perf_counter()
    out, st = snap.check_batch_reqs(reqs, n, a.depth)               # warm-up: builds the string / row indexes
    t_first = time.perf_counter() - t0
    ts, res, walls = [], [], []
    for _ in range(a.string_steps):
        t0 = time.perf_counter()
        out, st = snap.check_batch_reqs(reqs, n, a.depth)
        ts.append(time.perf_counter() - t0)
        t = snap.last_timing_full()
        res.append(t["resolve_ms"])
        walls.append(t["wall_ms"])
    ms = float(np.median(ts)) * 1e3
    # the same requests packed (every request's strings back to back in one pinned blob, 24-B records:
    # the Go batcher's C arena) and resolved on the GPU: keto_check_batch_packed
    t0 = time.perf_counter()
    blob, rec, used = g.pack_requests(reqs, n, threads=a.threads)
    t_pack = time.perf_counter() - t0
    hb = blob.array[:used]
    pa, ps_ = np.zeros(n, dtype=np.uint8), np.zeros(n, dtype=np.uint8)
    t0 = time.perf_counter()
    snap.check_batch_packed(hb, rec.array, a.depth, n=n, allowed=pa, status=ps_)     # warm-up: uploads the indexes
    t_pfirst = time.perf_counter() - t0
    pts = []
    for _ in range(a.string_steps):
        t0 = time.perf_counter()
        snap.check_batch_packed(hb, rec.array, a.depth, n=n, allowed=pa, status=ps_)
        pts.append(time.perf_counter() - t0)
    pms = float(np.median(pts)) * 1e3
    host = {"value": round(n / (ms * 1e-3), 1), "unit": "checks/s", "ms_per_batch": round(ms, 3),
            "resolve_ms": round(float(np.median(res)), 3), "device_wall_ms": round(float(np.median(walls)), 3),
            "threads": a.threads, "first_call_ms": round(t_first * 1e3, 1), "request_build_s": round(t_make, 2),
            "statuses_not_ok": int((st != 0).sum()),
            "what": "keto_check_batch: 128-B keto_check_req with namespace / object / relation / subject-id strings "
                    "in C memory -> name resolution on host threads (hashed string and row indexes) -> pipelined H2D "
                    "/ check / D2H; median of the timed batches; first_call_ms includes building the indexes",
            "_out": out.copy()}
    return {"value": round(n / (pms * 1e-3), 1), "unit": "checks/s", "ms_per_batch": round(pms, 3),
            "form": "keto_check_batch_packed (what the Go shim's gpu.Snapshot.CheckBatch calls)",
            "blob_bytes": int(used), "record_bytes": int(rec.array.nbytes), "pack_s": round(t_pack, 2),
            "first_call_ms": round(t_pfirst * 1e3, 1), "statuses_equal_host": bool((ps_ == st).all()),
            "decisions_equal_host": bool((pa == out).all()), "strings_in_snapshot": int(u.n_strings),
            "what": "the batch's strings back to back in one pinned blob + 24-B records (offset, six lengths, kind, "
                    "depth), as the Go batcher packs them -> H2D -> every request resolved on the GPU against the "
                    "snapshot's string / row indexes (uploaded once per version) -> check -> D2H; median of the timed "
                    "batches; first_call_ms includes the index upload; pack_s (the packing, untimed like the "
                    "request structs of host_resolution) for reference",
            "host_resolution": host, "_out": pa.copy()}


def rusage():
    import resource
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_maxrss / 1e6, r.ru_utime + r.ru_stime          # GB (ru_maxrss is in KB), CPU seconds


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU over RCCL; KETO_BENCH_BACKEND=gloo (rehearsal: several ranks sharing the
    # GPUs of a smaller box, the rank's device = LOCAL_RANK modulo the devices) -- never the driver's run
    backend = os.environ.get("KETO_BENCH_BACKEND", "nccl")
    if world > 1:
        local = local % max(1, torch.cuda.device_count()) if backend != "nccl" else local
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    from tools import synth

    params = synth.scaled(synth.POWERLAW_1B, a.scale) if a.scale != 1.0 else dict(synth.POWERLAW_1B)
    log(f"rank {rank}/{world}: generating the graph (scale {a.scale})")
    t0 = time.time()
    g = synth.SynthGraph(params, threads=a.threads)
    t_gen = time.time() - t0
    log(f"rank {rank}: {g.n_edges} tuples, {g.n_rows} rows; building + uploading the snapshot")
    t0 = time.time()
    migrate = a.partitioned and a.part_mode == "migrate"
    unified = None
    # collectives of the partitioned modes: on the GPU with RCCL, staged through the host with gloo
    comm = f"cuda:{dev}" if backend == "nccl" else "cpu"
    if migrate:
        from keto_amd.capi import PART_MIGRATE
        from keto_amd.multi import close_filters_dist
        snap = g.snapshot_part(rank, world, dev, mode=PART_MIGRATE, hot_bytes=int(a.hot_mb * 1e6))
        if world > 1:
            rounds = close_filters_dist(snap, device=comm)
            log(f"rank {rank}: closure filters exchanged in {rounds} rounds")
        else:
            snap.part_closure_done(True)
    else:
        if a.partitioned:
            snap = g.snapshot_part(rank, world, dev)
        elif world == 1 and a.string_steps > 0:
            # one string id space and the string table in the snapshot, for the string-form leg
            unified = g.unified(threads=a.threads)
            snap = g.snapshot_unified(unified, device=dev)
        else:
            snap = g.snapshot(device=dev)
    t_snap = time.time() - t0
    q = g.queries(a.batch, seed=1000 + rank, depth=a.depth, threads=a.threads)
    q_gen = q                                           # generator ids: the oracle legs' requests
    if not migrate and not a.partitioned and unified is not None:
        q = unified.to_device_targets(q)                # the snapshot's subject-id space
    d_out = torch.empty(a.batch, dtype=torch.uint8, device=f"cuda:{dev}")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    if a.partitioned:
        from keto_amd.multi import route_device, send_back
        # requests travel as row ids; the owner table routes them (root rows to their part)
        d_q = torch.from_numpy(q.view(np.int32).reshape(-1, 4).copy()).to(f"cuda:{dev}")
        owner_dev = torch.from_numpy(snap.row_owner(np.arange(g.n_rows, dtype=np.uint32), world).astype(np.int16)
                                     ).to(f"cuda:{dev}")
        routed = [0, None, 0]
        if migrate:
            from keto_amd.multi import SnapshotMigEngine, mig_check
            engine = SnapshotMigEngine(snap, f"cuda:{dev}")

        def step():
            recv, state = route_device(d_q, owner_dev, rank, world, comm_device=comm)
            if migrate:
                dec, routed[2] = mig_check(engine, recv, a.depth, device=f"cuda:{dev}", comm_device=comm)
            else:
                dec = torch.empty(len(recv), dtype=torch.uint8, device=d_q.device)
                snap.check_batch_rows_device(recv.data_ptr(), len(recv), dec.data_ptr(), a.depth, sp)
            send_back(dec, state, d_out, world, comm_device=comm)
            routed[0] = len(recv)
            routed[1] = recv
    else:
        qd = snap.with_handles(q)        # request resolution (row ids -> row handles), untimed
        d_q = torch.from_numpy(qd.view(np.uint8)).to(f"cuda:{dev}")

        def step():
            snap.check_batch_device(d_q.data_ptr(), a.batch, d_out.data_ptr(), a.depth, sp)

    strf = None
    if not migrate and not a.partitioned and unified is not None:
        strf = string_form(g, unified, snap, q_gen, a)
    rows_dev = None
    if not a.partitioned and not migrate and a.steps > 0:
        # the same batch resident in HBM by row id (what the resolution produces): keto_check_batch_rows_device,
        # the row id -> handle translation inside the timed region (detail only; value times the handle form)
        d_rows = torch.from_numpy(np.ascontiguousarray(q).view(np.uint8)).to(f"cuda:{dev}")
        d_rout = torch.empty(a.batch, dtype=torch.uint8, device=f"cuda:{dev}")
        for _ in range(2):
            snap.check_batch_rows_device(d_rows.data_ptr(), a.batch, d_rout.data_ptr(), a.depth, sp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            snap.check_batch_rows_device(d_rows.data_ptr(), a.batch, d_rout.data_ptr(), a.depth, sp)
        torch.cuda.synchronize()
        t_rows = (time.perf_counter() - t0) / a.steps
        rows_dev = {"value": round(a.batch / t_rows, 1), "unit": "checks/s", "ms_per_step": round(t_rows * 1e3, 3),
                    "what": "the batch resident in HBM as 16-B row-id requests through keto_check_batch_rows_device "
                            "(row id -> handle translation + the check, timed like value)", "_out": d_rout}
    e2e = None
    if not a.partitioned and a.e2e_steps > 0:
        e2e = end_to_end(snap, q, a, d_out)
        if a.e2e_only:
            e2e.pop("_out")
            if rank == 0:
                print(json.dumps({"end_to_end": e2e}), flush=True)
            return
    log(f"rank {rank}: warmup {a.warmup}, timed {a.steps} steps of {a.batch} checks")
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    tier_ms, tier_n = [], []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
        ms, n = snap.last_timing()
        tier_ms.append(ms)
        tier_n.append(n)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{dev}" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total = world * a.batch * a.steps
    value = total / elapsed

    # ---- roofline of the dominant kernel (tier-0 check kernel)
    tier0_ms = float(np.mean([m[0] for m in tier_ms]))
    tier1_ms = float(np.mean([m[1] for m in tier_ms]))
    overflow = int(np.mean([n[1] for n in tier_n]))
    roofline = None
    work = None
    allowed_rate = float(d_out.float().mean().item())
    gpu_out = d_out.cpu().numpy()
    cpu = None
    parity = None
    ref_sql = None
    if rank == 0 and not a.no_work and not migrate:
        # oracle table over a bounded sample of the batch: every tuple those requests can reach
        ns = min(a.cpu_sample, a.batch)
        sample = q_gen[:ns]
        log(f"oracle table over the first {ns} requests")
        t0 = time.perf_counter()
        tab = g.oracle_table(sample, a.depth)
        reqs = g.oracle_requests(tab, sample)
        t_tab = time.perf_counter() - t0
        # SURVEY.md 8(d) algorithmic bytes: B_check(q) = 14 + sum over BFS rows (8 + 4 deg), from the
        # oracle's BFS-count mode on a 1 % sample of the batch, scaled to the launch
        nb = min(ns, max(1, int(a.batch * a.bytes_sample)))
        log(f"{tab.t.n} tuples; pricing {nb} requests in BFS-count mode")
        t0 = time.perf_counter()
        bq = tab.bfs_bytes_reqs(tab.prefix(reqs, nb), a.depth, threads=a.threads)
        t_bfs = time.perf_counter() - t0
        alg = float(bq.mean()) * a.batch
        achieved = alg / (tier0_ms * 1e-3) / 1e9
        # bytes the tier-0 kernel's own traversal requests (instrumented pass, same decisions):
        # 32 B header + window per row visit, 16 B per id-table bucket, 16 B per edge-block reload,
        # 16 B per request in, 1 B per decision out
        if a.partitioned:
            # the instrumented pass takes handle-form requests: the batch this rank received, by handle
            from keto_amd.capi import CHECK_IDS_DTYPE
            rq = routed[1].cpu().numpy().view(CHECK_IDS_DTYPE).reshape(-1).copy()
            rq["row"] = snap.row_handles(rq["row"])
            d_h = torch.from_numpy(rq.view(np.uint8)).to(f"cuda:{dev}")
            d_w = torch.empty(len(rq), dtype=torch.uint8, device=f"cuda:{dev}")
            w = snap.check_work_device(d_h.data_ptr(), len(rq), d_w.data_ptr(), a.depth)
        else:
            w = snap.check_work_device(d_q.data_ptr(), a.batch, d_out.data_ptr(), a.depth)
        rows, edges, idreads, vprobes, vinserts, items = w[:6]
        nw = routed[0] if a.partitioned else a.batch        # requests the instrumented pass ran
        touched = (32 * w[0] + 16 * w[9] + 16 * w[8]) * a.batch / max(1, nw) + 17 * a.batch
        kname = snap.check_kernel_name(a.depth)
        traffic, tsrc = pmc_traffic(kname, {"tuples": int(g.n_edges), "checks_per_gpu_per_step": a.batch,
                                            "max_depth": a.depth, "scale": a.scale})
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": None if traffic is None else int(traffic),
                    "traffic_GBps": None if traffic is None else round(traffic / (tier0_ms * 1e-3) / 1e9, 1),
                    "traffic_source": tsrc, "kernel": kname, "kernel_ms": round(tier0_ms, 3),
                    "alg_bytes_per_launch": int(alg), "alg_bytes_per_check": round(float(bq.mean()), 1),
                    "alg_bytes_sample": f"SURVEY 8(d) B_check over the first {nb} requests (oracle BFS-count mode, "
                                        f"{a.threads} threads, {t_bfs:.1f} s)",
                    "traversal_bytes_per_launch": int(touched),
                    "traversal_GBps": round(touched / (tier0_ms * 1e-3) / 1e9, 1)}
        nwd = max(1, nw)
        work = {"rows_per_check": rows / nwd, "set_edges_per_check": edges / nwd,
                "id_words_per_check": idreads / nwd, "visited_hbm_probes_per_check": vprobes / nwd,
                "top_level_items_per_check": items / nwd, "instrumented_requests": int(nw),
                "line_touches_per_check": {k: round(v / nwd, 3) for k, v in zip(
                    ("request", "header", "edge", "id_table", "id_search", "frame_push", "frame_pop"), w[6:13])}}
        # ---- CPU baseline (N = 1): the oracle restatement timed on the sample, decisions compared
        if world == 1 and not a.no_cpu_baseline:
            log(f"cpu baseline over {ns} requests, {a.threads} threads")
            t0 = time.perf_counter()
            ref = tab.check_batch_reqs(reqs, a.depth, threads=a.threads)
            t_cpu = time.perf_counter() - t0
            parity = {"sample": int(ns), "mismatches": int((ref != gpu_out[:ns]).sum())}
            cpu = {"value": round(ns / t_cpu, 1), "unit": "checks/s", "cores": a.threads, "kind": "port",
                   "host": {**a.host, "threads_used": a.threads},
                   "sample": f"first {ns} requests of the rank-0 batch; oracle/keto_oracle.c over the "
                             f"{tab.t.n} tuples those requests can reach (extracted in {t_tab:.1f} s), "
                             f"{a.threads} host threads, {t_cpu:.2f} s"}
            # the reference engine's algorithm issuing its own SQL against SQLite, one worker process
            # per core (oracle/sql_bench.py), on a bounded sample
            if a.sql_sample > 0:
                ref_sql = sql_leg(g, q_gen, a, gpu_out)

    part_parity = None
    if a.partitioned and a.check_parity:
        full = g.snapshot(device=dev)
        want = full.check_batch_ids(full.with_handles(q), a.depth)
        bad = torch.tensor([int((want != gpu_out).sum())], dtype=torch.int64, device=comm if world > 1 else "cpu")
        if world > 1:
            dist.all_reduce(bad)
        part_parity = {"requests": world * a.batch, "mismatches_vs_replicated": int(bad.item())}
        del full
    if e2e is not None and roofline is not None:
        e2e["frac"] = round(roofline["alg_bytes_per_launch"] / (e2e["ms_per_batch"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if e2e is not None:
        e2e["decisions_equal_device_resident"] = all(bool((o == gpu_out).all()) for o in e2e.pop("_out"))
    if rows_dev is not None:
        rows_dev["decisions_equal_device_resident"] = bool((rows_dev.pop("_out").cpu().numpy() == gpu_out).all())
    if strf is not None:
        strf["decisions_equal_device_resident"] = bool((strf.pop("_out") == gpu_out).all())
        hr = strf["host_resolution"]
        hr["decisions_equal_device_resident"] = bool((hr.pop("_out") == gpu_out).all())
        if roofline is not None:
            for x in (strf, hr):
                x["frac"] = round(roofline["alg_bytes_per_launch"] / (x["ms_per_batch"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        if e2e is not None:
            e2e["string_form"] = strf
    # host resources per rank (the 8-rank run: every rank holds the graph and the snapshot's host tables)
    rss, cpu_s = rusage()
    host_ranks = [[rss, cpu_s]]
    if world > 1:
        t = torch.tensor([rss, cpu_s], dtype=torch.float64, device=f"cuda:{dev}" if backend == "nccl" else "cpu")
        allr = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allr, t)
        host_ranks = [x.tolist() for x in allr]
    if rank == 0:
        line = {
            "metric": "checks/sec (whole node) on 1B-tuple graph, max-depth 5; % of HBM roofline",
            "value": round(value, 1), "unit": "checks/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": "powerlaw-acl-1B (BASELINE config #4) on one GPU per rank, " +
                                   ("migrating partition (every row on one part, searches move between parts as "
                                    f"records, {a.hot_mb} MB of replicated hot rows per part)" if migrate else
                                    "edge-partitioned snapshot, requests routed by all-to-all" if a.partitioned
                                    else "replicated snapshot") +
                                   ("; value = requests resident in HBM by row id, routed and checked per step"
                                    if a.partitioned else
                                    "; value = a device-resident batch of pre-resolved requests (row handles in HBM, "
                                    "keto_check_batch_device; the row id -> handle resolution is untimed); "
                                    "detail.device_row_ids times the row-id form with its translation, and "
                                    "end_to_end.value is SURVEY 8(d) t_batch (host entry to decisions on the host)"),
                       "tuples": int(g.n_edges), "set_edge_fraction": round(g.n_set_edges / max(1, g.n_edges), 4),
                       "rows": int(g.n_rows), "checks_per_gpu_per_step": a.batch, "max_depth": a.depth,
                       "global_batch": a.batch * world,
                       "parallelism": (f"migrating-{world}" if migrate else f"partitioned-{world}" if a.partitioned
                                       else f"replicated-dp{world}"),
                       "scale": a.scale},
            "roofline": roofline,
            "end_to_end": e2e,
            "cpu_baseline": cpu,
            "ref_sql": ref_sql,
            "parity": parity if part_parity is None else part_parity,
            "detail": {"device_row_ids": rows_dev, "tier0_ms": round(tier0_ms, 3), "tier1_ms": round(tier1_ms, 3),
                       "tier0_overflow_requests": overflow, "allowed_fraction": round(allowed_rate, 4),
                       "gen_s": round(t_gen, 1), "snapshot_upload_s": round(t_snap, 1), "work": work,
                       "host_per_rank": [{"peak_rss_gb": round(r_, 2), "cpu_s": round(c_, 1)} for r_, c_ in host_ranks],
                       "host": a.host, "threads": a.threads,
                       "string_table": unified is not None if not migrate else False,
                       "migrate_rounds_last_step": routed[2] if migrate else None},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
