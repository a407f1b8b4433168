"""BASELINE config #4's edge-partitioned forms at the headline scale, on the box's one GPU.

north_star: "When [the graph] does not [fit one GPU], the graph is edge-partitioned by hash(namespace,
object)".  The 1B-tuple power-law graph (tools/synth.cpp, POWERLAW_1B; 155M rows) is cut into P
shared-rows parts (P = 2, 4: subject-set targets on every part, root rows by hash) and into 2 migrating
parts (every row on one part, searches travel between parts as continuation records), each part a
rank of the in-process transport (keto_comm_init_local) on device 0, as the Go server runs a graph
past one GPU's memory (integration/go/internal/gpu/partition.go).  For each form:

* the bench's 16,777,216-request batch (docs:d#view@u at max-depth 5, tools/synth.py queries seed
  1000) goes through keto_check_batch_routed (named, resolved on host threads) and
  keto_check_batch_routed_packed (packed, resolved on each rank's device: the Go Partition's call),
  each rank passing its own slice (most requests belong to other parts): every decision equals the
  replicated snapshot's, whose first 1,000,000 decisions equal oracle/keto_oracle.c
  (internal/check/engine.go:36-123);
* 5,000 expand roots (request rows owned by every part, and subject-set targets) go through
  keto_expand_batch_routed: every tree equals the replicated snapshot's node for node
  (internal/expand/engine.go:33-102);
* one 100-tuple transaction that adds root rows (new documents, owned by the parts their hash picks)
  with direct and subject-set subjects is applied to every part and to the replicated snapshot; the
  whole batch is checked again (unchanged) plus requests on the new rows, against the replicated
  snapshot (internal/persistence/sql/relationtuples.go:279-297).

Set KETO_PARTS_LOG=<path> to append one JSON line per form (per-part device GiB, host RSS, build /
upload / exchange / routed-batch times): profiles/r06*_config4_parts.log come from it."""
import ctypes as C
import json
import os
import resource
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BATCH = 16 * 1024 * 1024
N_ROOTS = 5_000


def _rss_gb():
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1e6
    return 0.0


def _log(rec):
    rec = {**rec, "rss_gb": round(_rss_gb(), 2),
           "peak_rss_gb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 2)}
    print("[config4-parts] " + json.dumps(rec), flush=True)
    path = os.environ.get("KETO_PARTS_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def _ranks(P, fn):
    res = [None] * P

    def run(r):
        try:
            res[r] = (True, fn(r))
        except Exception as e:          # noqa: BLE001 -- reported per rank
            res[r] = (False, e)

    ts = [threading.Thread(target=run, args=(r,)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    assert not any(t.is_alive() for t in ts), "a rank is still waiting"
    bad = [(r, v) for r, (ok, v) in enumerate(res) if not ok]
    assert not bad, bad
    return [v for _, v in res]


def _slice(arr, lo, hi):
    from keto_amd.capi import KCheckReq
    return (KCheckReq * max(1, hi - lo)).from_address(C.addressof(arr) + lo * C.sizeof(KCheckReq))


class Base:
    pass


@pytest.fixture(scope="module")
def base():
    import torch
    from keto_amd.capi import Snapshot
    from tools import synth
    b = Base()
    t0 = time.perf_counter()
    b.g = g = synth.SynthGraph(dict(synth.POWERLAW_1B), threads=16)
    assert g.n_edges == 1_000_000_000
    b.u = u = g.unified(threads=16)
    b.q = g.queries(BATCH, seed=1000, depth=5, threads=16)
    b.arr = g.string_requests(u.names, b.q, threads=16)
    b.full = g.snapshot_unified(u, device=0)
    t_full = time.perf_counter() - t0
    qd = b.full.with_handles(u.to_device_targets(b.q))
    d_q = torch.from_numpy(qd.view(np.uint8)).to("cuda:0")
    d_out = torch.full((BATCH,), 7, dtype=torch.uint8, device="cuda:0")
    b.full.check_batch_device(d_q.data_ptr(), BATCH, d_out.data_ptr(), 5, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    b.want = d_out.cpu().numpy()
    del d_q, d_out
    assert (b.want <= 1).all()
    # the replicated decisions themselves against the C restatement of the reference engine
    k = 1_000_000
    tab = g.oracle_table(b.q[:k], 5)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, b.q[:k]), 5, threads=16)
    assert (b.want[:k] == ref).all(), f"{int((b.want[:k] != ref).sum())} mismatches of {k}"
    del tab, ref
    # expand roots: rows of requests (root rows of every part) and subject-set targets (every part's)
    rng = np.random.default_rng(46)
    rel = g.relation_names()
    names = dict(g.namespaces)
    req_rows = b.q["row"][rng.integers(0, BATCH, size=N_ROOTS // 2)]
    set_rows = rng.integers(0, g.n_rows, size=N_ROOTS - len(req_rows)).astype(np.uint32)
    rows = np.concatenate([req_rows, set_rows])
    b.roots = [(("set", names[int(g.row_ns[r])], f"{int(g.row_obj[r]):08x}", rel[int(g.row_rel[r])]), 0)
               for r in rows.tolist()]
    b.want_trees = [(st, nodes) for st, _, nodes in b.full.expand_batch(b.roots, 5, want_nodes=True)]
    assert sum(len(n) for _, n in b.want_trees) > N_ROOTS
    # the write: 50 new documents, each with a direct user and a group subject set (root rows)
    wr = np.random.default_rng(47)
    b.new_objs = [f"w{i:07x}" for i in range(50)]
    users = wr.integers(0, g.params["n_users"], size=50)
    groups = [r for r in rng.integers(0, g.n_rows, size=4000).tolist() if names[int(g.row_ns[r])] == "groups"][:50]
    assert len(groups) == 50
    b.inserts = []
    for o, uid, gr in zip(b.new_objs, users.tolist(), groups):
        b.inserts.append((1, o, "view", f"u{uid:08x}"))
        b.inserts.append((1, o, "view", None, 3, f"{int(g.row_obj[gr]):08x}", rel[int(g.row_rel[gr])]))
    # requests on the new rows: the direct user, and members reached through the group (or not)
    members = wr.integers(0, g.params["n_users"], size=150)
    b.new_reqs = [("docs", o, "view", ("id", f"u{int(x):08x}"), 0)
                  for o, x in zip(b.new_objs * 4, users.tolist() + members.tolist())]
    b.full.apply(b.inserts, [])
    b.want_new, b.want_new_st = b.full.check_batch(b.new_reqs, 5)
    assert b.want_new[:50].all()
    _log({"form": "replicated", "arena_gib": round(b.full.stats()["device_bytes"] / 2**30, 2),
          "build_s": round(t_full, 1), "allowed_fraction": round(float(b.want.mean()), 4)})
    yield b
    b.full.close()
    u.free()
    g.close()


def _routed_batch(comms, parts, b):
    P = len(parts)
    bounds = [(r * BATCH // P, (r + 1) * BATCH // P) for r in range(P)]
    t0 = time.perf_counter()
    res = _ranks(P, lambda r: comms[r].check_batch_routed(parts[r], _slice(b.arr, *bounds[r]), 5,
                                                          n=bounds[r][1] - bounds[r][0]))
    dt = time.perf_counter() - t0
    got = np.concatenate([a for a, _ in res])
    st = np.concatenate([s for _, s in res])
    return got, st, dt


def _check_form(b, P, mode, label):
    from keto_amd.capi import PART_MIGRATE, Comm, Snapshot
    g, u = b.g, b.u
    rec = {"form": label, "parts": P}
    t0 = time.perf_counter()
    # the parts side by side (each a host-only snapshot of the whole graph, then its part uploaded)
    parts = _ranks(P, lambda r: Snapshot.from_csr(g.namespaces, g.row_ns, u.row_obj, u.row_rel, g.row_ptr, u.edges,
                                                  kstrs=(u.strs, u.n_strings), device=-1).upload_part(r, P, 0, mode=mode))
    rec["build_upload_s"] = round(time.perf_counter() - t0, 1)
    rec["part_gib"] = [round(p.stats()["device_bytes"] / 2**30, 2) for p in parts]
    cid = os.urandom(32)
    comms = [Comm(cid, P, r, 0, local=True) for r in range(P)]
    try:
        if mode == PART_MIGRATE:
            t0 = time.perf_counter()
            rounds = _ranks(P, lambda r: comms[r].close_filters(parts[r]))
            rec["filter_exchange_s"] = round(time.perf_counter() - t0, 1)
            rec["filter_rounds"] = rounds[0]
        got, st, dt = _routed_batch(comms, parts, b)       # first batch: builds the resolution indexes
        rec["first_routed_batch_s"] = round(dt, 2)
        assert (st == 0).all(), f"{int((st != 0).sum())} statuses not OK"
        assert (got == b.want).all(), f"{label}: {int((got != b.want).sum())} mismatches of {BATCH}"
        got, st, dt = _routed_batch(comms, parts, b)
        rec["routed_batch_ms"] = round(dt * 1e3, 1)
        rec["routed_checks_per_s"] = round(BATCH / dt, 1)
        assert (got == b.want).all()
        # the same batch packed (the Go Partition's call): every rank's slice resolved on its device
        bounds = [(r * BATCH // P, (r + 1) * BATCH // P) for r in range(P)]
        packs = [g.pack_requests(_slice(b.arr, lo, hi), hi - lo) for lo, hi in bounds]
        for rep in range(2):                             # the first call uploads each part's indexes
            t0 = time.perf_counter()
            res = _ranks(P, lambda r: comms[r].check_batch_routed_packed(
                parts[r], packs[r][0].array[:packs[r][2]], packs[r][1].array, 5, n=bounds[r][1] - bounds[r][0]))
            dt = time.perf_counter() - t0
            got = np.concatenate([x for x, _ in res])
            assert (got == b.want).all(), f"{label} packed: {int((got != b.want).sum())} mismatches"
            assert all((s_ == 0).all() for _, s_ in res)
        rec["routed_packed_batch_ms"] = round(dt * 1e3, 1)
        rec["routed_packed_checks_per_s"] = round(BATCH / dt, 1)
        del packs
        # expand: each rank its share of the roots
        shares = [list(range(r, N_ROOTS, P)) for r in range(P)]
        t0 = time.perf_counter()
        trees = _ranks(P, lambda r: comms[r].expand_batch_routed(parts[r], [b.roots[i] for i in shares[r]], 5,
                                                                 want_nodes=True))
        rec["routed_expand_s"] = round(time.perf_counter() - t0, 2)
        for r in range(P):
            for i, (st_, _, nodes) in zip(shares[r], trees[r]):
                assert (st_, nodes) == b.want_trees[i], (label, b.roots[i])
        # one write transaction on every part: root rows added on the parts their hash picks
        t0 = time.perf_counter()
        _ranks(P, lambda r: parts[r].apply(b.inserts, []))            # the parts side by side, as the Go Partition does
        rec["apply_all_parts_s"] = round(time.perf_counter() - t0, 2)
        # the write added exactly 50 rows (ids after the build's): their owners
        owners = parts[0].row_owner(np.arange(g.n_rows, g.n_rows + 50, dtype=np.uint32), P)
        rec["new_rows_per_part"] = np.bincount(owners[owners >= 0], minlength=P).tolist()
        got, st, dt = _routed_batch(comms, parts, b)
        rec["routed_batch_after_write_ms"] = round(dt * 1e3, 1)
        assert (got == b.want).all(), f"{label} after the write: {int((got != b.want).sum())} mismatches"
        mine = [b.new_reqs[r::P] for r in range(P)]
        res = _ranks(P, lambda r: comms[r].check_batch_routed(parts[r], mine[r], 5))
        for r, (a, s) in enumerate(res):
            assert (a == b.want_new[r::P]).all() and (s == b.want_new_st[r::P]).all(), (label, r)
    finally:
        for c in comms:
            c.close()
        for p in parts:
            p.close()
    _log(rec)


@pytest.mark.parametrize("P", [2, 4])
def test_shared_rows_parts_full_scale(base, P):
    from keto_amd.capi import PART_SHARED
    _check_form(base, P, PART_SHARED, "shared-rows")


def test_migrating_parts_full_scale(base):
    from keto_amd.capi import PART_MIGRATE
    _check_form(base, 2, PART_MIGRATE, "migrating")
