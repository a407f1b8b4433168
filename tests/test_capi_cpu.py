"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/keto_mi355x.h
declares, builds host-only snapshots (device = -1) with the reference ordering / poisoning /
collision bookkeeping, and refuses compute without a device."""
import os
import re

import pytest

import keto_amd
from keto_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exports_match_header():
    hdr = open(os.path.join(ROOT, "include", "keto_mi355x.h")).read()
    declared = set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(keto_[a-z_]+)\(", hdr, re.M))
    lib = keto_amd.load()
    for name in declared:
        assert hasattr(lib, name), name
    assert set(capi.EXPORTS) == declared


def test_abi_version():
    hdr = open(os.path.join(ROOT, "include", "keto_mi355x.h")).read()
    want = int(re.search(r"#define KETO_ABI_VERSION (\d+)", hdr).group(1))
    assert keto_amd.load().keto_abi_version() == want == capi.KETO_ABI_VERSION


def test_host_snapshot_stats():
    ns = [(1, "n")]
    rows = [(1, "a", "r", "u"), (1, "a", "r", None, 1, "b", "r"), (1, "b", "r", "v"),
            (1, "c", "r", None, 1, "", "r"),        # wildcard subject set -> materialized row
            (1, "d", "r", None, 99, "x", "y"),      # unknown subject-set namespace -> poisoned row
            (1, "e", "r", "n:b#r")]                 # subject id colliding with set n:b#r
    s = keto_amd.Snapshot.build(ns, rows, device=-1)
    st = s.stats()
    assert st["n_tuples"] == 6
    assert st["n_real_rows"] == 5
    assert st["n_wildcard_rows"] == 1
    assert st["n_poisoned_rows"] == 2      # the row itself and the wildcard row (n, *, r) that includes it
    assert st["n_collision_keys"] == 1
    assert st["device_bytes"] == 0


def test_duplicate_namespace_rejected():
    with pytest.raises(keto_amd.KetoError, match="-4"):
        keto_amd.Snapshot.build([(1, "n"), (2, "n")], [], device=-1)


def test_compute_without_device_fails_loudly():
    s = keto_amd.Snapshot.build([(1, "n")], [(1, "a", "r", "u")], device=-1)
    with pytest.raises(keto_amd.KetoError):
        s.check_batch([("n", "a", "r", ("id", "u"), 0)])


def test_csr_bulk_loader_validates_order():
    import numpy as np
    with pytest.raises(keto_amd.KetoError):
        keto_amd.Snapshot.from_csr([(1, "n")], np.array([1, 1]), np.array([2, 1]), np.array([0, 0]),
                                   np.array([0, 0, 0], dtype=np.uint64), np.zeros(0, np.uint32), device=-1)


def test_arena_layout_lines():
    """compute_layout on the power-law generator: rows some subject set points at carry a closure
    filter, and filter + header + window (CB + 8 words) fill exactly one 128-B line; every other
    row's header + window (8 words) never straddles a line; handles are distinct and increasing in
    arena order."""
    import numpy as np
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 8192), threads=2)
    s = g.host_snapshot()
    h = s.row_handles(np.arange(g.n_rows, dtype=np.uint32)).astype(np.int64)
    sets = g.edges[(g.edges & 0x80000000) != 0] & 0x7FFFFFFF
    target = np.zeros(g.n_rows, dtype=bool)
    target[sets.astype(np.int64)] = True
    assert target.any() and (~target).any()
    word = h * 4
    assert ((word[target] - 24) % 32 == 0).all()              # filter at a line start, header at +96 B
    assert (word[~target] % 32 <= 24).all()
    assert len(np.unique(h)) == len(h)


def test_route_argument_checks_need_no_gpu():
    """keto_route_work_bytes is host arithmetic (destination bytes + per-(part, 2048-request tile)
    counts + part starts, each 256-B aligned); keto_route_rows_device rejects bad part counts and a
    short workspace before touching the device."""
    import ctypes as C
    from keto_amd import capi
    lib = capi.load()
    assert capi.route_work_bytes(0, 1) == 0 + 0 + 256
    assert capi.route_work_bytes(4096, 3) == 4096 + 256 + 256
    assert capi.route_work_bytes(4097, 8) == 4352 + 256 + 256
    counts = (C.c_uint32 * 65)()
    for n_parts, self_part, wb in ((0, 0, 1 << 20), (65, 0, 1 << 20), (4, 4, 1 << 20), (4, 0, 10)):
        rc = lib.keto_route_rows_device(C.c_void_p(8), C.c_uint32(100), C.c_void_p(8), C.c_uint32(10),
                                        C.c_uint32(self_part), C.c_uint32(n_parts), C.c_void_p(8), C.c_uint64(wb),
                                        C.c_void_p(8), C.c_void_p(8), counts, None)
        assert rc == -1, (n_parts, self_part, wb)                 # KETO_E_INVALID


def test_host_apply_wildcard_sets():
    """keto_snapshot_apply on a host-only snapshot: new wildcard subject sets (empty object, empty
    relation, the namespace named "") become materialized rows and writes to the rows they match take
    the delta path (version + 1); a write to a row that a poisoned wildcard row matches is refused
    with KETO_E_REBUILD and leaves the snapshot unchanged."""
    ns = [(1, "n"), (2, "")]
    rows = [(1, "a", "r", "u"), (1, "b", "r", None, 1, "", "r"), (1, "c", "s", "v")]
    s = keto_amd.Snapshot.build(ns, rows, device=-1)
    assert s.stats()["n_wildcard_rows"] == 1
    assert s.apply([(1, "a", "r", "w")]) == 1                                   # matched by n:*#r
    assert s.apply([(1, "d", "r", None, 1, "c", ""), (1, "e", "r", None, 2, "a", "r"),
                    (1, "f", "r", None, 1, "", "")], [(1, "b", "r", None, 1, "", "r")]) == 2
    st = s.stats()
    assert st["n_wildcard_rows"] == 4 and st["n_tuples"] == 6, st
    assert s.apply([], [(1, "d", "r", None, 1, "c", "")]) == 3
    p = keto_amd.Snapshot.build(ns, [(1, "a", "r", None, 99, "x", "y"), (1, "b", "r", None, 1, "", "r")],
                                device=-1)
    with pytest.raises(keto_amd.KetoError, match="-6"):
        p.apply([(1, "c", "r", "u")])                                           # n:*#r holds a poisoned page
    assert p.version() == 0
    assert p.apply([(1, "c", "s", "u")]) == 1                                   # no wildcard row matches n:c#s


def test_apply_is_not_starved_by_readers():
    """The snapshot lock lets a waiting write in (RwGate, snapshot.hpp): four threads cloning a
    host-only snapshot back to back (each clone holds the lock shared) cannot keep keto_snapshot_apply
    waiting.  With a reader-preferring lock the writes could wait as long as the readers keep
    overlapping; here 30 transactions must commit while the readers run."""
    import threading
    import time
    ns = [(1, "docs"), (2, "groups")]
    rows = [(1, f"d{i}", "view", f"u{i % 97}") for i in range(20000)]
    rows += [(1, f"d{i}", "view", None, 2, f"g{i % 50}", "member") for i in range(0, 20000, 7)]
    s = keto_amd.Snapshot.build(ns, rows, device=-1)
    stop = threading.Event()
    clones = [0] * 4
    errors = []

    def reader(k):
        try:
            while not stop.is_set():
                s.clone(device=-1).close()
                clones[k] += 1
        except Exception as e:          # noqa: BLE001 -- reported below
            errors.append(repr(e))

    ts = [threading.Thread(target=reader, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    t0 = time.time()
    try:
        for k in range(30):
            s.apply([(1, f"w{k}", "view", f"wu{k}")])
    finally:
        stop.set()
        for t in ts:
            t.join(timeout=60)
    assert not errors, errors
    assert s.version() == 30
    assert time.time() - t0 < 60
    assert sum(clones) > 0
    s.close()


def test_string_table_grows_across_chunks(tmp_path):
    """Writes append strings to a chunked table (Chunked, snapshot.hpp: 2^16 strings a chunk, never
    moved) and rows to per-row tables grown before the exclusive lock (delta.cpp, Grown).  180,000
    new strings on a 140,003-string build cross two chunk boundaries; every added and built name
    still resolves and prints back, in the snapshot, a clone and a saved / loaded copy."""
    ns = [(1, "docs")]
    s = keto_amd.Snapshot.build(ns, [(1, f"d{i}", "view", f"u{i}") for i in range(70000)], device=-1)
    for k in range(3):
        s.apply([(1, f"n{k}_{i}", "view", f"w{k}_{i}") for i in range(30000)])
    st = s.stats()
    assert st["n_strings"] == 140003 + 180000 and st["n_rows"] == 160000, st
    picks = [(k, i) for k in range(3) for i in (0, 1, 21844, 21845, 29999)]
    reqs = [("docs", f"n{k}_{i}", "view", ("id", f"w{k}_{i}"), 0) for k, i in picks]
    reqs += [("docs", "d5", "view", ("id", "u5"), 0), ("docs", "zz", "view", ("id", "nope"), 0)]
    want = [("id", f"w{k}_{i}") for k, i in picks] + [("id", "u5")]
    path = str(tmp_path / "snap.bin")
    s.save(path)
    for snap in (s, s.clone(device=-1), keto_amd.Snapshot.load(path, device=-1)[0]):
        out, status = snap.resolve_checks(reqs)
        assert (status == 0).all()
        assert (out["row"][:-1] != 0xFFFFFFFF).all() and out["row"][-1] == 0xFFFFFFFF
        assert snap.subject_fields([int(x) for x in out["target"][:-1]]) == want
        assert snap.stats()["n_strings"] == st["n_strings"]
    s.apply([(1, "n0_0", "view", "late")])
    assert s.resolve_checks([("docs", "n0_0", "view", ("id", "late"), 0)])[0]["target"][0] == st["n_strings"]


def test_engine_build_id_keys_traffic_profiles():
    """The PMC traffic profiles bench.py reports as `roofline.traffic` are keyed on engine.hip and its
    compile flags (keto_amd/build.py SOURCE_FLAGS): the key changes with the flags, and a committed
    profile exists for the build as it stands, so the round's bench line carries measured traffic."""
    import glob
    import hashlib
    import json
    from keto_amd import build
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(build.CSRC, "engine.hip"), "rb").read()
    assert build.engine_build_id() != hashlib.sha256(src).hexdigest() or not build.SOURCE_FLAGS.get("engine.hip")
    keys = [json.load(open(p)).get("engine_sha256") for p in glob.glob(os.path.join(root, "profiles", "*_traffic.json"))]
    assert build.engine_build_id() in keys
