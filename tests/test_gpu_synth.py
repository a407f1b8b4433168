"""Large(r)-graph parity: the power-law ACL generator (BASELINE config #4 shape, scaled down) and a
nested-groups graph with cycles and depth up to 32 (config #3 shape), GPU vs the C oracle,
bit-exact decisions and exact expand trees."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def powerlaw():
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 256), threads=16)
    snap = g.snapshot(device=0)
    yield g, snap
    g.close()


@pytest.fixture(scope="module")
def nested():
    from tools import synth
    g = synth.SynthGraph(dict(n_docs=0, n_folders=0, n_groups=1 << 15, n_users=1 << 15, target_edges=0, seed=3),
                         threads=16, kind="nested", chain=32)
    snap = g.snapshot(device=0)
    yield g, snap
    g.close()


@pytest.mark.parametrize("gmd,wave", [(32, 0), (16, 0), (40, 0), (7, 0), (32, 1), (12, 1), (40, 1)])
def test_nested_deep_checks_match_oracle(nested, monkeypatch, gmd, wave):
    """Config #3 shape: chains of 32 nested groups with cycles; global max-depth up to 40 takes the
    deep (global-stack) kernel tiers, or deep_wave_kernel as tier 0 (KETO_DEEP_WAVE=1)."""
    g, snap = nested
    monkeypatch.setenv("KETO_DEEP_WAVE", str(wave))
    q = g.queries_nested(12000, seed=100 + gmd, depths=(5, 16, 32, 0, -1, 40))
    gpu = snap.check_batch_ids(snap.with_handles(q), gmd)
    tab = g.oracle_table(q, max(gmd, 1))
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), gmd, threads=16)
    assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)}"


@pytest.mark.parametrize("pool", [True, False])
def test_nested_tier1_borrowed_tables_match_oracle(nested, pool):
    """Tiny tier-0/1 visited tables (KETO_T0_CAP / KETO_T1_CAP) make thousands of deep requests
    outgrow tier 1: with the pool, a tier-1 lane borrows one of tier 2's direct tables and finishes
    the request itself (PromoVisited); requests that find every table borrowed, or all of them
    without the pool, restart on tier 2.  Every decision must equal the oracle's either way.  Whole
    requests (KETO_ITEMS=0): split into items and pretested, too few searches outgrow the tables
    (tests/test_gpu_items.py runs the items with these tables)."""
    g, snap = nested
    q = g.queries_nested(12000, seed=77, depths=(16, 32, 0, 40))
    env = {"KETO_T0_CAP": "256", "KETO_T1_CAP": "1024", "KETO_ITEMS": "0"}
    if not pool:
        env["KETO_NO_POOL"] = "1"
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        gpu = snap.check_batch_ids(snap.with_handles(q), 40)
        _, n = snap.last_timing()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    tab = g.oracle_table(q, 40)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), 40, threads=16)
    assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)} (pool {pool}, tiers {n})"
    assert n[1] > 0, f"no request reached tier 1: {n}"
    if not pool:
        assert n[2] > 0, f"no request reached tier 2 without the pool: {n}"


def test_nested_expand_matches_oracle(nested):
    g, snap = nested
    rng = np.random.default_rng(9)
    rows = rng.integers(0, g.n_rows, size=120).astype(np.uint32)
    depths = rng.choice([2, 5, 12, 20], size=120).astype(np.int32)
    status, offs, nodes = snap.expand_batch_ids(rows | np.uint32(0x80000000), depths, 20)
    q = np.zeros(len(rows), dtype=[("row", "<u4"), ("target", "<u4"), ("flags", "<u4"), ("max_depth", "<i4")])
    q["row"] = rows
    tab = g.oracle_table(q, 20)
    for i, (row, d) in enumerate(zip(rows, depths)):
        r, want = _oracle_expand_nodes(g, tab, int(row), int(d), 20)
        if r == 0:
            assert status[i] == 1
            continue
        assert r == 1 and status[i] == 0
        have = []
        for subj, info in nodes[offs[i]:offs[i + 1]]:
            leaf, nc = int(info >> 31), int(info & 0x7FFFFFFF)
            if subj >> 31:
                t = int(subj & 0x7FFFFFFF)
                have.append((leaf, 1, 0, 0xFFFF0000 + int(g.row_ns[t]), int(g.row_obj[t]), int(g.row_rel[t]), nc))
            else:
                have.append((leaf, 0, int(subj), 0, 0, 0, nc))
        assert have == want, f"root row {row} depth {d}"


def _gpu_check(snap, q, gmd):
    return snap.check_batch_ids(q, gmd)


@pytest.mark.parametrize("gmd", [5, 2, 8])
def test_powerlaw_checks_match_oracle(powerlaw, gmd):
    g, snap = powerlaw
    q = g.queries(40000, seed=11 + gmd, depth=gmd)
    rng = np.random.default_rng(gmd)
    q["max_depth"] = rng.integers(-1, gmd + 2, size=len(q))      # exercise the depth clamp
    gpu = _gpu_check(snap, snap.with_handles(q), gmd)
    tab = g.oracle_table(q, gmd)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), gmd, threads=16)
    assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)}"
    assert 0.05 < gpu.mean() < 0.95


def test_powerlaw_closure_filters_prune(powerlaw):
    """Subject sets whose closure filter rules the requested id out are skipped (work slot 15) --
    a large share of the row visits -- and every decision stays the oracle's."""
    import torch
    g, snap = powerlaw
    q = g.queries(20000, seed=77, depth=5)
    d = torch.from_numpy(snap.with_handles(q).view(np.int32).reshape(-1, 4).copy()).to("cuda:0")
    out = torch.empty(len(q), dtype=torch.uint8, device="cuda:0")
    w = snap.check_work_device(d.data_ptr(), len(q), out.data_ptr(), 5)
    torch.cuda.synchronize()
    gpu = out.cpu().numpy()
    tab = g.oracle_table(q, 5)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), 5, threads=16)
    assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)}"
    rows, pruned = w[0], w[15]
    assert pruned > 0.15 * rows, (rows, pruned)


def _oracle_expand_nodes(g, tab, row, depth, gmd):
    from oracle.oracle_c import OraNode, OraSubject, lib
    ns = int(g.row_ns[row])
    root = OraSubject(1, 0, 0xFFFF0000 + ns, int(g.row_obj[row]), int(g.row_rel[row]),
                      int(g.params["n_users"] + row))
    nodes = C.POINTER(OraNode)()
    nn = C.c_uint64()
    r = lib().ora_expand(C.byref(tab.t), C.byref(root), C.c_int32(depth), C.c_int32(gmd), C.byref(nodes),
                         C.byref(nn))
    out = [(nodes[i].type, nodes[i].kind, nodes[i].sid, nodes[i].name, nodes[i].obj, nodes[i].rel,
            nodes[i].n_children) for i in range(nn.value)]
    if nn.value:
        lib().ora_free(C.cast(nodes, C.c_void_p))
    return r, out


def test_powerlaw_expand_matches_oracle(powerlaw):
    _expand_matches_oracle(*powerlaw)


@pytest.mark.parametrize("pin_chunk", [None, 4096, 1 << 16])
def test_powerlaw_proto_all_device_equals_host(powerlaw, monkeypatch, pin_chunk):
    """keto_tree_proto_all_device (encoded on the GPU) gives the host encoder's bytes and offsets;
    pin_chunk: the D2H through many small pinned bounce chunks (KETO_PROTO_PIN_CHUNK)."""
    if pin_chunk:
        monkeypatch.setenv("KETO_PROTO_PIN_CHUNK", str(pin_chunk))
    g, snap = powerlaw
    rng = np.random.default_rng(19)
    n = 5000
    rows = rng.integers(0, g.n_rows, size=n).astype(np.uint32) | np.uint32(0x80000000)
    depths = rng.integers(-1, 7, size=n).astype(np.int32)
    for gmd in (5, 2):
        st_h, offs_h, blob_h, _, _ = snap.expand_batch_ids_proto(rows, depths, gmd)
        st_d, offs_d, blob_d, _, _ = snap.expand_batch_ids_proto(rows, depths, gmd, device=True)
        assert (st_h == st_d).all() and (offs_h == offs_d).all()
        assert len(blob_h) > 0 and blob_h == blob_d


def test_powerlaw_proto_all_equals_per_tree(powerlaw):
    """keto_tree_proto_all (every tree of an arena encoded on host threads into one buffer) gives
    byte for byte the per-tree keto_tree_proto encodings, at the offsets it reports; nil trees
    (rows with no tuples) are empty; the sizing call writes nothing."""
    g, snap = powerlaw
    rng = np.random.default_rng(9)
    n = 2000
    rows = rng.integers(0, g.n_rows, size=n).astype(np.uint32) | np.uint32(0x80000000)
    depths = rng.integers(0, 5, size=n).astype(np.int32)
    lib = snap.lib
    a = C.c_void_p()
    assert lib.keto_expand_batch_ids(snap.h, rows.ctypes.data_as(C.c_void_p), depths.ctypes.data_as(C.c_void_p),
                                     C.c_uint32(n), C.c_int32(5), C.byref(a)) == 0
    try:
        offs = np.zeros(n + 1, dtype=np.uint64)
        total = lib.keto_tree_proto_all(snap.h, a, None, C.c_uint64(0), offs.ctypes.data_as(C.c_void_p))
        assert total == int(offs[-1]) > 0
        blob = C.create_string_buffer(total)
        assert lib.keto_tree_proto_all(snap.h, a, blob, C.c_uint64(total), offs.ctypes.data_as(C.c_void_p)) == total
        nil = 0
        for i in range(n):
            pn = lib.keto_tree_proto(snap.h, a, C.c_uint32(i), None, C.c_uint64(0))
            one = b""
            if pn > 0:
                buf = C.create_string_buffer(pn)
                lib.keto_tree_proto(snap.h, a, C.c_uint32(i), buf, C.c_uint64(pn))
                one = buf.raw[:pn]
            else:
                nil += 1
            assert blob.raw[int(offs[i]):int(offs[i + 1])] == one, i
        assert nil < n
    finally:
        lib.keto_tree_arena_free(a)


def _expand_matches_oracle(g, snap):
    rng = np.random.default_rng(5)
    rows = rng.integers(0, g.n_rows, size=300).astype(np.uint32)
    depths = rng.integers(1, 5, size=300).astype(np.int32)
    status, offs, nodes = snap.expand_batch_ids(rows | np.uint32(0x80000000), depths, 5)
    q = np.zeros(len(rows), dtype=[("row", "<u4"), ("target", "<u4"), ("flags", "<u4"), ("max_depth", "<i4")])
    q["row"] = rows
    tab = g.oracle_table(q, 5)
    for i, (row, d) in enumerate(zip(rows, depths)):
        r, want = _oracle_expand_nodes(g, tab, int(row), int(d), 5)
        if r == 0:
            assert status[i] == 1
            continue
        assert r == 1 and status[i] == 0
        have = []
        for subj, info in nodes[offs[i]:offs[i + 1]]:
            leaf = int(info >> 31)
            nc = int(info & 0x7FFFFFFF)
            if subj >> 31:
                t = int(subj & 0x7FFFFFFF)
                have.append((leaf, 1, 0, 0xFFFF0000 + int(g.row_ns[t]), int(g.row_obj[t]), int(g.row_rel[t]), nc))
            else:
                have.append((leaf, 0, int(subj), 0, 0, 0, nc))
        assert have == want, f"root row {row} depth {d}"


@pytest.fixture(scope="module")
def powerlaw_seg1():
    """The power-law graph laid out from 2^32 - 64K words on: rows in both arena segments and rows
    bumped past the boundary (a 16 GiB arena on the device)."""
    import os
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 4096), threads=16)
    os.environ["KETO_TEST_ARENA_BASE"] = str((1 << 32) - (1 << 16))
    try:
        snap = g.snapshot(device=0)
    finally:
        del os.environ["KETO_TEST_ARENA_BASE"]
    yield g, snap
    snap.close()
    g.close()


@pytest.mark.parametrize("gmd", [5, 9, 16])
def test_segment1_checks_match_oracle(powerlaw_seg1, gmd):
    g, snap = powerlaw_seg1
    h = snap.row_handles(np.arange(g.n_rows, dtype=np.uint32)).astype(np.int64)
    assert (h < (1 << 30)).any() and (h >= (1 << 30)).mean() > 0.5
    q = g.queries(20000, seed=300 + gmd, depth=gmd)
    gpu = _gpu_check(snap, snap.with_handles(q), gmd)
    tab = g.oracle_table(q, gmd)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), gmd, threads=16)
    assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)}"
    assert 0.05 < gpu.mean() < 0.95


def test_segment1_expand_matches_oracle(powerlaw_seg1):
    _expand_matches_oracle(*powerlaw_seg1)


@pytest.mark.parametrize("dyn,static8,gmd,heads", [("32", "4", 5, "1"), ("4", "0", 5, "4"), ("16", "7", 8, "16"),
                                                    ("100", "2", 5, "2"), ("0", "4", 5, "4"), ("4", "2", 5, "4"),
                                                    ("4", "2", 8, "8")])
def test_powerlaw_dynamic_runs_match_oracle(powerlaw, monkeypatch, dyn, static8, gmd, heads):
    """Tier 0 with dynamic per-XCD request runs (TierArgs::dyn; forced on a batch far below the
    16-requests-per-lane threshold, so most lanes grab runs, several lanes find their XCD's range
    exhausted and a run ends at the batch end; grids of 4 and 20 workgroups split the batch into
    fewer or uneven XCD ranges; 1-16 heads per XCD deal the runs out interleaved, so waves move on
    to other heads once theirs is dealt out): every decision equals the oracle's.  Batch sizes
    that are not multiples of 4 exercise the byte-wise decision stores of a run's last group."""
    g, snap = powerlaw
    monkeypatch.setenv("KETO_T0_DYN_FORCE", "1")
    monkeypatch.setenv("KETO_T0_DYN", dyn)
    monkeypatch.setenv("KETO_T0_DYN_STATIC", static8)
    monkeypatch.setenv("KETO_T0_HEADS", heads)
    for n, seed in ((300_001, 70), (1_003, 71), (5_001, 72)):
        q = g.queries(n, seed=seed + gmd, depth=gmd)
        rng = np.random.default_rng(seed)
        q["max_depth"] = rng.integers(-1, gmd + 2, size=len(q))
        gpu = _gpu_check(snap, snap.with_handles(q), gmd)
        tab = g.oracle_table(q, gmd)
        ref = tab.check_batch_reqs(g.oracle_requests(tab, q), gmd, threads=16)
        assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)}"


@pytest.mark.parametrize("cap", ["1", "3"])
def test_powerlaw_walk_cap_matches_oracle(powerlaw, monkeypatch, cap):
    """Tier 0 walking at most `cap` window edges / pops per loop iteration (KETO_T0_WALK; a lane
    stopped early goes on next iteration without a global access): decisions equal the oracle's."""
    g, snap = powerlaw
    monkeypatch.setenv("KETO_T0_WALK", cap)
    for gmd in (5, 8):
        q = g.queries(100_003, seed=80 + gmd, depth=gmd)
        gpu = _gpu_check(snap, snap.with_handles(q), gmd)
        tab = g.oracle_table(q, gmd)
        ref = tab.check_batch_reqs(g.oracle_requests(tab, q), gmd, threads=16)
        assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)}"


@pytest.fixture(scope="module")
def drive():
    """BASELINE config #2 at 1/16 scale: files whose view row holds the file's own
    owner set (another relation of the same object, namespace 1 sorts first) before its folder; an
    8-ary folder tree of depth <= 6 with group grants; Zipf(1.1) group sizes."""
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.DRIVE_10M, 1 / 16), threads=16, kind="drive")
    snap = g.snapshot(device=0)
    yield g, snap
    snap.close()
    g.close()


@pytest.mark.parametrize("gmd", [5, 2, 3, 7])
def test_drive_checks_match_oracle(drive, gmd):
    g, snap = drive
    q = g.queries(40000, seed=20 + gmd, depth=gmd)
    rng = np.random.default_rng(gmd)
    q["max_depth"] = rng.integers(-1, gmd + 2, size=len(q))      # exercise the depth clamp
    gpu = _gpu_check(snap, snap.with_handles(q), gmd)
    tab = g.oracle_table(q, gmd)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), gmd, threads=16)
    assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)}"
    assert 0.05 < gpu.mean() < 0.95


def test_drive_owner_relation_decides(drive):
    """Requests for a file's own owner (reached only through files:d#view@(files:d#owner), the
    intra-object edge) are allowed at every depth >= 2 and denied at depth 1."""
    g, snap = drive
    rng = np.random.default_rng(1)
    files = rng.integers(0, g.params["n_docs"], size=5000)
    owner_rows = (2 * files).astype(np.int64)
    first_owner = g.edges[g.row_ptr[owner_rows].astype(np.int64)]
    q = np.zeros(len(files), dtype=[("row", "<u4"), ("target", "<u4"), ("flags", "<u4"), ("max_depth", "<i4")])
    q["row"] = 2 * files + 1
    q["target"] = first_owner
    for d, want in ((1, 0), (2, 1), (5, 1)):
        q["max_depth"] = d
        gpu = _gpu_check(snap, snap.with_handles(q), 5)
        assert (gpu == want).all(), (d, int((gpu != want).sum()))


def test_drive_expand_matches_oracle(drive):
    _expand_matches_oracle(*drive)


def test_drive_full_scale_matches_oracle():
    """Config #2 at its full size (exactly 10,000,000 tuples, seed 2): 1,000,000 checks on the GPU,
    the first 100,000 compared with the oracle."""
    from tools import synth
    g = synth.SynthGraph(dict(synth.DRIVE_10M), threads=16, kind="drive")
    try:
        assert g.n_edges == 10_000_000
        snap = g.snapshot(device=0)
        q = g.queries(1_000_000, seed=2, depth=5)
        gpu = _gpu_check(snap, snap.with_handles(q), 5)
        k = 100_000
        tab = g.oracle_table(q[:k], 5)
        ref = tab.check_batch_reqs(g.oracle_requests(tab, q[:k]), 5, threads=16)
        assert (gpu[:k] == ref).all(), f"{int((gpu[:k] != ref).sum())} mismatches of {k}"
        snap.close()
    finally:
        g.close()


@pytest.mark.parametrize("lanes,n", [(2048, 2 * 2048 - 3), (2048, 2 * 2048 + 1), (2048, 3 * 2048 - 1),
                                     (2048, 4 * 2048 + 5), (256, 1001)])
def test_static_runs_short_match_oracle(powerlaw, monkeypatch, lanes, n):
    """Static tier-0 runs (KETO_T0_DYN=0) on a pinned lane count (KETO_SLOTS): batches of 2 and 3
    requests per lane (runs of 1-3 requests, decisions stored byte by byte), a short final run, and
    runs rounded up to whole groups of 4; every decision equals the oracle's."""
    g, snap = powerlaw
    monkeypatch.setenv("KETO_T0_DYN", "0")
    monkeypatch.setenv("KETO_SLOTS", str(lanes))
    q = g.queries(n, seed=n, depth=5)
    gpu = _gpu_check(snap, snap.with_handles(q), 5)
    tab = g.oracle_table(q, 5)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q), 5, threads=16)
    assert (gpu == ref).all(), f"{int((gpu != ref).sum())} mismatches of {len(q)}"
