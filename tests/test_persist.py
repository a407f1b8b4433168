"""Persisted snapshots (keto_snapshot_save / keto_snapshot_load, persist.cpp; SURVEY 8(f) row 2, the
optional on-disk CSR): a snapshot written to a file and read back answers exactly like the one that
was saved, at the same version, after any writes.  CPU part: host-only snapshots; the loaded
snapshot's statistics, request resolution (row handles, subject ids) and subject strings equal a
clone's of the saved one (both are laid out afresh), and damaged, truncated or foreign files are
refused.  GPU part: checks and expands of loaded snapshots against the SQL oracle after writes
(internal/check/engine.go:36-123, internal/expand/engine.go:33-102,
internal/persistence/sql/relationtuples.go:128-149,200-223), and the power-law graph's decisions
before and after a save/load round trip."""
import os
import random

import numpy as np
import pytest

from tests.engine_util import rows_from_tuples, subj
from tests.randgraph import random_checks, random_expands, random_graph
from tests.test_gpu_lifecycle import _random_write, _row


def _graph_with_writes(seed, device, steps=4):
    """A random graph (wildcards, collisions) built on `device`, with `steps` random write
    transactions applied; returns (snapshot, store, alphabet, ns)."""
    import keto_amd
    from oracle.oracle_sql import SQLStore
    ns, tuples, raw, ps, alph = random_graph(seed, wide=seed % 4 == 3, allow_wildcards=seed % 3 == 0,
                                             allow_poison=False, allow_collisions=seed % 2 == 0)
    names, objs, rels, users = alph
    set_names = list(names)
    names = [n for n in names if n]
    store = SQLStore(ns, tuples, page_size=ps)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), page_size=ps, device=device)
    rng = random.Random(seed)
    if names:
        for _ in range(steps):
            cur = store.tuples()
            ins = [_random_write(rng, names, objs, rels, users, set_names, 0.1) for _ in range(rng.randint(1, 8))]
            dels = [rng.choice(cur) for _ in range(rng.randint(0, 3))] if cur else []
            snap.apply([_row(ns, t) for t in ins], [_row(ns, t) for t in dels])
            for t in ins:
                store.insert(t)
            for t in dels:
                store.delete(t)
    return snap, store, (names, objs, rels, users), ns


@pytest.mark.parametrize("seed", range(16))
def test_round_trip_host(tmp_path, seed):
    import keto_amd
    snap, store, (names, objs, rels, users), ns = _graph_with_writes(seed + 1300, device=-1)
    path = tmp_path / "snap.keto"
    snap.save(path, tag=0xABCDEF0123456789 + seed)
    assert path.exists() and not (tmp_path / "snap.keto.tmp").exists()
    got, tag = keto_amd.Snapshot.load(path, device=-1)
    assert tag == 0xABCDEF0123456789 + seed
    ref = snap.clone(-1)                                   # laid out afresh, like the loaded one
    assert got.version() == snap.version()
    st_got, st_ref = got.stats(), ref.stats()
    st_got.pop("device_bytes")
    st_ref.pop("device_bytes")
    assert st_got == st_ref
    if names:
        checks = random_checks(seed * 41, (names, objs + ["new1", "a0"], rels + ["q"], users + ["w001"]), k=64)
        reqs = [(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in checks]
        reqs = [r for r in reqs if not (r[0] == "" or r[1] == "" or r[2] == "")]   # wildcards need a device overlay
        if reqs:
            try:
                want = ref.resolve_checks(reqs)
            except keto_amd.KetoError:
                want = None
            if want is not None:
                have = got.resolve_checks(reqs)
                assert (have[0] == want[0]).all() and (have[1] == want[1]).all()
    # saving the loaded snapshot gives the same tables again
    path2 = tmp_path / "snap2.keto"
    got.save(path2, tag=7)
    again, tag2 = keto_amd.Snapshot.load(path2, device=-1)
    assert tag2 == 7 and again.stats() == got.stats() and again.version() == got.version()
    for s in (snap, got, ref, again):
        s.close()


def test_power_law_round_trip_host(tmp_path):
    """The generator's graph (CSR load with its string table): every request resolves to the same
    ids on the loaded snapshot as on the saved one."""
    import keto_amd
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 4096), threads=4)
    u = g.unified(threads=4)
    snap = g.snapshot_unified(u, device=-1)
    path = tmp_path / "pl.keto"
    snap.save(path, tag=1)
    got, tag = keto_amd.Snapshot.load(path, device=-1)
    q = g.queries(50_000, seed=5, depth=5, threads=4)
    reqs = g.string_requests(u.names, q, threads=4)
    a, sa = snap.resolve_checks_reqs(reqs, len(q))
    b, sb = got.resolve_checks_reqs(reqs, len(q))
    assert tag == 1 and (sa == sb).all() and (a == b).all()
    assert got.stats() == snap.stats()
    rows = np.arange(snap.stats()["n_rows"], dtype=np.uint32)
    assert (got.row_handles(rows) == snap.row_handles(rows)).all()     # the same arena layout
    # without a string table (keto_snapshot_from_csr, strings == NULL: subject ids name no string)
    bare = g.snapshot(device=-1)
    bare.save(path, tag=2)
    back, tag = keto_amd.Snapshot.load(path, device=-1)
    assert tag == 2 and back.stats() == bare.stats()
    assert (back.row_handles(rows) == bare.row_handles(rows)).all()
    for s in (snap, got, bare, back):
        s.close()
    u.free()
    g.close()


def _small(tmp_path):
    import keto_amd
    ns = [(1, "n"), (2, "m")]
    rows = [(1, "a", "r", "u"), (1, "b", "r", None, 1, "a", "r"), (2, "c", "s", "v")]
    snap = keto_amd.Snapshot.build(ns, rows, device=-1)
    path = tmp_path / "s.keto"
    snap.save(path, tag=3)
    snap.close()
    return path


def test_damaged_files_refused(tmp_path):
    import keto_amd
    path = _small(tmp_path)
    data = path.read_bytes()
    ok, tag = keto_amd.Snapshot.load(path, device=-1)
    assert tag == 3
    ok.close()
    bad = tmp_path / "bad.keto"
    for cut in (0, 10, 64, 100, len(data) - 30, len(data) - 1):        # truncated
        bad.write_bytes(data[:cut])
        with pytest.raises(keto_amd.KetoError) as e:
            keto_amd.Snapshot.load(bad, device=-1)
        assert e.value.code == -1
    for pos in range(64, len(data), max(1, (len(data) - 64) // 40)):  # one flipped byte anywhere past the header
        flip = bytearray(data)
        flip[pos] ^= 0x5A
        bad.write_bytes(bytes(flip))
        try:
            s, _ = keto_amd.Snapshot.load(bad, device=-1)
        except keto_amd.KetoError as x:
            assert x.code == -1
        else:                                            # a section's padding bytes carry no checksum
            s.close()
    import struct
    huge = bytearray(data)
    struct.pack_into("<Q", huge, 64 + 8, (1 << 64) - 8)  # a section's byte count near 2^64
    bad.write_bytes(bytes(huge))
    with pytest.raises(keto_amd.KetoError) as e:
        keto_amd.Snapshot.load(bad, device=-1)
    assert e.value.code == -1
    flip = bytearray(data)
    flip[0] ^= 1                                         # magic
    bad.write_bytes(bytes(flip))
    with pytest.raises(keto_amd.KetoError):
        keto_amd.Snapshot.load(bad, device=-1)
    flip = bytearray(data)
    flip[8] = 99                                         # format
    bad.write_bytes(bytes(flip))
    with pytest.raises(keto_amd.KetoError) as e:
        keto_amd.Snapshot.load(bad, device=-1)
    assert "format" in str(e.value)
    with pytest.raises(keto_amd.KetoError):
        keto_amd.Snapshot.load(tmp_path / "missing.keto", device=-1)


def test_save_refuses_parts_and_bad_paths(tmp_path):
    import keto_amd
    snap = keto_amd.Snapshot.build([(1, "n")], [(1, "a", "r", "u")], device=-1)
    with pytest.raises(keto_amd.KetoError):
        snap.save(tmp_path / "no_such_dir" / "x.keto")
    snap.close()


@pytest.mark.gpu
def test_save_refuses_parts(tmp_path):
    import keto_amd
    part = keto_amd.Snapshot.build([(1, "n")], [(1, "a", "r", "u")], device=-1).upload_part(0, 2, 0)
    with pytest.raises(keto_amd.KetoError):
        part.save(tmp_path / "p.keto")
    part.close()


def _want_tree(store, s, d, g):
    from oracle.oracle_sql import ExpandEngine, NotFoundError
    try:
        tr = ExpandEngine(store, g).build_tree(s, d)
        return ("tree", tr.to_json()) if tr is not None else ("nil", None)
    except NotFoundError:
        return ("error", None)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(16))
def test_loaded_snapshot_matches_oracle(tmp_path, seed):
    """Saved after writes on the GPU snapshot, loaded onto the GPU, written to again: checks and
    expands equal the SQL oracle's at every step."""
    import keto_amd
    from oracle.oracle_sql import CheckEngine
    snap, store, (names, objs, rels, users), ns = _graph_with_writes(seed + 1500, device=0)
    if not names:
        snap.close()
        pytest.skip("only a namespace named ''")
    path = tmp_path / "g.keto"
    snap.save(path, tag=seed)
    got, tag = keto_amd.Snapshot.load(path, device=0)
    assert tag == seed and got.version() == snap.version()
    snap.close()
    rng = random.Random(seed + 77)
    set_names = list(names)
    for step in range(3):
        if step:
            cur = store.tuples()
            ins = [_random_write(rng, names, objs, rels, users, set_names, 0.1) for _ in range(rng.randint(1, 6))]
            dels = [rng.choice(cur) for _ in range(rng.randint(0, 2))] if cur else []
            got.apply([_row(ns, t) for t in ins], [_row(ns, t) for t in dels])
            for t in ins:
                store.insert(t)
            for t in dels:
                store.delete(t)
        checks = random_checks(seed * 53 + step, (names, objs + ["new1", "a0"], rels + ["q"], users + ["w001"]), k=48)
        for g in sorted({c[2] for c in checks}):
            grp = [c for c in checks if c[2] == g]
            out = got.check_batch([(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in grp], g)[0]
            for (t, d, _), a in zip(grp, out):
                assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, step, t, d, g)
        exps = random_expands(seed * 23 + step, (names, objs + ["new3"], rels + ["q"], users), k=8)
        for g in sorted({e[2] for e in exps}):
            grp = [e for e in exps if e[2] == g]
            res = got.expand_batch([(subj(s), d) for s, d, _ in grp], g)
            for (s, d, _), (st, js) in zip(grp, res):
                have = {0: "tree", 1: "nil", 2: "error"}[st]
                assert (have, js) == _want_tree(store, s, d, g), (seed, step, s, d, g)
    got.close()


@pytest.mark.gpu
def test_power_law_decisions_survive_round_trip(tmp_path):
    import keto_amd
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 256), threads=8)
    snap = g.snapshot(device=0)
    q = g.queries(1 << 20, seed=9, depth=5, threads=8)
    want = snap.check_batch_ids(snap.with_handles(q), 5)
    path = tmp_path / "pl.keto"
    snap.save(path)
    got, _ = keto_amd.Snapshot.load(path, device=0)
    have = got.check_batch_ids(got.with_handles(q), 5)
    assert np.array_equal(np.asarray(want), np.asarray(have))
    for s in (snap, got):
        s.close()
    g.close()


def test_writes_staged_beside_readers_host():
    """keto_snapshot_apply stages a transaction under the shared lock and commits under the exclusive
    one (capi.cpp): readers resolving requests at the same time keep working and see versions only
    move forward, and every write lands.  Host-only snapshot, one writer thread, two reader threads."""
    import threading
    import keto_amd
    ns = [(1, "doc"), (2, "grp")]
    rows = [(1, f"d{i}", "view", None, 2, f"g{i % 7}", "member") for i in range(200)]
    rows += [(2, f"g{j}", "member", f"u{j}") for j in range(7)]
    snap = keto_amd.Snapshot.build(ns, rows, device=-1)
    reqs = [("doc", f"d{i}", "view", ("id", f"u{i % 7}"), 0) for i in range(200)]
    reqs += [("doc", "dnew", "view", ("id", "unew"), 0), ("grp", "gnew", "member", ("id", "unew"), 0)]
    stop = threading.Event()
    errors = []

    def writer():
        try:
            for k in range(150):
                t = [(1, "dnew", "view", "unew"), (2, "gnew", "member", "unew")]
                snap.apply(inserts=t)
                snap.apply(deletes=t)
        except Exception as e:            # noqa: BLE001 -- reported below
            errors.append(e)
        finally:
            stop.set()

    def reader():
        try:
            seen = 0
            while not stop.is_set():
                v0 = snap.version()
                out, st = snap.resolve_checks(reqs)
                assert (st == 0).all()
                assert v0 >= seen                     # versions only move forward
                seen = v0
                # the build's rows keep their handles through every write
                assert (out[:200]["row"] != 0xFFFFFFFF).all()
        except Exception as e:            # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=writer)] + [threading.Thread(target=reader) for _ in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors
    assert snap.version() == 300
    snap.close()


def _mix64(x):
    M = (1 << 64) - 1
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & M
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & M
    return x ^ (x >> 31)


def _section_hash(data: bytes) -> int:
    """persist.cpp section_hash restated (1-MiB blocks, four lanes per 32 B, folded in order)."""
    import struct
    M = (1 << 64) - 1
    B = 1 << 20
    hs = []
    for k in range(0, max(1, -(-len(data) // B))):
        p = data[k * B:(k + 1) * B]
        n = len(p)
        h = (k ^ ((n * 0x9E3779B97F4A7C15) & M)) & M
        i = 0
        while i + 32 <= n:
            a, b, c, d = struct.unpack_from("<4Q", p, i)
            h = (_mix64(h ^ a) + _mix64(b ^ 0x632BE59BD9B4E019) + _mix64((c + h) & M) + _mix64(d ^ (h >> 17))) & M
            i += 32
        while i + 8 <= n:
            h = _mix64(h ^ struct.unpack_from("<Q", p, i)[0])
            i += 8
        t = int.from_bytes(p[i:] + b"\0" * (8 - (n - i)), "little") if i < n else 0
        hs.append(_mix64(h ^ t ^ 0xD6E8FEB86659FD93))
    if not data:
        hs = []
    h = _mix64(len(data) + 1)
    for x in hs:
        h = (_mix64(h ^ x) * 0x94D049BB133111EB) & M
    return h


def test_crafted_files_refused(tmp_path):
    """Files whose checksums are right but whose contents are not: the ABI field of a newer library,
    and a scalars section (page_size 0, then an empty-string id past the string table) rewritten with
    a recomputed section hash.  Both fail with KETO_E_INVALID before anything indexes with them
    (persist.cpp trusted these fields)."""
    import struct
    import keto_amd
    path = _small(tmp_path)
    data = bytearray(path.read_bytes())
    bad = tmp_path / "crafted.keto"
    newer = bytearray(data)
    struct.pack_into("<I", newer, 12, 99)                # the header's abi
    bad.write_bytes(bytes(newer))
    with pytest.raises(keto_amd.KetoError) as e:
        keto_amd.Snapshot.load(bad, device=-1)
    assert "ABI" in str(e.value)
    sid, nbytes, h = struct.unpack_from("<3Q", data, 64)  # the first section: the scalars
    assert sid == 1 and _section_hash(bytes(data[88:88 + nbytes])) == h   # the restated hash is the library's
    for field, value in ((0, 0), (1, 0x7FFFFFF0)):       # page_size = 0; empty_str far past the strings
        crafted = bytearray(data)
        struct.pack_into("<I", crafted, 88 + 4 * field, value)
        struct.pack_into("<Q", crafted, 64 + 16, _section_hash(bytes(crafted[88:88 + nbytes])))
        bad.write_bytes(bytes(crafted))
        with pytest.raises(keto_amd.KetoError) as e:
            keto_amd.Snapshot.load(bad, device=-1)
        assert e.value.code == -1 and "bad scalars" in str(e.value), e.value
