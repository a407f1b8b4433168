"""Requests resolved on the GPU (keto_check_batch_packed, keto_amd/csrc/resolve_dev.hip): the same
decisions and statuses as keto_check_batch (host resolution, resolve.cpp) and as the SQL oracle
(whereQuery, internal/persistence/sql/relationtuples.go:178-198; check/engine.go:36-123) -- on
quirk-heavy random graphs (unknown namespaces and strings, subject sets, wildcard queries left to the
host, collisions, poisoned rows), on strings longer than a slot's 11 inline bytes that share their
first 11 bytes, after writes that add strings and rows, and on the power-law graph built from its
string tuples."""
import random

import numpy as np
import pytest

from oracle.oracle_sql import CheckEngine, RelationTuple, SQLStore, SubjectID, SubjectSet
from tests.engine_util import rows_from_tuples, subj
from tests.randgraph import random_checks, random_store

pytestmark = pytest.mark.gpu


def _same_as_host(snap, reqs, g):
    from keto_amd.capi import pack_requests
    want, want_st = snap.check_batch(reqs, g)
    blob, packed = pack_requests(reqs)
    got, st = snap.check_batch_packed(blob, packed, g)
    assert (got == want).all(), [(r, int(a), int(b)) for r, a, b in zip(reqs, got, want) if a != b][:5]
    assert (st == want_st).all(), [(r, int(a), int(b)) for r, a, b in zip(reqs, st, want_st) if a != b][:5]
    return got


@pytest.mark.parametrize("seed", range(5000, 5060))
def test_random_graphs_packed_equals_host(seed):
    import keto_amd
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=seed % 4 == 0)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples, raw), page_size=ps, device=0)
    checks = random_checks(seed, alph, k=80)
    for g in sorted({c[2] for c in checks}):
        grp = [c for c in checks if c[2] == g]
        reqs = [(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in grp]
        got = _same_as_host(snap, reqs, g)
        for (t, d, _), a in zip(grp, got):
            assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, t, d, g)
    snap.close()


def test_long_strings_sharing_a_prefix():
    """Objects, relations and subject ids longer than a string slot's 11 inline bytes, many sharing
    their first 11 bytes (the slot matches, the device compares the rest), and requests naming
    strings the snapshot does not hold but whose prefix it does."""
    import keto_amd
    rng = random.Random(7)
    ns = [(1, "files"), (2, "groups")]
    pre = "0123456789abcdef"
    objs = [pre + f"/doc/{i:05d}" for i in range(60)] + ["short"]
    users = [pre + f"user-{i}" * (1 + i % 5) for i in range(40)] + ["u"]
    grps = [pre + f"g{i:03d}" for i in range(20)]
    tuples = []
    for _ in range(600):
        if rng.random() < 0.6:
            tuples.append(RelationTuple("files", rng.choice(objs), "view", SubjectID(rng.choice(users))))
        elif rng.random() < 0.5:
            tuples.append(RelationTuple("files", rng.choice(objs), "view", SubjectSet("groups", rng.choice(grps), "member")))
        else:
            tuples.append(RelationTuple("groups", rng.choice(grps), "member", SubjectID(rng.choice(users))))
    store = SQLStore(ns, tuples)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), device=0)
    reqs, exp = [], []
    for _ in range(400):
        o = rng.choice(objs + [pre + "/doc/99999", pre])
        if rng.random() < 0.8:
            s = rng.choice(users + [pre + "user-", pre + "nobody"])
            reqs.append(("files", o, "view", ("id", s), 0))
            exp.append(RelationTuple("files", o, "view", SubjectID(s)))
        else:
            gname = rng.choice(grps + [pre + "g999"])
            reqs.append(("files", o, "view", ("set", "groups", gname, "member"), 0))
            exp.append(RelationTuple("files", o, "view", SubjectSet("groups", gname, "member")))
    got = _same_as_host(snap, reqs, 5)
    for t, a in zip(exp, got):
        assert bool(a) == CheckEngine(store, 5).subject_is_allowed(t, 0), t
    snap.close()


@pytest.mark.parametrize("seed", range(6))
def test_packed_after_writes(seed):
    """Writes add strings and rows the build's indexes do not hold (added_str, row_of): the build's
    device indexes stay, the tables of added strings and rows are rebuilt for each new version, and
    every version resolves exactly like the host."""
    import keto_amd
    from tests.test_gpu_lifecycle import _random_write, _row
    from tests.randgraph import random_graph
    ns, tuples, raw, ps, alph = random_graph(seed + 700, allow_poison=False)
    names, objs, rels, users = alph
    names = [n for n in names if n]
    if not names:
        pytest.skip("only a namespace named ''")
    store = SQLStore(ns, tuples, page_size=ps)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), page_size=ps, device=0)
    rng = random.Random(seed)
    # long names (past a slot's 11 inline bytes): an added string is verified against its own bytes
    objs = objs + ["an_object_name_longer_than_a_slot"]
    users = users + ["a_subject_id_longer_than_a_slot_0", "a_subject_id_longer_than_a_slot_1"]
    for step in range(8):
        ins = [_random_write(rng, names, objs, rels, users) for _ in range(rng.randint(2, 10))]
        snap.apply([_row(ns, t) for t in ins], [])
        for t in ins:
            store.insert(t)
        checks = random_checks(seed * 5 + step, (names, objs + ["new1", "new7", "a0", "Z"], rels + ["q"],
                                                 users + ["w001", "a", "zz"]), k=60)
        for g in sorted({c[2] for c in checks}):
            grp = [c for c in checks if c[2] == g]
            reqs = [(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in grp]
            got = _same_as_host(snap, reqs, g)
            for (t, d, _), a in zip(grp, got):
                assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, step, t, d)
    snap.close()


def test_powerlaw_packed_matches_host():
    """200,000 named requests on the power-law graph (1/256 scale) built from its string tuples,
    packed by the generator's packer, against keto_check_batch on the same snapshot."""
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 256), threads=16)
    st = g.string_tuples(seed=5)
    snap, _ = g.snapshot_from_strings(st, device=0)
    q = g.queries(200_000, seed=11, depth=5)
    arr = g.string_requests(st, q)
    want, want_st = snap.check_batch_reqs(arr, len(q), 5)
    blob, rec, used = g.pack_requests(arr, len(q))
    got, got_st = snap.check_batch_packed(blob.array[:used], rec.array, 5, n=len(q))
    assert (got == want).all() and (got_st == want_st).all()
    assert 0.05 < got.mean() < 0.95
    snap.close()
    g.close()


@pytest.mark.parametrize("layout", ["in_order", "shuffled"])
def test_packed_pipelined_pieces(layout, monkeypatch):
    """A batch of several pieces (KETO_PACKED_CHUNK) is uploaded piece by piece while earlier pieces
    are resolved and checked (resolve_dev.hip, device_check_packed).  In request order each piece's
    strings are in its window; shuffled records (fields anywhere in the blob) are found by the kernel
    and the batch is resolved and checked again over the whole blob.  Both equal keto_check_batch;
    a bounds error in the last piece still fails the call before any output is written."""
    from keto_amd.capi import KetoError
    from tools import synth
    monkeypatch.setenv("KETO_PACKED_CHUNK", "4096")
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 1024), threads=16)
    st = g.string_tuples(seed=5)
    snap, _ = g.snapshot_from_strings(st, device=0)
    q = g.queries(50_000, seed=13, depth=5)
    arr = g.string_requests(st, q)
    want, want_st = snap.check_batch_reqs(arr, len(q), 5)
    blob, rec, used = g.pack_requests(arr, len(q))
    b, r = blob.array[:used], rec.array[:len(q)]          # (pinned: the pieces' copies are asynchronous)
    if layout == "shuffled":                 # the same records, the blob's strings in another order
        perm = np.random.default_rng(3).permutation(len(q))
        lens = r["len"].astype(np.int64).sum(axis=1)
        parts, off, new_off = [], 0, np.zeros(len(q), dtype=np.uint32)
        for i in perm:
            parts.append(b[r["off"][i]:r["off"][i] + lens[i]])
            new_off[i] = off
            off += lens[i]
        b = np.concatenate(parts)
        r = r.copy()
        r["off"] = new_off
    got, got_st = snap.check_batch_packed(b, r, 5, n=len(q))
    assert (got == want).all() and (got_st == want_st).all()
    bad = r.copy()
    bad["off"][len(q) - 3] = len(b) - 1
    out = np.full(len(q), 7, dtype=np.uint8)
    with pytest.raises(KetoError, match=f"request {len(q) - 3}'s fields lie outside the blob"):
        snap.check_batch_packed(b, bad, 5, n=len(q), allowed=out)
    assert (out == 7).all()
    snap.close()
    g.close()


def test_packed_empty_batch_and_bad_offsets():
    import keto_amd
    from keto_amd.capi import CHECK_PACKED_DTYPE, KetoError, pack_requests
    snap = keto_amd.Snapshot.build([(1, "n")], [(1, "a", "r", "u")], device=0)
    got, st = snap.check_batch_packed(b"", np.zeros(0, dtype=CHECK_PACKED_DTYPE), 5)
    assert len(got) == 0
    blob, packed = pack_requests([("n", "a", "r", ("id", "u"), 0)])
    packed["off"][0] = 1000
    with pytest.raises(KetoError):
        snap.check_batch_packed(blob, packed, 5)
    # the bounds are checked on the device (resolve_packed): the first request past the blob is named,
    # no field of it is read, nothing is written to the outputs, and the snapshot answers afterwards
    reqs = [("n", "a", "r", ("id", "u"), 0), ("n", "a", "r", ("id", "x"), 0), ("n", "", "r", ("id", "u"), 0),
            ("n", "a", "r", ("set", "n", "a", "r"), 0)]
    blob, packed = pack_requests(reqs)
    for bad, (field, value) in ((1, ("off", len(blob) - 1)), (3, ("len", 0xFFFF))):
        p = packed.copy()
        if field == "off":
            p["off"][bad] = value
        else:
            p["len"][bad][5] = value
        allowed = np.full(len(reqs), 7, dtype=np.uint8)
        with pytest.raises(KetoError, match=f"request {bad}'s fields lie outside the blob"):
            snap.check_batch_packed(blob, p, 5, allowed=allowed)
        assert (allowed == 7).all()
    got, st = snap.check_batch_packed(blob, packed, 5)                    # (request 2: a wildcard, host)
    want, want_st = snap.check_batch(reqs, 5)
    assert (got == want).all() and (st == want_st).all() and got[0] == 1 and got[1] == 0
    snap.close()


def test_packed_batches_concurrent_with_writes():
    """Several threads run packed batches on one snapshot (its shared lock only) while writes add
    strings and rows: the device resolver's state is created once and its per-version tables are
    rebuilt under its own lock, never under a running resolve kernel (resolve_dev.hip rdev_get /
    rdev_refresh).  The requests name rows and strings the writes never touch, so every batch must
    decide exactly as before the first write; the written rows are checked after."""
    import threading
    import keto_amd
    from keto_amd.capi import pack_requests
    rng = random.Random(11)
    ns = [(1, "docs"), (2, "groups")]
    tuples = []
    for _ in range(3000):
        if rng.random() < 0.5:
            tuples.append(RelationTuple("docs", f"d{rng.randrange(400)}", "view", SubjectID(f"u{rng.randrange(300)}")))
        elif rng.random() < 0.5:
            tuples.append(RelationTuple("docs", f"d{rng.randrange(400)}", "view", SubjectSet("groups", f"g{rng.randrange(60)}", "member")))
        else:
            tuples.append(RelationTuple("groups", f"g{rng.randrange(60)}", "member", SubjectID(f"u{rng.randrange(300)}")))
    store = SQLStore(ns, tuples)
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), device=0)
    reqs = [("docs", f"d{rng.randrange(420)}", "view", ("id", f"u{rng.randrange(320)}"), 0) for _ in range(4000)]
    blob, packed = pack_requests(reqs)
    want, want_st = snap.check_batch(reqs, 5)
    errors, stop = [], threading.Event()

    def reader():
        try:
            while not stop.is_set():
                got, st = snap.check_batch_packed(blob, packed, 5)
                if not ((got == want).all() and (st == want_st).all()):
                    errors.append(int((got != want).sum()))
        except Exception as e:          # noqa: BLE001 -- reported below
            errors.append(repr(e))

    ts = [threading.Thread(target=reader) for _ in range(4)]
    for t in ts:
        t.start()
    written = []
    for k in range(40):
        ins = [RelationTuple("docs", f"w{k}_{j}", "view", SubjectID(f"wu{k}_{j}_with_a_long_suffix")) for j in range(5)]
        snap.apply(rows_from_tuples(ns, ins), [])
        written += ins
    stop.set()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[:5]
    for t in written:
        store.insert(t)
    wreq = [(t.namespace, t.object, t.relation, ("id", t.subject.id), 0) for t in written[::7]]
    got = _same_as_host(snap, wreq, 5)
    assert got.all()
    snap.close()


def test_packed_batches_in_flight_equal_sync(monkeypatch):
    """Packed batches of one piece keep up to KETO_PACKED_SLOTS in flight per snapshot (resolve_dev.hip
    device_check_packed_async): one batch's upload and resolution run while another's check does, and
    the check is enqueued without a host round trip.  Eight threads at once with 1, 2 and 4 slots,
    and the batch redone on the synchronous path when the check needs tier 2 (forced here by the test
    hook), all decide like keto_check_batch (host resolution) on the power-law graph."""
    import threading
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 256), threads=16)
    st = g.string_tuples(seed=5)
    snap, _ = g.snapshot_from_strings(st, device=0)
    q = g.queries(65_536, seed=13, depth=5)
    arr = g.string_requests(st, q)
    want, want_st = snap.check_batch_reqs(arr, len(q), 5)
    blob, rec, used = g.pack_requests(arr, len(q))
    for env in ({"KETO_PACKED_SLOTS": "0"}, {"KETO_PACKED_SLOTS": "1"}, {}, {"KETO_PACKED_SLOTS": "4"},
                {"KETO_TEST_PACKED_FALLBACK": "1"}):
        for k in ("KETO_PACKED_SLOTS", "KETO_TEST_PACKED_FALLBACK"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        errors = []

        def reader():
            try:
                for _ in range(6):
                    got, gst = snap.check_batch_packed(blob.array[:used], rec.array, 5, n=len(q))
                    if not ((got == want).all() and (gst == want_st).all()):
                        errors.append(int((got != want).sum()))
            except Exception as e:      # noqa: BLE001 -- reported below
                errors.append(repr(e))

        ts = [threading.Thread(target=reader) for _ in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in ts)
        assert not errors, (env, errors[:5])
    snap.close()
    g.close()


def test_packed_tier_overflow_in_flight_matches_oracle():
    """The hub graph of tests/test_gpu_overflow.py through packed batches: maps outgrow tier 0, so the
    in-flight check runs tier 1 behind tier 0 without reading its count back; every global max-depth
    from 1 to 7 (max-depth > 9 takes the synchronous path) against the SQL oracle."""
    import keto_amd
    from tests.test_gpu_overflow import _graph
    ns, tuples = _graph()
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), device=0)
    store = SQLStore(ns, tuples)
    rng = random.Random(5)
    for gmd in range(1, 8):
        reqs, items = [], []
        for _ in range(200):
            obj = rng.choice(["root", "hub", f"x{rng.randrange(150):04d}"])
            sub = SubjectID(f"u{rng.randrange(2000):05d}") if rng.random() < 0.8 else SubjectSet("n", f"y{rng.randrange(150):04d}", "r")
            d = rng.choice([0, 1, 2, 3, 5, 8])
            items.append((RelationTuple("n", obj, "r", sub), d))
            reqs.append(("n", obj, "r", subj(sub), d))
        got = _same_as_host(snap, reqs, gmd)
        eng = CheckEngine(store, gmd)
        bad = [(t, d) for (t, d), a in zip(items, got) if bool(a) != eng.subject_is_allowed(t, d)]
        assert not bad, (gmd, bad[:5])
    snap.close()
