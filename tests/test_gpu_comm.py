"""The library's own multi-GPU layer (keto_amd/csrc/comm.cpp: keto_comm_*, keto_check_batch_sharded,
keto_check_batch_routed, keto_comm_close_filters) on the box's one GPU.

* RCCL, as a one-rank communicator: the collectives run through RCCL for real.
* The local transport (keto_comm_init_local) with P = 2 and 3 ranks, each a thread of this process
  with its own stream and its own part on the one GPU: requests cross parts, migrating searches
  travel as continuation records between parts, the filter exchange converges across parts.  Every
  decision must equal the replicated snapshot's and the SQL oracle's
  (internal/check/engine.go:36-123).
* Error agreement: a failure on one rank (an injected one at every local phase, a NULL argument, a
  request it cannot route) makes every rank return the same code instead of leaving its peers
  waiting, and the communicator stays usable afterwards.
The same exchanges over gloo (multi.py) are tests/test_multi_cpu.py."""
import ctypes as C
import os
import threading

import pytest

from oracle.oracle_sql import CheckEngine
from tests.engine_util import rows_from_tuples, subj
from tests.randgraph import poisoned_wildcard_case, random_checks, random_store

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from keto_amd.capi import Comm
    c = Comm(Comm.make_id(), 1, 0, 0)
    yield c
    c.close()


@pytest.fixture(autouse=True)
def _short_timeout(monkeypatch):
    # a rank that never arrives fails its peers' calls after 60 s instead of hanging the run
    monkeypatch.setenv("KETO_COMM_TIMEOUT_MS", "60000")


def _reqs(seed, alph):
    checks = random_checks(seed, alph, k=48)
    return [(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in checks], checks


def _local_comms(P):
    from keto_amd.capi import Comm
    cid = os.urandom(32)
    return [Comm(cid, P, r, 0, local=True) for r in range(P)]


def _ranks(P, fn):
    """fn(rank) on P threads at once (a collective call per rank); [(ok, result or exception)]."""
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
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts), "a rank is still waiting"
    return res


def _ok(res):
    bad = [(r, v) for r, (ok, v) in enumerate(res) if not ok]
    assert not bad, bad
    return [v for _, v in res]


def _parts(ns, rows, ps, P, mode):
    import keto_amd
    return [keto_amd.Snapshot.build(ns, rows, page_size=ps, device=-1).upload_part(r, P, 0, mode=mode) for r in range(P)]


@pytest.mark.parametrize("seed", range(4000, 4030))
def test_sharded_and_routed_match_oracle(comm, seed):
    import keto_amd
    from keto_amd.capi import PART_MIGRATE, PART_SHARED, KetoError
    store, ns, tuples, raw, ps, alph = random_store(seed)
    rows = rows_from_tuples(ns, tuples, raw)
    full = keto_amd.Snapshot.build(ns, rows, page_size=ps, device=0)
    reqs, checks = _reqs(seed, alph)
    g = 5
    want, want_st = full.check_batch(reqs, g)
    got, st = comm.check_batch_sharded(full, reqs, g)
    assert (got == want).all() and (st == want_st).all(), seed
    for (t, d, _), a in zip(checks, got):
        assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, t, d)
    for mode in (PART_SHARED, PART_MIGRATE):
        part = keto_amd.Snapshot.build(ns, rows, page_size=ps, device=-1).upload_part(0, 1, 0, mode=mode)
        if mode == PART_MIGRATE:
            comm.close_filters(part)
        try:
            got_p, st_p = comm.check_batch_routed(part, reqs, g)
        except KetoError as e:                      # a wildcard request no stored set uses: not routable
            assert "wildcard" in str(e), e
            continue
        assert (got_p == want).all() and (st_p == want_st).all(), (seed, mode)
        part.close()
    full.close()


def test_routed_powerlaw_matches_replicated(comm):
    """The power-law generator at 1/256 scale, built from its string tuples: 200,000 named requests
    through the sharded path on the replicated snapshot and the routed path on a one-part shared and
    migrating partition, against keto_check_batch on the replicated snapshot."""
    from keto_amd.capi import PART_MIGRATE, PART_SHARED
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 256), threads=16)
    st = g.string_tuples(seed=5)
    full, _ = g.snapshot_from_strings(st, device=0)
    q = g.queries(200_000, seed=11, depth=5)
    arr = g.string_requests(st, q)
    want, want_st = full.check_batch_reqs(arr, len(q), 5)
    got, got_st = comm.check_batch_sharded(full, arr, 5, n=len(q))
    assert (got == want).all() and (got_st == want_st).all()
    for mode in (PART_SHARED, PART_MIGRATE):
        part, _ = g.snapshot_from_strings(st, device=-1)
        part.upload_part(0, 1, 0, mode=mode)
        if mode == PART_MIGRATE:
            comm.close_filters(part)
        got, got_st = comm.check_batch_routed(part, arr, 5, n=len(q))
        assert (got == want).all() and (got_st == want_st).all(), mode
        part.close()
    full.close()
    g.close()


# ------------------------------------------------------------------ local transport, P > 1
@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("seed", range(4100, 4120))
def test_local_ranks_match_oracle(P, seed):
    """P ranks on one GPU over the local transport: sharded on a shared replicated snapshot, routed on
    a shared-rows and a migrating partition (each rank its own part and its own batch; the last
    rank's batch is empty on odd seeds), every decision against the replicated snapshot and the SQL
    oracle."""
    import keto_amd
    from keto_amd.capi import PART_MIGRATE, PART_SHARED
    store, ns, tuples, raw, ps, alph = random_store(seed)
    rows = rows_from_tuples(ns, tuples, raw)
    full = keto_amd.Snapshot.build(ns, rows, page_size=ps, device=0)
    reqs, checks = _reqs(seed, alph)
    g = 5
    want, want_st = full.check_batch(reqs, g)
    for (t, d, _), a in zip(checks, want):
        assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, t, d)
    comms = _local_comms(P)
    for r, (got, st) in enumerate(_ok(_ranks(P, lambda r: comms[r].check_batch_sharded(full, reqs, g)))):
        assert (got == want).all() and (st == want_st).all(), (seed, r)
    ranks = P - (seed % 2)                          # odd seeds: the last rank passes no request
    for mode in (PART_SHARED, PART_MIGRATE):
        # wildcard queries no stored set uses: answered by the requesting shared-rows part; on a
        # migrating partition as one request per matching row (and, in the row a failing page cuts,
        # one per top-level tuple before the cut)
        mine = [list(range(r, len(reqs), ranks)) if r < ranks else [] for r in range(P)]
        parts = _parts(ns, rows, ps, P, mode)
        if mode == PART_MIGRATE:
            _ok(_ranks(P, lambda r: comms[r].close_filters(parts[r])))
        res = _ok(_ranks(P, lambda r: comms[r].check_batch_routed(parts[r], [reqs[i] for i in mine[r]], g)))
        for r, (got, st) in enumerate(res):
            for k, i in enumerate(mine[r]):
                assert got[k] == want[i] and st[k] == want_st[i], (seed, mode, r, reqs[i])
        for p in parts:
            p.close()
    for c in comms:
        c.close()
    full.close()


@pytest.mark.parametrize("P", [1, 2, 3])
@pytest.mark.parametrize("seed", range(4500, 4516))
def test_local_migrating_wildcard_over_failing_pages(P, seed):
    """Wildcard queries whose rows hold failing pages on a migrating partition: the query reads its
    rows' tuples in ORDER BY order a page at a time and stops at the first page that fails toInternal
    (relationtuples.go:64-71,250-277; engine.go:98-100), so the row the failing page cuts is read only
    in part.  Every decision (named and packed) against the replicated snapshot and the SQL oracle."""
    import keto_amd
    from keto_amd.capi import PART_MIGRATE, pack_requests
    store, ns, tuples, raw, ps, reqs, checks = poisoned_wildcard_case(seed)
    rows = rows_from_tuples(ns, tuples, raw)
    g = 5
    full = keto_amd.Snapshot.build(ns, rows, page_size=ps, device=0)
    want, want_st = full.check_batch(reqs, g)
    for (t, d), a in zip(checks, want):
        assert bool(a) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, t, d)
    mine = [list(range(r, len(reqs), P)) for r in range(P)]
    comms = _local_comms(P)
    parts = _parts(ns, rows, ps, P, PART_MIGRATE)
    _ok(_ranks(P, lambda r: comms[r].close_filters(parts[r])))
    named = _ok(_ranks(P, lambda r: comms[r].check_batch_routed(parts[r], [reqs[i] for i in mine[r]], g)))
    packed = [pack_requests([reqs[i] for i in m]) for m in mine]
    pk = _ok(_ranks(P, lambda r: comms[r].check_batch_routed_packed(parts[r], packed[r][0], packed[r][1], g)))
    for r in range(P):
        for k, i in enumerate(mine[r]):
            assert named[r][0][k] == want[i] and named[r][1][k] == want_st[i], (seed, P, r, reqs[i])
            assert pk[r][0][k] == want[i] and pk[r][1][k] == want_st[i], (seed, P, r, reqs[i])
    for p in parts:
        p.close()
    for c in comms:
        c.close()
    full.close()


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("seed", range(4300, 4308))
def test_local_routed_packed_equals_named(P, seed):
    """keto_check_batch_routed_packed (each rank's batch packed and resolved on its device) against
    keto_check_batch_routed (resolved on host threads) on quirk-heavy random graphs, shared-rows and
    migrating parts: the same decisions and statuses for every request -- unknown namespaces and
    strings, subject sets, wildcard queries (left to the host by the device) -- and both equal the SQL
    oracle (internal/check/engine.go:36-123, relationtuples.go:178-198)."""
    import keto_amd
    from keto_amd.capi import PART_MIGRATE, PART_SHARED, pack_requests
    store, ns, tuples, raw, ps, alph = random_store(seed)
    rows = rows_from_tuples(ns, tuples, raw)
    reqs, checks = _reqs(seed, alph)
    g = 5
    mine = [list(range(r, len(reqs), P)) for r in range(P)]
    if seed % 2:
        mine[-1] = []                                   # the last rank passes no request
    packed = [pack_requests([reqs[i] for i in m]) for m in mine]
    comms = _local_comms(P)
    for mode in (PART_SHARED, PART_MIGRATE):
        parts = _parts(ns, rows, ps, P, mode)
        if mode == PART_MIGRATE:
            _ok(_ranks(P, lambda r: comms[r].close_filters(parts[r])))
        named = _ok(_ranks(P, lambda r: comms[r].check_batch_routed(parts[r], [reqs[i] for i in mine[r]], g)))
        pk = _ok(_ranks(P, lambda r: comms[r].check_batch_routed_packed(parts[r], packed[r][0], packed[r][1], g)))
        for r, ((a, st), vp) in enumerate(zip(named, pk)):
            assert (vp[0] == a).all() and (vp[1] == st).all(), (seed, mode, r)
            for k, i in enumerate(mine[r]):
                t, d, _ = checks[i]
                assert bool(a[k]) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, mode, t, d)
        for p in parts:
            p.close()
    for c in comms:
        c.close()


@pytest.fixture(scope="module")
def powerlaw_strings():
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 256), threads=16)
    st = g.string_tuples(seed=5)
    full, _ = g.snapshot_from_strings(st, device=0)
    q = g.queries(240_000, seed=12, depth=5)
    arr = g.string_requests(st, q)
    want, want_st = full.check_batch_reqs(arr, len(q), 5)
    yield g, st, full, arr, len(q), want, want_st
    full.close()
    g.close()


def _slice(arr, lo, hi):
    from keto_amd.capi import KCheckReq
    return (KCheckReq * max(1, hi - lo)).from_address(C.addressof(arr) + lo * C.sizeof(KCheckReq))


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("mode", ["shared", "migrate"])
def test_local_routed_powerlaw_matches_replicated(powerlaw_strings, P, mode):
    """The power-law graph (1/256 scale, from string tuples) on P parts over the local transport: each
    rank passes its own 240,000 / P named requests, most of which belong to other parts; on the
    migrating partition searches cross parts as records (many rounds).  Decisions equal the
    replicated snapshot's."""
    from keto_amd.capi import PART_MIGRATE, PART_SHARED
    g, st, full, arr, n, want, want_st = powerlaw_strings
    m = PART_MIGRATE if mode == "migrate" else PART_SHARED
    parts = []
    for r in range(P):
        part, _ = g.snapshot_from_strings(st, device=-1)
        parts.append(part.upload_part(r, P, 0, mode=m))
    comms = _local_comms(P)
    if m == PART_MIGRATE:
        rounds = _ok(_ranks(P, lambda r: comms[r].close_filters(parts[r])))
        assert len(set(rounds)) == 1 and rounds[0] >= 1
    bounds = [(r * n // P, (r + 1) * n // P) for r in range(P)]
    res = _ok(_ranks(P, lambda r: comms[r].check_batch_routed(parts[r], _slice(arr, *bounds[r]), 5,
                                                              n=bounds[r][1] - bounds[r][0])))
    for r, (got, gst) in enumerate(res):
        lo, hi = bounds[r]
        assert (got == want[lo:hi]).all(), (mode, P, r, int((got != want[lo:hi]).sum()))
        assert (gst == want_st[lo:hi]).all()
    # the sharded path on the replicated snapshot, every rank the whole batch
    res = _ok(_ranks(P, lambda r: comms[r].check_batch_sharded(full, arr, 5, n=n)))
    for got, gst in res:
        assert (got == want).all() and (gst == want_st).all()
    for c in comms:
        c.close()
    for p in parts:
        p.close()


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("mode", ["shared", "migrate"])
def test_local_routed_packed_powerlaw_matches_replicated(powerlaw_strings, P, mode):
    """The power-law graph (1/256 scale) on P parts: every rank's 240,000 / P requests packed by the
    generator's packer and resolved on its device (keto_check_batch_routed_packed), decisions equal
    the replicated snapshot's; a request whose fields lie outside its blob on one rank fails every
    rank alike, and the next call answers exactly."""
    from keto_amd.capi import PART_MIGRATE, PART_SHARED
    g, st, full, arr, n, want, want_st = powerlaw_strings
    m = PART_MIGRATE if mode == "migrate" else PART_SHARED
    parts = []
    for r in range(P):
        part, _ = g.snapshot_from_strings(st, device=-1)
        parts.append(part.upload_part(r, P, 0, mode=m))
    comms = _local_comms(P)
    if m == PART_MIGRATE:
        _ok(_ranks(P, lambda r: comms[r].close_filters(parts[r])))
    bounds = [(r * n // P, (r + 1) * n // P) for r in range(P)]
    packs = [g.pack_requests(_slice(arr, lo, hi), hi - lo) for lo, hi in bounds]
    res = _ok(_ranks(P, lambda r: comms[r].check_batch_routed_packed(parts[r], packs[r][0].array[:packs[r][2]],
                                                                     packs[r][1].array, 5, n=bounds[r][1] - bounds[r][0])))
    for r, (got, gst) in enumerate(res):
        lo, hi = bounds[r]
        assert (got == want[lo:hi]).all() and (gst == want_st[lo:hi]).all(), (mode, P, r)
    bad = packs[1][1].array.copy()
    bad["off"][5] = packs[1][2]                         # request 5's fields past rank 1's blob
    _agreed_failure(_ranks(P, lambda r: comms[r].check_batch_routed_packed(
        parts[r], packs[r][0].array[:packs[r][2]], bad if r == 1 else packs[r][1].array, 5,
        n=bounds[r][1] - bounds[r][0])), 1, "outside the blob")
    res = _ok(_ranks(P, lambda r: comms[r].check_batch_routed_packed(parts[r], packs[r][0].array[:packs[r][2]],
                                                                     packs[r][1].array, 5, n=bounds[r][1] - bounds[r][0])))
    for r, (got, _) in enumerate(res):
        assert (got == want[bounds[r][0]:bounds[r][1]]).all()
    for c in comms:
        c.close()
    for p in parts:
        p.close()


# ------------------------------------------------------------------ error agreement
def _agreed_failure(res, bad_rank, needle):
    codes = set()
    for r, (ok, v) in enumerate(res):
        assert not ok, f"rank {r} returned normally while rank {bad_rank} failed"
        codes.add(v.code)
        if r == bad_rank:
            assert needle in str(v), (r, v)
        else:
            assert f"rank {bad_rank} failed" in str(v), (r, v)
    assert len(codes) == 1, codes


@pytest.mark.parametrize("point", ["resolve", "check", "mig_begin", "mig_round", "filters", "sharded"])
def test_local_error_agreement(powerlaw_strings, monkeypatch, point):
    """A failure injected on rank 1 of 3 (KETO_COMM_INJECT) at each local phase: every rank returns
    the same code, rank 1 its own message, the others name rank 1; no rank waits.  The communicator
    and the parts then answer the next call exactly."""
    from keto_amd.capi import PART_MIGRATE, PART_SHARED
    g, st, full, arr, n, want, want_st = powerlaw_strings
    P = 3
    m = PART_SHARED if point in ("check", "resolve", "sharded") else PART_MIGRATE
    parts = []
    for r in range(P):
        part, _ = g.snapshot_from_strings(st, device=-1)
        parts.append(part.upload_part(r, P, 0, mode=m))
    comms = _local_comms(P)
    k = 30_000
    bounds = [(r * k, (r + 1) * k) for r in range(P)]

    def routed(r):
        return comms[r].check_batch_routed(parts[r], _slice(arr, *bounds[r]), 5, n=k)

    if point == "filters":
        monkeypatch.setenv("KETO_COMM_INJECT", "1:filters")
        _agreed_failure(_ranks(P, lambda r: comms[r].close_filters(parts[r])), 1, "injected")
        monkeypatch.delenv("KETO_COMM_INJECT")
    if m == PART_MIGRATE:
        _ok(_ranks(P, lambda r: comms[r].close_filters(parts[r])))
    monkeypatch.setenv("KETO_COMM_INJECT", f"1:{'check' if point == 'sharded' else point}")
    if point == "sharded":
        _agreed_failure(_ranks(P, lambda r: comms[r].check_batch_sharded(full, _slice(arr, 0, k), 5, n=k)), 1,
                        "injected")
    elif point != "filters":
        _agreed_failure(_ranks(P, routed), 1, "injected")
    monkeypatch.delenv("KETO_COMM_INJECT")
    for r, (got, gst) in enumerate(_ok(_ranks(P, routed))):
        lo, hi = bounds[r]
        assert (got == want[lo:hi]).all() and (gst == want_st[lo:hi]).all(), (point, r)
    for c in comms:
        c.close()
    for p in parts:
        p.close()


@pytest.mark.parametrize("mode", ["shared", "migrate"])
def test_local_parts_at_different_versions_refused(powerlaw_strings, mode):
    """A write applied to one part but not yet to the other: the routed check and the routed expand
    refuse the batch on every rank (KETO_E_INVALID, agreed: the version travels with the counts)
    instead of sending a migrating part's records, which name rows by their owners' handles of
    another layout.  Once every part has the write, the same batch answers like the replicated
    snapshot (the write adds a new document only, so no earlier decision changes)."""
    from keto_amd.capi import PART_MIGRATE, PART_SHARED, KetoError
    g, st, full, arr, n, want, want_st = powerlaw_strings
    P = 2
    m = PART_MIGRATE if mode == "migrate" else PART_SHARED
    parts = []
    for r in range(P):
        part, _ = g.snapshot_from_strings(st, device=-1)
        parts.append(part.upload_part(r, P, 0, mode=m))
    comms = _local_comms(P)
    if m == PART_MIGRATE:
        _ok(_ranks(P, lambda r: comms[r].close_filters(parts[r])))
    k = 20_000
    write = [(1, "zz000001", "view", "u00000001")]
    parts[0].apply(write, [])

    def routed(r):
        return comms[r].check_batch_routed(parts[r], _slice(arr, r * k, (r + 1) * k), 5, n=k)

    for fn in (routed, lambda r: comms[r].expand_batch_routed(parts[r], [(("set", "docs", "zz000001", "view"), 0)], 5)):
        res = _ranks(P, fn)
        for r, (ok, v) in enumerate(res):
            assert not ok and isinstance(v, KetoError) and "different snapshot versions" in str(v), (mode, r, v)
    parts[1].apply(write, [])
    for r, (got, gst) in enumerate(_ok(_ranks(P, routed))):
        assert (got == want[r * k:(r + 1) * k]).all() and (gst == want_st[r * k:(r + 1) * k]).all(), (mode, r)
    got, _ = _ok(_ranks(P, lambda r: comms[r].check_batch_routed(
        parts[r], [("docs", "zz000001", "view", ("id", "u00000001"), 0)] if r == 1 else [], 5)))[1]
    assert list(got) == [1], mode
    for c in comms:
        c.close()
    for p in parts:
        p.close()


def test_local_error_agreement_bad_arguments(powerlaw_strings):
    """Real rank-local errors, no injection: rank 2 passes a NULL request array with n > 0.  Every
    rank returns the code, and the communicator stays usable.  Rank 0 then passes a wildcard query
    (empty object) that no stored set uses: the shared-rows part answers it from its batch-local row,
    the migrating part as one request per matching row, both like the replicated snapshot."""
    from keto_amd.capi import PART_MIGRATE, PART_SHARED, KCheckReq
    g, st, full, arr, n, want, want_st = powerlaw_strings
    P = 3
    k = 1000
    wild = (KCheckReq * k)()
    C.memmove(wild, _slice(arr, 0, k), C.sizeof(wild))
    wild[7].object.n = 0                                  # docs:#view@u -- a wildcard query
    wild_want, wild_st = full.check_batch_reqs(wild, k, 5)
    for mode in (PART_SHARED, PART_MIGRATE):
        parts = []
        for r in range(P):
            part, _ = g.snapshot_from_strings(st, device=-1)
            parts.append(part.upload_part(r, P, 0, mode=mode))
        comms = _local_comms(P)
        if mode == PART_MIGRATE:
            _ok(_ranks(P, lambda r: comms[r].close_filters(parts[r])))

        def null_on_2(r):
            c = comms[r]
            if r == 2:
                from keto_amd.capi import _check
                import numpy as np
                a = np.zeros(k, dtype=np.uint8)
                _check(c.lib.keto_check_batch_routed(c.h, parts[r].h, None, C.c_uint32(k), C.c_int32(5),
                                                     a.ctypes.data_as(C.c_void_p), a.ctypes.data_as(C.c_void_p)))
            return c.check_batch_routed(parts[r], _slice(arr, r * k, (r + 1) * k), 5, n=k)

        _agreed_failure(_ranks(P, null_on_2), 2, "NULL")

        def wild_on_0(r):
            return comms[r].check_batch_routed(parts[r], wild if r == 0 else _slice(arr, r * k, (r + 1) * k), 5, n=k)

        got, gst = _ok(_ranks(P, wild_on_0))[0]
        assert (got == wild_want).all() and (gst == wild_st).all(), mode
        for r, (got, gst) in enumerate(_ok(_ranks(P, lambda r: comms[r].check_batch_routed(
                parts[r], _slice(arr, r * k, (r + 1) * k), 5, n=k)))):
            assert (got == want[r * k:(r + 1) * k]).all(), (mode, r)
        for c in comms:
            c.close()
        for p in parts:
            p.close()


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("seed", range(4200, 4216))
def test_local_migrating_parts_follow_writes(P, seed):
    """Write transactions on a migrating partition (KETO_PART_MIGRATE): every part applies every
    transaction to its host tables (the whole graph's) and is laid out afresh, since its stubs name
    rows by their owners' handles; the next routed batch sees the stale filters on some rank and every
    rank runs the closure-filter exchange again before the records travel.  After each write the
    routed checks of every rank equal the SQL oracle's (relationtuples.go:128-149,200-223,
    check/engine.go:36-123), wildcard queries included (one request per matching row).  Expands from every rank (set
    roots any part owns, subject ids, wildcard queries, unknown rows) equal the oracle's trees: each
    part copies the other parts' rows its trees reach into the call's overlay
    (expand/engine.go:33-102)."""
    import random
    from oracle.oracle_sql import ExpandEngine, NotFoundError, SQLStore
    from tests.randgraph import random_expands
    from tests.randgraph import random_graph
    from tests.test_gpu_lifecycle import _random_write, _row
    import keto_amd
    from keto_amd.capi import PART_MIGRATE
    ns, tuples, raw, ps, alph = random_graph(seed, wide=seed % 4 == 3, allow_wildcards=seed % 3 == 0,
                                             allow_poison=False, allow_collisions=seed % 2 == 0)
    names, objs, rels, users = alph
    set_names = list(names)
    names = [n_ for n_ in names if n_]
    if not names:
        pytest.skip("only a namespace named ''")
    store = SQLStore(ns, tuples, page_size=ps)
    rows = rows_from_tuples(ns, tuples)
    parts = [keto_amd.Snapshot.build(ns, rows, page_size=ps, device=-1).upload_part(r, P, 0, mode=PART_MIGRATE)
             for r in range(P)]
    comms = _local_comms(P)
    _ok(_ranks(P, lambda r: comms[r].close_filters(parts[r])))
    rng = random.Random(seed)
    g = 5
    for step in range(5):
        cur = store.tuples()
        ins = [_random_write(rng, names, objs, rels, users, set_names, 0.1) for _ in range(rng.randint(1, 8))]
        dels = [rng.choice(cur) for _ in range(rng.randint(0, 3))] if cur else []
        for p in parts:
            p.apply([_row(ns, t) for t in ins], [_row(ns, t) for t in dels])
        for t in ins:
            store.insert(t)
        for t in dels:
            store.delete(t)
        checks = random_checks(seed * 41 + step, (names, objs + ["new1", "a0"], rels + ["q"], users + ["w001"]), k=60)
        reqs = [(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in checks]
        mine = [list(range(r, len(reqs), P)) for r in range(P)]      # wildcard queries included
        res = _ok(_ranks(P, lambda r: comms[r].check_batch_routed(parts[r], [reqs[i] for i in mine[r]], g)))
        for r, (got, _) in enumerate(res):
            for k, i in enumerate(mine[r]):
                t, d, _ = checks[i]
                assert bool(got[k]) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, step, r, t, d)
        exps = random_expands(seed * 23 + step, (names, objs + ["new3"], rels + ["q"], users), k=12)
        shares = [exps[r::P] for r in range(P)]
        res = _ok(_ranks(P, lambda r: comms[r].expand_batch_routed(parts[r], [(subj(s_), d) for s_, d, _ in shares[r]], g)))
        for r, got in enumerate(res):
            for (s_, d, _), (st_, js) in zip(shares[r], got):
                try:
                    tr = ExpandEngine(store, g).build_tree(s_, d)
                    want_t = ("tree", tr.to_json()) if tr is not None else ("nil", None)
                except NotFoundError:
                    want_t = ("error", None)
                assert ({0: "tree", 1: "nil", 2: "error"}[st_], js) == want_t, (seed, step, r, s_, d)
    for c in comms:
        c.close()
    for p in parts:
        p.close()


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("seed", range(4200, 4216))
def test_local_shared_parts_follow_writes(P, seed):
    """Write transactions on an edge-partitioned snapshot (KETO_PART_SHARED): every part applies every
    transaction (its host tables are the whole graph's) and writes the rows it holds -- subject-set
    targets on every part, root rows on their owner, a root row that becomes a target joins every part.
    After each write the routed checks of every rank (wildcard queries included) and the expands of
    each part's own roots equal the SQL oracle's (relationtuples.go:128-149,200-223,
    check/engine.go:36-123, expand/engine.go:33-102)."""
    import random
    from oracle.oracle_sql import ExpandEngine, NotFoundError, SQLStore
    from tests.randgraph import random_expands, random_graph
    from tests.test_gpu_lifecycle import _random_write, _row
    import keto_amd
    from keto_amd.capi import PART_SHARED
    ns, tuples, raw, ps, alph = random_graph(seed, wide=seed % 4 == 3, allow_wildcards=seed % 3 == 0,
                                             allow_poison=False, allow_collisions=seed % 2 == 0)
    names, objs, rels, users = alph
    set_names = list(names)
    names = [n_ for n_ in names if n_]
    if not names:
        pytest.skip("only a namespace named ''")
    store = SQLStore(ns, tuples, page_size=ps)
    rows = rows_from_tuples(ns, tuples)
    parts = [keto_amd.Snapshot.build(ns, rows, page_size=ps, device=-1).upload_part(r, P, 0, mode=PART_SHARED)
             for r in range(P)]
    comms = _local_comms(P)
    rng = random.Random(seed)
    g = 5
    for step in range(6):
        cur = store.tuples()
        ins = [_random_write(rng, names, objs, rels, users, set_names, 0.1) for _ in range(rng.randint(1, 8))]
        dels = [rng.choice(cur) for _ in range(rng.randint(0, 3))] if cur else []
        for p in parts:
            p.apply([_row(ns, t) for t in ins], [_row(ns, t) for t in dels])
        for t in ins:
            store.insert(t)
        for t in dels:
            store.delete(t)
        checks = random_checks(seed * 41 + step, (names, objs + ["new1", "a0"], rels + ["q"], users + ["w001"]), k=60)
        reqs = [(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in checks]
        mine = [list(range(r, len(reqs), P)) for r in range(P)]
        res = _ok(_ranks(P, lambda r: comms[r].check_batch_routed(parts[r], [reqs[i] for i in mine[r]], g)))
        for r, (got, _) in enumerate(res):
            for k, i in enumerate(mine[r]):
                t, d, _ = checks[i]
                assert bool(got[k]) == CheckEngine(store, g).subject_is_allowed(t, d), (seed, step, r, t, d)
        # expands of set roots on the part owning the root row (any part for a subject-set target)
        exps = random_expands(seed * 23 + step, (names, objs + ["new3"], rels + ["q"], users), k=10)
        for s_, d, _ in exps:
            if not hasattr(s_, "namespace") or "" in (s_.namespace, s_.object, s_.relation):
                continue
            try:
                tr = ExpandEngine(store, g).build_tree(s_, d)
                want_t = ("tree", tr.to_json()) if tr is not None else ("nil", None)
            except NotFoundError:
                want_t = ("error", None)
            answered = False
            for p in parts:
                try:
                    (st_, js), = p.expand_batch([(subj(s_), d)], g)
                except keto_amd.KetoError:
                    continue                                # another part's root row
                answered = True
                assert ({0: "tree", 1: "nil", 2: "error"}[st_], js) == want_t, (seed, step, s_, d)
            assert answered, s_
        # the same roots and more (subject ids, wildcard queries, unknown rows) from every rank through
        # keto_expand_batch_routed: each rank's share, root rows expanded on their owners
        shares = [exps[r::P] for r in range(P)]
        res = _ok(_ranks(P, lambda r: comms[r].expand_batch_routed(parts[r], [(subj(s_), d) for s_, d, _ in shares[r]], g)))
        for r, got in enumerate(res):
            for (s_, d, _), (st_, js) in zip(shares[r], got):
                try:
                    tr = ExpandEngine(store, g).build_tree(s_, d)
                    want_t = ("tree", tr.to_json()) if tr is not None else ("nil", None)
                except NotFoundError:
                    want_t = ("error", None)
                assert ({0: "tree", 1: "nil", 2: "error"}[st_], js) == want_t, (seed, step, r, s_, d)
    for c in comms:
        c.close()
    for p in parts:
        p.close()


@pytest.mark.parametrize("P", [2, 3])
def test_shared_parts_new_root_rows_never_read_stale_handles(P, monkeypatch):
    """The write-path bug behind r04f6 / r04f7, made deterministic.  A write that adds root rows owned
    by another part gives them no handle on this part; their row -> handle entries must read NO_UNIT.
    KETO_DEBUG_FILL fills every fresh device allocation with the handle of groups:g#member (the set
    every docs:yJ row points at), so an entry nothing wrote names that set: a subject-set request
    docs:yJ#view@(docs:nK#view) would then be allowed on every run, where the reference denies it
    (check/engine.go:36-80: typed equality of the subject set).  Then the new rows become subject-set
    targets (they join every part) and requests reach them through groups:g.  An expand runs first on
    every part, so both lazily built maps exist and the write patches them in place (the path of the
    bug).  The same test on the library built from before the fix fails every run
    (profiles/r05b_slack_prefix.log)."""
    from oracle.oracle_sql import RelationTuple, SQLStore, SubjectID, SubjectSet
    import keto_amd
    from keto_amd.capi import PART_SHARED
    ns = [(0, "docs"), (1, "groups")]
    tuples = [RelationTuple("groups", "g", "member", SubjectID("alice"))]
    tuples += [RelationTuple("docs", f"y{j}", "view", SubjectSet("groups", "g", "member")) for j in range(8)]
    tuples += [RelationTuple("docs", f"d{j}", "view", SubjectID("carol")) for j in range(8)]
    store = SQLStore(ns, tuples)
    rows = rows_from_tuples(ns, tuples)
    parts = [keto_amd.Snapshot.build(ns, rows, device=-1).upload_part(r, P, 0, mode=PART_SHARED) for r in range(P)]
    # the handle of groups:g#member on every part (a subject-set target: every part holds it, same layout)
    hs = {int(p.resolve_checks([("groups", "g", "member", ("id", "alice"), 0)])[0]["row"][0]) for p in parts}
    assert len(hs) == 1, hs
    monkeypatch.setenv("KETO_DEBUG_FILL", str(hs.pop()))
    comms = _local_comms(P)
    g = 5

    def routed_vs_oracle(reqs, step):
        mine = [list(range(r, len(reqs), P)) for r in range(P)]
        res = _ok(_ranks(P, lambda r: comms[r].check_batch_routed(parts[r], [reqs[i] for i in mine[r]], g)))
        for r, (got, st) in enumerate(res):
            for k, i in enumerate(mine[r]):
                ns_, o, rel, s_, d = reqs[i]
                sub = SubjectID(s_[1]) if s_[0] == "id" else SubjectSet(*s_[1:])
                want = CheckEngine(store, g).subject_is_allowed(RelationTuple(ns_, o, rel, sub), d)
                assert bool(got[k]) == want and st[k] == 0, (P, step, r, reqs[i])

    news = [f"n{k}" for k in range(16)]
    probe = [("docs", f"y{j}", "view", ("set", "docs", nk, "view"), 0) for j in range(8) for nk in news]
    probe += [("docs", f"y{j}", "view", ("id", u), 0) for j in range(8) for u in ("alice", "bob")]
    probe += [("docs", nk, "view", ("id", "bob"), 0) for nk in news]
    routed_vs_oracle(probe, "before")                 # allocates each part's row -> handle map
    # an expand builds each part's handle -> row map: with both maps present a write patches them in
    # place (without it the maps were dropped and rebuilt whole, which hid the bug)
    roots = [(("set", "docs", f"y{j}", "view"), 3) for j in range(8)]
    _ok(_ranks(P, lambda r: comms[r].expand_batch_routed(parts[r], roots[r::P], g)))
    ins = [RelationTuple("docs", nk, "view", SubjectID("bob")) for nk in news]
    for p in parts:
        p.apply([rows_from_tuples(ns, [t])[0] for t in ins], [])
    for t in ins:
        store.insert(t)
    routed_vs_oracle(probe, "new root rows")
    # the new rows become subject-set targets: every part now holds them, reached through groups:g
    sets = [RelationTuple("groups", "g", "member", SubjectSet("docs", nk, "view")) for nk in news[::3]]
    for p in parts:
        p.apply([rows_from_tuples(ns, [t])[0] for t in sets], [])
    for t in sets:
        store.insert(t)
    routed_vs_oracle(probe, "new targets")
    for c in comms:
        c.close()
    for p in parts:
        p.close()


@pytest.fixture(scope="module")
def powerlaw_parts():
    """The power-law graph (1/1024 scale) with its strings: a replicated snapshot, shared-rows parts
    for P = 3, and expand roots of every kind (folders and groups, which every part keeps, and docs,
    which one part owns)."""
    from keto_amd.capi import PART_SHARED
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 1024), threads=8)
    st = g.string_tuples(seed=3, threads=8)
    full, _ = g.snapshot_from_strings(st, device=0)
    P = 3
    parts = []
    for r in range(P):
        part, _ = g.snapshot_from_strings(st, device=-1)
        parts.append(part.upload_part(r, P, 0, mode=PART_SHARED))
    q = g.queries(600, seed=17, depth=5, threads=8)
    arr = g.string_requests(st, q, threads=8)

    def text(k):
        return k.p[:k.n].decode() if k.n else ""

    roots = [(("set", text(arr[i].namespace_), text(arr[i].object), text(arr[i].relation)), 1 + i % 5)
             for i in range(len(q))]
    user = text(arr[0].subject.id)
    roots += [(("id", user), 3), (("set", "nope", "x", "y"), 3), (("set", roots[0][0][1], "no such object", roots[0][0][3]), 3)]
    yield g, st, full, parts, roots
    full.close()
    for p in parts:
        p.close()
    g.free_strings(st)
    g.close()


def test_local_expand_routed_powerlaw(powerlaw_parts):
    """Three ranks' expand batches over shared-rows parts: every tree (nodes in pre-order, status)
    equals the replicated snapshot's; roots owned by other parts cross."""
    g, st, full, parts, roots = powerlaw_parts
    P = len(parts)
    want = full.expand_batch(roots, 5, want_nodes=True)
    comms = _local_comms(P)
    shares = [list(range(r, len(roots), P)) for r in range(P)]
    res = _ok(_ranks(P, lambda r: comms[r].expand_batch_routed(parts[r], [roots[i] for i in shares[r]], 5,
                                                               want_nodes=True)))
    crossed = 0
    for r, got in enumerate(res):
        for k, i in enumerate(shares[r]):
            assert got[k] == want[i], (r, i, roots[i])
            crossed += 1
    assert crossed == len(roots)
    # an empty batch on one rank still takes part
    res = _ok(_ranks(P, lambda r: comms[r].expand_batch_routed(parts[r], [] if r == 1 else roots[:50], 5)))
    assert res[1] == [] and res[0] == res[2] == [w[:2] for w in want[:50]]
    for c in comms:
        c.close()


@pytest.mark.parametrize("point", ["resolve", "expand", "roots_alloc", "owner", "trees_alloc"])
def test_local_expand_error_agreement(powerlaw_parts, monkeypatch, point):
    """A failure injected on rank 1 before the roots leave (resolve, local expand, the roots' exchange
    buffers) or while it expands other ranks' roots (owner) or sets up the trees' exchange: every rank
    returns the same code; the next call answers exactly."""
    g, st, full, parts, roots = powerlaw_parts
    P = len(parts)
    comms = _local_comms(P)
    monkeypatch.setenv("KETO_COMM_INJECT", f"1:{point}")
    _agreed_failure(_ranks(P, lambda r: comms[r].expand_batch_routed(parts[r], roots[r::P], 5)), 1, "injected")
    monkeypatch.delenv("KETO_COMM_INJECT")
    want = full.expand_batch(roots, 5)
    res = _ok(_ranks(P, lambda r: comms[r].expand_batch_routed(parts[r], roots[r::P], 5)))
    for r, got in enumerate(res):
        assert got == want[r::P], r
    for c in comms:
        c.close()


@pytest.mark.parametrize("P", [2, 3])
def test_expand_routed_migrating_parts(powerlaw_parts, P):
    """Migrating parts expand every root themselves, copying the other parts' rows a tree reaches
    into the call's overlay: each rank's share of the roots (folders and groups, docs of every part)
    gives the replicated snapshot's trees, node for node (expand/engine.go:33-102)."""
    from keto_amd.capi import PART_MIGRATE
    g, st, full, parts, roots = powerlaw_parts
    mig = []
    for r in range(P):
        sn, _ = g.snapshot_from_strings(st, device=-1)
        mig.append(sn.upload_part(r, P, 0, mode=PART_MIGRATE))
    comms = _local_comms(P)
    _ok(_ranks(P, lambda r: comms[r].close_filters(mig[r])))
    want = full.expand_batch(roots, 5, want_nodes=True)
    res = _ok(_ranks(P, lambda r: comms[r].expand_batch_routed(mig[r], roots[r::P], 5, want_nodes=True)))
    for r, got in enumerate(res):
        assert got == want[r::P], r
    for c in comms:
        c.close()
    for p in mig:
        p.close()


def test_expand_routed_one_rank(comm, powerlaw_parts):
    """Over RCCL with one rank and one shared-rows part (P = 1): the trees equal keto_expand_batch's."""
    from keto_amd.capi import PART_SHARED
    g, st, full, parts, roots = powerlaw_parts
    one, _ = g.snapshot_from_strings(st, device=-1)
    one = one.upload_part(0, 1, 0, mode=PART_SHARED)
    assert comm.expand_batch_routed(one, roots, 5, want_nodes=True) == full.expand_batch(roots, 5, want_nodes=True)
    one.close()
