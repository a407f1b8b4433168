"""The library's own RCCL layer (keto_amd/csrc/comm.cpp: keto_comm_*, keto_check_batch_sharded,
keto_check_batch_routed, keto_comm_close_filters) on the box's one GPU, as a one-rank communicator:
the collectives run through RCCL for real (all-gather, grouped send/recv all-to-alls, all-reduce),
and every decision must equal the replicated snapshot's and the SQL oracle's.  Runs with more ranks
are the driver's multi-GPU node; the same exchanges over gloo are tests/test_multi_cpu.py."""
import pytest

from oracle.oracle_sql import CheckEngine
from tests.engine_util import rows_from_tuples, subj
from tests.randgraph import random_checks, random_store

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from keto_amd.capi import Comm
    c = Comm(Comm.make_id(), 1, 0, 0)
    yield c
    c.close()


def _reqs(seed, alph):
    checks = random_checks(seed, alph, k=48)
    return [(t.namespace, t.object, t.relation, subj(t.subject), d) for t, d, _ in checks], checks


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
