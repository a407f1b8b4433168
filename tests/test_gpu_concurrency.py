"""Writes concurrent with the tree encoders (keto_snapshot_apply against keto_tree_json /
keto_tree_json_all / keto_tree_proto_all / keto_tree_proto_all_device / keto_subject_fields on an
arena built before the writes).  apply appends strings and row keys (vector reallocation), so an
encoder that read them without the snapshot's shared lock would read freed memory; with the lock
every encoding of the old arena stays byte-identical while the writes land."""
import ctypes as C
import threading

import numpy as np
import pytest

from tests.engine_util import rows_from_tuples, subj
from tests.randgraph import random_expands, random_store

pytestmark = pytest.mark.gpu


def _arena(snap, reqs, g):
    from keto_amd.capi import KExpandReq, _check, _Keep, subject_struct
    keep = _Keep()
    arr = (KExpandReq * len(reqs))()
    for k, (sub, d) in enumerate(reqs):
        arr[k].subject = subject_struct(keep, sub)
        arr[k].max_depth = d
    a = C.c_void_p()
    _check(snap.lib.keto_expand_batch(snap.h, arr, C.c_uint32(len(reqs)), C.c_int32(g), C.byref(a)))
    return a


@pytest.mark.parametrize("seed", [3001, 3002, 3003])
def test_apply_concurrent_with_encoders(seed):
    from oracle.oracle_sql import RelationTuple, SubjectID
    store, ns, tuples, raw, ps, alph = random_store(seed, wide=True, allow_wildcards=False, allow_poison=False,
                                                   allow_collisions=False)
    import keto_amd
    snap = keto_amd.Snapshot.build(ns, rows_from_tuples(ns, tuples), page_size=ps, device=0)
    names = [n for n in alph[0] if n]
    reqs = [(subj(s), d) for s, d, _ in random_expands(seed, alph, k=64)]
    a = _arena(snap, reqs, 5)
    n = len(reqs)
    try:
        base_json = snap._json_all(a, n)
        base_proto = snap._proto_all(a, n)[1]
        base_dev = snap._proto_all(a, n, device=True)[1]
        nodes = []
        for i in range(n):
            nn = C.c_uint64()
            ptr = snap.lib.keto_tree_nodes(a, C.c_uint32(i), C.byref(nn))
            nodes += [ptr[j].subject for j in range(nn.value)]
        base_fields = snap.subject_fields(nodes, arena=a) if nodes else []
        errors = []
        stop = threading.Event()

        def writer():
            try:
                for k in range(60):
                    new = [RelationTuple(names[0], f"zz{seed}_{k}_{j}", "r", SubjectID(f"new-user-{k}-{j}" * 3))
                           for j in range(50)]
                    snap.apply(rows_from_tuples(ns, new))
            except Exception as e:             # noqa: BLE001 - surfaced below
                errors.append(("writer", e))
            finally:
                stop.set()

        def reader(kind):
            try:
                while not stop.is_set():
                    if kind == "json":
                        assert snap._json_all(a, n) == base_json
                    elif kind == "proto":
                        assert snap._proto_all(a, n)[1] == base_proto
                    elif kind == "device":
                        assert snap._proto_all(a, n, device=True)[1] == base_dev
                    else:
                        assert not nodes or snap.subject_fields(nodes, arena=a) == base_fields
            except Exception as e:             # noqa: BLE001
                errors.append((kind, e))

        ts = [threading.Thread(target=writer)] + [threading.Thread(target=reader, args=(k,))
                                                   for k in ("json", "proto", "device", "fields")]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=110)
        assert not any(t.is_alive() for t in ts), "a thread did not finish"
        assert not errors, errors
        assert snap.version() == 60
    finally:
        snap.lib.keto_tree_arena_free(a)
        snap.close()
