"""The snapshot builder's parallel paths (sharded interning, sample-sorted ORDER BY, hash-filtered
collision classes; keto_amd/csrc/parallel.hpp) produce exactly the snapshot of the sequential
paths: same strings, rows, layout, subject strings and collision classes, on quirk-heavy random
tables (empty fields, '#' in objects, ids equal to a set's String(), poisoned rows, duplicates),
in any commit order.  Host-only snapshots: no GPU."""
import ctypes as C
import random

import pytest

import keto_amd
from tests.engine_util import rows_from_tuples
from tests.randgraph import random_graph


def _fingerprint(s):
    lib = keto_amd.load()
    st = s.stats()
    import numpy as np
    h = s.row_handles(np.arange(st["n_rows"], dtype=np.uint32))
    buf = C.create_string_buffer(4096)
    strs = []
    for ref in [0x80000000 | r for r in range(st["n_rows"])] + list(range(st["n_strings"])):
        n = lib.keto_subject_string(s.h, C.c_uint32(ref), buf, C.c_uint64(4096))
        strs.append(buf.raw[:n])
    return st, h.tolist(), strs


def _build(monkeypatch, ns, rows, ps, par, threads=3):
    monkeypatch.setenv("KETO_BUILD_PAR_MIN", "1" if par else str(1 << 40))
    monkeypatch.setenv("KETO_BUILD_THREADS", str(threads))
    return keto_amd.Snapshot.build(ns, rows, page_size=ps, device=-1)


@pytest.mark.parametrize("seed", list(range(60)) + [1000 + s for s in range(12)])
def test_parallel_builder_equals_sequential(monkeypatch, seed):
    ns, tuples, raw, ps, _ = random_graph(seed, wide=seed >= 1000)
    rows = rows_from_tuples(ns, tuples, raw)
    random.Random(seed).shuffle(rows)
    a = _fingerprint(_build(monkeypatch, ns, rows, ps, par=False, threads=1))
    for th in (2, 5):
        b = _fingerprint(_build(monkeypatch, ns, rows, ps, par=True, threads=th))
        assert a == b, (seed, th)


def test_parallel_builder_large_table(monkeypatch):
    """3,000 tuples over many objects with dozens of colliding ids: sample sort with several
    buckets per thread, shards that all see traffic."""
    rng = random.Random(5)
    ns = [(1, "n"), (2, "m")]
    rows = []
    for i in range(3000):
        o = f"o{rng.randrange(300)}"
        if rng.random() < 0.5:
            sid = f"u{rng.randrange(500)}" if rng.random() < 0.9 else f"n:o{rng.randrange(300)}#r"
            rows.append((rng.choice([1, 2]), o, rng.choice(["r", "s"]), sid))
        else:
            rows.append((rng.choice([1, 2]), o, rng.choice(["r", "s"]), None, rng.choice([1, 2]),
                         f"o{rng.randrange(300)}", rng.choice(["r", "s"])))
    a = _fingerprint(_build(monkeypatch, ns, rows, 100, par=False, threads=1))
    b = _fingerprint(_build(monkeypatch, ns, rows, 100, par=True, threads=7))
    assert a == b
    assert a[0]["n_collision_keys"] > 10
