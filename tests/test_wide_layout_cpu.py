"""Wide arenas (past 64 GiB; snapshot.hpp hword) laid out on the host, no device needed.

A handle below 2^31 is a 16-B unit (targets, and roots below word 2^33); a handle h >= 2^31 names a
root whose header lies at word 2^33 + ((h - 2^31) << (2 + g)).  KETO_TEST_ROOT_BASE places the roots
of a small graph from a given word on (the gap is never built on the host); KETO_TEST_ROOT_G forces
the coarser units below 64 GiB too.  Checked here: every row keeps a distinct header word, handles
and header words increase together (the host's handle -> row lookup binary-searches them), roots
past 2^33 sit on their unit, no row crosses a 2^32-word segment, targets stay below 2^31, and the
part statistics report the arena's real size."""
import os

import numpy as np
import pytest

T = 1 << 33


def hword(h, g):
    h = np.asarray(h, dtype=np.uint64)
    return np.where(h < (1 << 31), h * np.uint64(4),
                    np.uint64(T) + ((h - np.uint64(1 << 31)) << np.uint64(2 + g)))


@pytest.fixture(scope="module")
def graph():
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 8192), threads=8)
    yield g
    g.close()


def _layout(graph, monkeypatch, base, force_g=None):
    monkeypatch.setenv("KETO_TEST_ROOT_BASE", str(base))
    if force_g is not None:
        monkeypatch.setenv("KETO_TEST_ROOT_G", str(force_g))
    snap = graph.snapshot(device=-1)
    h = snap.row_handles(np.arange(graph.n_rows, dtype=np.uint32)).astype(np.uint64)
    arena = snap.part_stats(0, 1)["arena_bytes"]
    snap.close()
    return h, arena


def _infer_g(h, arena_bytes):
    # the last root lies in the arena's far half: the largest unit that keeps it inside the arena
    fits = [g for g in range(1, 4) if int(hword(h.max(), g)) + 4 <= arena_bytes // 4]
    assert fits, f"no root unit places handle {int(h.max()):#x} inside {arena_bytes} B"
    return max(fits)


@pytest.mark.parametrize("base,force_g,want_g", [
    ((1 << 34) + (1 << 32) - (1 << 16), None, 1),   # ~80 GiB: roots in segments 4 and 5, 32-B units
    (25 << 30, None, 2),                            # ~100 GiB: 64-B units
    (3 * (1 << 32) - (1 << 16), 3, 3),              # 48 GiB forced to 128-B units
])
def test_wide_layout_invariants(graph, monkeypatch, base, force_g, want_g):
    h, arena = _layout(graph, monkeypatch, base, force_g)
    assert arena > base * 4
    g = _infer_g(h, arena)
    assert g == want_g
    roots = h >= (1 << 31)
    assert roots.mean() > 0.5 and (~roots).any()
    w = hword(h, g)
    order = np.argsort(h)
    assert (np.diff(w[order].astype(np.int64)) > 0).all()           # distinct, increasing with the handle
    assert ((w[roots] - np.uint64(T)) % np.uint64(4 << g) == 0).all()
    assert (w[roots] >= np.uint64(base)).all()
    # header + window never cross a segment (rows never do)
    assert ((w >> np.uint64(32)) == ((w + np.uint64(7)) >> np.uint64(32))).all()
    if base >= 1 << 34:
        assert (w[roots] >> np.uint64(32)).max() >= 4


def test_narrow_layout_unchanged(graph, monkeypatch):
    """Below 64 GiB the layout stays narrow: every handle is a 16-B unit."""
    h, arena = _layout(graph, monkeypatch, 3 * (1 << 32) - (1 << 16))
    assert arena < 64 << 30
    assert int(h.max()) * 16 < arena


def test_past_288_gib_refused(graph, monkeypatch):
    from keto_amd.capi import KetoError
    monkeypatch.setenv("KETO_TEST_ROOT_BASE", str(72 << 30))          # roots from 288 GiB on
    with pytest.raises(KetoError):
        graph.snapshot(device=-1)
