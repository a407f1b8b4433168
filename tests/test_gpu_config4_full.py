"""BASELINE config #4 at its full size in the driver's -m gpu run (before round 4 its parity lived only
in bench.py's leg): the 1B-tuple power-law ACL graph (tools/synth.cpp, seed of POWERLAW_1B, 155M rows)
bulk-loaded through keto_snapshot_from_csr, one 16,777,216-request batch of docs:d#view@u checks at
max-depth 5 through keto_check_batch_device (the bench's step), no request left undecided, the first
1,000,000 decisions compared with oracle/keto_oracle.c over the tuples they can reach
(internal/check/engine.go:36-123), and 5,000 expand roots on the same graph compared node for node
with the oracle's BuildTree (internal/expand/engine.go:33-102, pre-order, child order included)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BATCH = 16 * 1024 * 1024
ORA_NODE = np.dtype([("type", "u1"), ("kind", "u1"), ("sid", "<u4"), ("name", "<u4"), ("obj", "<u4"),
                     ("rel", "<u4"), ("n_children", "<u4")], align=True)


@pytest.fixture(scope="module")
def powerlaw_1b():
    from tools import synth
    g = synth.SynthGraph(dict(synth.POWERLAW_1B), threads=16)
    snap = g.snapshot(device=0)
    yield g, snap
    snap.close()
    g.close()


def test_config4_full_scale_matches_oracle(powerlaw_1b):
    import torch
    g, snap = powerlaw_1b
    assert g.n_edges == 1_000_000_000
    q = g.queries(BATCH, seed=1000, depth=5, threads=16)
    d_q = torch.from_numpy(snap.with_handles(q).view(np.uint8)).to("cuda:0")
    d_out = torch.full((BATCH,), 7, dtype=torch.uint8, device="cuda:0")
    snap.check_batch_device(d_q.data_ptr(), BATCH, d_out.data_ptr(), 5, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    gpu = d_out.cpu().numpy()
    _, tiers = snap.last_timing()
    assert (gpu <= 1).all(), f"{int((gpu > 1).sum())} requests undecided or unwritten (tiers {tiers})"
    k = 1_000_000
    tab = g.oracle_table(q[:k], 5)
    ref = tab.check_batch_reqs(g.oracle_requests(tab, q[:k]), 5, threads=16)
    assert (gpu[:k] == ref).all(), f"{int((gpu[:k] != ref).sum())} mismatches of {k}"
    assert 0.2 < gpu.mean() < 0.8


def _oracle_nodes(g, tab, row, gmd):
    from oracle.oracle_c import OraNode, OraSubject, lib
    root = OraSubject(1, 0, 0xFFFF0000 + int(g.row_ns[row]), int(g.row_obj[row]), int(g.row_rel[row]),
                      int(g.params["n_users"] + row))
    nodes = C.POINTER(OraNode)()
    nn = C.c_uint64()
    r = lib().ora_expand(C.byref(tab.t), C.byref(root), C.c_int32(gmd), C.c_int32(gmd), C.byref(nodes), C.byref(nn))
    out = np.zeros(0, dtype=ORA_NODE)
    if nn.value:
        assert C.sizeof(OraNode) == ORA_NODE.itemsize
        out = np.frombuffer(C.string_at(nodes, nn.value * ORA_NODE.itemsize), dtype=ORA_NODE).copy()
        lib().ora_free(C.cast(nodes, C.c_void_p))
    return r, out


def test_config4_full_scale_expand_matches_oracle(powerlaw_1b):
    g, snap = powerlaw_1b
    rng = np.random.default_rng(44)
    n = 5_000
    rows = rng.integers(0, g.n_rows, size=n).astype(np.uint32)
    status, offs, nodes = snap.expand_batch_ids(rows | np.uint32(0x80000000), np.zeros(n, dtype=np.int32), 5)
    assert len(status) == n and (status <= 1).all()
    q = np.zeros(n, dtype=[("row", "<u4"), ("target", "<u4"), ("flags", "<u4"), ("max_depth", "<i4")])
    q["row"] = rows
    tab = g.oracle_table(q, 5)
    n_nodes = 0
    for i in range(n):
        r, want = _oracle_nodes(g, tab, int(rows[i]), 5)
        if r == 0:
            assert status[i] == 1, i
            continue
        assert r == 1 and status[i] == 0, i
        have = nodes[offs[i]:offs[i + 1]]
        assert len(have) == len(want), f"root row {rows[i]}: {len(have)} nodes, oracle {len(want)}"
        subj, info = have[:, 0], have[:, 1]
        is_set = (subj >> 31).astype(bool)
        t = (subj & 0x7FFFFFFF).astype(np.int64)
        ts = np.where(is_set, t, 0)
        assert (want["type"] == (info >> 31)).all(), f"root row {rows[i]}: leaf flags"
        assert (want["n_children"] == (info & 0x7FFFFFFF)).all(), f"root row {rows[i]}: child counts"
        assert (want["kind"] == is_set).all(), f"root row {rows[i]}: node kinds"
        assert (want["sid"] == np.where(is_set, 0, subj)).all(), f"root row {rows[i]}: subject ids"
        assert (want["name"] == np.where(is_set, 0xFFFF0000 + g.row_ns[ts].astype(np.int64), 0)).all()
        assert (want["obj"] == np.where(is_set, g.row_obj[ts], 0)).all(), f"root row {rows[i]}: objects"
        assert (want["rel"] == np.where(is_set, g.row_rel[ts], 0)).all(), f"root row {rows[i]}: relations"
        n_nodes += len(have)
    assert n_nodes > 5_000
