"""Edge partitioning on one GPU with P logical parts and a loopback exchange (SURVEY.md section 4:
test partitioning on one device before RCCL): every part's snapshot (keto_snapshot_upload_part)
must answer the requests routed to it exactly as the replicated snapshot does, a part must refuse
another part's root row, and every part must hold fewer rows than the whole graph."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_parts", [2, 3])
def test_parts_match_replicated(n_parts):
    from keto_amd.capi import KetoError
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 512), threads=16)
    full = g.snapshot(device=0)
    q = g.queries(60000, seed=40 + n_parts, depth=5)
    rng = np.random.default_rng(n_parts)
    q["max_depth"] = rng.integers(-1, 7, size=len(q))
    want = full.check_batch_ids(full.with_handles(q), 5)
    own = full.row_owner(q["row"], n_parts)
    got = np.full(len(q), 255, dtype=np.uint8)
    rows_per_part = []
    for p in range(n_parts):
        part = g.snapshot_part(p, n_parts, device=0)
        sel = (own == p) | (own < 0)
        sel &= (np.arange(len(q)) % n_parts == p) | (own >= 0)     # shared rows: any one part
        mine = q[sel]
        got[sel] = part.check_batch_ids(part.with_handles(mine), 5)
        rows_per_part.append(part.stats()["device_bytes"])
        other = q[own == (p + 1) % n_parts][:4]
        if len(other):
            with pytest.raises(KetoError):
                part.with_handles(other)
        del part
    assert (got != 255).all()
    assert (got == want).all(), f"{int((got != want).sum())} mismatches"
    assert max(rows_per_part) < full.stats()["device_bytes"]


def test_row_id_requests_on_device():
    """keto_check_batch_rows_device (requests as they travel between parts) equals the handle form,
    and a request for another part's root row fails loudly."""
    import torch
    from keto_amd.capi import KetoError
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 1024), threads=16)
    q = g.queries(20000, seed=77, depth=5)
    full = g.snapshot(device=0)
    want = full.check_batch_ids(full.with_handles(q), 5)
    part = g.snapshot_part(1, 2, device=0)
    own = part.row_owner(q["row"], 2)
    mine = q[own != 0]
    d = torch.from_numpy(mine.view(np.int32).reshape(-1, 4).copy()).to("cuda:0")
    out = torch.empty(len(mine), dtype=torch.uint8, device="cuda:0")
    part.check_batch_rows_device(d.data_ptr(), len(mine), out.data_ptr(), 5)
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == want[own != 0]).all()
    other = q[own == 0][:8]
    d2 = torch.from_numpy(other.view(np.int32).reshape(-1, 4).copy()).to("cuda:0")
    out2 = torch.empty(len(other), dtype=torch.uint8, device="cuda:0")
    with pytest.raises(KetoError):
        part.check_batch_rows_device(d2.data_ptr(), len(other), out2.data_ptr(), 5)


def test_device_routing_world1_is_identity():
    import torch
    from keto_amd.multi import route_device, send_back
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 1024), threads=16)
    q = g.queries(5000, seed=78, depth=5)
    snap = g.snapshot_part(0, 1, device=0)
    want = snap.check_batch_ids(snap.with_handles(q), 5)
    d = torch.from_numpy(q.view(np.int32).reshape(-1, 4).copy()).to("cuda:0")
    owner = torch.from_numpy(snap.row_owner(np.arange(g.n_rows, dtype=np.uint32), 1).astype(np.int16)).to("cuda:0")
    recv, state = route_device(d, owner, 0, 1)
    dec = torch.empty(len(recv), dtype=torch.uint8, device="cuda:0")
    snap.check_batch_rows_device(recv.data_ptr(), len(recv), dec.data_ptr(), 5)
    out = torch.empty(len(q), dtype=torch.uint8, device="cuda:0")
    send_back(dec, state, out, 1)
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == want).all()


def _np_route(rows, owner, self_part, n_parts):
    """numpy statement of keto_route_rows_device: destination = owner[row] when in range and
    0 <= owner < n_parts, else self_part; a stable sort by destination."""
    dest = np.full(len(rows), self_part, dtype=np.int64)
    ok = rows < len(owner)
    o = np.where(ok, owner[np.minimum(rows, max(len(owner) - 1, 0))].astype(np.int64), -1)
    good = ok & (o >= 0) & (o < n_parts)
    dest[good] = o[good]
    order = np.argsort(dest, kind="stable")
    return order, np.bincount(dest, minlength=n_parts)


@pytest.mark.parametrize("n,n_parts,self_part", [(0, 3, 1), (1, 1, 0), (2047, 2, 1), (2049, 3, 0),
                                                  (100_003, 8, 5), (300_000, 64, 63), (70_000, 7, 0)])
def test_route_rows_device_matches_stable_sort(n, n_parts, self_part):
    """keto_route_rows_device against a numpy stable sort: every request lands in its owner's
    group in batch order; shared rows (-1), KETO_NO_ROW, out-of-range rows and out-of-range owner
    values stay on self_part; keto_unroute_device inverts the permutation."""
    import torch
    from keto_amd import capi
    rng = np.random.default_rng(n + 31 * n_parts)
    n_rows = 5000
    owner = rng.integers(-1, n_parts, size=n_rows).astype(np.int16)
    owner[:3] = n_parts                                        # out-of-range owner values
    reqs = rng.integers(0, 2**31, size=(n, 4)).astype(np.int32)
    rows = rng.integers(0, n_rows + 40, size=n).astype(np.uint32)
    rows[rng.random(n) < 0.01] = 0xFFFFFFFF                    # KETO_NO_ROW
    reqs[:, 0] = rows.view(np.int32)
    order, counts = _np_route(rows.astype(np.int64), owner, self_part, n_parts)
    dev = "cuda:0"
    d_reqs = torch.from_numpy(reqs).to(dev)
    d_owner = torch.from_numpy(owner).to(dev)
    wb = capi.route_work_bytes(n, n_parts)
    work = torch.empty(max(wb, 1), dtype=torch.uint8, device=dev)
    send = torch.empty((max(n, 1), 4), dtype=torch.int32, device=dev)
    d_order = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    cs = capi.route_rows_device(d_reqs.data_ptr(), n, d_owner.data_ptr(), n_rows, self_part, n_parts,
                                work.data_ptr(), wb, send.data_ptr(), d_order.data_ptr())
    assert cs == counts.tolist()
    if n == 0:
        return
    torch.cuda.synchronize()
    assert (d_order.cpu().numpy()[:n] == order).all()
    assert (send.cpu().numpy()[:n] == reqs[order]).all()
    back = torch.from_numpy((np.arange(n) % 251).astype(np.uint8)).to(dev)
    out = torch.full((n,), 255, dtype=torch.uint8, device=dev)
    capi.unroute_device(back.data_ptr(), d_order.data_ptr(), n, out.data_ptr())
    torch.cuda.synchronize()
    want = np.empty(n, dtype=np.uint8)
    want[order] = np.arange(n) % 251
    assert (out.cpu().numpy() == want).all()


def test_route_rows_device_rejects_bad_arguments():
    import torch
    from keto_amd import capi
    from keto_amd.capi import KetoError
    d = torch.zeros((10, 4), dtype=torch.int32, device="cuda:0")
    own = torch.zeros(4, dtype=torch.int16, device="cuda:0")
    wb = capi.route_work_bytes(10, 2)
    work = torch.empty(wb, dtype=torch.uint8, device="cuda:0")
    o = torch.empty(10, dtype=torch.int32, device="cuda:0")
    with pytest.raises(KetoError):                             # workspace too small
        capi.route_rows_device(d.data_ptr(), 10, own.data_ptr(), 4, 0, 2, work.data_ptr(), wb - 1,
                               d.data_ptr(), o.data_ptr())
    with pytest.raises(KetoError):                             # self_part out of range
        capi.route_rows_device(d.data_ptr(), 10, own.data_ptr(), 4, 2, 2, work.data_ptr(), wb,
                               d.data_ptr(), o.data_ptr())
    with pytest.raises(KetoError):                             # more than 64 parts
        capi.route_rows_device(d.data_ptr(), 10, own.data_ptr(), 4, 0, 65, work.data_ptr(), 1 << 20,
                               d.data_ptr(), o.data_ptr())


@pytest.mark.parametrize("n_parts", [2, 3])
def test_device_routing_loopback_matches_replicated(n_parts):
    """Every rank's routing on one GPU (loopback exchange): rank r routes its batch with
    keto_route_rows_device, the requests bound for part p are checked on part p's snapshot, and
    keto_unroute_device puts the decisions back; the result equals the replicated snapshot's."""
    import torch
    from keto_amd import capi
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 1024), threads=16)
    full = g.snapshot(device=0)
    parts = [g.snapshot_part(p, n_parts, device=0) for p in range(n_parts)]
    owner = torch.from_numpy(parts[0].row_owner(np.arange(g.n_rows, dtype=np.uint32), n_parts).astype(np.int16)
                             ).to("cuda:0")
    for rank in range(n_parts):
        q = g.queries(20000, seed=90 + rank, depth=5)
        want = full.check_batch_ids(full.with_handles(q), 5)
        d = torch.from_numpy(q.view(np.int32).reshape(-1, 4).copy()).to("cuda:0")
        n = len(q)
        wb = capi.route_work_bytes(n, n_parts)
        work = torch.empty(wb, dtype=torch.uint8, device="cuda:0")
        send = torch.empty_like(d)
        order = torch.empty(n, dtype=torch.int32, device="cuda:0")
        cs = capi.route_rows_device(d.data_ptr(), n, owner.data_ptr(), len(owner), rank, n_parts,
                                    work.data_ptr(), wb, send.data_ptr(), order.data_ptr())
        dec = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        off = 0
        for p in range(n_parts):
            if cs[p]:
                parts[p].check_batch_rows_device(send[off:].data_ptr(), cs[p], dec[off:].data_ptr(), 5)
            off += cs[p]
        out = torch.full((n,), 255, dtype=torch.uint8, device="cuda:0")
        capi.unroute_device(dec.data_ptr(), order.data_ptr(), n, out.data_ptr())
        torch.cuda.synchronize()
        assert (out.cpu().numpy() == want).all()


@pytest.mark.parametrize("n_parts", [2, 3])
def test_expand_on_parts_matches_replicated(n_parts):
    """Expand on a shared-rows partition (the PartitionedExpander's local step, loopback on one GPU):
    every root expanded on the part that owns its row gives the replicated snapshot's tree, node for
    node; a part refuses another part's root row."""
    from keto_amd.capi import KetoError
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 512), threads=16)
    full = g.snapshot(device=0)
    rng = np.random.default_rng(50 + n_parts)
    n = 6000
    rows = rng.integers(0, g.n_rows, size=n).astype(np.uint32)
    roots = rows | np.uint32(0x80000000)
    depths = rng.integers(-1, 7, size=n).astype(np.int32)
    st_w, off_w, nd_w = full.expand_batch_ids(roots, depths, 5)
    own = full.row_owner(rows, n_parts)
    assert (own >= 0).any() and (own < 0).any()
    for p in range(n_parts):
        part = g.snapshot_part(p, n_parts, device=0)
        sel = np.flatnonzero((own == p) | ((own < 0) & (np.arange(n) % n_parts == p)))
        st, off, nd = part.expand_batch_ids(roots[sel], depths[sel], 5)
        assert (st == st_w[sel]).all()
        for j, i in enumerate(sel):
            assert (nd[off[j]:off[j + 1]] == nd_w[off_w[i]:off_w[i + 1]]).all(), (p, int(rows[i]))
        other = roots[own == (p + 1) % n_parts][:4]
        if len(other):
            with pytest.raises(KetoError):
                part.expand_batch_ids(other, np.zeros(len(other), dtype=np.int32), 5)
        del part
