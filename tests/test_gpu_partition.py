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
