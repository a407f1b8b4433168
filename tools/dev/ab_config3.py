"""A/B of tuning builds on config #3 (tooling): the 1M-request nested-groups batch, best of --reps
runs, with a hash of the decisions so variants can be compared for identical answers.

  KETO_LIB=keto_amd/variants/lib_<name>.so python tools/dev/ab_config3.py --label <name>
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default=os.environ.get("KETO_LIB", "default"))
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from tools import synth
    g = synth.SynthGraph(dict(synth.NESTED_100M), threads=16, kind="nested", chain=32)
    snap = g.snapshot(device=0)
    q = g.queries_nested(1_000_000, seed=3, depths=(5, 16, 32), threads=16)
    qd = snap.with_handles(q)
    sp = torch.cuda.current_stream().cuda_stream
    d_q = torch.from_numpy(np.ascontiguousarray(qd).view(np.uint8)).to("cuda:0")
    d_o = torch.empty(len(qd), dtype=torch.uint8, device="cuda:0")
    times = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        snap.check_batch_device(d_q.data_ptr(), len(qd), d_o.data_ptr(), 32, sp)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
    ms, cnt = snap.last_timing()
    out = d_o.cpu().numpy()
    print(json.dumps({"label": a.label, "wall_ms": [round(t, 2) for t in times], "best_ms": round(min(times), 2),
                      "tier_ms": [round(x, 2) for x in ms], "tier_requests": [int(x) for x in cnt],
                      "decisions_sha": hashlib.sha256(out.tobytes()).hexdigest()[:16],
                      "allowed": int(out.sum())}), flush=True)


if __name__ == "__main__":
    main()
