"""Config #3 deep-tier sweep (tooling): the full 1M-request batch at global max-depth 32 under
combinations of KETO_DEEP_WAVE (deep_wave_kernel vs check_kernel as tier 0), KETO_SLOTS and
KETO_T0_CAP; one JSON line per combination, decisions checked equal across all of them.

  python tools/deep_sweep.py "KETO_DEEP_WAVE=0" "KETO_DEEP_WAVE=1,KETO_SLOTS=229376,KETO_T0_CAP=65536" ...
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.set_device(0)
    from tools import synth
    g = synth.SynthGraph(dict(synth.NESTED_100M), threads=16, kind="nested", chain=32)
    snap = g.snapshot(device=0)
    q = g.queries_nested(1_000_000, seed=3, depths=(5, 16, 32), threads=16)
    qd = snap.with_handles(q)
    d_q = torch.from_numpy(qd.view(np.uint8)).to("cuda:0")
    d_o = torch.empty(len(q), dtype=torch.uint8, device="cuda:0")
    sp = torch.cuda.current_stream().cuda_stream
    ref = None
    for combo in sys.argv[1:]:
        env = dict(kv.split("=") for kv in combo.split(",") if kv)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            best = None
            for _ in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                snap.check_batch_device(d_q.data_ptr(), len(q), d_o.data_ptr(), 32, sp)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                ms, cnt = snap.last_timing()
                if best is None or dt < best[0]:
                    best = (dt, ms, cnt)
            out = d_o.cpu().numpy()
            if ref is None:
                ref = out
            print(json.dumps({"env": env, "wall_ms": round(best[0] * 1e3, 3), "tier_ms": [round(x, 3) for x in best[1]],
                              "tier_requests": [int(x) for x in best[2]], "kernel": snap.check_kernel_name(32),
                              "same_decisions": bool((out == ref).all())}), flush=True)
        finally:
            for k, v in old.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v


if __name__ == "__main__":
    main()
