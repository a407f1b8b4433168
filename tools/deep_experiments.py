"""Config #3 deep-kernel experiments (tooling): how the 1M-request batch's time splits between the
longest searches and the rest, and what the step latency is with the chip loaded vs idle.

  python tools/deep_experiments.py
prints JSON lines: the full batch; the top-k longest requests alone (k = 1, 100, 10000); the batch
without them; and the full batch under tier-0 table / lane-count knobs (KETO_T0_CAP, KETO_SLOTS).
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
    sp = torch.cuda.current_stream().cuda_stream

    def run(sub, label, reps=2, **env):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update({k: str(v) for k, v in env.items()})
        try:
            d_q = torch.from_numpy(np.ascontiguousarray(sub).view(np.uint8)).to("cuda:0")
            d_o = torch.empty(len(sub), dtype=torch.uint8, device="cuda:0")
            best = None
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                snap.check_batch_device(d_q.data_ptr(), len(sub), d_o.data_ptr(), 32, sp)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                ms, cnt = snap.last_timing()
                best = dt if best is None else min(best, dt)
            return {"run": label, "requests": len(sub), "wall_ms": round(best * 1e3, 3),
                    "tier_ms": [round(x, 3) for x in ms], "tier_requests": [int(x) for x in cnt], "env": env}, \
                d_o.cpu().numpy()
        finally:
            for k, v in old.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v

    base, out = run(qd, "full batch")
    print(json.dumps(base), flush=True)
    d_q = torch.from_numpy(qd.view(np.uint8)).to("cuda:0")
    d_o = torch.empty(len(q), dtype=torch.uint8, device="cuda:0")
    d_s = torch.zeros(len(q), dtype=torch.int32, device="cuda:0")
    snap.check_steps_device(d_q.data_ptr(), len(q), d_o.data_ptr(), d_s.data_ptr(), 32)
    torch.cuda.synchronize()
    steps = d_s.cpu().numpy().astype(np.int64)
    order = np.argsort(-steps, kind="stable")
    for k in (1, 100, 10000):
        r, o = run(qd[order[:k]], f"top {k} longest alone")
        r["steps_max"] = int(steps[order[0]])
        r["us_per_step_of_longest"] = round(r["tier_ms"][0] * 1e3 / steps[order[0]], 3)
        r["same_decisions"] = bool((o == out[order[:k]]).all())
        print(json.dumps(r), flush=True)
    rest = np.sort(order[10000:])
    r, o = run(qd[rest], "without the 10000 longest")
    r["same_decisions"] = bool((o == out[rest]).all())
    print(json.dumps(r), flush=True)
    if "--no-knobs" in sys.argv:
        return
    for env in ({"KETO_T0_CAP": 65536}, {"KETO_T0_CAP": 4096}, {"KETO_NO_POOL": 1},
                {"KETO_SLOTS": 229376}, {"KETO_SLOTS": 917504}):
        r, o = run(qd, "full batch, knob", **env)
        r["same_decisions"] = bool((o == out).all())
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
