"""Tier 0 on a wide arena against the same graph's narrow layout (dev tooling, not the product).

The power-law graph at --scale, laid out twice on device 0: the ordinary layout, and a wide one whose
root rows start past 64 GiB (KETO_TEST_ROOT_BASE; 32-B root units, check_wave_kernel_wide) -- a real
device allocation of that size.  The same device-resident batch of --batch requests (handles of each
layout) is checked --steps times on each, alternating; prints both per-batch times (HIP-synchronized
wall, median) and whether the decisions are equal.

  python tools/dev/wide_ab.py [--scale 0.125] [--batch 4194304] [--steps 20]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.125)
    ap.add_argument("--batch", type=int, default=4 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--root-base", type=int, default=(1 << 34) + (1 << 30))
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from tools import synth
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, a.scale), threads=16)
    narrow = g.snapshot(device=0)
    os.environ["KETO_TEST_ROOT_BASE"] = str(a.root_base)
    try:
        wide = g.snapshot(device=0)
    finally:
        del os.environ["KETO_TEST_ROOT_BASE"]
    q = g.queries(a.batch, seed=77, depth=5)
    out = {}
    d_out = {}
    snaps = {"narrow": narrow, "wide": wide}
    d_q = {k: torch.from_numpy(s.with_handles(q).view(np.uint8)).cuda() for k, s in snaps.items()}
    for k in snaps:
        d_out[k] = torch.empty(a.batch, dtype=torch.uint8, device="cuda")
        out[k] = []
    for k, s in snaps.items():                                   # warmup
        for _ in range(3):
            s.check_batch_device(d_q[k].data_ptr(), a.batch, d_out[k].data_ptr(), 5)
    torch.cuda.synchronize()
    for _ in range(a.steps):
        for k, s in snaps.items():
            t = time.perf_counter()
            s.check_batch_device(d_q[k].data_ptr(), a.batch, d_out[k].data_ptr(), 5)
            torch.cuda.synchronize()
            out[k].append((time.perf_counter() - t) * 1e3)
    h = wide.row_handles(np.arange(g.n_rows, dtype=np.uint32)).astype(np.int64)
    res = {"tuples": g.n_edges, "batch": a.batch, "root_base_words": a.root_base,
           "wide_device_bytes": wide.stats()["device_bytes"], "wide_root_handles_past_2^31": int((h >= 1 << 31).sum()),
           "narrow_kernel": narrow.check_kernel_name(5),
           "ms_median": {k: round(float(np.median(v)), 3) for k, v in out.items()},
           "ms_min": {k: round(float(np.min(v)), 3) for k, v in out.items()},
           "decisions_equal": bool((d_out["narrow"].cpu() == d_out["wide"].cpu()).all()),
           "allowed_fraction": round(float(d_out["narrow"].float().mean()), 4)}
    print(json.dumps(res), flush=True)
    wide.close()
    narrow.close()
    g.close()


if __name__ == "__main__":
    main()
