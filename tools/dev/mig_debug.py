"""Debug helper: migrating-partition decisions vs the replicated snapshot, per batch."""
import sys
import numpy as np
import torch
torch.cuda.init()
sys.path.insert(0, ".")
from tests.test_gpu_migrate import _parts_from_csr, _mig_decide
from tools import synth

P = int(sys.argv[1]) if len(sys.argv) > 1 else 1
g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 512), threads=16)
full = g.snapshot(device=0)
parts = _parts_from_csr(g, P)
q = g.queries(60000, seed=141, depth=5)
rng = np.random.default_rng(1)
q["max_depth"] = rng.integers(-1, 7, size=len(q))
for gmd in (3, 5, 3, 5, 2):
    want = full.check_batch_ids(full.with_handles(q), gmd)
    got, rounds = _mig_decide(parts, q, gmd)
    bad = got != want
    d = q["max_depth"].copy()
    d[(d <= 0) | (d > gmd)] = gmd
    print(f"gmd {gmd} rounds {rounds} mismatches {int(bad.sum())} got-values {np.bincount(got[bad], minlength=3)[:4]} "
          f"want-values {np.bincount(want[bad], minlength=2)} eff-depths {np.bincount(d[bad], minlength=gmd + 1)}",
          flush=True)
