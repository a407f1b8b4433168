"""Debug helper: run the migrating partition with a tiny record pool (KETO_MIG_POOL_UNITS) and the
nested graph (big-lane tier) with KETO_MIG_DEBUG=1, so the per-round counters show the rerun paths."""
import os
import sys

import numpy as np
import torch

torch.cuda.init()
sys.path.insert(0, ".")
from tests.test_gpu_migrate import _mig_decide, _parts_from_csr  # noqa: E402
from tools import synth  # noqa: E402

os.environ["KETO_MIG_POOL_UNITS"] = "64"
g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, 1 / 1024), threads=16)
full = g.snapshot(device=0)
parts = _parts_from_csr(g, 3)
q = g.queries(30000, seed=12, depth=5)
want = full.check_batch_ids(full.with_handles(q), 5)
got, rounds = _mig_decide(parts, q, 5)
print("tiny pool: rounds", rounds, "mismatches", int((got != want).sum()), flush=True)
del os.environ["KETO_MIG_POOL_UNITS"]
g = synth.SynthGraph(dict(n_docs=0, n_folders=0, n_groups=1 << 14, n_users=1 << 14, target_edges=0, seed=3),
                     threads=16, kind="nested", chain=32)
full = g.snapshot(device=0)
parts = _parts_from_csr(g, 3, hot_bytes=64 << 10)
q = g.queries_nested(6000, seed=5, depths=(5, 16, 32, 0, 40))
want = full.check_batch_ids(full.with_handles(q), 40)
got, rounds = _mig_decide(parts, q, 40)
print("nested: rounds", rounds, "mismatches", int((got != want).sum()), flush=True)
