"""keto_amd -- MI355X-native batched check / expand engine for Keto's read hot path.

The product is the HIP library ``keto_amd/libketo_mi355x.so`` behind the C-ABI in
``include/keto_mi355x.h``.  ``keto_amd.capi`` is its ctypes binding (``Snapshot``: build / upload /
apply, check and expand batches, tree encoders), ``keto_amd.multi`` the multi-GPU drivers
(replicated sharding, partitioned routing over torch.distributed) and ``keto_amd.build`` the
in-tree gfx950 build.
"""
from keto_amd.capi import KetoError, Snapshot, load  # noqa: F401

__all__ = ["KetoError", "Snapshot", "load"]
