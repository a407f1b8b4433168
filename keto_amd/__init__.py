"""keto_amd -- MI355X-native batched check / expand engine for Keto's read hot path.

The product is the HIP library ``keto_amd/libketo_mi355x.so`` behind the C-ABI in
``include/keto_mi355x.h``; ``keto_amd.capi`` is its ctypes binding and ``keto_amd.engine`` the
host-side mirror of the reference engine interfaces.
"""
from keto_amd.capi import KetoError, Snapshot, load  # noqa: F401

__all__ = ["KetoError", "Snapshot", "load"]
