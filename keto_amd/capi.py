"""ctypes binding of libketo_mi355x.so (include/keto_mi355x.h).

Plumbing for tests and bench.py.  Loading fails loudly when the library is missing: there is no
Python or CPU fallback of the engine anywhere in this package.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KETO_LIB") or os.path.join(HERE, "libketo_mi355x.so")   # KETO_LIB: tuning builds

KETO_ABI_VERSION = 6          # include/keto_mi355x.h KETO_ABI_VERSION: load() refuses any other library
KETO_OK = 0
E_REBUILD = -6
CHECK_OK, CHECK_UNKNOWN_NAMESPACE, CHECK_UNDECIDED = 0, 1, 2
UNDECIDED = 2                 # decision byte of the ids / device entry points
EXPAND_TREE, EXPAND_NIL, EXPAND_NOT_FOUND, EXPAND_UNDECIDED = 0, 1, 2, 3
NO_ROW = 0xFFFFFFFF
NO_TARGET = 0xFFFFFFFF

EXPORTS = [
    "keto_abi_version", "keto_last_error", "keto_snapshot_build", "keto_snapshot_from_csr",
    "keto_snapshot_release", "keto_snapshot_get_stats", "keto_resolve_checks", "keto_check_batch",
    "keto_check_batch_ids", "keto_check_batch_device", "keto_expand_batch", "keto_tree_arena_free",
    "keto_tree_count", "keto_tree_status", "keto_tree_nodes", "keto_tree_json", "keto_subject_string",
    "keto_last_batch_timing", "keto_check_work_device", "keto_expand_batch_ids", "keto_row_handles",
    "keto_check_kernel_name", "keto_snapshot_upload_part", "keto_row_owner", "keto_check_batch_rows_device",
    "keto_route_work_bytes", "keto_route_rows_device", "keto_unroute_device", "keto_check_batch_rows",
    "keto_host_alloc", "keto_host_free", "keto_check_batch_pairs", "keto_tree_proto", "keto_tree_proto_all",
    "keto_check_steps_device", "keto_snapshot_part_stats", "keto_snapshot_apply", "keto_snapshot_version",
    "keto_snapshot_upload_part_mode", "keto_snapshot_part_stats_mode", "keto_part_stubs", "keto_part_filters",
    "keto_part_close", "keto_part_closure_done", "keto_mig_begin", "keto_mig_round", "keto_device_copy", "keto_device_memory", "keto_snapshot_upload_part_migrate",
    "keto_tree_proto_all_device", "keto_tree_json_all", "keto_subject_fields",
    "keto_comm_id", "keto_comm_init", "keto_comm_free", "keto_check_batch_sharded", "keto_check_batch_routed",
    "keto_check_batch_routed_packed",
    "keto_comm_close_filters", "keto_comm_init_local", "keto_snapshot_clone", "keto_check_batch_packed",
    "keto_snapshot_save", "keto_snapshot_load", "keto_expand_batch_routed",
]
PART_SHARED, PART_MIGRATE = 0, 1
MIG_MAX_PARTS = 30
FILTER_WORDS = 22


class KetoError(RuntimeError):
    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


class KStr(C.Structure):
    _fields_ = [("p", C.c_char_p), ("n", C.c_uint32)]


class KNamespace(C.Structure):
    _fields_ = [("id", C.c_int32), ("name", KStr)]


class KTuple(C.Structure):
    _fields_ = [("namespace_id", C.c_int32), ("object", KStr), ("relation", KStr), ("subject_kind", C.c_uint8),
                ("subject_id", KStr), ("set_namespace_id", C.c_int32), ("set_object", KStr),
                ("set_relation", KStr)]


class KSubject(C.Structure):
    _fields_ = [("kind", C.c_uint8), ("id", KStr), ("set_namespace", KStr), ("set_object", KStr),
                ("set_relation", KStr)]


class KCheckReq(C.Structure):
    _fields_ = [("namespace_", KStr), ("object", KStr), ("relation", KStr), ("subject", KSubject),
                ("max_depth", C.c_int32)]


class KCheckIds(C.Structure):
    _fields_ = [("row", C.c_uint32), ("target", C.c_uint32), ("flags", C.c_uint32), ("max_depth", C.c_int32)]


CHECK_IDS_DTYPE = np.dtype([("row", "<u4"), ("target", "<u4"), ("flags", "<u4"), ("max_depth", "<i4")])
CHECK_PAIR_DTYPE = np.dtype([("row", "<u4"), ("subject", "<u4")])
# keto_check_packed: a request's fields back to back in a blob (offset, six lengths, kind, depth)
CHECK_PACKED_DTYPE = np.dtype([("off", "<u4"), ("len", "<u2", (6,)), ("kind", "u1"), ("reserved", "u1"),
                               ("max_depth", "<i4")], align=True)
assert CHECK_PACKED_DTYPE.itemsize == 24


def pack_requests(reqs):
    """reqs as in Snapshot.check_batch -> (blob bytes, CHECK_PACKED_DTYPE array) for
    keto_check_batch_packed: every request's strings back to back."""
    parts, out = [], np.zeros(len(reqs), dtype=CHECK_PACKED_DTYPE)
    off = 0
    for i, (ns, obj, rel, sub, depth) in enumerate(reqs):
        fields = [ns, obj, rel] + ([sub[1]] if sub[0] == "id" else list(sub[1:4]))
        enc = [f.encode() for f in fields]
        out[i]["off"] = off
        out[i]["len"][:len(enc)] = [len(x) for x in enc]
        out[i]["kind"] = 0 if sub[0] == "id" else 1
        out[i]["max_depth"] = depth
        for x in enc:
            parts.append(x)
            off += len(x)
    return b"".join(parts), out


def pairs_of(q: np.ndarray) -> np.ndarray:
    """keto_check_ids by row id (subject sets flagged) -> 8-B keto_check_pair."""
    p = np.empty(len(q), dtype=CHECK_PAIR_DTYPE)
    p["row"] = q["row"]
    sets = (q["flags"] & 1) != 0
    p["subject"] = np.where(sets & (q["target"] != NO_TARGET), q["target"] | np.uint32(0x80000000), q["target"])
    return p


class KExpandReq(C.Structure):
    _fields_ = [("subject", KSubject), ("max_depth", C.c_int32)]


class KTreeNode(C.Structure):
    _fields_ = [("subject", C.c_uint32), ("info", C.c_uint32)]


class KOpts(C.Structure):
    _fields_ = [("page_size", C.c_uint32), ("device", C.c_int32), ("flags", C.c_uint32)]


class KTiming(C.Structure):
    _fields_ = [("tier_ms", C.c_float * 3), ("requests", C.c_uint32 * 3), ("undecided", C.c_uint32),
                ("chunks", C.c_uint32), ("wall_ms", C.c_float), ("resolve_ms", C.c_float),
                ("items_ms", C.c_float), ("items", C.c_uint32), ("items_kept", C.c_uint32),
                ("index_ms", C.c_float), ("streamed", C.c_uint32), ("stream_stalls", C.c_uint32),
                ("stream_fallbacks", C.c_uint32)]


class KPartStats(C.Structure):
    _fields_ = [("arena_bytes", C.c_uint64), ("shared_bytes", C.c_uint64), ("rows", C.c_uint32),
                ("shared_rows", C.c_uint32), ("root_rows", C.c_uint32), ("stub_rows", C.c_uint64)]


class KMigOut(C.Structure):
    _fields_ = [("units", C.c_uint64 * 30), ("records", C.c_uint32 * 30), ("d_records", C.c_void_p),
                ("d_offsets", C.c_void_p), ("decided", C.c_uint32), ("undecided", C.c_uint32),
                ("processed", C.c_uint32), ("reruns", C.c_uint32)]


class KStats(C.Structure):
    _fields_ = [("n_tuples", C.c_uint64), ("n_edges", C.c_uint64), ("n_rows", C.c_uint32),
                ("n_real_rows", C.c_uint32), ("n_wildcard_rows", C.c_uint32), ("n_seq_rows", C.c_uint32),
                ("n_poisoned_rows", C.c_uint32), ("n_strings", C.c_uint32), ("n_collision_keys", C.c_uint32),
                ("device_bytes", C.c_uint64)]


_lib = None


def load():
    """Load the engine.  In a process that also uses PyTorch-ROCm (which ships its own HIP runtime),
    torch's runtime must be initialized before the engine's: if torch is already imported, this
    initializes it first."""
    global _lib
    if _lib is not None:
        return _lib
    torch = sys.modules.get("torch")
    if torch is not None:
        try:
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass
    if not os.path.exists(LIB_PATH):
        raise KetoError(f"{LIB_PATH} is missing: build it with `python keto_amd/build.py` "
                        "(the engine has no non-HIP implementation)")
    lib = C.CDLL(LIB_PATH)
    # KETO_LIB_PARTIAL=1 (tooling only: a comparison build that predates entry points its run does not
    # call) skips the export check; the ABI version is checked whatever library KETO_LIB names
    if not hasattr(lib, "keto_abi_version") or lib.keto_abi_version() != KETO_ABI_VERSION:
        raise KetoError(f"{LIB_PATH} is not ABI {KETO_ABI_VERSION} (rebuild it with `python keto_amd/build.py`)")
    for name in EXPORTS:
        if not hasattr(lib, name) and not os.environ.get("KETO_LIB_PARTIAL"):
            raise KetoError(f"{LIB_PATH} does not export {name}")
    lib.keto_last_error.restype = C.c_char_p
    lib.keto_check_kernel_name.restype = C.c_char_p
    lib.keto_tree_count.restype = C.c_uint32
    lib.keto_tree_nodes.restype = C.POINTER(KTreeNode)
    lib.keto_tree_json.restype = C.c_int64
    lib.keto_tree_proto.restype = C.c_int64
    lib.keto_tree_proto_all.restype = C.c_int64
    lib.keto_tree_proto_all_device.restype = C.c_int64
    lib.keto_tree_json_all.restype = C.c_int64
    lib.keto_subject_string.restype = C.c_int64
    lib.keto_subject_fields.restype = C.c_int64
    lib.keto_route_work_bytes.restype = C.c_uint64
    lib.keto_snapshot_version.restype = C.c_uint64
    lib.keto_part_stubs.restype = C.c_int64
    lib.keto_route_work_bytes.argtypes = [C.c_uint32, C.c_uint32]
    _lib = lib
    return lib


def _check(rc):
    if rc != KETO_OK:
        raise KetoError(f"keto error {rc}: {load().keto_last_error().decode(errors='replace')}", rc)


def route_work_bytes(n: int, n_parts: int) -> int:
    """Device scratch bytes keto_route_rows_device needs for n requests over n_parts parts."""
    return int(load().keto_route_work_bytes(n, n_parts))


def route_rows_device(d_reqs_ptr: int, n: int, d_owner_ptr: int, n_rows: int, self_part: int, n_parts: int,
                      d_work_ptr: int, work_bytes: int, d_send_ptr: int, d_order_ptr: int, stream=0) -> list:
    """keto_route_rows_device: group n row-id requests by owner part on the device (stable);
    returns the per-part counts (the all-to-all split sizes)."""
    counts = (C.c_uint32 * n_parts)()
    _check(load().keto_route_rows_device(C.c_void_p(d_reqs_ptr), C.c_uint32(n), C.c_void_p(d_owner_ptr),
                                         C.c_uint32(n_rows), C.c_uint32(self_part), C.c_uint32(n_parts),
                                         C.c_void_p(d_work_ptr), C.c_uint64(work_bytes), C.c_void_p(d_send_ptr),
                                         C.c_void_p(d_order_ptr), counts, C.c_void_p(stream)))
    return list(counts)


def device_copy(dst_ptr: int, src_ptr: int, nbytes: int, stream=0) -> None:
    """keto_device_copy: synchronous device-to-device copy on `stream`."""
    _check(load().keto_device_copy(C.c_void_p(dst_ptr), C.c_void_p(src_ptr), C.c_uint64(nbytes), C.c_void_p(stream)))


def unroute_device(d_back_ptr: int, d_order_ptr: int, n: int, d_out_ptr: int, stream=0) -> None:
    """keto_unroute_device: d_out[d_order[j]] = d_back[j]."""
    _check(load().keto_unroute_device(C.c_void_p(d_back_ptr), C.c_void_p(d_order_ptr), C.c_uint32(n),
                                      C.c_void_p(d_out_ptr), C.c_void_p(stream)))


class HostBuffer:
    """Pinned host memory from keto_host_alloc, viewed as a numpy array (freed with the object)."""

    def __init__(self, n: int, dtype):
        lib = load()
        self.dtype = np.dtype(dtype)
        self.n = n
        self.p = C.c_void_p()
        _check(lib.keto_host_alloc(C.c_uint64(max(1, n) * self.dtype.itemsize), C.byref(self.p)))
        buf = (C.c_char * (max(1, n) * self.dtype.itemsize)).from_address(self.p.value)
        self.array = np.frombuffer(buf, dtype=self.dtype, count=n)

    def __del__(self):
        try:
            if self.p:
                load().keto_host_free(self.p)
                self.p = None
        except Exception:
            pass


class _Keep:
    """Keeps encoded strings alive while a call borrows them."""

    def __init__(self):
        self.items = []

    def s(self, x: str) -> KStr:
        b = x.encode()
        self.items.append(b)
        return KStr(b, len(b))


def subject_struct(keep: _Keep, sub) -> KSubject:
    """sub: ("id", str) or ("set", ns, obj, rel), or any object with .id / .namespace fields."""
    if isinstance(sub, tuple):
        if sub[0] == "id":
            return KSubject(0, keep.s(sub[1]), KStr(None, 0), KStr(None, 0), KStr(None, 0))
        return KSubject(1, KStr(None, 0), keep.s(sub[1]), keep.s(sub[2]), keep.s(sub[3]))
    if hasattr(sub, "id"):
        return KSubject(0, keep.s(sub.id), KStr(None, 0), KStr(None, 0), KStr(None, 0))
    return KSubject(1, KStr(None, 0), keep.s(sub.namespace), keep.s(sub.object), keep.s(sub.relation))


class Snapshot:
    def __init__(self, handle, lib):
        self.h = handle
        self.lib = lib

    def close(self):
        """Release the snapshot (host tables and device arena) now."""
        if self.h:
            self.lib.keto_snapshot_release(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ builders
    @staticmethod
    def _tuples(keep: "_Keep", rows):
        tt = (KTuple * max(1, len(rows)))()
        for k, r in enumerate(rows):
            t = tt[k]
            t.namespace_id = r[0]
            t.object = keep.s(r[1])
            t.relation = keep.s(r[2])
            if r[3] is not None:
                t.subject_kind = 0
                t.subject_id = keep.s(r[3])
            else:
                t.subject_kind = 1
                t.set_namespace_id = r[4]
                t.set_object = keep.s(r[5])
                t.set_relation = keep.s(r[6])
        return tt

    def apply(self, inserts=(), deletes=()) -> int:
        """keto_snapshot_apply: one TransactRelationTuples (inserts, then deletes), rows as in build();
        returns the new version.  Raises KetoError (code -6 = KETO_E_REBUILD: rebuild instead)."""
        keep = _Keep()
        ins, dels = list(inserts), list(deletes)
        ver = C.c_uint64()
        _check(self.lib.keto_snapshot_apply(self.h, self._tuples(keep, ins), C.c_uint64(len(ins)),
                                            self._tuples(keep, dels), C.c_uint64(len(dels)), C.byref(ver)))
        return ver.value

    def version(self) -> int:
        return int(self.lib.keto_snapshot_version(self.h))

    @classmethod
    def build(cls, namespaces: Sequence[Tuple[int, str]], rows: Iterable[tuple], page_size=100, device=0):
        """rows: (ns_id, obj, rel, sid) for subject ids, (ns_id, obj, rel, None, sns_id, sobj, srel) for sets,
        in commit order."""
        lib = load()
        keep = _Keep()
        ns = (KNamespace * max(1, len(namespaces)))(*[KNamespace(i, keep.s(n)) for i, n in namespaces])
        rows = list(rows)
        tt = cls._tuples(keep, rows)
        h = C.c_void_p()
        opts = KOpts(page_size, device, 0)
        _check(lib.keto_snapshot_build(ns, len(namespaces), tt, C.c_uint64(len(rows)), C.byref(opts), C.byref(h)))
        return cls(h, lib)

    def clone(self, device: int = 0) -> "Snapshot":
        """keto_snapshot_clone: a replica of this snapshot (current version) on another device."""
        h = C.c_void_p()
        _check(self.lib.keto_snapshot_clone(self.h, C.c_int32(device), C.byref(h)))
        return Snapshot(h, self.lib)

    def save(self, path, tag: int = 0) -> None:
        """keto_snapshot_save: the host tables at the current version to `path`, with the caller's tag."""
        _check(self.lib.keto_snapshot_save(self.h, os.fsencode(path), C.c_uint64(tag)))

    @classmethod
    def load(cls, path, device: int = 0):
        """keto_snapshot_load: a snapshot read back from `path` (device -1: host only); returns
        (snapshot, tag)."""
        lib = load()
        h = C.c_void_p()
        tag = C.c_uint64()
        _check(lib.keto_snapshot_load(os.fsencode(path), C.c_int32(device), C.byref(h), C.byref(tag)))
        return cls(h, lib), tag.value

    def upload_part(self, part: int, n_parts: int, device: int = 0, mode: int = PART_SHARED, hot_bytes: int = 0):
        """Edge-partitioned upload of a host-only snapshot (keto_snapshot_upload_part_mode; a migrating
        partition with hot_bytes > 0 replicates its hottest rows: keto_snapshot_upload_part_migrate)."""
        if mode == PART_MIGRATE and hot_bytes:
            _check(self.lib.keto_snapshot_upload_part_migrate(self.h, C.c_uint32(part), C.c_uint32(n_parts),
                                                              C.c_int32(device), C.c_uint64(hot_bytes)))
        else:
            _check(self.lib.keto_snapshot_upload_part_mode(self.h, C.c_uint32(part), C.c_uint32(n_parts),
                                                           C.c_int32(device), C.c_uint32(mode)))
        self.part, self.n_parts, self.part_mode = part, n_parts, mode
        return self

    def part_stats(self, part: int, n_parts: int, mode: int = PART_SHARED) -> dict:
        """keto_snapshot_part_stats_mode: the arena part `part` of n_parts would hold (host-only snapshot)."""
        st = KPartStats()
        _check(self.lib.keto_snapshot_part_stats_mode(self.h, C.c_uint32(part), C.c_uint32(n_parts), C.c_uint32(mode),
                                                      C.byref(st)))
        return {f: getattr(st, f) for f, _ in KPartStats._fields_}

    # ---- migrating partition (keto_part_* / keto_mig_*)
    def part_stubs(self) -> np.ndarray:
        """Row ids of this migrating part's stubs (other parts' rows its subject sets point at)."""
        n = int(self.lib.keto_part_stubs(self.h, None, C.c_uint64(0)))
        _check(0 if n >= 0 else n)
        out = np.empty(n, dtype=np.uint32)
        if n:
            self.lib.keto_part_stubs(self.h, out.ctypes.data_as(C.c_void_p), C.c_uint64(n))
        return out

    def part_filters(self, rows: np.ndarray) -> np.ndarray:
        """Current closure filters [n, FILTER_WORDS] of rows this part owns."""
        rows = np.ascontiguousarray(rows, dtype=np.uint32)
        out = np.empty((len(rows), FILTER_WORDS), dtype=np.uint32)
        _check(self.lib.keto_part_filters(self.h, rows.ctypes.data_as(C.c_void_p), C.c_uint64(len(rows)),
                                          out.ctypes.data_as(C.c_void_p)))
        return out

    def part_close(self, stub_rows: np.ndarray, filters: np.ndarray) -> int:
        """OR the owners' filters into these stubs and re-close this part's filters; returns changes."""
        stub_rows = np.ascontiguousarray(stub_rows, dtype=np.uint32)
        filters = np.ascontiguousarray(filters, dtype=np.uint32)
        ch = C.c_uint64(0)
        _check(self.lib.keto_part_close(self.h, stub_rows.ctypes.data_as(C.c_void_p), C.c_uint64(len(stub_rows)),
                                        filters.ctypes.data_as(C.c_void_p), C.byref(ch)))
        return int(ch.value)

    def part_closure_done(self, converged: bool = True):
        _check(self.lib.keto_part_closure_done(self.h, C.c_int(1 if converged else 0)))

    @staticmethod
    def _mig_out(o: "KMigOut", n_parts: int) -> dict:
        return {"units": [int(o.units[p]) for p in range(n_parts)],
                "records": [int(o.records[p]) for p in range(n_parts)],
                "d_records": int(o.d_records or 0), "d_offsets": int(o.d_offsets or 0),
                "decided": int(o.decided), "undecided": int(o.undecided), "processed": int(o.processed),
                "reruns": int(o.reruns)}

    def mig_begin(self, d_reqs_ptr: int, n: int, d_out_ptr: int, global_max_depth=5, stream=0) -> dict:
        """keto_mig_begin: start the searches of the row-id requests routed to this part."""
        o = KMigOut()
        _check(self.lib.keto_mig_begin(self.h, C.c_void_p(d_reqs_ptr), C.c_uint32(n), C.c_int32(global_max_depth),
                                       C.c_void_p(d_out_ptr), C.c_void_p(stream), C.byref(o)))
        return self._mig_out(o, self.n_parts)

    def mig_round(self, d_records_ptr: int, d_offsets_ptr: int, in_records, in_units, stream=0) -> dict:
        """keto_mig_round: continue the searches of the records received from every source part."""
        rec = (C.c_uint32 * MIG_MAX_PARTS)(*[int(x) for x in in_records])
        uni = (C.c_uint64 * MIG_MAX_PARTS)(*[int(x) for x in in_units])
        o = KMigOut()
        _check(self.lib.keto_mig_round(self.h, C.c_void_p(d_records_ptr), C.c_void_p(d_offsets_ptr), rec, uni,
                                       C.c_void_p(stream), C.byref(o)))
        return self._mig_out(o, self.n_parts)

    def row_owner(self, rows: np.ndarray, n_parts: int) -> np.ndarray:
        """Owner part of each row id (-1: held by every part)."""
        rows = np.ascontiguousarray(rows, dtype=np.uint32)
        out = np.empty(len(rows), dtype=np.int32)
        _check(self.lib.keto_row_owner(self.h, rows.ctypes.data_as(C.c_void_p), C.c_uint64(len(rows)),
                                       C.c_uint32(n_parts), out.ctypes.data_as(C.c_void_p)))
        return out

    @classmethod
    def from_csr(cls, namespaces, row_ns, row_obj, row_rel, row_ptr, edges, strings=None, page_size=100, device=0,
                 kstrs=None):
        """kstrs: (KStr array, n) string table already in C memory (large graphs), instead of strings."""
        lib = load()
        keep = _Keep()
        ns = (KNamespace * max(1, len(namespaces)))(*[KNamespace(i, keep.s(n)) for i, n in namespaces])
        row_ns = np.ascontiguousarray(row_ns, dtype=np.int32)
        row_obj = np.ascontiguousarray(row_obj, dtype=np.uint32)
        row_rel = np.ascontiguousarray(row_rel, dtype=np.uint32)
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.uint64)
        edges = np.ascontiguousarray(edges, dtype=np.uint32)
        strs = None
        n_str = 0
        if strings is not None:
            strs = (KStr * max(1, len(strings)))(*[keep.s(x) for x in strings])
            n_str = len(strings)
        elif kstrs is not None:
            strs, n_str = kstrs
        h = C.c_void_p()
        opts = KOpts(page_size, device, 0)
        p = lambda a: a.ctypes.data_as(C.c_void_p)
        _check(lib.keto_snapshot_from_csr(ns, len(namespaces), C.c_uint32(len(row_ns)), p(row_ns), p(row_obj),
                                          p(row_rel), p(row_ptr), p(edges), strs, C.c_uint32(n_str),
                                          C.byref(opts), C.byref(h)))
        return cls(h, lib)

    def stats(self) -> dict:
        st = KStats()
        _check(self.lib.keto_snapshot_get_stats(self.h, C.byref(st)))
        return {f: getattr(st, f) for f, _ in KStats._fields_}

    # ------------------------------------------------------------------ check
    def _check_reqs(self, keep, reqs):
        arr = (KCheckReq * max(1, len(reqs)))()
        for k, (ns, obj, rel, sub, depth) in enumerate(reqs):
            arr[k].namespace_ = keep.s(ns)
            arr[k].object = keep.s(obj)
            arr[k].relation = keep.s(rel)
            arr[k].subject = subject_struct(keep, sub)
            arr[k].max_depth = depth
        return arr

    def check_batch_reqs(self, arr, n: int, global_max_depth=5):
        """keto_check_batch on a prepared KCheckReq array (string requests: in-library resolution)."""
        allowed = np.zeros(max(1, n), dtype=np.uint8)
        status = np.zeros(max(1, n), dtype=np.uint8)
        _check(self.lib.keto_check_batch(self.h, arr, C.c_uint32(n), C.c_int32(global_max_depth),
                                         allowed.ctypes.data_as(C.c_void_p), status.ctypes.data_as(C.c_void_p)))
        return allowed[:n], status[:n]

    def check_batch_packed(self, blob, packed: np.ndarray, global_max_depth=5, n=None, allowed=None, status=None):
        """keto_check_batch_packed: requests resolved on the GPU from one string blob (bytes, a numpy
        uint8 array or a HostBuffer array) and CHECK_PACKED_DTYPE records.  Returns (allowed, status)."""
        n = len(packed) if n is None else n
        packed = np.ascontiguousarray(packed, dtype=CHECK_PACKED_DTYPE)
        blob, blen = _blob_array(blob)
        if allowed is None:
            allowed = np.zeros(max(1, n), dtype=np.uint8)
        if status is None:
            status = np.zeros(max(1, n), dtype=np.uint8)
        _check(self.lib.keto_check_batch_packed(self.h, blob.ctypes.data_as(C.c_void_p), C.c_uint64(blen),
                                                packed.ctypes.data_as(C.c_void_p), C.c_uint32(n),
                                                C.c_int32(global_max_depth), allowed.ctypes.data_as(C.c_void_p),
                                                status.ctypes.data_as(C.c_void_p)))
        return allowed[:n], status[:n]

    def check_batch(self, reqs, global_max_depth=5):
        """reqs: list of (namespace, object, relation, subject, max_depth). Returns (allowed, status)."""
        keep = _Keep()
        arr = self._check_reqs(keep, reqs)
        n = len(reqs)
        allowed = np.zeros(max(1, n), dtype=np.uint8)
        status = np.zeros(max(1, n), dtype=np.uint8)
        _check(self.lib.keto_check_batch(self.h, arr, C.c_uint32(n), C.c_int32(global_max_depth),
                                         allowed.ctypes.data_as(C.c_void_p), status.ctypes.data_as(C.c_void_p)))
        return allowed[:n], status[:n]

    def resolve_checks_reqs(self, arr, n: int):
        """keto_resolve_checks on a prepared KCheckReq array: (device-form requests, statuses)."""
        out = np.zeros(max(1, n), dtype=CHECK_IDS_DTYPE)
        status = np.zeros(max(1, n), dtype=np.uint8)
        _check(self.lib.keto_resolve_checks(self.h, arr, C.c_uint32(n), out.ctypes.data_as(C.c_void_p),
                                            status.ctypes.data_as(C.c_void_p)))
        return out[:n], status[:n]

    def resolve_checks(self, reqs):
        keep = _Keep()
        arr = self._check_reqs(keep, reqs)
        n = len(reqs)
        out = np.zeros(max(1, n), dtype=CHECK_IDS_DTYPE)
        status = np.zeros(max(1, n), dtype=np.uint8)
        _check(self.lib.keto_resolve_checks(self.h, arr, C.c_uint32(n), out.ctypes.data_as(C.c_void_p),
                                            status.ctypes.data_as(C.c_void_p)))
        return out[:n], status[:n]

    def row_handles(self, rows: np.ndarray) -> np.ndarray:
        rows = np.ascontiguousarray(rows, dtype=np.uint32)
        out = np.empty_like(rows)
        _check(self.lib.keto_row_handles(self.h, rows.ctypes.data_as(C.c_void_p), C.c_uint64(len(rows)),
                                         out.ctypes.data_as(C.c_void_p)))
        return out

    def with_handles(self, q: np.ndarray) -> np.ndarray:
        """Requests whose `row` holds row ids (and subject-id targets) -> device form."""
        d = np.array(q, dtype=CHECK_IDS_DTYPE, copy=True)
        d["row"] = self.row_handles(d["row"])
        return d

    def check_batch_ids(self, ids: np.ndarray, global_max_depth=5):
        ids = np.ascontiguousarray(ids, dtype=CHECK_IDS_DTYPE)
        n = len(ids)
        allowed = np.zeros(max(1, n), dtype=np.uint8)
        _check(self.lib.keto_check_batch_ids(self.h, ids.ctypes.data_as(C.c_void_p), C.c_uint32(n),
                                             C.c_int32(global_max_depth), allowed.ctypes.data_as(C.c_void_p)))
        return allowed[:n]

    def check_batch_rows(self, ids: np.ndarray, global_max_depth=5, out: Optional[np.ndarray] = None):
        """keto_check_batch_rows: host requests naming rows by row id (translated on the device),
        pipelined H2D / check / D2H.  `ids` / `out` may live in pinned memory (HostBuffer)."""
        ids = np.ascontiguousarray(ids, dtype=CHECK_IDS_DTYPE)
        n = len(ids)
        if out is None:
            out = np.zeros(max(1, n), dtype=np.uint8)
        _check(self.lib.keto_check_batch_rows(self.h, ids.ctypes.data_as(C.c_void_p), C.c_uint32(n),
                                              C.c_int32(global_max_depth), out.ctypes.data_as(C.c_void_p)))
        return out[:n]

    def check_batch_pairs(self, pairs: np.ndarray, max_depth=0, global_max_depth=5, out: Optional[np.ndarray] = None):
        """keto_check_batch_pairs: 8-B requests by row id, one request max-depth for the batch."""
        pairs = np.ascontiguousarray(pairs, dtype=CHECK_PAIR_DTYPE)
        n = len(pairs)
        if out is None:
            out = np.zeros(max(1, n), dtype=np.uint8)
        _check(self.lib.keto_check_batch_pairs(self.h, pairs.ctypes.data_as(C.c_void_p), C.c_uint32(n),
                                               C.c_int32(max_depth), C.c_int32(global_max_depth),
                                               out.ctypes.data_as(C.c_void_p)))
        return out[:n]

    def check_batch_device(self, d_ids_ptr: int, n: int, d_out_ptr: int, global_max_depth=5, stream=0):
        _check(self.lib.keto_check_batch_device(self.h, C.c_void_p(d_ids_ptr), C.c_uint32(n),
                                                C.c_int32(global_max_depth), C.c_void_p(d_out_ptr),
                                                C.c_void_p(stream)))

    def check_batch_rows_device(self, d_ids_ptr: int, n: int, d_out_ptr: int, global_max_depth=5, stream=0):
        """Device-resident requests naming rows by row id (partitioned mode)."""
        _check(self.lib.keto_check_batch_rows_device(self.h, C.c_void_p(d_ids_ptr), C.c_uint32(n),
                                                     C.c_int32(global_max_depth), C.c_void_p(d_out_ptr),
                                                     C.c_void_p(stream)))

    def last_timing(self):
        t = KTiming()
        _check(self.lib.keto_last_batch_timing(self.h, C.byref(t)))
        return list(t.tier_ms), list(t.requests)

    def last_timing_full(self) -> dict:
        t = KTiming()
        _check(self.lib.keto_last_batch_timing(self.h, C.byref(t)))
        return {"tier_ms": list(t.tier_ms), "requests": list(t.requests), "undecided": t.undecided,
                "chunks": t.chunks, "wall_ms": t.wall_ms, "resolve_ms": t.resolve_ms,
                "items_ms": t.items_ms, "items": t.items, "items_kept": t.items_kept, "index_ms": t.index_ms,
                "streamed": t.streamed, "stream_stalls": t.stream_stalls, "stream_fallbacks": t.stream_fallbacks}

    @staticmethod
    def check_kernel_name(global_max_depth=5) -> str:
        """Tier-0 check kernel a batch at this global max-depth launches (profile matching)."""
        return load().keto_check_kernel_name(C.c_int32(global_max_depth)).decode()

    def check_work_device(self, d_ids_ptr: int, n: int, d_out_ptr: int, global_max_depth=5):
        out = (C.c_uint64 * 16)()
        _check(self.lib.keto_check_work_device(self.h, C.c_void_p(d_ids_ptr), C.c_uint32(n),
                                               C.c_int32(global_max_depth), C.c_void_p(d_out_ptr), out))
        return list(out)

    def check_steps_device(self, d_ids_ptr: int, n: int, d_out_ptr: int, d_steps_ptr: int, global_max_depth=32):
        _check(self.lib.keto_check_steps_device(self.h, C.c_void_p(d_ids_ptr), C.c_uint32(n),
                                                C.c_int32(global_max_depth), C.c_void_p(d_out_ptr),
                                                C.c_void_p(d_steps_ptr)))

    # ------------------------------------------------------------------ expand
    def expand_batch_ids(self, roots: np.ndarray, depths: np.ndarray, global_max_depth=5):
        """Pre-resolved roots (bit31 = subject set row). Returns (status[n], offsets[n+1], nodes[m,2])."""
        roots = np.ascontiguousarray(roots, dtype=np.uint32)
        depths = np.ascontiguousarray(depths, dtype=np.int32)
        n = len(roots)
        a = C.c_void_p()
        _check(self.lib.keto_expand_batch_ids(self.h, roots.ctypes.data_as(C.c_void_p),
                                              depths.ctypes.data_as(C.c_void_p), C.c_uint32(n),
                                              C.c_int32(global_max_depth), C.byref(a)))
        try:
            status = np.array([self.lib.keto_tree_status(a, C.c_uint32(i)) for i in range(n)], dtype=np.int32)
            offs = np.zeros(n + 1, dtype=np.int64)
            chunks = []
            for i in range(n):
                nn = C.c_uint64()
                ptr = self.lib.keto_tree_nodes(a, C.c_uint32(i), C.byref(nn))
                offs[i + 1] = offs[i] + nn.value
                if nn.value:
                    buf = (C.c_uint32 * (2 * nn.value)).from_address(C.cast(ptr, C.c_void_p).value)
                    chunks.append(np.frombuffer(buf, dtype=np.uint32).copy().reshape(-1, 2))
            nodes = np.concatenate(chunks) if chunks else np.zeros((0, 2), dtype=np.uint32)
        finally:
            self.lib.keto_tree_arena_free(a)
        return status, offs, nodes

    def expand_batch_ids_proto(self, roots: np.ndarray, depths: np.ndarray, global_max_depth=5, device=False):
        """Pre-resolved roots -> every tree's SubjectTree proto in one buffer (keto_tree_proto_all, or
        keto_tree_proto_all_device).  Returns (status[n], offsets[n+1] into the blob, blob, expand seconds,
        encode seconds)."""
        import time
        roots = np.ascontiguousarray(roots, dtype=np.uint32)
        depths = np.ascontiguousarray(depths, dtype=np.int32)
        n = len(roots)
        a = C.c_void_p()
        t0 = time.perf_counter()
        _check(self.lib.keto_expand_batch_ids(self.h, roots.ctypes.data_as(C.c_void_p),
                                              depths.ctypes.data_as(C.c_void_p), C.c_uint32(n),
                                              C.c_int32(global_max_depth), C.byref(a)))
        t1 = time.perf_counter()
        try:
            offs, blob, t_enc = self._proto_all(a, n, device=device)
            status = np.array([self.lib.keto_tree_status(a, C.c_uint32(i)) for i in range(n)], dtype=np.int32)
        finally:
            self.lib.keto_tree_arena_free(a)
        return status, offs, blob, t1 - t0, t_enc

    def _proto_all(self, a, n, device=False):
        """(offsets[n+1], blob, seconds of the sizing + filling calls, as a caller pays them) of
        keto_tree_proto_all[_device] (the host encoder keeps a sizing call's encodings for the fill)."""
        import time
        fn = self.lib.keto_tree_proto_all_device if device else self.lib.keto_tree_proto_all
        offs = np.zeros(n + 1, dtype=np.uint64)
        t0 = time.perf_counter()
        total = fn(self.h, a, None, C.c_uint64(0), offs.ctypes.data_as(C.c_void_p))
        _check(min(0, total))
        blob = np.empty(max(1, total), dtype=np.uint8)
        got = fn(self.h, a, blob.ctypes.data_as(C.c_void_p), C.c_uint64(total), offs.ctypes.data_as(C.c_void_p))
        dt = time.perf_counter() - t0
        _check(min(0, got))
        assert got == total
        return offs, blob[:total].tobytes(), dt

    def _json_all(self, a, n):
        """Every tree's JSON text from keto_tree_json_all ("null" for nil trees, "" for errors)."""
        offs = np.zeros(n + 1, dtype=np.uint64)
        total = self.lib.keto_tree_json_all(self.h, a, None, C.c_uint64(0), offs.ctypes.data_as(C.c_void_p))
        _check(min(0, total))
        blob = C.create_string_buffer(max(1, total))
        got = self.lib.keto_tree_json_all(self.h, a, blob, C.c_uint64(total), offs.ctypes.data_as(C.c_void_p))
        _check(min(0, got))
        raw = blob.raw[:total]
        return [raw[int(offs[i]):int(offs[i + 1])].decode() for i in range(n)]

    def subject_fields(self, refs, arena=None):
        """keto_subject_fields: per subject reference ("id", id) or ("set", namespace, object, relation)."""
        refs = np.ascontiguousarray(refs, dtype=np.uint32)
        n = len(refs)
        lens = np.zeros(max(1, 3 * n), dtype=np.uint32)
        a = arena if arena is not None else None
        total = self.lib.keto_subject_fields(self.h, a, refs.ctypes.data_as(C.c_void_p), C.c_uint64(n), None,
                                             C.c_uint64(0), lens.ctypes.data_as(C.c_void_p))
        _check(min(0, total))
        buf = C.create_string_buffer(max(1, total))
        got = self.lib.keto_subject_fields(self.h, a, refs.ctypes.data_as(C.c_void_p), C.c_uint64(n), buf,
                                           C.c_uint64(total), lens.ctypes.data_as(C.c_void_p))
        _check(min(0, got))
        raw, at, out = buf.raw[:total], 0, []
        for i in range(n):
            parts = []
            for k in range(3 if refs[i] & 0x80000000 else 1):
                ln = int(lens[3 * i + k])
                parts.append(raw[at:at + ln].decode())
                at += ln
            out.append(("set", *parts) if refs[i] & 0x80000000 else ("id", parts[0]))
        return out

    def _tree_via_fields(self, a, i):
        """Tree i as the Go shim builds expand.Tree: pre-order nodes (keto_tree_nodes) + their subjects'
        fields (keto_subject_fields), as Tree.MarshalJSON's structure (a dict)."""
        nn = C.c_uint64()
        ptr = self.lib.keto_tree_nodes(a, C.c_uint32(i), C.byref(nn))
        nodes = [(ptr[j].subject, ptr[j].info) for j in range(nn.value)]
        fields = self.subject_fields([x for x, _ in nodes], arena=a) if nodes else []
        root, stack = None, []
        for (subj_ref, info), f in zip(nodes, fields):
            leaf = bool(info & 0x80000000)
            t = {"type": "leaf" if leaf else "union"}
            if f[0] == "id":
                t["subject_id"] = f[1]
            else:
                t["subject_set"] = {"namespace": f[1], "object": f[2], "relation": f[3]}
            if stack:
                stack[-1][0].setdefault("children", []).append(t)
                stack[-1][1] -= 1
            else:
                root = t
            if not leaf and info & 0x7FFFFFFF:
                stack.append([t, info & 0x7FFFFFFF])
            while stack and stack[-1][1] == 0:
                stack.pop()
        return root

    def expand_batch(self, reqs, global_max_depth=5, want_nodes=False, want_proto=False, proto_all=None,
                     json_all=False, via_fields=False):
        """reqs: list of (subject, max_depth). Returns list of (status, json_or_None[, nodes][, proto]);
        proto_all = "host" / "device": also every tree's bytes from keto_tree_proto_all[_device]
        (returned as (list, per-tree bytes list)); json_all: also every tree's JSON text from
        keto_tree_json_all (returned as (list, per-tree text list)); via_fields: also each tree rebuilt
        from its nodes and keto_subject_fields (the Go shim's path), as a dict."""
        keep = _Keep()
        n = len(reqs)
        arr = self._expand_reqs(keep, reqs)
        a = C.c_void_p()
        _check(self.lib.keto_expand_batch(self.h, arr, C.c_uint32(n), C.c_int32(global_max_depth), C.byref(a)))
        return self._arena_results(a, n, want_nodes, want_proto, proto_all, json_all, via_fields)

    @staticmethod
    def _expand_reqs(keep, reqs):
        arr = (KExpandReq * max(1, len(reqs)))()
        for k, (sub, depth) in enumerate(reqs):
            arr[k].subject = subject_struct(keep, sub)
            arr[k].max_depth = depth
        return arr

    def _arena_results(self, a, n, want_nodes=False, want_proto=False, proto_all=None, json_all=False,
                       via_fields=False):
        """The trees of arena `a` (freed here) as expand_batch returns them."""
        out = []
        try:
            for i in range(n):
                st = self.lib.keto_tree_status(a, C.c_uint32(i))
                js = None
                if st == EXPAND_TREE:
                    ln = self.lib.keto_tree_json(self.h, a, C.c_uint32(i), None, C.c_uint64(0))
                    buf = C.create_string_buffer(ln + 1)
                    self.lib.keto_tree_json(self.h, a, C.c_uint32(i), buf, C.c_uint64(ln + 1))
                    js = json.loads(buf.raw[:ln].decode())
                item = (st, js)
                if via_fields:
                    item = item + (self._tree_via_fields(a, i) if st == EXPAND_TREE else None,)
                if want_nodes:
                    nn = C.c_uint64()
                    ptr = self.lib.keto_tree_nodes(a, C.c_uint32(i), C.byref(nn))
                    nodes = [(ptr[j].subject, ptr[j].info) for j in range(nn.value)] if nn.value else []
                    item = item + (nodes,)
                if want_proto:
                    pn = self.lib.keto_tree_proto(self.h, a, C.c_uint32(i), None, C.c_uint64(0))
                    pb = None
                    if pn >= 0:
                        buf = C.create_string_buffer(max(1, pn))
                        self.lib.keto_tree_proto(self.h, a, C.c_uint32(i), buf, C.c_uint64(pn))
                        pb = buf.raw[:pn]
                    item = item + (pb,)
                out.append(item)
            if proto_all:
                offs, blob, _ = self._proto_all(a, n, device=proto_all == "device")
                return out, [blob[int(offs[i]):int(offs[i + 1])] for i in range(n)]
            if json_all:
                return out, self._json_all(a, n)
        finally:
            self.lib.keto_tree_arena_free(a)
        return out


def _blob_array(blob):
    """A packed batch's string blob (bytes, a numpy uint8 array or a HostBuffer array) -> (array, bytes used)."""
    if isinstance(blob, (bytes, bytearray)):
        blen = len(blob)
        return (np.frombuffer(blob, dtype=np.uint8) if blen else np.zeros(1, dtype=np.uint8)), blen
    return blob, blob.nbytes


class Comm:
    """A keto_comm: multi-GPU batches over RCCL behind the C-ABI (keto_amd/csrc/comm.cpp), one process
    per GPU.  Every rank builds it with the id one rank made (Comm.make_id) and distributed."""

    @staticmethod
    def make_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        _check(load().keto_comm_id(buf))
        return bytes(buf)

    def __init__(self, comm_id: bytes, n_ranks: int, rank: int, device: int = 0, local: bool = False):
        """local: keto_comm_init_local (the ranks are threads of this process; comm_id any 128 bytes)."""
        self.lib = load()
        self.h = C.c_void_p()
        self.rank, self.n_ranks = rank, n_ranks
        idb = (C.c_uint8 * 128).from_buffer_copy(comm_id.ljust(128, b"\0")[:128])
        init = self.lib.keto_comm_init_local if local else self.lib.keto_comm_init
        _check(init(idb, C.c_int32(n_ranks), C.c_int32(rank), C.c_int32(device), C.byref(self.h)))

    def close(self):
        if self.h:
            self.lib.keto_comm_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _batch(self, fn, snap, reqs, global_max_depth, n=None):
        """reqs: a list as in Snapshot.check_batch, or a prepared KCheckReq array of n requests."""
        keep = _Keep()
        if n is None:
            arr = snap._check_reqs(keep, reqs)
            n = len(reqs)
        else:
            arr = reqs
        allowed = np.zeros(max(1, n), dtype=np.uint8)
        status = np.zeros(max(1, n), dtype=np.uint8)
        _check(fn(self.h, snap.h, arr, C.c_uint32(n), C.c_int32(global_max_depth), allowed.ctypes.data_as(C.c_void_p),
                  status.ctypes.data_as(C.c_void_p)))
        return allowed[:n], status[:n]

    def check_batch_sharded(self, snap, reqs, global_max_depth=5, n=None):
        """keto_check_batch_sharded (replicated snapshot): reqs as in Snapshot.check_batch."""
        return self._batch(self.lib.keto_check_batch_sharded, snap, reqs, global_max_depth, n)

    def check_batch_routed(self, snap, reqs, global_max_depth=5, n=None):
        """keto_check_batch_routed (this rank's part of an edge-partitioned snapshot)."""
        return self._batch(self.lib.keto_check_batch_routed, snap, reqs, global_max_depth, n)

    def check_batch_routed_packed(self, snap, blob, packed: np.ndarray, global_max_depth=5, n=None):
        """keto_check_batch_routed_packed: a packed batch (as Snapshot.check_batch_packed takes it),
        resolved on this rank's device and routed to the parts owning its rows."""
        n = len(packed) if n is None else n
        packed = np.ascontiguousarray(packed, dtype=CHECK_PACKED_DTYPE)
        blob, blen = _blob_array(blob)
        allowed = np.zeros(max(1, n), dtype=np.uint8)
        status = np.zeros(max(1, n), dtype=np.uint8)
        _check(self.lib.keto_check_batch_routed_packed(self.h, snap.h, blob.ctypes.data_as(C.c_void_p), C.c_uint64(blen),
                                                       packed.ctypes.data_as(C.c_void_p), C.c_uint32(n),
                                                       C.c_int32(global_max_depth), allowed.ctypes.data_as(C.c_void_p),
                                                       status.ctypes.data_as(C.c_void_p)))
        return allowed[:n], status[:n]

    def expand_batch_routed(self, snap, reqs, global_max_depth=5, **kw):
        """keto_expand_batch_routed (this rank's shared-rows or migrating part): reqs and results as
        in Snapshot.expand_batch."""
        keep = _Keep()
        arr = snap._expand_reqs(keep, reqs)
        a = C.c_void_p()
        _check(self.lib.keto_expand_batch_routed(self.h, snap.h, arr, C.c_uint32(len(reqs)),
                                                 C.c_int32(global_max_depth), C.byref(a)))
        return snap._arena_results(a, len(reqs), **kw)

    def close_filters(self, snap) -> int:
        rounds = C.c_uint32(0)
        _check(self.lib.keto_comm_close_filters(self.h, snap.h, C.byref(rounds)))
        return rounds.value
