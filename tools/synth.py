"""ctypes front-end of tools/synth.cpp: synthetic ACL graphs / request batches (bench tooling)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "synth.cpp")
LIB = os.path.join(HERE, "libketo_synth.so")

NAMESPACES = [(1, "docs"), (2, "folders"), (3, "groups")]
DRIVE_NAMESPACES = [(1, "files"), (2, "folders"), (3, "groups")]


def build(force=False):
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", SRC, "-o", LIB])
    return LIB


class Params(C.Structure):
    _fields_ = [("n_docs", C.c_uint64), ("n_folders", C.c_uint64), ("n_groups", C.c_uint64),
                ("n_users", C.c_uint64), ("target_edges", C.c_uint64), ("seed", C.c_uint64)]


class Graph(C.Structure):
    _fields_ = [("n_rows", C.c_uint32), ("row_ns", C.POINTER(C.c_int32)), ("row_obj", C.POINTER(C.c_uint32)),
                ("row_rel", C.POINTER(C.c_uint32)), ("row_ptr", C.POINTER(C.c_uint64)),
                ("edges", C.POINTER(C.c_uint32)), ("n_edges", C.c_uint64), ("n_set_edges", C.c_uint64)]


class Strings(C.Structure):
    _fields_ = [("n", C.c_uint64), ("tuples", C.c_void_p), ("names", C.c_void_p), ("obj_base", C.c_uint64),
                ("user_base", C.c_uint64), ("rel_base", C.c_uint64), ("rel_off", C.c_uint32 * 8),
                ("rel_len", C.c_uint32 * 8)]


class Table(C.Structure):
    _fields_ = [("n", C.c_uint64), ("ns", C.c_void_p), ("obj", C.c_void_p), ("rel", C.c_void_p),
                ("kind", C.c_void_p), ("sid", C.c_void_p), ("sns", C.c_void_p), ("sobj", C.c_void_p),
                ("srel", C.c_void_p), ("key", C.c_void_p)]


# BASELINE.json config #4: 1,000,000,000 tuples, ~30 % subject-set edges (seed 4)
POWERLAW_1B = dict(n_docs=1 << 27, n_folders=1 << 24, n_groups=1 << 22, n_users=1 << 26,
                   target_edges=1_000_000_000, seed=4)


def scaled(params: dict, scale: float) -> dict:
    p = dict(params)
    for k in ("n_docs", "n_folders", "n_groups", "n_users"):
        p[k] = max(64, int(p[k] * scale))
    p["target_edges"] = int(p["target_edges"] * scale)
    return p


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = C.CDLL(LIB)
        _lib.synth_pack_reqs.restype = C.c_int64
    return _lib


# BASELINE.json config #3: nested group membership, chains up to 32, cycles (seed 3)
NESTED_100M = dict(n_docs=0, n_folders=0, n_groups=1 << 24, n_users=1 << 24, target_edges=100_000_000, seed=3)

# BASELINE.json config #2 / SURVEY.md 8(d): Drive-like files / folder forest (fan-out 8, depth <= 6) /
# Zipf(1.1) groups, exactly 10,000,000 tuples (seed 2); n_docs = files, folders = 8 full trees
DRIVE_10M = dict(n_docs=2_000_000, n_folders=8 * 37449, n_groups=50_000, n_users=1 << 20,
                 target_edges=10_000_000, seed=2)


class Unified:
    """SynthGraph.unified(): from_csr arrays in one string id space plus the string table."""

    def to_device_targets(self, q: np.ndarray) -> np.ndarray:
        """Requests of SynthGraph.queries (user targets) in the unified id space."""
        out = q.copy()
        out["target"] = q["target"] + np.uint32(self.user_base)
        return out

    def free(self):
        if getattr(self, "names", None) is not None and self.names.names:
            lib().synth_strings_free(C.byref(self.names))
            self.names = None


class SynthGraph:
    def __init__(self, params: dict, threads: int = 16, kind: str = "powerlaw", chain: int = 32):
        self.params = params
        self.kind = kind
        self.p = Params(**{k: params[k] for k, _ in Params._fields_})
        self.g = Graph()
        self.namespaces = DRIVE_NAMESPACES if kind == "drive" else NAMESPACES
        if kind == "nested":
            rc = lib().synth_generate_nested(C.byref(self.p), C.c_uint32(chain), C.c_int(threads), C.byref(self.g))
        elif kind == "drive":
            rc = lib().synth_generate_drive(C.byref(self.p), C.c_int(threads), C.byref(self.g))
        else:
            rc = lib().synth_generate(C.byref(self.p), C.c_int(threads), C.byref(self.g))
        if rc != 0:
            raise RuntimeError(f"synth_generate failed: {rc}")
        R, E = self.g.n_rows, self.g.n_edges
        self.row_ns = np.ctypeslib.as_array(self.g.row_ns, shape=(R,))
        self.row_obj = np.ctypeslib.as_array(self.g.row_obj, shape=(R,))
        self.row_rel = np.ctypeslib.as_array(self.g.row_rel, shape=(R,))
        self.row_ptr = np.ctypeslib.as_array(self.g.row_ptr, shape=(R + 1,))
        self.edges = np.ctypeslib.as_array(self.g.edges, shape=(max(E, 1),))[:E]

    @property
    def n_rows(self):
        return self.g.n_rows

    @property
    def n_edges(self):
        return self.g.n_edges

    @property
    def n_set_edges(self):
        return self.g.n_set_edges

    def close(self):
        if self.g.row_ptr:
            lib().synth_free(C.byref(self.g))

    def queries(self, n: int, seed: int, depth: int = 5, threads: int = 16) -> np.ndarray:
        from keto_amd.capi import CHECK_IDS_DTYPE
        out = np.zeros(n, dtype=CHECK_IDS_DTYPE)
        fn = lib().synth_queries_drive if self.kind == "drive" else lib().synth_queries
        fn(C.byref(self.g), C.byref(self.p), C.c_uint64(n), C.c_uint64(seed), C.c_int32(depth),
                            out.ctypes.data_as(C.c_void_p), C.c_int(threads))
        return out

    def queries_nested(self, n: int, seed: int, depths=(5, 16, 32), threads: int = 16) -> np.ndarray:
        from keto_amd.capi import CHECK_IDS_DTYPE
        out = np.zeros(n, dtype=CHECK_IDS_DTYPE)
        d = np.ascontiguousarray(depths, dtype=np.int32)
        lib().synth_queries_nested(C.byref(self.g), C.byref(self.p), C.c_uint64(n), C.c_uint64(seed),
                                   d.ctypes.data_as(C.c_void_p), C.c_uint32(len(d)), out.ctypes.data_as(C.c_void_p),
                                   C.c_int(threads))
        return out

    def snapshot(self, device=0):
        from keto_amd.capi import Snapshot
        return Snapshot.from_csr(self.namespaces, self.row_ns, self.row_obj, self.row_rel, self.row_ptr, self.edges,
                                 device=device)

    def snapshot_part(self, part: int, n_parts: int, device=0, mode=0, hot_bytes=0):
        """This part's share of the edge-partitioned snapshot (keto_snapshot_upload_part_mode; mode 1 =
        the migrating partition, with hot_bytes of replicated hot rows)."""
        from keto_amd.capi import Snapshot
        s = Snapshot.from_csr(self.namespaces, self.row_ns, self.row_obj, self.row_rel, self.row_ptr, self.edges,
                              device=-1)
        return s.upload_part(part, n_parts, device, mode=mode, hot_bytes=hot_bytes)

    def relation_names(self):
        """Relation names by id (byte order = id order): the generators' relation ids."""
        return ["member", "owner", "view"] if self.kind == "drive" else ["member", "view"]

    def string_tuples(self, seed=7, threads=16):
        """The graph as keto_relation_tuples rows with strings, in a seeded commit order
        (synth_emit_strings); kept alive by the returned object."""
        rel = self.relation_names()
        arr = (C.c_char_p * len(rel))(*[x.encode() for x in rel])
        st = Strings()
        rc = lib().synth_emit_strings(C.byref(self.g), C.byref(self.p), arr, C.c_uint32(len(rel)), C.c_uint64(seed),
                                      C.c_int(threads), C.byref(st))
        if rc != 0:
            raise RuntimeError(f"synth_emit_strings failed: {rc}")
        self._strings = st
        return st

    def snapshot_from_strings(self, st, device=0):
        """keto_snapshot_build (the product's builder: interning, ORDER BY, collision classes) over
        the string rows; returns (Snapshot, build seconds)."""
        import time
        from keto_amd.capi import KNamespace, KOpts, Snapshot, _Keep, _check, load
        keep = _Keep()
        ns = (KNamespace * len(self.namespaces))(*[KNamespace(i, keep.s(n)) for i, n in self.namespaces])
        h = C.c_void_p()
        opts = KOpts(100, device, 0)
        t0 = time.perf_counter()
        _check(load().keto_snapshot_build(ns, len(self.namespaces), C.c_void_p(st.tuples), C.c_uint64(st.n),
                                          C.byref(opts), C.byref(h)))
        return Snapshot(h, load()), time.perf_counter() - t0

    def unified(self, threads=16):
        """The graph in one byte-ordered string id space, for a snapshot that holds its strings
        (keto_snapshot_from_csr with a string table): objects, relation names and users each keep
        their order; returns a Unified (arrays for from_csr, the string table, the user id offset)."""
        rel = self.relation_names()
        st = Strings()
        arr = (C.c_char_p * len(rel))(*[x.encode() for x in rel])
        if lib().synth_emit_names(C.byref(self.g), C.byref(self.p), arr, C.c_uint32(len(rel)), C.c_int(threads),
                                  C.byref(st)) != 0:
            raise RuntimeError("synth_emit_names failed")
        n_objs = int(self.row_obj.max()) + 1 if self.n_rows else 0
        n_users = int(self.params["n_users"])
        blocks = [("obj", f"{0:08x}", f"{max(n_objs - 1, 0):08x}", n_objs),
                  ("user", f"u{0:08x}", f"u{max(n_users - 1, 0):08x}", n_users)]
        for i, r in enumerate(rel):
            for _, lo, hi, _n in blocks[:2]:
                if lo < r < hi:
                    raise ValueError(f"relation name {r!r} sorts inside a generated string block")
            blocks.append((f"rel{i}", r, r, 1))
        at, base = 0, {}
        for name, lo, _hi, cnt in sorted(blocks, key=lambda b: b[1]):
            base[name] = at
            at += cnt
        from keto_amd.capi import KStr
        u = Unified()
        u.n_strings = at
        u.strs = (KStr * max(1, at))()
        u.row_obj = np.empty(self.n_rows, dtype=np.uint32)
        u.row_rel = np.empty(self.n_rows, dtype=np.uint32)
        u.edges = np.empty(max(1, self.n_edges), dtype=np.uint32)[: self.n_edges]
        u.user_base = base["user"]
        rel_id = np.array([base[f"rel{i}"] for i in range(len(rel))], dtype=np.uint32)
        lib().synth_unify(C.byref(self.g), C.byref(st), C.c_uint64(n_objs), C.c_uint64(n_users),
                          C.c_uint32(base["obj"]), C.c_uint32(base["user"]), rel_id.ctypes.data_as(C.c_void_p),
                          C.c_uint32(len(rel)), u.strs, u.row_obj.ctypes.data_as(C.c_void_p),
                          u.row_rel.ctypes.data_as(C.c_void_p), u.edges.ctypes.data_as(C.c_void_p), C.c_int(threads))
        u.names = st                       # the string bytes the table points into
        u.graph = self
        return u

    def snapshot_unified(self, u, device=0):
        """The graph's snapshot with its string table (string-form requests resolve against it);
        the device arena equals snapshot()'s up to the subject-id values."""
        from keto_amd.capi import Snapshot
        return Snapshot.from_csr(self.namespaces, self.row_ns, u.row_obj, u.row_rel, self.row_ptr, u.edges,
                                 kstrs=(u.strs, u.n_strings), device=device)

    def string_requests(self, st, q: np.ndarray, threads=16):
        """keto_check_ids (CSR row ids, user targets) -> keto_check_req by name, for keto_check_batch."""
        from keto_amd.capi import KCheckReq
        names = [b""] * 4
        for i, n in self.namespaces:
            names[i] = n.encode()
        na = (C.c_char_p * 4)(*names)
        out = (KCheckReq * len(q))()
        qa = np.ascontiguousarray(q)
        lib().synth_check_reqs(C.byref(self.g), C.byref(st), qa.ctypes.data_as(C.c_void_p), C.c_uint64(len(q)), na,
                               out, C.c_int(threads))
        out._keep = (na, names)
        return out

    @staticmethod
    def pack_requests(arr, n, threads=16, pinned=True):
        """A keto_check_req array -> (blob, keto_check_packed records, bytes used) for
        keto_check_batch_packed, packed on host threads; pinned: both in page-locked memory
        (keto_host_alloc, .array holds the numpy view), else plain numpy arrays."""
        from keto_amd.capi import CHECK_PACKED_DTYPE, HostBuffer

        class _Plain:
            def __init__(self, k, dt):
                self.array = np.zeros(k, dtype=dt)
        buf = HostBuffer if pinned else _Plain
        total = 0
        cap = max(1, n) * 64
        while True:
            blob = buf(cap, np.uint8)
            rec = buf(max(1, n), CHECK_PACKED_DTYPE)
            used = lib().synth_pack_reqs(arr, C.c_uint64(n), blob.array.ctypes.data_as(C.c_void_p), C.c_uint64(cap),
                                         rec.array.ctypes.data_as(C.c_void_p), C.c_int(threads))
            if used >= 0:
                total = used
                break
            if cap >= (1 << 32):
                raise ValueError("requests do not pack below 4 GiB (or a field exceeds 65535 bytes)")
            cap = min(cap * 2, 1 << 32)
        return blob, rec, int(total)

    def free_strings(self, st):
        lib().synth_strings_free(C.byref(st))

    def host_snapshot(self):
        """Host-only snapshot (no device): resolution, row owners."""
        from keto_amd.capi import Snapshot
        return Snapshot.from_csr(self.namespaces, self.row_ns, self.row_obj, self.row_rel, self.row_ptr, self.edges,
                                 device=-1)

    def oracle_table(self, q: np.ndarray, depth: int):
        """OracleTable over every row a depth-bounded check of the sample can query."""
        from oracle.oracle_c import OracleTable
        t = Table()
        lib().synth_extract(C.byref(self.g), C.byref(self.p), q.ctypes.data_as(C.c_void_p), C.c_uint64(len(q)),
                            C.c_int32(depth), C.byref(t))
        n = t.n

        def arr(ptr, dt):
            buf = (C.c_char * (max(n, 1) * np.dtype(dt).itemsize)).from_address(ptr)
            return np.frombuffer(buf, dtype=dt, count=n).copy()

        arrays = dict(ns=arr(t.ns, np.int32), obj=arr(t.obj, np.uint32), rel=arr(t.rel, np.uint32),
                      kind=arr(t.kind, np.uint8), sid=arr(t.sid, np.uint32), sns=arr(t.sns, np.int32),
                      sobj=arr(t.sobj, np.uint32), srel=arr(t.srel, np.uint32), key=arr(t.key, np.uint32))
        lib().synth_table_free(C.byref(t))
        # string space: objects / relations are per-row ids; namespace names and "" get ids above them
        strings = {"": 0xFFFFFFF0, **{n: 0xFFFF0000 + i for i, n in self.namespaces}}
        return OracleTable(self.namespaces, arrays, strings, {}, page_size=100)

    def sql_store(self, tab):
        """The oracle table's tuples in an in-memory SQLite store with the reference schema
        (oracle/oracle_sql.py's SQLStore; strings are the ids as 8-digit hex, so byte order = id order)."""
        from oracle.oracle_sql import SQLStore, _NID
        n = tab.t.n
        a = tab.arr
        hx = lambda v: f"{v:08x}"
        ns, obj, rel = a["ns"].tolist(), a["obj"].tolist(), a["rel"].tolist()
        kind, sid, sns, sobj, srel = (a[k].tolist() for k in ("kind", "sid", "sns", "sobj", "srel"))

        def rows():
            for i in range(n):
                if kind[i]:
                    yield (f"s{i:010d}", _NID, ns[i], hx(obj[i]), hx(rel[i]), None, sns[i], hx(sobj[i]), hx(srel[i]), i)
                else:
                    yield (f"s{i:010d}", _NID, ns[i], hx(obj[i]), hx(rel[i]), hx(sid[i]), None, None, None, i)
        return SQLStore(self.namespaces, bulk_rows=rows())

    def sql_requests(self, q: np.ndarray):
        """keto_check_ids -> (RelationTuple, request max-depth) for oracle_sql.CheckEngine."""
        from oracle.oracle_sql import RelationTuple, SubjectID
        names = dict(self.namespaces)
        return [(RelationTuple(names[int(self.row_ns[r["row"]])], f"{int(self.row_obj[r['row']]):08x}",
                               f"{int(self.row_rel[r['row']]):08x}", SubjectID(f"{int(r['target']):08x}")),
                 int(r["max_depth"])) for r in q]

    def oracle_requests(self, tab, q: np.ndarray):
        """keto_check_ids -> oracle requests (docs:d#view@u, request max-depth kept), as one ctypes array."""
        from oracle.oracle_c import OraCheckReq
        arr = (OraCheckReq * len(q))()
        v = np.frombuffer(arr, dtype=np.dtype(OraCheckReq))
        rows = q["row"].astype(np.int64)
        v["q"]["ns"] = self.row_ns[rows]
        v["q"]["obj"] = self.row_obj[rows]
        v["q"]["rel"] = self.row_rel[rows]
        v["q_ns_unknown"] = 0
        v["t"]["kind"] = 0
        v["t"]["sid"] = q["target"]
        v["t"]["key"] = q["target"]
        v["max_depth"] = q["max_depth"]
        return arr
