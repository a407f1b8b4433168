"""ctypes front-end of the C restatement (oracle/keto_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Builds the ordered, interned tuple table the C oracle walks, from either
  * an ``oracle_sql.SQLStore`` (rows fetched with the reference ORDER BY, so the order
    comes from SQLite itself, not from any code of the product), or
  * numpy arrays already in ORDER BY order (synthetic graphs whose string naming makes
    numeric id order equal byte order).
Only tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from oracle.oracle_sql import SQLStore, SubjectID, SubjectSet, Tree, _ORDER

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libketo_oracle.so")
ANY_NS = -(2 ** 63)


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.ora_check.restype = C.c_int
        _lib.ora_check_batch.restype = C.c_int
        _lib.ora_expand.restype = C.c_int
        _lib.ora_bfs_bytes.restype = C.c_uint64
        _lib.ora_bfs_bytes_batch.restype = C.c_int
    return _lib


class OraTable(C.Structure):
    _fields_ = [("n", C.c_uint64), ("ns", C.c_void_p), ("obj", C.c_void_p), ("rel", C.c_void_p),
                ("kind", C.c_void_p), ("sid", C.c_void_p), ("sns", C.c_void_p), ("sobj", C.c_void_p),
                ("srel", C.c_void_p), ("key", C.c_void_p), ("n_ns", C.c_uint32), ("ns_ids", C.c_void_p),
                ("ns_name", C.c_void_p), ("empty_str", C.c_uint32), ("page_size", C.c_uint32)]


class OraQuery(C.Structure):
    _fields_ = [("ns", C.c_int64), ("obj", C.c_uint32), ("rel", C.c_uint32)]


class OraSubject(C.Structure):
    _fields_ = [("kind", C.c_uint8), ("sid", C.c_uint32), ("name", C.c_uint32), ("obj", C.c_uint32),
                ("rel", C.c_uint32), ("key", C.c_uint32)]


class OraCheckReq(C.Structure):
    _fields_ = [("q", OraQuery), ("q_ns_unknown", C.c_int32), ("t", OraSubject), ("max_depth", C.c_int32)]


class OraNode(C.Structure):
    _fields_ = [("type", C.c_uint8), ("kind", C.c_uint8), ("sid", C.c_uint32), ("name", C.c_uint32),
                ("obj", C.c_uint32), ("rel", C.c_uint32), ("n_children", C.c_uint32)]


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class OracleTable:
    """Interned, ordered tuple table + string dictionaries."""

    def __init__(self, namespaces, arrays, strings, keys, page_size=100):
        self.namespaces = list(namespaces)
        self.arr = arrays            # dict of numpy arrays (kept alive)
        self.strings = strings       # str -> id (byte-order preserving)
        self.keys = keys             # String() -> key id
        self.page_size = page_size
        self.ns_ids = np.array([i for i, _ in self.namespaces] or [0], dtype=np.int32)
        self.ns_name = np.array([self.sid(n) for _, n in self.namespaces] or [0], dtype=np.uint32)
        a = self.arr
        self.t = OraTable(len(a["ns"]), _p(a["ns"]), _p(a["obj"]), _p(a["rel"]), _p(a["kind"]), _p(a["sid"]),
                          _p(a["sns"]), _p(a["sobj"]), _p(a["srel"]), _p(a["key"]), len(self.namespaces),
                          _p(self.ns_ids), _p(self.ns_name), self.sid(""), page_size)

    # string / key ids; unknown strings get ids that match nothing in the table
    def sid(self, s):
        v = self.strings.get(s)
        if v is None:
            v = self.strings[s] = len(self.strings) + 0x40000000
        return v

    def kid(self, k):
        v = self.keys.get(k)
        if v is None:
            v = self.keys[k] = len(self.keys) + 0x40000000
        return v

    def ns_id_by_name(self, name):
        for i, n in self.namespaces:
            if n == name:
                return i
        return None

    # ---------------------------------------------------------------- builders
    @classmethod
    def from_store(cls, store: SQLStore):
        rows = store.conn.execute(
            "SELECT namespace_id, object, relation, subject_id, subject_set_namespace_id, subject_set_object, "
            f"subject_set_relation FROM keto_relation_tuples ORDER BY {_ORDER}").fetchall()
        names = {n: i for i, n in store.nm.items}
        strs = {"", *[n for _, n in store.nm.items]}
        for r in rows:
            strs.update(x for x in (r[1], r[2], r[3], r[5], r[6]) if x is not None)
        order = sorted(strs, key=lambda s: s.encode())
        strings = {s: i for i, s in enumerate(order)}
        keys = {}

        def key_of(r):
            if r[3] is not None:
                k = r[3]
            else:
                nm = next((n for i, n in store.nm.items if i == r[4]), None)
                k = f"{nm}:{r[5]}#{r[6]}" if nm is not None else f"\x00poison:{r[4]}:{r[5]}#{r[6]}"
            if k not in keys:
                keys[k] = len(keys)
            return keys[k]

        n = len(rows)
        arr = {
            "ns": np.array([r[0] for r in rows], dtype=np.int32).reshape(n),
            "obj": np.array([strings[r[1]] for r in rows], dtype=np.uint32).reshape(n),
            "rel": np.array([strings[r[2]] for r in rows], dtype=np.uint32).reshape(n),
            "kind": np.array([0 if r[3] is not None else 1 for r in rows], dtype=np.uint8).reshape(n),
            "sid": np.array([strings[r[3]] if r[3] is not None else 0 for r in rows], dtype=np.uint32).reshape(n),
            "sns": np.array([r[4] if r[4] is not None else 0 for r in rows], dtype=np.int32).reshape(n),
            "sobj": np.array([strings[r[5]] if r[5] is not None else 0 for r in rows], dtype=np.uint32).reshape(n),
            "srel": np.array([strings[r[6]] if r[6] is not None else 0 for r in rows], dtype=np.uint32).reshape(n),
            "key": np.array([key_of(r) for r in rows], dtype=np.uint32).reshape(n),
        }
        del names
        return cls(store.nm.items, arr, strings, keys, store.page_size)

    # ---------------------------------------------------------------- requests
    def subject(self, s):
        if isinstance(s, SubjectID):
            return OraSubject(0, self.sid(s.id), 0, 0, 0, self.kid(s.string()))
        return OraSubject(1, 0, self.sid(s.namespace), self.sid(s.object), self.sid(s.relation),
                          self.kid(s.string()))

    def check_req(self, tup, max_depth):
        r = OraCheckReq()
        if tup.namespace == "":
            r.q.ns = ANY_NS
        else:
            nid = self.ns_id_by_name(tup.namespace)
            r.q_ns_unknown = 1 if nid is None else 0
            r.q.ns = 0 if nid is None else nid
        r.q.obj = self.sid(tup.object)
        r.q.rel = self.sid(tup.relation)
        r.t = self.subject(tup.subject)
        r.max_depth = max_depth
        return r

    def check(self, tup, max_depth, global_max_depth=5) -> bool:
        r = self.check_req(tup, max_depth)
        return bool(lib().ora_check(C.byref(self.t), C.byref(r), C.c_int32(global_max_depth)))

    @staticmethod
    def prefix(reqs, n):
        """The first n requests of a ctypes request array, as a view (no copy)."""
        return (OraCheckReq * n).from_address(C.addressof(reqs))

    @staticmethod
    def _req_array(reqs):
        if isinstance(reqs, C.Array):
            return reqs
        return (OraCheckReq * len(reqs))(*reqs)

    def check_batch_reqs(self, reqs, global_max_depth=5, threads=1):
        n = len(reqs)
        arr = self._req_array(reqs)
        out = np.zeros(n, dtype=np.uint8)
        lib().ora_check_batch(C.byref(self.t), arr, C.c_uint64(n), C.c_int32(global_max_depth), _p(out),
                              C.c_int(threads))
        return out

    def bfs_bytes_reqs(self, reqs, global_max_depth=5, threads=1):
        """SURVEY.md 8(d) algorithmic bytes of each check (BFS-count mode; measurement only)."""
        n = len(reqs)
        arr = self._req_array(reqs)
        out = np.zeros(n, dtype=np.uint64)
        lib().ora_bfs_bytes_batch(C.byref(self.t), arr, C.c_uint64(n), C.c_int32(global_max_depth), _p(out),
                                  C.c_int(threads))
        return out

    def expand(self, subject, max_depth, global_max_depth=5):
        """Returns ("tree", json) | ("nil", None) | ("error", None)."""
        root = self.subject(subject)
        nodes = C.POINTER(OraNode)()
        nn = C.c_uint64()
        r = lib().ora_expand(C.byref(self.t), C.byref(root), C.c_int32(max_depth), C.c_int32(global_max_depth),
                             C.byref(nodes), C.byref(nn))
        if r < 0:
            return "error", None
        if r == 0:
            return "nil", None
        inv = {v: k for k, v in self.strings.items()}
        pos = [0]

        def rec():
            nd = nodes[pos[0]]
            pos[0] += 1
            if nd.kind == 0:
                sub = SubjectID(inv[nd.sid])
            else:
                sub = SubjectSet(inv[nd.name], inv[nd.obj], inv[nd.rel])
            t = Tree("union" if nd.type == 0 else "leaf", sub)
            for _ in range(nd.n_children):
                t.children.append(rec())
            return t

        tree = rec()
        lib().ora_free(C.cast(nodes, C.c_void_p))
        return "tree", tree.to_json()
