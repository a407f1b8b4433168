"""SQL-level CPU restatement of Keto's check / expand engines -- TEST INFRASTRUCTURE ONLY.

This module is the *oracle*: a line-by-line restatement of the reference Go code
(icyphox/keto, fork of ory/keto v0.8.1) executed against the stdlib ``sqlite3``
driver with the reference's own schema, WHERE clause, ORDER BY and LIMIT/OFFSET
pagination.  It exists so that tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg can check the MI355X engine; the product path
(``keto_amd``) never imports it.

Parity status: pinned against the reference's own golden vectors (engine tests,
handler tests and docs-code-samples expected outputs) transcribed into
``tests/golden/reference_cases.json``; the Go reference itself cannot run in this
container (no Go toolchain).

Followed reference lines (relative to /root/reference):
  * schema      internal/persistence/sql/migrations/sql/20210623162417000000_relationtuple.sqlite3.up.sql:3-24
  * row         internal/persistence/sql/relationtuples.go:19-31
  * toInternal  internal/persistence/sql/relationtuples.go:43-80
  * whereQuery  internal/persistence/sql/relationtuples.go:178-198
  * GetRelationTuples internal/persistence/sql/relationtuples.go:238-277 (ORDER BY :250, TotalPages :262-265)
  * pagination  internal/persistence/sql/persister.go:46,106-134
  * namespaces  internal/driver/config/namespace_memory.go:30-48 (linear scan, first match)
  * check       internal/check/engine.go:36-123
  * expand      internal/expand/engine.go:33-102
  * visited     internal/x/graph/graph_utils.go:13-35
  * subjects    internal/relationtuple/definitions.go:163-169 (String), :252-266 (Equals)
"""
from __future__ import annotations

import sqlite3
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple, Union

DEFAULT_PAGE_SIZE = 100  # internal/persistence/sql/persister.go:46


class NotFoundError(Exception):
    """herodot.ErrNotFound (unknown namespace name or id)."""


# --------------------------------------------------------------------------------------
# domain model (internal/relationtuple/definitions.go)
# --------------------------------------------------------------------------------------
@dataclass(frozen=True)
class SubjectID:
    id: str

    def string(self) -> str:  # definitions.go:163-165
        return self.id

    def equals(self, other) -> bool:  # definitions.go:252-258
        return isinstance(other, SubjectID) and other.id == self.id


@dataclass(frozen=True)
class SubjectSet:
    namespace: str
    object: str
    relation: str

    def string(self) -> str:  # definitions.go:167-169
        return f"{self.namespace}:{self.object}#{self.relation}"

    def equals(self, other) -> bool:  # definitions.go:260-266
        return (isinstance(other, SubjectSet) and other.relation == self.relation
                and other.object == self.object and other.namespace == self.namespace)


Subject = Union[SubjectID, SubjectSet]


@dataclass(frozen=True)
class RelationTuple:
    namespace: str
    object: str
    relation: str
    subject: Subject


@dataclass
class Tree:
    type: str  # "union" | "leaf"  (internal/expand/tree.go:16-23)
    subject: Subject
    children: List["Tree"] = field(default_factory=list)

    def to_json(self):
        """Mirror of Tree.MarshalJSON (internal/expand/tree.go:85-90,156-163)."""
        out = {"type": self.type}
        if self.children:
            out["children"] = [c.to_json() for c in self.children]
        if isinstance(self.subject, SubjectID):
            out["subject_id"] = self.subject.id
        else:
            out["subject_set"] = {"namespace": self.subject.namespace,
                                  "object": self.subject.object,
                                  "relation": self.subject.relation}
        return out


def subject_from_json(d) -> Subject:
    if "subject_id" in d and d["subject_id"] is not None:
        return SubjectID(d["subject_id"])
    s = d["subject_set"]
    return SubjectSet(s.get("namespace", ""), s.get("object", ""), s.get("relation", ""))


def tuple_from_json(d) -> RelationTuple:
    return RelationTuple(d.get("namespace", ""), d.get("object", ""), d.get("relation", ""),
                         subject_from_json(d))


def tree_from_json(d) -> Optional[Tree]:
    if d is None:
        return None
    sub = subject_from_json(d)
    return Tree(d["type"], sub, [tree_from_json(c) for c in d.get("children", []) or []])


# --------------------------------------------------------------------------------------
# persistence: SQLite store with the reference schema and queries
# --------------------------------------------------------------------------------------
_SCHEMA = """
CREATE TABLE keto_relation_tuples
(
    shard_id                 TEXT        NOT NULL,
    nid                      TEXT        NOT NULL,
    namespace_id             INTEGER     NOT NULL,
    object                   VARCHAR(64) NOT NULL,
    relation                 VARCHAR(64) NOT NULL,
    subject_id               VARCHAR(64) NULL,
    subject_set_namespace_id INTEGER NULL,
    subject_set_object       VARCHAR(64) NULL,
    subject_set_relation     VARCHAR(64) NULL,
    commit_time              INTEGER     NOT NULL,
    PRIMARY KEY (shard_id, nid),
    CONSTRAINT chk_keto_rt_subject_type CHECK
        ((subject_id IS NULL AND
          subject_set_namespace_id IS NOT NULL AND subject_set_object IS NOT NULL AND subject_set_relation IS NOT NULL)
            OR
         (subject_id IS NOT NULL AND
          subject_set_namespace_id IS NULL AND subject_set_object IS NULL AND subject_set_relation IS NULL))
);
"""
_INDEX = """
CREATE INDEX keto_relation_tuples_full_idx ON keto_relation_tuples
    (nid, namespace_id, object, relation, subject_id, subject_set_namespace_id, subject_set_object,
     subject_set_relation, commit_time);
"""

_ORDER = ("nid, namespace_id, object, relation, subject_id, subject_set_namespace_id, "
          "subject_set_object, subject_set_relation, commit_time")  # relationtuples.go:250

_NID = "00000000-0000-0000-0000-000000000000"


class Namespaces:
    """memoryNamespaceManager: ordered list, linear scan, first match (namespace_memory.go:30-48)."""

    def __init__(self, namespaces: Sequence[Tuple[int, str]]):
        self.items = [(int(i), str(n)) for i, n in namespaces]

    def by_name(self, name: str) -> Tuple[int, str]:
        for i, n in self.items:
            if n == name:
                return i, n
        raise NotFoundError(f"Unknown namespace with name {name}.")

    def by_id(self, nid: int) -> Tuple[int, str]:
        for i, n in self.items:
            if i == nid:
                return i, n
        raise NotFoundError(f"Unknown namespace with id {nid}.")


class SQLStore:
    """Persister.GetRelationTuples over an in-memory SQLite DB with the reference schema.

    ``raw_rows`` may be given instead of ``tuples`` to insert rows whose namespace ids are
    not (or no longer) configured -- this is how poisoned pages (SURVEY A.Q8) arise.
    """

    def __init__(self, namespaces: Sequence[Tuple[int, str]], tuples: Sequence[RelationTuple] = (),
                 page_size: int = DEFAULT_PAGE_SIZE, raw_rows: Sequence[tuple] = (), bulk_rows=None):
        self.nm = Namespaces(namespaces)
        self.page_size = page_size
        self.conn = sqlite3.connect(":memory:")
        self.conn.executescript(_SCHEMA)
        if bulk_rows is not None:       # full keto_relation_tuples rows, indexed after the insert (bench)
            self.conn.executemany("INSERT INTO keto_relation_tuples VALUES (?,?,?,?,?,?,?,?,?,?)", bulk_rows)
        self.conn.executescript(_INDEX)
        self._seq = 0
        self.requested_pages: List[int] = []  # ManagerWrapper.RequestedPages analogue
        for t in tuples:
            self.insert(t)
        for r in raw_rows:
            self.insert_raw(*r)

    # RelationTuple.FromInternal / insertSubject (relationtuples.go:82-124)
    def insert(self, t: RelationTuple):
        ns_id, _ = self.nm.by_name(t.namespace)
        if isinstance(t.subject, SubjectID):
            self.insert_raw(ns_id, t.object, t.relation, t.subject.id, None, None, None)
        else:
            sns, _ = self.nm.by_name(t.subject.namespace)
            self.insert_raw(ns_id, t.object, t.relation, None, sns, t.subject.object, t.subject.relation)

    def insert_raw(self, ns_id, obj, rel, sid, sns, sobj, srel):
        self._seq += 1
        self.conn.execute(
            "INSERT INTO keto_relation_tuples VALUES (?,?,?,?,?,?,?,?,?,?)",
            (f"shard-{self._seq}", _NID, ns_id, obj, rel, sid, sns, sobj, srel, self._seq))

    def delete(self, t: RelationTuple):
        """DeleteRelationTuples for one tuple (relationtuples.go:200-223, whereSubject :151-176):
        every row with its namespace, object, relation and exact subject."""
        ns_id, _ = self.nm.by_name(t.namespace)
        if isinstance(t.subject, SubjectID):
            self.conn.execute("DELETE FROM keto_relation_tuples WHERE nid = ? AND namespace_id = ? AND object = ? AND "
                              "relation = ? AND subject_id = ? AND subject_set_namespace_id IS NULL AND "
                              "subject_set_object IS NULL AND subject_set_relation IS NULL",
                              (_NID, ns_id, t.object, t.relation, t.subject.id))
        else:
            sns, _ = self.nm.by_name(t.subject.namespace)
            self.conn.execute("DELETE FROM keto_relation_tuples WHERE nid = ? AND namespace_id = ? AND object = ? AND "
                              "relation = ? AND subject_id IS NULL AND subject_set_namespace_id = ? AND "
                              "subject_set_object = ? AND subject_set_relation = ?",
                              (_NID, ns_id, t.object, t.relation, sns, t.subject.object, t.subject.relation))

    def tuples(self):
        """Every row in commit order, as RelationTuples (rows with unknown namespaces skipped)."""
        out = []
        for ns_id, obj, rel, sid, sns, sobj, srel in self.conn.execute(
                "SELECT namespace_id, object, relation, subject_id, subject_set_namespace_id, subject_set_object, "
                "subject_set_relation FROM keto_relation_tuples ORDER BY commit_time"):
            _, nm = self.nm.by_id(ns_id)
            if sid is not None:
                out.append(RelationTuple(nm, obj, rel, SubjectID(sid)))
            else:
                _, snm = self.nm.by_id(sns)
                out.append(RelationTuple(nm, obj, rel, SubjectSet(snm, sobj, srel)))
        return out

    def _to_internal(self, row) -> RelationTuple:  # relationtuples.go:43-80
        ns_id, obj, rel, sid, sns, sobj, srel = row
        _, ns_name = self.nm.by_id(ns_id)
        if sid is not None:
            sub = SubjectID(sid)
        else:
            nid, _ = self.nm.by_id(sns)
            _, sname = self.nm.by_id(nid)
            sub = SubjectSet(sname, sobj, srel)
        return RelationTuple(ns_name, obj, rel, sub)

    def get_relation_tuples(self, namespace: str, obj: str, relation: str, token: str = ""):
        """Returns (tuples, next_page_token). Raises NotFoundError like the reference."""
        page = 1 if token == "" else int(token)  # persister.go:119-134
        self.requested_pages.append(page)
        where, args = ["nid = ?"], [_NID]
        if namespace != "":  # whereQuery :179-185
            ns_id, _ = self.nm.by_name(namespace)
            where.append("namespace_id = ?")
            args.append(ns_id)
        if obj != "":
            where.append("object = ?")
            args.append(obj)
        if relation != "":
            where.append("relation = ?")
            args.append(relation)
        w = " AND ".join(where)
        total = self.conn.execute(f"SELECT COUNT(*) FROM keto_relation_tuples WHERE {w}", args).fetchone()[0]
        rows = self.conn.execute(
            f"SELECT namespace_id, object, relation, subject_id, subject_set_namespace_id, "
            f"subject_set_object, subject_set_relation FROM keto_relation_tuples WHERE {w} "
            f"ORDER BY {_ORDER} LIMIT ? OFFSET ?",
            args + [self.page_size, (page - 1) * self.page_size]).fetchall()
        total_pages = -(-total // self.page_size)  # pop Paginator.TotalPages
        next_token = "" if page >= total_pages else str(page + 1)
        return [self._to_internal(r) for r in rows], next_token


# --------------------------------------------------------------------------------------
# engines
# --------------------------------------------------------------------------------------
class _Ctx:
    """context.Context carrying the visited map (graph_utils.go); None = no map yet."""
    __slots__ = ("visited",)

    def __init__(self, visited=None):
        self.visited = visited


def check_and_add_visited(ctx: _Ctx, s: Subject):  # graph_utils.go:13-35
    if ctx.visited is None:
        return _Ctx({s.string()}), False
    k = s.string()
    if k in ctx.visited:
        return ctx, True
    ctx.visited.add(k)
    return _Ctx(ctx.visited), False


class CheckEngine:
    """check.Engine (internal/check/engine.go)."""

    def __init__(self, store: SQLStore, global_max_depth: int = 5):
        self.store = store
        self.global_max_depth = global_max_depth

    def _subject_is_allowed(self, ctx, requested: RelationTuple, rels, rest_depth) -> bool:  # :36-80
        for sr in rels:
            ctx2, seen = check_and_add_visited(ctx, sr.subject)  # shadowing: ctx stays the outer one
            if seen:
                continue
            if requested.subject.equals(sr.subject):
                return True
            if not isinstance(sr.subject, SubjectSet):
                continue
            s = sr.subject
            if self._check_one_indirection_further(ctx2, requested, (s.namespace, s.object, s.relation),
                                                   rest_depth - 1):
                return True
        return False

    def _check_one_indirection_further(self, ctx, requested, query, rest_depth) -> bool:  # :82-114
        if rest_depth <= 0:
            return False
        prev = ""
        while True:
            try:
                rels, nxt = self.store.get_relation_tuples(*query, token=prev)
            except NotFoundError:
                return False
            allowed = self._subject_is_allowed(ctx, requested, rels, rest_depth)
            if allowed or nxt == "":
                return allowed
            prev = nxt

    def subject_is_allowed(self, r: RelationTuple, rest_depth: int) -> bool:  # :116-123
        g = self.global_max_depth
        if rest_depth <= 0 or g < rest_depth:
            rest_depth = g
        return self._check_one_indirection_further(_Ctx(), r, (r.namespace, r.object, r.relation), rest_depth)


class ExpandEngine:
    """expand.Engine (internal/expand/engine.go). Errors propagate as NotFoundError."""

    def __init__(self, store: SQLStore, global_max_depth: int = 5):
        self.store = store
        self.global_max_depth = global_max_depth

    def build_tree(self, subject: Subject, rest_depth: int, ctx: Optional[_Ctx] = None) -> Optional[Tree]:
        ctx = ctx or _Ctx()
        g = self.global_max_depth
        if rest_depth <= 0 or g < rest_depth:  # :35-37
            rest_depth = g
        if isinstance(subject, SubjectSet):
            ctx, seen = check_and_add_visited(ctx, subject)  # :40-43
            if seen:
                return None
            tree = Tree("union", subject)
            nxt = ""
            first = True
            while first or nxt != "":  # :55-92
                first = False
                rels, nxt = self.store.get_relation_tuples(subject.namespace, subject.object, subject.relation,
                                                           token=nxt)
                if len(rels) == 0:
                    return None
                if rest_depth <= 1:
                    tree.type = "leaf"
                    return tree
                children = []
                for r in rels:
                    c = self.build_tree(r.subject, rest_depth - 1, ctx)
                    if c is None:
                        c = Tree("leaf", r.subject)
                    children.append(c)
                tree.children.extend(children)
            return tree
        return Tree("leaf", subject)  # :97-101


def canonical_tree(t):
    """Order-insensitive canonical form of a JSON tree (children sorted recursively),
    the comparison used by internal/e2e/cases_test.go:91-93."""
    if t is None:
        return None
    import json
    c = dict(t)
    if "children" in c:
        c["children"] = sorted((canonical_tree(x) for x in c["children"]),
                               key=lambda x: json.dumps(x, sort_keys=True))
    return c
