"""Feed the same relation tuples to the oracle and to the MI355X engine."""
from oracle.oracle_sql import SubjectID, SubjectSet


def rows_from_tuples(namespaces, tuples, raw=()):
    """RelationTuples (+ raw SQL rows) -> keto_tuple rows in commit order (names resolved like
    RelationTuple.FromInternal, internal/persistence/sql/relationtuples.go:114-124)."""
    by_name = {}
    for i, n in namespaces:
        by_name.setdefault(n, i)
    out = []
    for t in tuples:
        if isinstance(t.subject, SubjectID):
            out.append((by_name[t.namespace], t.object, t.relation, t.subject.id))
        else:
            s = t.subject
            out.append((by_name[t.namespace], t.object, t.relation, None, by_name[s.namespace], s.object, s.relation))
    for ns_id, obj, rel, sid, sns, sobj, srel in raw:
        if sid is not None:
            out.append((ns_id, obj, rel, sid))
        else:
            out.append((ns_id, obj, rel, None, sns, sobj, srel))
    return out


def subj(s):
    return ("id", s.id) if isinstance(s, SubjectID) else ("set", s.namespace, s.object, s.relation)
