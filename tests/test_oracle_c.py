"""Cross-check the C restatement against the SQL-level restatement (which is pinned to the
reference's golden vectors) on the golden cases and on random quirk-heavy graphs."""
import pytest

from oracle.oracle_c import OracleTable
from oracle.oracle_sql import CheckEngine, ExpandEngine, NotFoundError, SQLStore, subject_from_json, tuple_from_json
from tests.golden_util import case_namespaces, case_tuples, load_cases
from tests.randgraph import random_checks, random_expands, random_store


@pytest.mark.parametrize("case", load_cases(), ids=lambda c: c["name"])
def test_c_oracle_golden(case):
    store = SQLStore(case_namespaces(case), case_tuples(case), page_size=case.get("page_size", 100))
    tab = OracleTable.from_store(store)
    for chk in case.get("checks", []):
        assert tab.check(tuple_from_json(chk["tuple"]), chk["max_depth"], chk["global_max_depth"]) == chk["expected"]
    for ex in case.get("expands", []):
        kind, got = tab.expand(subject_from_json(ex["subject"]), ex["max_depth"], ex["global_max_depth"])
        if ex.get("expected_error"):
            assert kind == "error"
        elif ex["expected"] is None:
            assert kind == "nil"
        else:
            assert kind == "tree" and got == ex["expected"]


def _sql_expand(store, sub, d, g):
    try:
        t = ExpandEngine(store, g).build_tree(sub, d)
    except NotFoundError:
        return "error", None
    return ("nil", None) if t is None else ("tree", t.to_json())


@pytest.mark.parametrize("seed,wide", [(s, False) for s in range(400)] + [(s, True) for s in range(1000, 1040)])
def test_c_oracle_matches_sql_oracle(seed, wide):
    store, _ns, _t, _raw, _ps, alph = random_store(seed, wide=wide)
    tab = OracleTable.from_store(store)
    for tup, d, g in random_checks(seed, alph):
        want = CheckEngine(store, g).subject_is_allowed(tup, d)
        assert tab.check(tup, d, g) == want, (seed, tup, d, g)
    for sub, d, g in random_expands(seed, alph):
        assert tab.expand(sub, d, g) == _sql_expand(store, sub, d, g), (seed, sub, d, g)
