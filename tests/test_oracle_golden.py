"""Pin the SQL-level oracle against the reference's own golden vectors."""
import pytest

from oracle.oracle_sql import (CheckEngine, ExpandEngine, NotFoundError, SQLStore, canonical_tree,
                               subject_from_json, tuple_from_json)
from tests.golden_util import case_namespaces, case_tuples, load_cases

CASES = load_cases()


def _checks():
    for c in CASES:
        for i, chk in enumerate(c.get("checks", [])):
            yield pytest.param(c, chk, id=f"{c['name']}#{i}")


def _expands():
    for c in CASES:
        for i, ex in enumerate(c.get("expands", [])):
            yield pytest.param(c, ex, id=f"{c['name']}#{i}")


@pytest.mark.parametrize("case,chk", list(_checks()))
def test_oracle_check_golden(case, chk):
    store = SQLStore(case_namespaces(case), case_tuples(case), page_size=case.get("page_size", 100))
    eng = CheckEngine(store, chk["global_max_depth"])
    got = eng.subject_is_allowed(tuple_from_json(chk["tuple"]), chk["max_depth"])
    assert got == chk["expected"]
    if "expected_pages" in chk:  # engine_test.go:468-482 (RequestedPages)
        assert len(store.requested_pages) == chk["expected_pages"]


@pytest.mark.parametrize("case,ex", list(_expands()))
def test_oracle_expand_golden(case, ex):
    store = SQLStore(case_namespaces(case), case_tuples(case), page_size=case.get("page_size", 100))
    eng = ExpandEngine(store, ex["global_max_depth"])
    sub = subject_from_json(ex["subject"])
    if ex.get("expected_error") == "not_found":
        with pytest.raises(NotFoundError):
            eng.build_tree(sub, ex["max_depth"])
        return
    tree = eng.build_tree(sub, ex["max_depth"])
    got = None if tree is None else tree.to_json()
    if ex.get("ordered"):
        assert got == ex["expected"]
    else:
        assert canonical_tree(got) == canonical_tree(ex["expected"])
    if "expected_pages" in ex:
        assert len(store.requested_pages) == ex["expected_pages"]
