"""Helpers that load tests/golden/reference_cases.json into oracle / engine inputs."""
import json
import os

from oracle.oracle_sql import tuple_from_json, subject_from_json

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_cases.json")


def load_cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


def case_tuples(case):
    return [tuple_from_json(t) for t in case["tuples"]]


def case_namespaces(case):
    return [(int(i), n) for i, n in case["namespaces"]]
