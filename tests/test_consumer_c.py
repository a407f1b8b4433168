"""A C program written against include/keto_mi355x.h only (integration/c/keto_consumer.c), compiled
with gcc here: it builds snapshots from strings, checks, expands, reads JSON and protobuf trees,
exercises an error path and frees everything.  On the CPU it runs host-only (compute must fail
with KETO_E_HIP); on the GPU it runs every golden case of the reference's tests
(tests/golden/reference_cases.json) and its decisions / trees must equal the expected ones."""
import json
import os
import subprocess

import pytest

from oracle.oracle_sql import subject_from_json, tuple_from_json, SubjectID
from tests.golden_util import case_namespaces, case_tuples, load_cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "integration", "c", "keto_consumer.c")


@pytest.fixture(scope="module")
def consumer(tmp_path_factory):
    import keto_amd
    keto_amd.load()                      # builds nothing; the library must exist
    exe = str(tmp_path_factory.mktemp("consumer") / "keto_consumer")
    libdir = os.path.join(ROOT, "keto_amd")
    subprocess.check_call(["gcc", "-std=c99", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                           SRC, "-o", exe, "-L", libdir, "-lketo_mi355x", f"-Wl,-rpath,{libdir}"])
    return exe


def _input(case, device):
    ns = case_namespaces(case)
    ids = {n: i for i, n in reversed(ns)}
    lines = [f"P\t{case.get('page_size', 100)}", f"V\t{device}"]
    lines += [f"N\t{i}\t{n}" for i, n in ns]
    for t in case_tuples(case):
        if isinstance(t.subject, SubjectID):
            lines.append(f"T\t{ids[t.namespace]}\t{t.object}\t{t.relation}\tI\t{t.subject.id}")
        else:
            s = t.subject
            lines.append(f"T\t{ids[t.namespace]}\t{t.object}\t{t.relation}\tS\t{ids[s.namespace]}\t{s.object}\t{s.relation}")
    for c in case.get("checks", []):
        t = tuple_from_json(c["tuple"])
        sub = (f"I\t{t.subject.id}" if isinstance(t.subject, SubjectID)
               else f"S\t{t.subject.namespace}\t{t.subject.object}\t{t.subject.relation}")
        lines.append(f"C\t{t.namespace}\t{t.object}\t{t.relation}\t{sub}\t{c['max_depth']}\t{c['global_max_depth']}")
    for e in case.get("expands", []):
        s = subject_from_json(e["subject"])
        sub = f"I\t{s.id}" if isinstance(s, SubjectID) else f"S\t{s.namespace}\t{s.object}\t{s.relation}"
        lines.append(f"E\t{sub}\t{e['max_depth']}\t{e['global_max_depth']}")
    for ln in lines:
        assert "\n" not in ln and ln.count("\t") < 12
    return "\n".join(lines) + "\n"


def _run(exe, tmp_path, case, device):
    p = tmp_path / "in.tsv"
    p.write_text(_input(case, device))
    r = subprocess.run([exe, str(p)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout.splitlines()


@pytest.mark.parametrize("case", [c for c in load_cases() if c.get("checks")][:6], ids=lambda c: c["name"])
def test_consumer_host_only(consumer, tmp_path, case):
    out = _run(consumer, tmp_path, case, -1)
    assert out[0].startswith("stats tuples=")
    assert out[1] == "nodevice -2"                      # KETO_E_HIP: no compute without a device
    assert out[-1] == "done"


@pytest.mark.gpu
@pytest.mark.parametrize("case", load_cases(), ids=lambda c: c["name"])
def test_consumer_golden_on_gpu(consumer, tmp_path, case):
    from tests.proto_util import tree_json_to_proto
    out = _run(consumer, tmp_path, case, 0)
    checks = [ln.split("\t") for ln in out if ln.startswith("check\t")]
    assert len(checks) == len(case.get("checks", []))
    for c, (_, _, allowed, status) in zip(case.get("checks", []), checks):
        assert bool(int(allowed)) == c["expected"], c
    exps = [ln.split("\t") for ln in out if ln.startswith("expand\t")]
    assert len(exps) == len(case.get("expands", []))
    for e, (_, _, status, js, pb) in zip(case.get("expands", []), exps):
        if e.get("expected_error"):
            assert int(status) == 2 and js == "error"
        elif e["expected"] is None:
            assert int(status) == 1 and js == "null" and pb == "-"
        else:
            assert int(status) == 0 and json.loads(js) == e["expected"]
            assert bytes.fromhex(pb) == tree_json_to_proto(e["expected"])
    assert out[-1] == "done"
