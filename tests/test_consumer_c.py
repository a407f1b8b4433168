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


def _input(case, device, replicas=1):
    ns = case_namespaces(case)
    ids = {n: i for i, n in reversed(ns)}
    lines = [f"P\t{case.get('page_size', 100)}", f"V\t{device}", "R" + f"\t{device}" * replicas]
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


def _run(exe, tmp_path, case, device, replicas=1):
    p = tmp_path / "in.tsv"
    p.write_text(_input(case, device, replicas))
    r = subprocess.run([exe, str(p)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout.splitlines()


@pytest.mark.parametrize("case", [c for c in load_cases() if c.get("checks")][:6], ids=lambda c: c["name"])
def test_consumer_host_only(consumer, tmp_path, case):
    out = _run(consumer, tmp_path, case, -1, replicas=2)      # host-only replicas clone too
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


def _tuple_fields(ids, t):
    if isinstance(t.subject, SubjectID):
        return f"{ids[t.namespace]}\t{t.object}\t{t.relation}\tI\t{t.subject.id}"
    s = t.subject
    return f"{ids[t.namespace]}\t{t.object}\t{t.relation}\tS\t{ids[s.namespace]}\t{s.object}\t{s.relation}"


@pytest.mark.gpu
@pytest.mark.parametrize("replicas", [1, 2, 3, "parts2", "parts3"])
@pytest.mark.parametrize("seed", range(24))
def test_consumer_writes_checks_expands_on_gpu(consumer, tmp_path, seed, replicas):
    """The whole Go call sequence from C: build -> check / expand micro-batches -> write transactions
    applied after they commit (KETO_E_REBUILD -> rebuild from the consumer's table, as the registry's
    persister wrapper does) -> checks and expands again; trees also rebuilt from keto_tree_nodes +
    keto_subject_fields (the Go shim's path) and re-encoded byte-equal.  With replicas > 1 the consumer
    is one server process over several devices (here all device 0): replicas cloned from the first
    build, batches dealt round-robin, every write applied to each.  With "partsP" the graph is
    partitioned instead (the server's mode for a graph past one device's memory): P shared-rows parts,
    one local rank per part on its own thread, every batch split over the ranks and routed
    (keto_check_batch_routed / keto_expand_batch_routed), every write applied to every part, restarts
    through a host-only saved snapshot partitioned again.  Every decision and tree is compared with the
    SQL oracle replaying the same transactions."""
    import random
    from oracle.oracle_sql import CheckEngine, ExpandEngine, NotFoundError, SQLStore
    from tests.proto_util import tree_json_to_proto
    from tests.randgraph import random_checks, random_expands, random_graph
    from tests.test_gpu_lifecycle import _random_write
    ns, tuples, _raw, ps, alph = random_graph(seed + 900, wide=seed % 4 == 3, allow_wildcards=seed % 5 == 0,
                                              allow_poison=False, allow_collisions=seed % 3 == 0)
    names, objs, rels, users = alph
    names = [n for n in names if n]
    if not names:
        pytest.skip("only a namespace named ''")
    ids = {n: i for i, n in reversed(ns)}
    store = SQLStore(ns, tuples, page_size=ps)
    topo = ("Q" + "\t0" * int(replicas[5:])) if isinstance(replicas, str) else ("R" + "\t0" * replicas)
    lines = [f"P\t{ps}", "V\t0", topo]
    lines += [f"N\t{i}\t{n}" for i, n in ns] + [f"T\t{_tuple_fields(ids, t)}" for t in tuples]
    want = []                                  # expected output lines, in order
    rng = random.Random(seed)
    for step in range(6):
        checks = random_checks(seed * 13 + step, (names, objs + ["new1", "a0"], rels + ["q"], users + ["w001"]), k=16)
        for g in sorted({c[2] for c in checks}):
            for t, d, _ in (c for c in checks if c[2] == g):
                sub = (f"I\t{t.subject.id}" if isinstance(t.subject, SubjectID)
                       else f"S\t{t.subject.namespace}\t{t.subject.object}\t{t.subject.relation}")
                lines.append(f"C\t{t.namespace}\t{t.object}\t{t.relation}\t{sub}\t{d}\t{g}")
                want.append(("check", CheckEngine(store, g).subject_is_allowed(t, d)))
        exps = random_expands(seed * 7 + step, (names, objs + ["new3"], rels + ["q"], users), k=6)
        for g in sorted({e[2] for e in exps}):
            for s, d, _ in (e for e in exps if e[2] == g):
                sub = f"I\t{s.id}" if isinstance(s, SubjectID) else f"S\t{s.namespace}\t{s.object}\t{s.relation}"
                lines.append(f"E\t{sub}\t{d}\t{g}")
                try:
                    tr = ExpandEngine(store, g).build_tree(s, d)
                    want.append(("expand", tr.to_json() if tr is not None else None))
                except NotFoundError:
                    want.append(("expand", "error"))
        cur = store.tuples()
        ins = [_random_write(rng, names, objs, rels, users) for _ in range(rng.randint(1, 8))]
        dels = [rng.choice(cur) for _ in range(rng.randint(0, 3))] if cur else []
        lines += [f"A+\t{_tuple_fields(ids, t)}" for t in ins] + [f"A-\t{_tuple_fields(ids, t)}" for t in dels]
        lines.append("A!")
        want.append(("apply", None))
        for t in ins:
            store.insert(t)
        for t in dels:
            store.delete(t)
        if step in (2, 4):                             # a server restart from its persisted snapshot
            lines.append(f"S\t{tmp_path / 'snap.keto'}")
    p = tmp_path / "in.tsv"
    p.write_text("\n".join(lines) + "\n")
    r = subprocess.run([consumer, str(p)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    got = [ln.split("\t") for ln in r.stdout.splitlines() if ln.split("\t")[0] in ("check", "expand", "apply")]
    restarts = [ln.split("\t") for ln in r.stdout.splitlines() if ln.startswith("restart")]
    assert len(restarts) == 2 and all(x[1] == x[2] for x in restarts)
    # the consumer runs a batch of checks before the expands of a step: same order as `want`
    assert [g[0] for g in got] == [w[0] for w in want]
    versions = 0
    for g, (kind, exp) in zip(got, want):
        if kind == "check":
            assert bool(int(g[2])) == exp, (seed, g)
        elif kind == "expand":
            _, _, status, js, pb = g
            if exp == "error":
                assert int(status) == 2 and js == "error"
            elif exp is None:
                assert int(status) == 1 and js == "null" and pb == "-"
            else:
                assert int(status) == 0 and json.loads(js) == exp, (seed, js, exp)
                assert bytes.fromhex(pb) == tree_json_to_proto(exp)
        else:
            assert int(g[1]) in (0, -6)                  # applied, or KETO_E_REBUILD -> rebuilt
            versions += int(g[3]) == 0
    assert r.stdout.splitlines()[-1] == "done"
