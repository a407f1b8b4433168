"""Consistency of the Go integration sources (integration/go, not compiled here: no Go toolchain)
with the C-ABI they bind and with each other: every C.keto_* / C.KETO_* name they use is declared in
include/keto_mi355x.h, every exported gpu.X another package uses is declared in package gpu, the
package graph has no cycle (gpu imports none of the packages that import it), and the sources stay
within Go 1.17 (the reference's go.mod:221)."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "integration", "go")
MODULE = "github.com/ory/keto/"


def _go_files():
    return sorted(glob.glob(os.path.join(GO, "**", "*.go"), recursive=True))


def _code(src):
    return "\n".join(ln.split("//")[0] for ln in src.splitlines())     # comments may name anything


def _imports(src):
    m = re.search(r"^import \((.*?)^\)", src, re.S | re.M)
    block = m.group(1) if m else ""
    single = re.findall(r'^import\s+"([^"]+)"', src, re.M)
    return set(re.findall(r'"([^"]+)"', block)) | set(single)


def test_go_sources_use_declared_c_names():
    hdr = open(os.path.join(ROOT, "include", "keto_mi355x.h")).read()
    declared = set(re.findall(r"\b((?:keto|KETO)_[A-Za-z0-9_]+)\b", hdr))
    files = _go_files()
    assert len(files) >= 8
    for f in files:
        src = open(f).read()
        for name in set(re.findall(r"\bC\.(?:sizeof_)?((?:keto|KETO)_[A-Za-z0-9_]+)", src)):
            assert name in declared, (os.path.relpath(f, ROOT), name)


def test_go_sources_stay_on_go_1_17():
    for f in _go_files():
        src = open(f).read()
        code = _code(src)
        for banned in ("runtime.Pinner", "unsafe.StringData", "unsafe.SliceData", "unsafe.String(", "[T any]",
                       "min(", "max(", "clear(", "atomic.Pointer", "atomic.Int64", "errors.Join", "slices.",
                       "maps."):
            assert banned not in code, (os.path.relpath(f, ROOT), banned)
        # cgo files and their importers are behind the keto_gpu tag, in both build-constraint forms
        # (Go 1.17 reads // +build); cmd/check's batch mode is a plain gRPC client and builds always
        if 'import "C"' in src or MODULE + "internal/gpu" in src:
            assert "//go:build keto_gpu" in src and "// +build keto_gpu" in src, f


def test_go_package_graph():
    pkgs = {}
    for f in _go_files():
        src = open(f).read()
        rel = os.path.relpath(os.path.dirname(f), GO).replace(os.sep, "/")
        pkg = re.search(r"^package (\w+)", src, re.M).group(1)
        assert pkg == rel.split("/")[-1], (f, pkg)             # the package of its drop-in directory
        pkgs.setdefault(rel, set()).update(i[len(MODULE):] for i in _imports(src) if i.startswith(MODULE))
    # internal/gpu is imported by check, expand, driver and persistence/sql: it must import none of them
    assert not (pkgs["internal/gpu"] & {"internal/check", "internal/expand", "internal/driver",
                                        "internal/persistence/sql"}), pkgs["internal/gpu"]
    for p, deps in pkgs.items():
        for d in deps:
            assert p not in pkgs.get(d, set()), (p, d)          # no two-package cycle among our files
    assert "internal/gpu" in pkgs["internal/expand"] and "internal/gpu" in pkgs["internal/check"]
    assert "internal/gpu" in pkgs["internal/driver"] and "internal/gpu" in pkgs["internal/persistence/sql"]


def test_exported_gpu_names_exist():
    decl = set()
    for f in glob.glob(os.path.join(GO, "internal", "gpu", "*.go")):
        code = _code(open(f).read())
        decl |= set(re.findall(r"^func (?:\([^)]*\) )?([A-Z]\w*)", code, re.M))
        decl |= set(re.findall(r"^type ([A-Z]\w*)", code, re.M))
        decl |= set(re.findall(r"^\s*([A-Z]\w*)\s*=", code, re.M))          # var / const blocks
        decl |= set(re.findall(r"^(?:var|const) ([A-Z]\w*)", code, re.M))
    for f in _go_files():
        if os.sep + os.path.join("internal", "gpu") + os.sep in f:
            continue
        for name in set(re.findall(r"\bgpu\.([A-Z]\w*)", _code(open(f).read()))):
            assert name in decl, (os.path.relpath(f, ROOT), name)


def test_engine_dispatch_hooks_match_the_registry():
    """The providers the engines look for are the methods registry_gpu.go adds to RegistryDefault."""
    reg = _code(open(os.path.join(GO, "internal", "driver", "registry_gpu.go")).read())
    for eng, method in (("check", "GPUCheckBatcher"), ("expand", "GPUExpandBatcher")):
        src = _code(open(os.path.join(GO, "internal", eng, "engine_gpu.go")).read())
        assert f"{method}() *gpu." in src
        assert re.search(r"func \(r \*RegistryDefault\) " + method + r"\(\) \*gpu\.", reg), method
    # the persister wrapper overrides every write method of relationtuple.Manager
    # (internal/relationtuple/definitions.go:28-34)
    for m in ("WriteRelationTuples", "DeleteRelationTuples", "DeleteAllRelationTuples", "TransactRelationTuples"):
        assert re.search(r"func \(p \*gpuPersister\) " + m + r"\(", reg), m


def test_multi_gpu_server_process():
    """One server process drives every GPU (the reference is one process, internal/driver/daemon.go:62-69):
    EnableGPU takes the device list, builds one replica per device (sorted once, the others cloned
    with keto_snapshot_clone), the batchers deal batches over the replica set, and every write
    transaction reaches every replica before it returns."""
    reg = _code(open(os.path.join(GO, "internal", "driver", "registry_gpu.go")).read())
    assert re.search(r"func EnableGPU\(ctx context\.Context, reg Registry, devices \[\]int\) error", reg)
    assert "gpu.BuildReplicas(" in reg and "gpu.ApplyAll(" in reg and "func GPUDevicesFromEnv() []int" in reg
    gpu_go = _code(open(os.path.join(GO, "internal", "gpu", "gpu.go")).read())
    assert "C.keto_snapshot_clone(" in gpu_go
    assert re.search(r"func BuildReplicas\(nss \[\]\*namespace\.Namespace, rows \[\]Row, devices \[\]int\)", gpu_go)
    bat = _code(open(os.path.join(GO, "internal", "gpu", "batcher.go")).read())
    assert re.search(r"func NewBatcher\(snaps \[\]\*Snapshot,", bat)
    assert re.search(r"func NewExpandBatcher\(snaps \[\]\*Snapshot,", bat)
    assert "r.idle" in bat                              # a batch goes to a replica with none in flight


def test_persisted_snapshot_at_startup():
    """A server started with KETO_GPU_SNAPSHOT_FILE loads the persisted snapshot (keto_snapshot_load)
    when its tag is the table's current fingerprint (row count + newest commit_time), clones it to
    the other devices, and otherwise scans, builds and saves the file again (keto_snapshot_save)."""
    reg = _code(open(os.path.join(GO, "internal", "driver", "registry_gpu.go")).read())
    gpu_go = _code(open(os.path.join(GO, "internal", "gpu", "gpu.go")).read())
    sql = _code(open(os.path.join(GO, "internal", "persistence", "sql", "snapshot_gpu.go")).read())
    assert "C.keto_snapshot_save(" in gpu_go and "C.keto_snapshot_load(" in gpu_go
    assert re.search(r"func \(s \*Snapshot\) Save\(path string, tag uint64\) error", gpu_go)
    assert re.search(r"func Load\(path string, device int\) \(\*Snapshot, uint64, error\)", gpu_go)
    assert re.search(r"func \(p \*Persister\) SnapshotFingerprint\(ctx context\.Context\) \(uint64, error\)", sql)
    assert "SnapshotFingerprint(ctx context.Context) (uint64, error)" in reg      # part of the row source
    load_at = reg.index("g.loadFile(path, fp)")
    scan_at = reg.index("src.SnapshotRows(ctx)")
    assert load_at < scan_at                                                    # the file first
    assert ".Save(path, fp)" in reg and "tag != fp" in reg


def test_collective_calls_never_skip_an_empty_batch():
    """keto_check_batch_sharded / _routed are collective: a rank with no request must still call them,
    or its peers wait (checkWith's collective flag)."""
    comm = _code(open(os.path.join(GO, "internal", "gpu", "comm.go")).read())
    gpu_go = _code(open(os.path.join(GO, "internal", "gpu", "gpu.go")).read())
    assert len(re.findall(r"checkWith\(reqs, depths, true,", comm)) == 2
    assert "if n == 0 && !collective {" in gpu_go
    assert "C.keto_comm_init_local(" in comm
