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
    EnableGPU takes the device list and places the snapshot (gpu.Place): one replica per device while
    the replicated arena fits each of them (sized with keto_snapshot_part_stats_mode and
    keto_device_memory), else one Partition over all of them; the batchers deal batches over the
    engine set, and every write transaction reaches every replica or part before it returns."""
    reg = _code(open(os.path.join(GO, "internal", "driver", "registry_gpu.go")).read())
    assert re.search(r"func EnableGPU\(ctx context\.Context, reg Registry, devices \[\]int\) error", reg)
    assert "gpu.Place(" in reg and "gpu.ApplyEngines(" in reg and "func GPUDevicesFromEnv() []int" in reg
    assert "func GPUPlacementFromEnv() string" in reg
    gpu_go = _code(open(os.path.join(GO, "internal", "gpu", "gpu.go")).read())
    assert "C.keto_snapshot_clone(" in gpu_go
    part = _code(open(os.path.join(GO, "internal", "gpu", "partition.go")).read())
    assert re.search(r"func Place\(base \*Snapshot, devices \[\]int, mode string\) \(\[\]Engine, error\)", part)
    assert "C.keto_device_memory(" in part and "C.keto_snapshot_part_stats_mode(" in part
    # past the arena cap a replica cannot take (KETO_ARENA_MAX_BYTES), the snapshot is partitioned
    # even onto one device: PlanParts deals parts to the devices in turn, several per device if need be
    assert "C.KETO_ARENA_MAX_BYTES" in part and "arena <= arenaCap" in part
    assert re.search(r"func PlanParts\(base \*Snapshot, devices \[\]int\) \(\[\]int, error\)", part)
    assert "plan[k] = devices[k%len(devices)]" in part and "NewPartition(base, plan)" in part
    hdr = open(os.path.join(ROOT, "include", "keto_mi355x.h")).read()
    assert re.search(r"#define KETO_ARENA_MAX_BYTES \(288ull << 30\)", hdr)
    bat = _code(open(os.path.join(GO, "internal", "gpu", "batcher.go")).read())
    assert re.search(r"func NewBatcher\(snaps \[\]Engine,", bat)
    assert re.search(r"func NewExpandBatcher\(snaps \[\]Engine,", bat)
    assert "set.idle" in bat                            # a batch goes to an engine with none in flight
    # both engine kinds answer the batchers: a replica and a partition
    for recv in (r"\(s \*Snapshot\)", r"\(p \*Partition\)"):
        for m in ("CheckBatch", "ExpandBatch", "Apply", "Close"):
            assert re.search(r"^func " + recv + " " + m + r"\(", gpu_go + "\n" + part + "\n" +
                             _code(open(os.path.join(GO, "internal", "gpu", "apply.go")).read()), re.M), (recv, m)


def test_partitioned_serving():
    """A graph past one GPU's memory is served partitioned from the same process: shared-rows parts
    (keto_snapshot_upload_part_mode, KETO_PART_SHARED) on the devices, one in-process communicator
    rank per part (NewLocalComm), every batch split over the ranks and routed collectively -- every
    rank calls, an empty slice too -- and every write applied to every part."""
    part = _code(open(os.path.join(GO, "internal", "gpu", "partition.go")).read())
    assert "C.keto_snapshot_upload_part_mode(" in part and "C.KETO_PART_SHARED" in part
    assert "NewLocalComm(" in part
    assert "call(p.parts[k], reqs[lo:hi]" in part                       # every rank, its slice
    assert "call = p.comms[k].CheckBatchRoutedPacked" in part and "packedFits(reqs)" in part   # resolved on the device
    comm = _code(open(os.path.join(GO, "internal", "gpu", "comm.go")).read())
    assert "C.keto_check_batch_routed_packed(" in comm
    assert ".ExpandBatchRouted(p.parts[k], subs[lo:hi]" in part
    assert "wg.Wait()" in part                                           # the ranks' calls run at once
    apply_at = part.index("func (p *Partition) Apply(")
    assert "p.parts[k].Apply(inserts, deletes)" in part[apply_at:apply_at + 400]       # every part, side by side
    assert "p.ranks(" in part[apply_at:apply_at + 400]


def test_persisted_snapshot_at_startup():
    """A server started with KETO_GPU_SNAPSHOT_FILE scans the table, and loads the persisted snapshot
    (keto_snapshot_load, host-only, then placed) when its tag is the fingerprint of the scanned rows'
    contents (gpu.Fingerprint: an order-independent hash of the row multiset, so no committed write
    leaves it unchanged); otherwise it builds and saves the file again (keto_snapshot_save)."""
    reg = _code(open(os.path.join(GO, "internal", "driver", "registry_gpu.go")).read())
    gpu_go = _code(open(os.path.join(GO, "internal", "gpu", "gpu.go")).read())
    part = _code(open(os.path.join(GO, "internal", "gpu", "partition.go")).read())
    assert "C.keto_snapshot_save(" in gpu_go and "C.keto_snapshot_load(" in gpu_go
    assert re.search(r"func \(s \*Snapshot\) Save\(path string, tag uint64\) error", gpu_go)
    assert re.search(r"func Load\(path string, device int\) \(\*Snapshot, uint64, error\)", gpu_go)
    assert re.search(r"func Fingerprint\(rows \[\]Row\) uint64", part)
    scan_at = reg.index("src.SnapshotRows(ctx)")
    load_at = reg.index("g.loadFile(path, gpu.Fingerprint(rows))")
    assert scan_at < load_at                                                    # the rows' contents first
    assert ".Save(path, gpu.Fingerprint(rows))" in reg and "tag != fp" in reg
    assert "gpu.Load(path, -1)" in reg


def test_fingerprint_is_order_independent_and_content_sensitive():
    """gpu.Fingerprint restated in Python (FNV-1a per field with length separators, a splitmix64
    finalizer, a wrapping sum over rows): the same multiset in another order gives the same value;
    deleting a tuple and inserting another (same count) changes it; a duplicate counts."""
    M = (1 << 64) - 1

    def mix64(x):
        x ^= x >> 31
        x = (x * 0xBF58476D1CE4E5B9) & M
        x ^= x >> 29
        x = (x * 0x94D049BB133111EB) & M
        return x ^ (x >> 32)

    def row_hash(r):
        h = 1469598103934665603

        def step(v):
            nonlocal h
            h = ((h ^ v) * 1099511628211) & M

        def add(b):
            for c in b.encode():
                step(c)
            step(len(b.encode()))
        step(r[0] & 0xFFFFFFFF)
        add(r[1])
        add(r[2])
        if r[3] is not None:
            step(1)
            add(r[3])
        else:
            step(2 ^ ((r[4] & 0xFFFFFFFF) << 8))
            add(r[5])
            add(r[6])
        return h

    def fp(rows):
        s = sum(mix64(row_hash(r)) for r in rows) & M
        return mix64(s ^ mix64((len(rows) + 0x9E3779B97F4A7C15) & M))

    a = [(1, "d", "view", "u1"), (1, "d", "view", None, 2, "g", "member"), (2, "g", "member", "u2")]
    assert fp(a) == fp(list(reversed(a)))
    assert fp(a) != fp(a[:2] + [(2, "g", "member", "u3")])
    assert fp(a) != fp(a + [a[0]])
    assert fp([(1, "ab", "c", "x")]) != fp([(1, "a", "bc", "x")])
    part = open(os.path.join(GO, "internal", "gpu", "partition.go")).read()
    for const in ("1469598103934665603", "1099511628211", "0xBF58476D1CE4E5B9", "0x94D049BB133111EB",
                  "0x9E3779B97F4A7C15"):
        assert const in part, const


def test_collective_calls_never_skip_an_empty_batch():
    """keto_check_batch_sharded / _routed are collective: a rank with no request must still call them,
    or its peers wait (checkWith's collective flag)."""
    comm = _code(open(os.path.join(GO, "internal", "gpu", "comm.go")).read())
    gpu_go = _code(open(os.path.join(GO, "internal", "gpu", "gpu.go")).read())
    assert len(re.findall(r"checkWith\(reqs, depths, true,", comm)) == 2
    assert "if n == 0 && !collective {" in gpu_go
    assert "C.keto_comm_init_local(" in comm


def test_packed_batches_use_a_reused_pinned_arena():
    """A large packed batch goes up from a page-locked arena (keto_host_alloc) the snapshot keeps
    from call to call, so keto_check_batch_packed can upload it asynchronously under the resolution
    and check of earlier pieces.  The snapshot keeps one arena per batch in flight (a pool of
    InflightFromEnv arenas, each locked for its call), frees them all with the snapshot, and the
    batchers deal InflightFromEnv batches to an engine at once (KETO_GPU_INFLIGHT)."""
    src = _code(open(os.path.join(GO, "internal", "gpu", "gpu.go")).read())
    body = src[src.index("func (s *Snapshot) checkPacked("):]
    body = body[:body.index("\nfunc ")]
    assert "s.arenas.get(" in body and "defer s.arenas.put(a)" in body
    assert body.index("s.arenas.get(") < body.index("C.keto_check_batch_packed(")
    arena = src[src.index("func (a *pinnedArena) get("):]
    assert "C.keto_host_alloc(" in arena and "C.keto_host_free(" in arena and "a.mu.Lock()" in arena
    pool = src[src.index("func (p *arenaPool) init("):]
    assert "InflightFromEnv()" in pool[:pool.index("\n}")]
    close = src[src.index("func (s *Snapshot) Close()"):]
    assert "s.arenas.freeAll()" in close[:close.index("\n}")]
    bat = _code(open(os.path.join(GO, "internal", "gpu", "batcher.go")).read())
    es = bat[bat.index("func newEngineSet("):]
    es = es[:es.index("\n}")]
    assert "InflightFromEnv()" in es and "per*len(snaps)" in es


def test_check_flush_size_from_env():
    """The check batcher's flush size is KETO_GPU_CHECK_BATCH (default 65,536, capped at 2^24)."""
    src = _code(open(os.path.join(GO, "internal", "gpu", "batcher.go")).read())
    fn = src[src.index("func CheckFlushFromEnv() int {"):]
    fn = fn[:fn.index("\n}\n")]
    assert 'os.Getenv("KETO_GPU_CHECK_BATCH")' in fn and "return 1 << 16" in fn and "1<<24" in fn
    assert "newCoalescer(CheckFlushFromEnv()," in src
