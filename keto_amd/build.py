"""Build recipe for the in-tree HIP library keto_amd/libketo_mi355x.so (gfx950 only)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libketo_mi355x.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
SOURCES = ["snapshot.cpp", "resolve.cpp", "delta.cpp", "persist.cpp", "capi.cpp", "engine.hip", "route.hip", "migrate.hip", "proto.hip", "reach.hip", "resolve_dev.hip", "comm.cpp"]
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]
HOST_HIP = ["-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"]   # host-only sources using the HIP / RCCL APIs
# engine.hip (tier 0, the deep tier, expand) and migrate.hip (the migrating walk) are scheduled for
# memory clauses: the latency-bound walks' independent loads issue back to back (config #3 126-128 ->
# 121 ms, P = 8 migrating parts 18.1-19.2 -> 17.3-18.1 ms; tier 0 and config #5 unchanged; A/B on one
# box: profiles/r06zzc_configs_compiler_flags.txt, r06zze_migrate_compiler_flags.txt, r06zzb_*)
_MEM_CLAUSE = ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]
SOURCE_FLAGS = {"engine.hip": _MEM_CLAUSE, "migrate.hip": _MEM_CLAUSE}


def engine_build_id():
    """sha256 of engine.hip and its compile flags: keys the committed PMC traffic profiles
    (tools/traffic.py writes it, bench.py matches it)."""
    import hashlib
    h = hashlib.sha256(open(os.path.join(CSRC, "engine.hip"), "rb").read())
    flags = SOURCE_FLAGS.get("engine.hip", [])
    if flags:
        h.update(b"\0" + " ".join(flags).encode())
    return h.hexdigest()


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose=False, force=False):
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, "parallel.hpp"), os.path.join(CSRC, "snapshot.hpp"), os.path.join(CSRC, "capi_internal.hpp"),
                                                        os.path.join(HERE, "..", "include", "keto_mi355x.h"), os.path.abspath(__file__)]
    if not force and not _stale(OUT, deps):
        return OUT
    objs = []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(CSRC, src + ".o")
        objs.append(obj)
        if not force and not _stale(obj, [path] + deps[len(SOURCES):]):
            continue
        cmd = [HIPCC, f"--offload-arch={ARCH}", *CXXFLAGS, *SOURCE_FLAGS.get(src, []), "-c", path, "-o", obj]
        if src.endswith(".cpp"):
            cmd = [HIPCC, *CXXFLAGS, *HOST_HIP, "-x", "c++", "-c", path, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT, *objs, "-L/opt/rocm/lib", "-lrccl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return OUT


if __name__ == "__main__":
    build(verbose=True, force="--force" in sys.argv)


def build_variant(name, defines):
    """Tuning build with -D defines into keto_amd/variants/lib_<name>.so (select with KETO_LIB)."""
    vdir = os.path.join(HERE, "variants")
    os.makedirs(vdir, exist_ok=True)
    objs = []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(vdir, f"{name}_{src}.o")
        flags = [f"-D{d}" for d in defines]
        if src.endswith(".cpp"):
            cmd = [HIPCC, *CXXFLAGS, *HOST_HIP, *flags, "-x", "c++", "-c", path, "-o", obj]
        else:
            cmd = [HIPCC, f"--offload-arch={ARCH}", *CXXFLAGS, *SOURCE_FLAGS.get(src, []), *flags, "-c", path, "-o", obj]
        subprocess.check_call(cmd)
        objs.append(obj)
    out = os.path.join(vdir, f"lib_{name}.so")
    subprocess.check_call([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs, "-L/opt/rocm/lib", "-lrccl"])
    return out
