"""Tuning build: one source (engine.hip by default) compiled with extra compiler flags, linked with the default build's other
objects into keto_amd/variants/lib_<name>.so (select with KETO_LIB).  Run after build() so the other
objects exist.  Usage: [SRC=migrate.hip] python tools/dev/build_flag_variant.py <name> <flag> [<flag> ...]
(SRC names the one source compiled with the flags, engine.hip by default)."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from keto_amd import build as B  # noqa: E402


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    target = os.environ.get("SRC", "engine.hip")
    vdir = os.path.join(B.HERE, "variants")
    os.makedirs(vdir, exist_ok=True)
    objs = []
    for src in B.SOURCES:
        obj = os.path.join(B.CSRC, src + ".o")
        if src == target:
            obj = os.path.join(vdir, f"{name}_{src}.o")
            subprocess.check_call([B.HIPCC, f"--offload-arch={B.ARCH}", *B.CXXFLAGS, *flags, "-c",
                                   os.path.join(B.CSRC, src), "-o", obj])
        objs.append(obj)
    out = os.path.join(vdir, f"lib_{name}.so")
    subprocess.check_call([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out, *objs,
                           "-L/opt/rocm/lib", "-lrccl"])
    print(out)


if __name__ == "__main__":
    main()
