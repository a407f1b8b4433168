"""Consistency of the Go integration sources (integration/go, not compiled here: no Go toolchain)
with the C-ABI they bind: every C.keto_* / C.KETO_* name they use is declared in
include/keto_mi355x.h, and they stay within Go 1.17 (the reference's go.mod:221)."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _go_files():
    return sorted(glob.glob(os.path.join(ROOT, "integration", "go", "**", "*.go"), recursive=True))


def test_go_sources_use_declared_c_names():
    hdr = open(os.path.join(ROOT, "include", "keto_mi355x.h")).read()
    declared = set(re.findall(r"\b((?:keto|KETO)_[A-Za-z0-9_]+)\b", hdr))
    files = _go_files()
    assert len(files) >= 5
    for f in files:
        src = open(f).read()
        for name in set(re.findall(r"\bC\.(?:sizeof_)?((?:keto|KETO)_[A-Za-z0-9_]+)", src)):
            assert name in declared, (os.path.relpath(f, ROOT), name)


def test_go_sources_stay_on_go_1_17():
    for f in _go_files():
        src = open(f).read()
        code = "\n".join(ln.split("//")[0] for ln in src.splitlines())     # comments may name them
        for banned in ("runtime.Pinner", "unsafe.StringData", "unsafe.SliceData", "unsafe.String(", "[T any]",
                       "min(", "max(", "clear("):
            assert banned not in code, (os.path.relpath(f, ROOT), banned)
        # cgo files carry both build-constraint forms (the // +build line is what Go 1.17 reads)
        if 'import "C"' in src:
            assert "//go:build keto_gpu" in src and "// +build keto_gpu" in src, f
