"""Host-side ThreadSanitizer run of the library's concurrency (tests/tsan/snapshot_tsan.cpp): a writer
applying transactions, readers resolving named requests (the lazily built resolution indexes),
mapping rows and reading stats, a copier cloning / saving / loading, and a planner computing partition
statistics, all on one host-only snapshot at once.  The library's host code is built with
-fsanitize=thread (-Xarch_host for the .hip sources, whose kernels never run here); any data race
fails the test.  The reference runs its whole suite under Go's race detector (.circleci/config.yml:63)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_host_library_under_tsan(tmp_path):
    from concurrent.futures import ThreadPoolExecutor
    from keto_amd.build import HOST_HIP, SOURCES
    csrc = os.path.join(ROOT, "keto_amd", "csrc")
    san = ["-fsanitize=thread", "-fno-omit-frame-pointer"]

    def compile_one(f):
        o = str(tmp_path / (f + ".o"))
        if f.endswith(".cpp"):
            cmd = [HIPCC, "-O1", "-g", "-std=c++17", "-x", "c++", *HOST_HIP, *san, "-c", os.path.join(csrc, f), "-o", o]
        else:
            cmd = [HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-Xarch_host",
                   "-fsanitize=thread", "-fno-omit-frame-pointer", "-w", "-c", os.path.join(csrc, f), "-o", o]
        subprocess.check_call(cmd)
        return o

    with ThreadPoolExecutor(4) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    d = str(tmp_path / "drv.o")
    subprocess.check_call([HIPCC, "-O1", "-g", "-std=c++17", "-x", "c++", *san, "-c",
                           os.path.join(ROOT, "tests", "tsan", "snapshot_tsan.cpp"), "-o", d])
    exe = str(tmp_path / "snapshot_tsan")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-fsanitize=thread", "-fno-gpu-sanitize", d, *objs, "-o", exe,
                           "-L/opt/rocm/lib", "-lrccl"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1", KETO_BUILD_THREADS="4")
    r = subprocess.run([exe, "60", str(tmp_path)], capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-6000:]
    assert "tsan host rounds ok: 60 writes" in r.stdout
