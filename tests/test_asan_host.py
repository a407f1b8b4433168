"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer run of the library's C++ host code
(snapshot builder, interning, collision classes, resolution, C-ABI error paths) on random
quirk-heavy tuple tables and CSR graphs (tests/asan/snapshot_asan.cpp).  Only host code is
instrumented (-Xarch_host for the HIP source); no GPU is used: the snapshots are host-only and
compute calls must fail loudly with KETO_E_HIP (sanitizers on the host library)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_host_library_under_asan(tmp_path):
    csrc = os.path.join(ROOT, "keto_amd", "csrc")
    san = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    objs = []
    from keto_amd.build import HOST_HIP, SOURCES
    for f in [s for s in SOURCES if s.endswith(".cpp")]:
        o = str(tmp_path / (f + ".o"))
        subprocess.check_call([HIPCC, "-O1", "-g", "-std=c++17", "-x", "c++", *HOST_HIP, *san, "-c", os.path.join(csrc, f),
                               "-o", o])
        objs.append(o)
    for f in [s for s in SOURCES if s.endswith(".hip")]:
        o = str(tmp_path / (f + ".o"))
        subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-Xarch_host",
                               "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-fno-omit-frame-pointer",
                               "-w", "-c", os.path.join(csrc, f), "-o", o])
        objs.append(o)
    d = str(tmp_path / "drv.o")
    subprocess.check_call([HIPCC, "-O1", "-g", "-std=c++17", "-x", "c++", *san, "-c",
                           os.path.join(ROOT, "tests", "asan", "snapshot_asan.cpp"), "-o", d])
    exe = str(tmp_path / "snapshot_asan")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-fsanitize=address,undefined", "-fno-gpu-sanitize",
                           d, *objs, "-o", exe, "-L/opt/rocm/lib", "-lrccl"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "300"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "asan host rounds ok: 300" in r.stdout
