#!/bin/bash
# The packed-path tests on the build with resolve_packed templated (its opt-in clock mode).
set -e
o=gpurun_out/r05bb; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resolve_device.py tests/test_gpu_comm.py tests/test_gpu_concurrency.py tests/test_gpu_lifecycle.py > $o/pytest_packed.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
