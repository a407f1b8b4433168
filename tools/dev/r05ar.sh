#!/bin/bash
# Pipelined packed batches (pieces uploaded on a copy stream while earlier pieces resolve and check):
# the device-resolution tests, then the bench's string-form leg and a kernel / copy trace of it.
set -e
o=gpurun_out/r05ar; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resolve_device.py tests/test_gpu_concurrency.py tests/test_gpu_comm.py > $o/pytest_packed.log 2>&1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $o/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $o/tr -o tr -- python -u bench.py --no-work --steps 2 --warmup 1 --e2e-steps 0 --string-steps 3 > $o/tr.log 2>&1
