#!/bin/bash
# resolve_packed_quad (four lanes per request) for batches up to 2^18 requests:
# batch latency (r05as 0.34 ms), the bench's string-form leg, and a kernel trace of the 65k batches.
set -e
o=gpurun_out/r05az; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resolve_device.py tests/test_gpu_comm.py tests/test_gpu_concurrency.py > $o/pytest_packed.log 2>&1
timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 2 --requests 65536 > $o/packed_65k.log 2> $o/packed_65k.err
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $o/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr -o tr -- python -u tools/apply_concurrent.py --graph drive10m --packed --seconds 1 --requests 65536 > $o/tr.log 2>&1
