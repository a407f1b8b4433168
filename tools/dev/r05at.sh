#!/bin/bash
# One host round trip fewer per packed batch on an unpartitioned snapshot: the resolution tests,
# then the 65,536-request batch latency again (r05as had 0.34 ms).
set -e
o=gpurun_out/r05at; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resolve_device.py tests/test_gpu_comm.py > $o/pytest_packed.log 2>&1
timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 2 --requests 65536 > $o/packed_65k.log 2> $o/packed_65k.err
