#!/bin/bash
# Row/handle maps patched independently (no re-upload of the row map after row-adding writes):
# new-rows writes under 4 readers.
set -e
o=gpurun_out/r05an; mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lifecycle.py tests/test_gpu_arena_split.py tests/test_gpu_items.py tests/test_gpu_concurrency.py tests/test_gpu_resolve_device.py tests/test_gpu_replicas.py tests/test_gpu_comm.py > $o/pytest_writes.log 2>&1
KETO_APPLY_TRACE=1 timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 8 --readers 4 --new-rows > $o/apply_1b_r4_rows.log 2> $o/apply_1b_r4_rows.err
