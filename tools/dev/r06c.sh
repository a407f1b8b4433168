#!/bin/bash
# Packed batches in flight (KETO_PACKED_SLOTS): the packed / concurrency / migrating tests, then the
# 65,536-request packed reads on the 1B graph with 1-4 reader threads and 0 (one batch at a time),
# 2 and 4 slots, with 100-tuple writes every 20 ms (KETO_APPLY_TRACE on the 2-reader run).
o=gpurun_out/r06c
mkdir -p $o
bash tools/gpu_steps.sh r06c \
  "pytest|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resolve_device.py tests/test_gpu_concurrency.py tests/test_gpu_migrate.py -m gpu" \
  "s0_r2|300|KETO_PACKED_SLOTS=0 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 2" \
  "s2_r2|300|KETO_APPLY_TRACE=1 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 2" \
  "s2_r1|300|python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 1" \
  "s2_r4|300|python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 4" \
  "s4_r4|300|KETO_PACKED_SLOTS=4 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 4"
