#!/bin/bash
# Packed batches in flight, second form: resolution straight to handles, tier 0 only on two check
# streams, one D2H, no memsets per batch.  Tests, then the 65,536-request sweep on the 1B graph, then
# a kernel + copy trace of the 4-reader / 4-slot run.
o=gpurun_out/r06e
mkdir -p $o
bash tools/gpu_steps.sh r06e \
  "pytest|600|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resolve_device.py tests/test_gpu_concurrency.py tests/test_gpu_overflow.py -m gpu" \
  "s2_r2|300|KETO_APPLY_TRACE=1 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 2" \
  "s4_r4|300|KETO_PACKED_SLOTS=4 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 4" \
  "s4_r8|300|KETO_PACKED_SLOTS=4 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 8" \
  "trace|300|cd /tmp && export TMPDIR=/tmp && cd - && KETO_PACKED_SLOTS=4 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/tr -o t -- python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 1 --requests 65536 --readers 4"
