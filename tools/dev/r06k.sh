#!/bin/bash
# keto_check_batch_routed_packed (ABI 6): the local-transport routed tests (new packed ones included),
# the consumer (packed batches from 4 threads), then config #4's partitioned forms at full scale with
# the packed routed batch timed.
o=gpurun_out/r06k
mkdir -p $o
bash tools/gpu_steps.sh r06k \
  "comm|500|python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_comm.py tests/test_consumer_c.py -m gpu" \
  "parts|900|KETO_PARTS_LOG=$o/config4_parts.log python -u -m pytest -x -v -s --timeout 850 --timeout-method thread tests/test_gpu_config4_parts.py -m gpu"
