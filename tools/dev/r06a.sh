#!/bin/bash
# Round 6 first GPU call: the routed exchanges with the version agreement (test_gpu_comm.py, incl. the
# new refused-at-different-versions test), then config #4's partitioned forms at the full 1B scale
# (tests/test_gpu_config4_parts.py) with their per-part log.
o=gpurun_out/r06a
mkdir -p $o
bash tools/gpu_steps.sh r06a \
  "comm|400|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_comm.py -m gpu" \
  "parts|1000|KETO_PARTS_LOG=$o/config4_parts.log python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_config4_parts.py -m gpu"
