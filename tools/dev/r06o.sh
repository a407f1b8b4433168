#!/bin/bash
# Migrating parts answer wildcard queries over rows with failing pages: the comm and migrate suites.
o=gpurun_out/r06o
mkdir -p $o
bash tools/gpu_steps.sh r06o \
  "comm|600|python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_migrate.py -m gpu"
