#!/bin/bash
# Migrating walk with its visited map's first 16 ids in LDS behind a register filter: the comm /
# migrate suites, then the local-transport bench.
o=gpurun_out/r06y
mkdir -p $o
bash tools/gpu_steps.sh r06y \
  "tests|600|python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_migrate.py -m gpu" \
  "mig_local|400|python -u tools/bench_migrate_local.py --scale 0.125 --parts 1 2 4 8 --hot-mb 0 300"
