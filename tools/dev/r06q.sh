#!/bin/bash
# Migrating rounds without global-atomic grouping, one-launch local exchanges, fused round words:
# the comm / migrate suites, then the local-transport bench and a P = 8 kernel trace.
o=gpurun_out/r06q
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06q \
  "tests|600|python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_migrate.py -m gpu" \
  "mig_local|400|python -u tools/bench_migrate_local.py --scale 0.125 --parts 1 2 4 8 --hot-mb 0 300" \
  "mig_trace|300|rocprofv3 --kernel-trace --memory-copy-trace --stats -d $o/tr -o t -- python -u tools/bench_migrate_local.py --scale 0.125 --parts 8 --hot-mb 300 --steps 3"
