#!/bin/bash
# Migrating parts through the product path (local transport ranks, routed packed), P = 1/2/4/8, then
# a kernel trace of the P = 8 run.
o=gpurun_out/r06p
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06p \
  "mig_local|400|python -u tools/bench_migrate_local.py --scale 0.125 --parts 1 2 4 8 --hot-mb 0 300" \
  "mig_trace|300|rocprofv3 --kernel-trace --memory-copy-trace --stats -d $o/tr -o t -- python -u tools/bench_migrate_local.py --scale 0.125 --parts 8 --hot-mb 300 --steps 3"
