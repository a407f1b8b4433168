#!/bin/bash
# Migrating parts (P = 8 local-transport ranks, routed packed batches) with migrate.hip built under
# memory-clause scheduling (SRC=migrate.hip tools/dev/build_flag_variant.py migmcl), alternating with
# the default build on one box; then the comm / migrate suites on the variant.
export TMPDIR=/tmp
M="python -u tools/bench_migrate_local.py --scale 0.125 --parts 8 --hot-mb 300"
L="KETO_LIB=keto_amd/variants/lib_migmcl.so"
bash tools/gpu_steps.sh r06zze \
  "base1|300|$M" "mcl1|300|$L $M" "base2|300|$M" "mcl2|300|$L $M" \
  "tests_mcl|400|$L python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_migrate.py -m gpu"
