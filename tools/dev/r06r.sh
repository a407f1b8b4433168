#!/bin/bash
# Migrating small tier: lanes x visited-table entries sweep at P = 8 (local transport, hot 300 MB).
o=gpurun_out/r06r
mkdir -p $o
run() { echo "KETO_MIG_LANES=$1 KETO_MIG_VCAP=$2"; KETO_MIG_LANES=$1 KETO_MIG_VCAP=$2 python -u tools/bench_migrate_local.py --scale 0.125 --parts 8 --hot-mb 300 --steps 5; }
export -f run
bash tools/gpu_steps.sh r06r \
  "l256k_v512|200|run 262144 512" \
  "l64k_v512|200|run 65536 512" \
  "l64k_v128|200|run 65536 128" \
  "l256k_v128|200|run 262144 128" \
  "l32k_v256|200|run 32768 256" \
  "debug|200|KETO_MIG_DEBUG=1 run 262144 512"
