#!/bin/bash
# Configs #3 (deep check) and #5 (expand) with engine.hip built under compiler flags
# (tools/dev/build_flag_variant.py: sur / ilp / mcl as in r06zzb.sh), alternating with the
# default build on one box; each run keeps its oracle parity legs.
export TMPDIR=/tmp
C="python -u tools/bench_configs.py --configs 3,5 --reps3 3"
L="KETO_LIB=keto_amd/variants/lib_"
bash tools/gpu_steps.sh r06zzc \
  "base1|300|$C" "sur1|300|${L}sur.so $C" "ilp1|300|${L}ilp.so $C" "mcl1|300|${L}mcl.so $C" \
  "base2|300|$C" "sur2|300|${L}sur.so $C" "ilp2|300|${L}ilp.so $C" "mcl2|300|${L}mcl.so $C"
