#!/bin/bash
# Config #3: more tier-0 lanes with 64K-entry tables (a bigger deep budget), one process, decisions
# compared across all combos.
o=gpurun_out/r06i
mkdir -p $o
timeout -k 10 500 python -u tools/deep_sweep.py "" "KETO_DEEP_BUDGET_GB=200" "KETO_DEEP_BUDGET_GB=240" \
  "KETO_DEEP_BUDGET_GB=100" "KETO_T0_CAP=32768" "KETO_T0_CAP=131072,KETO_DEEP_BUDGET_GB=240" "" > $o/sweep.log 2> $o/sweep.err || { tail -20 $o/sweep.err; exit 1; }
cat $o/sweep.log
