#!/bin/bash
# Config #3 with the targets-only reachability index: the pretest's bounds (KETO_REACH_WORK edges,
# KETO_REACH_CAP marks) and minimum depth swept in one process, decisions compared across legs.
o=gpurun_out/r06zw
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06zw \
  "sweep|500|KETO_REACH_TRACE=1 python -u tools/deep_sweep.py '' 'KETO_REACH_WORK=2048' 'KETO_REACH_WORK=8192' 'KETO_REACH_CAP=4096,KETO_REACH_WORK=8192' 'KETO_REACH_MIN_DEPTH=12' ''"
