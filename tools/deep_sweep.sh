#!/bin/bash
# Config #3 tier-geometry sweep (tuning): bash tools/deep_sweep.sh <tag> "<env settings>"...
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
i=0
for envs in "$@"; do
  echo "== $(date +%T) [$envs]" | tee -a $out/sweep.log
  env $envs timeout -k 10 300 python -u tools/bench_configs.py --configs 3 --no-parity $EXTRA >> $out/sweep.log 2> $out/sweep_$i.err || { tail -20 $out/sweep_$i.err; exit 1; }
  tail -1 $out/sweep.log
  i=$((i+1))
done
