#!/bin/bash
# Second GPU-box pass of a round: BASELINE configs #2 / #3 / #5 with parity, the config #3 kernel trace
# and step histogram, and an end-to-end chunking sweep.  Usage: bash tools/gpu_extra.sh <tag>
set -o pipefail
tag=${1:-extra}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { echo "== $(date +%T) $1"; }
step configs
timeout -k 10 500 python -u tools/bench_configs.py --configs 2,3,5 --reps3 3 > $out/configs.log 2>&1 || { tail -30 $out/configs.log; exit 1; }
grep "^{" $out/configs.log | cut -c1-400
step deep-profile
timeout -k 10 300 python -u tools/deep_profile.py > $out/deep_profile.log 2>&1 || { tail -30 $out/deep_profile.log; exit 1; }
step config3-kernel-trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt3 -o kt -- python -u tools/bench_configs.py --configs 3 --no-parity > $out/kt3.log 2>&1 || { tail -30 $out/kt3.log; exit 1; }
step e2e-sweep
timeout -k 10 400 python -u tools/e2e_sweep.py --reps 5 --settings "X=0;KETO_CHUNK_FIRST=1048576;KETO_CHUNK=2097152;KETO_PIPE_STREAMS=2;KETO_PIPE_STREAMS=2,KETO_CHUNK_LANES=262144;KETO_PIPE_STREAMS=2,KETO_CHUNK_LANES=262144,KETO_CHUNK=2097152;KETO_PIPE_STREAMS=2,KETO_CHUNK_LANES=131072,KETO_CHUNK=2097152,KETO_T0_DYN_FORCE=1" > $out/e2e_sweep.log 2>&1 || { tail -30 $out/e2e_sweep.log; exit 1; }
grep "^{" $out/e2e_sweep.log | cut -c1-200
step done
