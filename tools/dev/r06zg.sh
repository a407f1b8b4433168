#!/bin/bash
# Expand config #5: runs over 256 ids to the shared big-run queue (pieces a wave each; a build with
# KETO_BIG_RUN=256) against the default 1024, kernel stats of both, trees checked against the oracle.
o=gpurun_out/r06zg
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06zg \
  "check256|240|KETO_LIB=keto_amd/variants/lib_bigrun256.so python -u tools/dev/expand_prof.py --reps 3 --check 5000" \
  "ks_256|200|KETO_LIB=keto_amd/variants/lib_bigrun256.so rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_256 -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "ks_1024|200|rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_1024 -o p -- python -u tools/dev/expand_prof.py --reps 10"
