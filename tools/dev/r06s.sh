#!/bin/bash
# Expand config #5: the spread-4 tier 0 forced to 6 waves per SIMD (80 VGPRs, spilling) against the
# default, phase trace and kernel stats.
o=gpurun_out/r06s
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06s \
  "trace_default|240|KETO_EXPAND_TRACE=1 python -u tools/dev/expand_prof.py --reps 6" \
  "trace_spread4|240|KETO_EXPAND_SPREAD=4 KETO_EXPAND_TRACE=1 python -u tools/dev/expand_prof.py --reps 6 --check 5000" \
  "ks_default|300|rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks1 -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "ks_spread4|300|KETO_EXPAND_SPREAD=4 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks4 -o p -- python -u tools/dev/expand_prof.py --reps 10"
