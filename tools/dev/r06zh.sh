#!/bin/bash
# Expand config #5: the lane-run copy with 1 / 4 / 8 half-waves per lane (KETO_EXPAND_RUN_SPLIT),
# kernel stats of each, trees checked against the oracle at the default.
o=gpurun_out/r06zh
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06zh \
  "check|240|python -u tools/dev/expand_prof.py --reps 3 --check 5000" \
  "ks_1|200|KETO_EXPAND_RUN_SPLIT=1 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_1 -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "ks_4|200|rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_4 -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "ks_8|200|KETO_EXPAND_RUN_SPLIT=8 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_8 -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "tests|400|python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_synth.py -m gpu -k expand"
