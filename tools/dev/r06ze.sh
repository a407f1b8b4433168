#!/bin/bash
# Expand config #5: staged trees over 256 nodes copied as 512-node pieces (a wave each) instead of by
# their 16-lane gather group, and the lane-run copy with 4 ids per thread in flight; kernel stats of
# the new default and of KETO_EXPAND_GATHER_BIG=0 (every single-piece tree in the gather), trees
# checked against the oracle, then the expand parity suites.
o=gpurun_out/r06ze
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06ze \
  "check|240|python -u tools/dev/expand_prof.py --reps 3 --check 5000" \
  "ks_new|300|rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_new -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "ks_gather_all|300|KETO_EXPAND_GATHER_BIG=0 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_all -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "tests|400|python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_synth.py tests/test_gpu_configs_full.py -m gpu -k expand"
