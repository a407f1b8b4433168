#!/bin/bash
# Expand config #5: a leaf-level union's set children walked a 4-edge group per trip (expand_sm,
# KETO_EXPAND_LEAF4) against one edge per trip (a KETO_EXPAND_LEAF4=0 build), kernel stats of both,
# trees checked against the oracle, then the expand parity suites.
o=gpurun_out/r06zi
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06zi \
  "check|240|python -u tools/dev/expand_prof.py --reps 3 --check 5000" \
  "ks_leaf4|200|rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_leaf4 -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "ks_off|200|KETO_LIB=keto_amd/variants/lib_leaf4off.so rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_off -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "tests|400|python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_synth.py tests/test_gpu_configs_full.py tests/test_gpu_arena_split.py -m gpu -k expand"
