#!/bin/bash
# The reachability index without root rows (targets only, exact): the items / deep suites, the
# arena-split suite (deep checks on split and wide arenas now take the pretest), then config #3 with
# the new index against KETO_REACH_ROOTS=1 (roots too, as before) in one process.
o=gpurun_out/r06zt
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06zt \
  "items|500|python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_items.py tests/test_gpu_configs_full.py tests/test_gpu_arena_split.py -m gpu" \
  "config3|400|python -u tools/deep_sweep.py '' 'KETO_REACH_ROOTS=1' '' 'KETO_REACH_ROOTS=1'"
