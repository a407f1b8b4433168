#!/bin/bash
# Wide arenas (past 64 GiB): the arena split tests over the narrow 48 GiB layout and the wide 48 GiB
# (128-B units), ~80 GiB (32-B units) and ~112 GiB (64-B units) layouts, then the lifecycle suite.
bash tools/gpu_steps.sh r06z \
  "arena|700|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_arena_split.py -m gpu --durations=20" \
  "lifecycle|400|python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_lifecycle.py -m gpu"
