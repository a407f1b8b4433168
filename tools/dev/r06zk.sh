#!/bin/bash
# Final evidence of round 6: the bench's kernel-trace and PMC passes (traffic of this engine.hip),
# then configs #2, #3 and #5 through tools/bench_configs.py.
PROFILE_ONLY=1 bash tools/gpu_round.sh r06zj || exit $?
bash tools/gpu_steps.sh r06zj "configs|600|python -u tools/bench_configs.py --configs 2,3,5"
