#!/bin/bash
# Expand config #5: the copy kernels' grid cap (KETO_EXPAND_COPY_BLOCKS, default 16384) at 1024 / 2048 /
# 4096 blocks -- kernel stats of each (the copies are dispatch- and latency-bound).
o=gpurun_out/r06zf
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06zf \
  "ks_1024|200|KETO_EXPAND_COPY_BLOCKS=1024 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_1024 -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "ks_2048|200|KETO_EXPAND_COPY_BLOCKS=2048 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_2048 -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "ks_4096|200|KETO_EXPAND_COPY_BLOCKS=4096 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_4096 -o p -- python -u tools/dev/expand_prof.py --reps 10" \
  "ks_default|200|rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_def -o p -- python -u tools/dev/expand_prof.py --reps 10"
