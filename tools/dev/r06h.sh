#!/bin/bash
# End-to-end leg (pinned 8-B pairs H2D -> check -> D2H, one streamed launch): which copy engine the
# runtime uses.  The box's HSA / HIP environment, then --e2e-only under SDMA settings.
o=gpurun_out/r06h
mkdir -p $o
env | grep -iE "^(HSA|HIP|GPU_|ROC|AMD_)" | sort > $o/env.txt
cat $o/env.txt
for v in default sdma1 sdma0; do
  case $v in
    default) e="";;
    sdma1) e="HSA_ENABLE_SDMA=1";;
    sdma0) e="HSA_ENABLE_SDMA=0";;
  esac
  env $e timeout -k 10 200 python -u bench.py --e2e-only --e2e-steps 5 --string-steps 0 > $o/e2e_$v.log 2> $o/e2e_$v.err || { tail -20 $o/e2e_$v.err; exit 1; }
  echo "== $v"; cut -c1-700 $o/e2e_$v.log
done
