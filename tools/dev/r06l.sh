#!/bin/bash
# Tier 0 A/B on one box: one request prefetch slot (KETO_NQ_SLOTS=1: 20 KB of LDS per block) at 6 and
# 7 waves per SIMD against the default (two slots, 24 KB, 6 waves); 16.7M checks on the 1B graph,
# interleaved, 2 reps.
o=gpurun_out/r06l
mkdir -p $o
for rep in 1 2; do
  for v in main nq1w6 nq1w7; do
    if [ $v = main ]; then L=""; else L="KETO_LIB=keto_amd/variants/lib_$v.so"; fi
    env $L timeout -k 10 300 python -u bench.py --no-work --no-cpu-baseline --e2e-steps 0 --string-steps 0 --steps 30 --warmup 5 > $o/b_${v}_$rep.log 2> $o/b_${v}_$rep.err || { tail -20 $o/b_${v}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$o/b_${v}_$rep.log').read().strip().splitlines()[-1]); print('$v', $rep, d['value'], d['detail']['tier0_ms'])"
  done
done
