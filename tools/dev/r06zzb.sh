#!/bin/bash
# Tier 0 built with compiler scheduling / CFG flags (engine.hip only, tools/dev/build_flag_variant.py):
# sur = -structurizecfg-skip-uniform-regions, ilp = -amdgpu-sched-strategy=max-ilp,
# mcl = -amdgpu-sched-strategy=max-memory-clause; alternating with the default build on one box,
# then the parity suite on the CFG variant.
export TMPDIR=/tmp
B="python -u bench.py --no-work --e2e-steps 0 --string-steps 0"
L="KETO_LIB=keto_amd/variants/lib_"
bash tools/gpu_steps.sh r06zzb \
  "base1|240|$B" "sur1|240|${L}sur.so $B" "ilp1|240|${L}ilp.so $B" "mcl1|240|${L}mcl.so $B" \
  "base2|240|$B" "sur2|240|${L}sur.so $B" "ilp2|240|${L}ilp.so $B" "mcl2|240|${L}mcl.so $B" \
  "parity_sur|300|${L}sur.so python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_synth.py -m gpu"
