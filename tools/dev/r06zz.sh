#!/bin/bash
# Tier 0 with T's closure-filter word/bit hashed once per request and kept in a register
# (KETO_T0_TCW=1, a variant library) against the default build, alternating on one box; the
# parity suite on the variant.
o=gpurun_out/r06zz
mkdir -p $o
export TMPDIR=/tmp
B="python -u bench.py --no-work --e2e-steps 0 --string-steps 0"
V="KETO_LIB=keto_amd/variants/lib_tcw.so"
bash tools/gpu_steps.sh r06zz \
  "base1|240|$B" "tcw1|240|$V $B" "base2|240|$B" "tcw2|240|$V $B" \
  "parity|300|$V python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_synth.py -m gpu"
