#!/bin/bash
# Tier 0 compiled with SimplifyCFG's phi-node folding thresholds raised (more branches as selects:
# -mllvm -two-entry-phi-node-folding-threshold=128 -phi-node-folding-threshold=64, a variant
# library) against the default build, alternating on one box; the parity suite on the variant.
o=gpurun_out/r06zs
mkdir -p $o
export TMPDIR=/tmp
B="python -u bench.py --no-work --e2e-steps 0 --string-steps 0"
V="KETO_LIB=keto_amd/variants/lib_phi2.so"
bash tools/gpu_steps.sh r06zs \
  "base1|240|$B" "phi1|240|$V $B" "base2|240|$B" "phi2|240|$V $B" \
  "parity|300|$V python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_synth.py -m gpu"
