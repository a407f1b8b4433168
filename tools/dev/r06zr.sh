#!/bin/bash
# Tier 0's bound by footprint (the line waste): the bench's 16.7M-check batch on
# the power-law graph at 1, 1/16 and 1/128 scale (the last inside the 256 MB Infinity Cache) on one
# box, back to back -- what removing every HBM line could save at most.
o=gpurun_out/r06zr
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06zr \
  "s1|300|python -u bench.py --no-work --e2e-steps 0 --string-steps 0 --scale 1.0" \
  "s16|200|python -u bench.py --no-work --e2e-steps 0 --string-steps 0 --scale 0.0625" \
  "s128|200|python -u bench.py --no-work --e2e-steps 0 --string-steps 0 --scale 0.0078125" \
  "s1b|300|python -u bench.py --no-work --e2e-steps 0 --string-steps 0 --scale 1.0"
