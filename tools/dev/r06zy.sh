#!/bin/bash
# A real wide arena: the power-law graph at 4x (4B tuples, ~73 GiB arena: root rows past 32 GiB in
# 32-B units) on one MI355X through bench.py -- the headline batch of 16,777,216 device-resident
# checks, 200,000 of them against the C restatement -- with host peak RSS (the box allows 270 GiB).
o=gpurun_out/r06zy
mkdir -p $o
export TMPDIR=/tmp
bash tools/gpu_steps.sh r06zy \
  "bench4b|900|python -u bench.py --scale 4.0 --steps 10 --warmup 5 --e2e-steps 0 --string-steps 0 --cpu-sample 200000 --sql-sample 0"
