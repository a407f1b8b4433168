#!/bin/bash
# End-to-end streamed batch: tier 0 reading the requests straight from mapped host memory
# (KETO_STREAM_ZERO_COPY=1) against the chunked copies; a small run first.
o=gpurun_out/r06x
mkdir -p $o
bash tools/gpu_steps.sh r06x \
  "zc_small|200|KETO_STREAM_ZERO_COPY=1 python -u bench.py --e2e-only --e2e-steps 3 --scale 0.0625 --batch 2097152" \
  "copy_a|300|python -u bench.py --e2e-only --e2e-steps 10" \
  "zc_a|300|KETO_STREAM_ZERO_COPY=1 python -u bench.py --e2e-only --e2e-steps 10" \
  "copy_b|300|python -u bench.py --e2e-only --e2e-steps 10" \
  "zc_b|300|KETO_STREAM_ZERO_COPY=1 python -u bench.py --e2e-only --e2e-steps 10"
