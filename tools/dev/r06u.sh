#!/bin/bash
# End-to-end streamed batch: request chunks over one copy stream or alternating over two.
o=gpurun_out/r06u
mkdir -p $o
bash tools/gpu_steps.sh r06u \
  "one_a|300|KETO_STREAM_COPY_STREAMS=1 python -u bench.py --e2e-only --e2e-steps 10" \
  "two_a|300|KETO_STREAM_COPY_STREAMS=2 python -u bench.py --e2e-only --e2e-steps 10" \
  "one_b|300|KETO_STREAM_COPY_STREAMS=1 python -u bench.py --e2e-only --e2e-steps 10" \
  "two_b|300|KETO_STREAM_COPY_STREAMS=2 python -u bench.py --e2e-only --e2e-steps 10"
