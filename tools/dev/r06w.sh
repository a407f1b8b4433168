#!/bin/bash
# End-to-end streamed batch: request chunk size sweep (KETO_STREAM_CHUNK_LOG2; 2^20 pairs = 8 MB default).
o=gpurun_out/r06w
mkdir -p $o
bash tools/gpu_steps.sh r06w \
  "c20|300|KETO_STREAM_CHUNK_LOG2=20 python -u bench.py --e2e-only --e2e-steps 10" \
  "c21|300|KETO_STREAM_CHUNK_LOG2=21 python -u bench.py --e2e-only --e2e-steps 10" \
  "c22|300|KETO_STREAM_CHUNK_LOG2=22 python -u bench.py --e2e-only --e2e-steps 10" \
  "c23|300|KETO_STREAM_CHUNK_LOG2=23 python -u bench.py --e2e-only --e2e-steps 10" \
  "c19|300|KETO_STREAM_CHUNK_LOG2=19 python -u bench.py --e2e-only --e2e-steps 10"
