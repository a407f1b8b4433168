#!/bin/bash
# The whole -m gpu suite on the current build (round-6 changes: version agreement, exclusive filter
# exchange, locked part / mig entry points, packed batches in flight, batched write images), then the
# 2-reader packed run with writes (KETO_APPLY_TRACE).
o=gpurun_out/r06f
mkdir -p $o
bash tools/gpu_steps.sh r06f \
  "pytest_gpu|1050|python -u -m pytest -x -q --timeout 900 --timeout-method thread tests -m gpu" \
  "s2_r2|120|KETO_APPLY_TRACE=1 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 2"
