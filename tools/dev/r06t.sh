#!/bin/bash
# After the migrating-round and failing-page changes: the whole -m gpu suite, smoke, and the bench.
o=gpurun_out/r06t
mkdir -p $o
bash tools/gpu_steps.sh r06t \
  "pytest_gpu|1000|python -u -m pytest -x -q --timeout 900 --timeout-method thread --durations=30 tests -m gpu" \
  "smoke|180|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|400|python -u bench.py"
