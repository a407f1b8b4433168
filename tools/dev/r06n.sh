#!/bin/bash
# The whole -m gpu suite with durations (routed packed, consumer partition packed, in-flight packed),
# then smoke, then 1M-request packed batches in flight on the 1B graph.
o=gpurun_out/r06n
mkdir -p $o
bash tools/gpu_steps.sh r06n \
  "pytest_gpu|1000|python -u -m pytest -x -q --timeout 900 --timeout-method thread --durations=40 tests -m gpu" \
  "smoke|180|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "packed_1m|150|python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 1048576 --readers 2"
