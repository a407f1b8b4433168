#!/bin/bash
# Packed batches: blob and records uploaded side by side; tests, the 2- and 4-reader 65,536-request
# runs on the 1B graph, then the default bench line (new device_row_ids leg).
o=gpurun_out/r06g
mkdir -p $o
bash tools/gpu_steps.sh r06g \
  "pytest|300|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_resolve_device.py -m gpu" \
  "s2_r2|120|python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 2" \
  "s4_r4|120|KETO_PACKED_SLOTS=4 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 4 --requests 65536 --readers 4" \
  "bench|400|python -u bench.py"
