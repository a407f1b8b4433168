#!/bin/bash
# Packed (string-form) batches: bounds check, undecided fold and wildcard count on the device instead
# of host loops over every record.  The device-resolution tests, then the bench's string-form leg.
set -e
o=gpurun_out/r05ap; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resolve_device.py tests/test_gpu_concurrency.py > $o/pytest_packed.log 2>&1
timeout -k 10 400 python -u bench.py > $o/bench.log 2>&1
