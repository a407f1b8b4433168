#!/bin/bash
# Where a 16.7M-request packed (string-form) batch spends its 21 ms: kernels and copies traced.
set -e
o=gpurun_out/r05aq; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $o/tr -o tr -- python -u bench.py --no-work --steps 2 --warmup 1 --e2e-steps 0 --string-steps 3 > $o/tr.log 2>&1
