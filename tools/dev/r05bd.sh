#!/bin/bash
# Kernel + copy timeline of 65,536-request packed batches on the 1B graph (where the 0.34 ms goes).
set -e
o=gpurun_out/r05bd; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/tr -o tr -- python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 1 --requests 65536 > $o/tr.log 2>&1
