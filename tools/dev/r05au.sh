#!/bin/bash
# Where a 65,536-request packed batch's ~0.34 ms goes: the lock / phase trace, and a kernel + copy trace.
set -e
o=gpurun_out/r05au; mkdir -p $o
KETO_TRACE_LOCKS=1 timeout -k 10 600 python -u tools/apply_concurrent.py --graph drive10m --packed --seconds 1 --requests 65536 > $o/trace_65k.log 2> $o/trace_65k.err
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/tr -o tr -- python -u tools/apply_concurrent.py --graph drive10m --packed --seconds 1 --requests 65536 > $o/tr.log 2>&1
