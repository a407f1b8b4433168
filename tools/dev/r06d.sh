#!/bin/bash
# Kernel + copy trace of 65,536-request packed batches in flight (4 readers, 4 slots) on the 1B graph.
o=gpurun_out/r06d
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
KETO_PACKED_SLOTS=4 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $o/tr -o t -- python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 1 --requests 65536 --readers 4 > $o/run.log 2>&1 || { tail -20 $o/run.log; exit 1; }
ls -la $o/tr/*/ 2>/dev/null | head; ls -laR $o/tr | head -20
