#!/bin/bash
# Final engine evidence: the default bench line, then the rocprofv3 kernel-trace summary of the bench
# command and the FETCH_SIZE / WRITE_SIZE PMC passes (tools/traffic.py turns them into the profiles/
# files bench.py's roofline.traffic reads for this engine.hip).
o=gpurun_out/r06m
mkdir -p $o
timeout -k 10 400 python -u bench.py > $o/bench.log 2>&1 || { tail -30 $o/bench.log; exit 1; }
tail -1 $o/bench.log | cut -c1-400
PROFILE_ONLY=1 bash tools/gpu_round.sh r06m
