#!/bin/bash
# Packed path without the misrouted-row readback on unpartitioned snapshots: the full gpu round
# (tests, smoke, bench, kernel trace, PMC passes), then the 65,536-request packed latency (r05as 0.34 ms).
set -e
bash tools/gpu_round.sh r05bc
o=gpurun_out/r05bc
timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 2 --requests 65536 > $o/packed_65k.log 2> $o/packed_65k.err
