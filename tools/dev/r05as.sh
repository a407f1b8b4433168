#!/bin/bash
# Packed batch latency at the Go batcher's flush size (65,536 requests) and at 1M, 1B graph, one
# reader, no writes worth noting (--seconds 2: the quiet half is what is read).
set -e
o=gpurun_out/r05as; mkdir -p $o
timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 2 --requests 65536 > $o/packed_65k.log 2> $o/packed_65k.err
timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 2 --requests 1000000 > $o/packed_1m.log 2> $o/packed_1m.err
