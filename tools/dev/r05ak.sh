#!/bin/bash
# First-write stall fix (Chunked string table, per-row tables grown before the exclusive lock):
# writes of new subject ids, then writes that add rows, 4 reader threads, the 1B graph.
set -e
o=gpurun_out/r05ak; mkdir -p $o
KETO_APPLY_TRACE=1 timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 8 --readers 4 > $o/apply_1b_r4.log 2> $o/apply_1b_r4.err
KETO_APPLY_TRACE=1 timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 8 --readers 4 --new-rows > $o/apply_1b_r4_rows.log 2> $o/apply_1b_r4_rows.err
