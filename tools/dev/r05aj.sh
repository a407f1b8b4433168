#!/bin/bash
# Writes under read load on the 1B graph with the writer-preferring snapshot lock: 1 and 4 reader threads.
set -e
o=gpurun_out/r05aj; mkdir -p $o
KETO_APPLY_TRACE=1 timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 8 --readers 4 > $o/apply_1b_r4.log 2> $o/apply_1b_r4.err
