#!/bin/bash
# Lock timeline of row-adding writes under 4 readers (1B graph): where a batch after an insert waits.
set -e
o=gpurun_out/r05am; mkdir -p $o
KETO_TRACE_LOCKS=1 KETO_APPLY_TRACE=1 timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 3 --readers 4 --new-rows > $o/apply_rows.log 2> $o/apply_rows.err
