#!/bin/bash
# Per-step clocks of resolve_packed (KETO_RESOLVE_CLOCKS) on 65,536-request packed batches, 1B graph
# and drive10m: when lanes start, their record load, row query and subject lookup (us).
set -e
o=gpurun_out/r05ba; mkdir -p $o
KETO_RESOLVE_CLOCKS=1 timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 1 --requests 65536 > $o/clk_1b.log 2> $o/clk_1b.err
KETO_RESOLVE_CLOCKS=1 timeout -k 10 600 python -u tools/apply_concurrent.py --graph drive10m --packed --seconds 1 --requests 65536 > $o/clk_10m.log 2> $o/clk_10m.err
