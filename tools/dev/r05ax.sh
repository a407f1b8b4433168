#!/bin/bash
# Packed pipeline piece size: 2^21 (default) against 2^19 and 2^20, on 1M-request batches (1B graph,
# apply_concurrent quiet phase) and on the bench's 16.7M string-form leg.
set -e
o=gpurun_out/r05ax; mkdir -p $o
for c in 2097152 1048576 524288; do
  KETO_PACKED_CHUNK=$c timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 2 --requests 1000000 > $o/packed_1m_$c.log 2> $o/packed_1m_$c.err
done
for c in 2097152 524288; do
  KETO_PACKED_CHUNK=$c timeout -k 10 400 python -u bench.py --no-work --steps 2 --warmup 1 --e2e-steps 0 --string-steps 3 > $o/bench_$c.log 2>&1
done
