#!/bin/bash
# Config #3 (nested groups, 100M tuples, 1M checks at depths 5/16/32): the deep tier's visited-table
# footprint.  Tier-0 tables of 64K (default) / 16K / 4K / 1K entries, with the deep budget as is and
# scaled down, in one process (decisions compared across all); then PMC passes (L2 read requests,
# fetch size, waits) for the default and the 4K-entry tables.
o=gpurun_out/r06b
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u tools/deep_sweep.py "" "KETO_T0_CAP=16384" "KETO_T0_CAP=4096" "KETO_T0_CAP=1024" \
  "KETO_T0_CAP=4096,KETO_DEEP_BUDGET_GB=16" "KETO_T0_CAP=1024,KETO_DEEP_BUDGET_GB=4" "" > $o/sweep.log 2> $o/sweep.err || { tail -20 $o/sweep.err; exit 1; }
cat $o/sweep.log
for c in default cap4k; do
  if [ $c = default ]; then combo=""; else combo="KETO_T0_CAP=4096"; fi
  i=0
  for grp in "TCC_EA0_RDREQ_sum FETCH_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $o/pmc_${c}_$i -o p -- python -u tools/deep_sweep.py "$combo" > $o/pmc_${c}_$i.log 2>&1 || { tail -20 $o/pmc_${c}_$i.log; exit 1; }
  done
done
echo done
