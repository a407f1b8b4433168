#!/bin/bash
# PMC passes over the bench command (one counter group per rocprofv3 run; see MI355X guide slot table).
# Usage: bash tools/pmc_passes.sh <tag> [bench args...]
set -o pipefail
tag=${1:-pmc}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "== $(date +%T) pass $i: $grp"
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o p -- python -u bench.py --no-cpu-baseline --no-work "$@" > $out/p$i.log 2>&1 || { tail -20 $out/p$i.log; exit 1; }
done <<'GROUPS'
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_ACTIVE_INST_ANY
GROUPS
echo "== done"
