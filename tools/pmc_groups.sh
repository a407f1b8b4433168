#!/bin/bash
# PMC passes with caller-chosen counter groups over any command (one rocprofv3 run per group).
# Usage: bash tools/pmc_groups.sh <tag> "<group1>" "<group2>" ... -- <command...>
set -o pipefail
tag=$1; shift
groups=()
while [ "$1" != "--" ]; do groups+=("$1"); shift; done
shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  echo "== $(date +%T) pass $i: $grp"
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o p -- "$@" > $out/p$i.log 2>&1 || { tail -20 $out/p$i.log; exit 1; }
done
echo "== done"
