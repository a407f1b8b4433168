#!/bin/bash
# Kernel traces of config #5's expand under staging / run-queue settings given as arguments,
# e.g. "staged_ri0:KETO_EXPAND_STAGE=1,KETO_EXPAND_RUN_INLINE=0" (dev A/B).
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/exab
mkdir -p $out
for spec in "$@"; do
    tag=${spec%%:*}
    for kv in $(echo "${spec#*:}" | tr ',' ' '); do export "$kv"; done
    echo "== $tag ${spec#*:}"
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/$tag -o kt -- python -u tools/bench_configs.py --configs 5 --no-parity > $out/$tag.log 2>&1
done
