#!/bin/bash
# Run GPU steps one after another on the box, each under its own time limit, its output in
# gpurun_out/<tag>/<name>.log.  A step that fails its tests (exit 1) lets the next one run; a step
# that times out, aborts or crashes (any other non-zero status) ends the script there.
# Usage: bash tools/gpu_steps.sh <tag> "<name>|<seconds>|<command>" ...
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
worst=0
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}
  secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $(date +%T) $name ($secs s)"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  tail -4 "$out/$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping: $name ended with status $rc"
    exit $rc
  fi
  [ $rc -ne 0 ] && worst=$rc
done
exit $worst
