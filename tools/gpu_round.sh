#!/bin/bash
# One GPU-box pass: gpu parity tests, smoke, bench, rocprofv3 kernel-trace stats, PMC traffic passes.
# Usage (from the repo root on the box): bash tools/gpu_round.sh <tag> [bench args...]
# (the trace and PMC passes skip the end-to-end leg, so every traced tier-0 launch is a full batch;
# PROFILE_ONLY=1 runs just those passes, SKIP_PROFILE=1 everything but them)
set -o pipefail
tag=${1:-run}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { echo "== $(date +%T) $1"; }
if [ -z "$PROFILE_ONLY" ]; then
step pytest
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread --durations=30 > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
step smoke
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -30 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
step bench
timeout -k 10 400 python -u bench.py "$@" > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log
fi
[ -n "$SKIP_PROFILE" ] && { step done; exit 0; }
step kernel-trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python -u bench.py --no-work --e2e-steps 0 --string-steps 0 "$@" > $out/kt.log 2>&1 || { tail -30 $out/kt.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  step "pmc $c"
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $out/pmc_$c -o pmc -- python -u bench.py --no-work --e2e-steps 0 --string-steps 0 "$@" > $out/pmc_$c.log 2>&1 || { tail -30 $out/pmc_$c.log; exit 1; }
done
step done
