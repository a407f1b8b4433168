set -o pipefail
tag=r05af
o=gpurun_out/$tag; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== bench $(date +%T)"
timeout -k 10 420 python -u bench.py > $o/bench.log 2>&1 || { tail -30 $o/bench.log; exit 1; }
tail -1 $o/bench.log | cut -c1-300
PROFILE_ONLY=1 bash tools/gpu_round.sh $tag
