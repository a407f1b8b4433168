set -o pipefail
o=gpurun_out/r05j; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for e in "" "KETO_REACH_WORK=2048" "KETO_REACH_WORK=1024" "KETO_REACH_WORK=512" "KETO_REACH_WAVE_SLOTS=2048" "KETO_REACH_MIN_DEPTH=24" "KETO_REACH_MIN_DEPTH=33"; do
  echo "== batch [$e] $(date +%T)"
  env $e timeout -k 10 200 python -u tools/dev/chain_probe.py --batch-only > $o/b.log 2>&1 || { tail -20 $o/b.log; exit 1; }
  tail -1 $o/b.log | tee -a $o/sweep.log
done
