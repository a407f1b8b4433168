set -o pipefail
o=gpurun_out/r05g; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== items parity on the deep wave kernel $(date +%T)"
KETO_DEEP_WAVE=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_items.py -m gpu > $o/pytest_dw.log 2>&1 || { tail -30 $o/pytest_dw.log; exit 1; }
tail -2 $o/pytest_dw.log
for dw in 0 1; do
  echo "== chain deep_wave=$dw $(date +%T)"
  KETO_DEEP_WAVE=$dw timeout -k 10 300 python -u tools/dev/chain_probe.py --top 1 --reps 3 > $o/chain_dw$dw.log 2>&1 || { tail -20 $o/chain_dw$dw.log; exit 1; }
  tail -1 $o/chain_dw$dw.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($dw, d['single'][0]['us_per_step_tier0'], {k: (v['tier_ms'][0], v['items_ms']) for k, v in d.items() if k.startswith('batch')})"
done
echo "== config 3 deep wave $(date +%T)"
KETO_DEEP_WAVE=1 timeout -k 10 300 python -u tools/bench_configs.py --configs 3 > $o/config3_dw.log 2>&1 || { tail -20 $o/config3_dw.log; exit 1; }
tail -1 $o/config3_dw.log | cut -c1-700
