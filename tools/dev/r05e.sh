set -o pipefail
o=gpurun_out/r05e; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in main ck_r0l16 ck_r4l8 ck_r0l8 ck_r0l16w6; do
  echo "== chain $v $(date +%T)"
  if [ $v = main ]; then L=""; else L=keto_amd/variants/lib_$v.so; fi
  KETO_LIB=$L timeout -k 10 300 python -u tools/dev/chain_probe.py --top 1 --reps 3 > $o/chain_$v.log 2>&1 || { tail -20 $o/chain_$v.log; exit 1; }
  tail -1 $o/chain_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['single'][0]['us_per_step_tier0'], {k: v['tier_ms'][0] for k, v in d.items() if k.startswith('batch')})"
done
echo "== config 5 $(date +%T)"
timeout -k 10 300 python -u tools/bench_configs.py --configs 5 > $o/config5.log 2>&1 || { tail -20 $o/config5.log; exit 1; }
tail -1 $o/config5.log | cut -c1-400
echo "== parity $(date +%T)"
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_items.py tests/test_gpu_parity.py tests/test_gpu_synth.py -m gpu > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
