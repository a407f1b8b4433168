set -o pipefail
o=gpurun_out/r05i; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for k in 1 2; do
for v in main ck_pf; do
  if [ $v = main ]; then L=""; else L=keto_amd/variants/lib_$v.so; fi
  echo "== chain $v #$k $(date +%T)"
  KETO_REACH_TRACE=1 KETO_LIB=$L timeout -k 10 300 python -u tools/dev/chain_probe.py --top 1 --reps 3 > $o/chain_${v}_$k.log 2>&1 || { tail -20 $o/chain_${v}_$k.log; exit 1; }
  tail -1 $o/chain_${v}_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['single'][0]['us_per_step_tier0'], {k: (v['tier_ms'][0], v['items_ms']) for k, v in d.items() if k.startswith('batch')})"
done
done
grep "^reach:" $o/chain_main_1.log | tail -3
echo "== pf parity $(date +%T)"
KETO_LIB=keto_amd/variants/lib_ck_pf.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_items.py tests/test_gpu_overflow.py -m gpu > $o/pytest_pf.log 2>&1 || { tail -30 $o/pytest_pf.log; exit 1; }
tail -2 $o/pytest_pf.log
echo "== writes under packed reads on the 1B graph $(date +%T)"
KETO_APPLY_TRACE=1 timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 8 > $o/apply_1b.log 2> $o/apply_1b.err || { tail -20 $o/apply_1b.err; exit 1; }
tail -1 $o/apply_1b.log
python tools/dev/apply_trace_sum.py $o/apply_1b.err | tee $o/apply_1b_trace.json
echo "== lifecycle parity $(date +%T)"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lifecycle.py tests/test_gpu_comm.py -k "lifecycle or follow_writes or collisions or wildcard or stale" -m gpu > $o/pytest_life.log 2>&1 || { tail -30 $o/pytest_life.log; exit 1; }
tail -2 $o/pytest_life.log
