set -o pipefail
o=gpurun_out/r05ab; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== expand parity $(date +%T)"
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_synth.py tests/test_gpu_configs_full.py tests/test_gpu_lifecycle.py -m gpu -k "expand or config or lifecycle or writes" > $o/pytest_exp.log 2>&1 || { tail -30 $o/pytest_exp.log; exit 1; }
tail -2 $o/pytest_exp.log
echo "== comm expand $(date +%T)"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_comm.py tests/test_consumer_c.py -m gpu -k "expand or migrating or parts" > $o/pytest_comm.log 2>&1 || { tail -30 $o/pytest_comm.log; exit 1; }
tail -2 $o/pytest_comm.log
echo "== expand prof $(date +%T)"
KETO_EXPAND_TRACE=1 timeout -k 10 240 python -u tools/dev/expand_prof.py --reps 6 --check 5000 > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
tail -3 $o/trace.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks -o p -- python -u tools/dev/expand_prof.py --reps 10 > $o/ks.log 2>&1 || { tail -20 $o/ks.log; exit 1; }
cut -c1-180 $o/ks/p_kernel_stats.csv | grep -v "closure_pass\|sig_pass\|scatter_unit" | head -14
echo "== configs 2,5 $(date +%T)"
timeout -k 10 400 python -u tools/bench_configs.py --configs 2,5 > $o/configs.log 2>&1 || { tail -20 $o/configs.log; exit 1; }
grep '^{' $o/configs.log | cut -c1-400
