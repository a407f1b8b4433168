set -o pipefail
o=gpurun_out/r05q; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== migrating expand $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_comm.py -m gpu -k "migrating or expand" > $o/pytest_mig.log 2>&1 || { tail -40 $o/pytest_mig.log; exit 1; }
tail -2 $o/pytest_mig.log
echo "== expand parity + synth $(date +%T)"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_synth.py tests/test_gpu_configs_full.py -m gpu -k "expand or config" > $o/pytest_exp.log 2>&1 || { tail -30 $o/pytest_exp.log; exit 1; }
tail -2 $o/pytest_exp.log
echo "== config 5 $(date +%T)"
timeout -k 10 300 python -u tools/bench_configs.py --configs 5 > $o/config5.log 2>&1 || { tail -20 $o/config5.log; exit 1; }
grep '^{' $o/config5.log | cut -c1-300
