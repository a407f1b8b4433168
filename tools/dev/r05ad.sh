set -o pipefail
o=gpurun_out/r05ad; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== comm $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_migrate.py -m gpu > $o/pytest_comm.log 2>&1 || { tail -40 $o/pytest_comm.log; exit 1; }
tail -2 $o/pytest_comm.log
echo "== config 2 $(date +%T)"
timeout -k 10 200 python -u tools/bench_configs.py --configs 2 > $o/c2.log 2>&1 || { tail -20 $o/c2.log; exit 1; }
grep '^{' $o/c2.log | cut -c1-300
