set -o pipefail
o=gpurun_out/r05k; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== migrating writes + migrate + comm $(date +%T)"
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_migrate.py -m gpu > $o/pytest_mig.log 2>&1 || { tail -30 $o/pytest_mig.log; exit 1; }
tail -2 $o/pytest_mig.log
echo "== config 5 $(date +%T)"
timeout -k 10 300 python -u tools/bench_configs.py --configs 5 > $o/config5.log 2>&1 || { tail -20 $o/config5.log; exit 1; }
tail -1 $o/config5.log | cut -c1-500
echo "== config 3 $(date +%T)"
timeout -k 10 200 python -u tools/dev/chain_probe.py --batch-only > $o/c3.log 2>&1 || { tail -20 $o/c3.log; exit 1; }
tail -1 $o/c3.log
echo "== parity $(date +%T)"
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_items.py tests/test_gpu_parity.py tests/test_gpu_synth.py -m gpu > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
