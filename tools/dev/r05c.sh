set -o pipefail
o=gpurun_out/r05c; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== chain probe $(date +%T)"
timeout -k 10 300 python -u tools/dev/chain_probe.py --top 2 > $o/chain.log 2>&1 || { tail -20 $o/chain.log; exit 1; }
tail -1 $o/chain.log
echo "== config 3 $(date +%T)"
timeout -k 10 400 python -u tools/bench_configs.py --configs 3 > $o/config3.log 2>&1 || { tail -20 $o/config3.log; exit 1; }
tail -1 $o/config3.log | cut -c1-600
echo "== deep parity $(date +%T)"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_items.py tests/test_gpu_overflow.py tests/test_gpu_consumer_c.py tests/test_consumer_c.py -m gpu > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
