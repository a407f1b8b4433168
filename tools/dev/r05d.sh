set -o pipefail
o=gpurun_out/r05d; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== chain probe $(date +%T)"
timeout -k 10 300 python -u tools/dev/chain_probe.py --top 2 > $o/chain.log 2>&1 || { tail -20 $o/chain.log; exit 1; }
grep batch_without $o/chain.log | tail -3
echo "== deep parity + consumer $(date +%T)"
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_items.py tests/test_gpu_overflow.py tests/test_consumer_c.py -m gpu > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
