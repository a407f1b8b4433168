set -o pipefail
o=gpurun_out/r05u; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== parity+partition+replicas $(date +%T)"
timeout -k 10 1000 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_partition.py tests/test_gpu_replicas.py -m gpu > $o/p.log 2>&1; echo "rc=$?"
grep -c PASSED $o/p.log; grep -v PASSED $o/p.log | tail -60
