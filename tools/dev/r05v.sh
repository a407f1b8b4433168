set -o pipefail
o=gpurun_out/r05v; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== pytest -m gpu -v $(date +%T)"
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $o/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc"
tail -3 $o/pytest_gpu.log
exit $rc
