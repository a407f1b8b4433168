set -o pipefail
o=gpurun_out/r05s; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== pytest -m gpu $(date +%T)"
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
tail -3 $o/pytest_gpu.log
