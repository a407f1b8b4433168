set -o pipefail
tag=r05ae
o=gpurun_out/$tag; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== pytest -m gpu $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { grep -v PASSED $o/pytest_gpu.log | tail -40; exit 1; }
tail -1 $o/pytest_gpu.log
echo "== smoke $(date +%T)"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -30 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
