set -o pipefail
o=gpurun_out/r05t; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== replicas $(date +%T)"
timeout -k 10 170 python -u -m pytest -x -v --timeout 100 --timeout-method thread "tests/test_gpu_replicas.py::test_replicas_follow_writes[22]" "tests/test_gpu_replicas.py::test_replicas_follow_writes[21]" > $o/rep.log 2>&1; echo "rc=$?"
tail -80 $o/rep.log
