set -o pipefail
o=gpurun_out/r05x; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== concurrent packed + writes loop $(date +%T)"
timeout -k 10 400 python -u tools/dev/hang_loop.py tests.test_gpu_resolve_device:test_packed_batches_concurrent_with_writes --n 25 --limit 40 > $o/loop.log 2> $o/trace.log; rc=$?; echo "rc=$rc"
tail -3 $o/loop.log
tail -c 100000 $o/trace.log > $o/trace_tail.log; rm -f $o/trace.log
[ $rc -eq 0 ] || exit 1
echo "== concurrency + lifecycle + replicas + resolve $(date +%T)"
timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_concurrency.py tests/test_gpu_lifecycle.py tests/test_gpu_replicas.py tests/test_gpu_resolve_device.py tests/test_gpu_host_api.py -m gpu > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
