set -o pipefail
o=gpurun_out/r05w; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== concurrent packed + writes loop $(date +%T)"
timeout -k 10 600 python -u tools/dev/hang_loop.py tests.test_gpu_resolve_device:test_packed_batches_concurrent_with_writes --n 25 --limit 40 > $o/loop.log 2> $o/trace.log; echo "rc=$?"
tail -5 $o/loop.log
tail -c 200000 $o/trace.log > $o/trace_tail.log; rm -f $o/trace.log
tail -40 $o/trace_tail.log
