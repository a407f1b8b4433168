set -o pipefail
o=gpurun_out/r05h; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== stream tests $(date +%T)"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_stream.py -m gpu > $o/pytest_stream.log 2>&1 || { tail -30 $o/pytest_stream.log; exit 1; }
tail -2 $o/pytest_stream.log
echo "== writes under packed reads on the 1B graph $(date +%T)"
KETO_APPLY_TRACE=1 timeout -k 10 600 python -u tools/apply_concurrent.py --graph powerlaw1b --packed --seconds 8 > $o/apply_1b.log 2> $o/apply_1b.err || { tail -20 $o/apply_1b.err; exit 1; }
tail -1 $o/apply_1b.log
python tools/dev/apply_trace_sum.py $o/apply_1b.err | tee $o/apply_1b_trace.json
