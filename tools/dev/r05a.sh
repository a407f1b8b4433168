set -o pipefail
o=gpurun_out/r05a; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== probe $(date +%T)"
timeout -k 10 240 ./tools/dev/latency_probe > $o/probe.log 2>&1 || { echo probe failed; tail $o/probe.log; exit 1; }
echo "== tests $(date +%T)"
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_comm.py -k "never_read_stale or follow_writes or expand_error_agreement" tests/test_gpu_resolve_device.py > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
echo "== pre-fix build under the new test (expected to fail) $(date +%T)"
KETO_LIB=keto_amd/variants/lib_prefix_slack.so timeout -k 10 200 python -u -m pytest -v --timeout 100 --timeout-method thread tests/test_gpu_comm.py -k "never_read_stale" > $o/prefix.log 2>&1; echo "prefix exit $?"
grep -E "PASS|FAIL|Error|assert" $o/prefix.log | head -20
echo "== config 2 $(date +%T)"
timeout -k 10 300 python -u tools/bench_configs.py --configs 2 > $o/config2.log 2>&1 || { tail -30 $o/config2.log; exit 1; }
tail -5 $o/config2.log
