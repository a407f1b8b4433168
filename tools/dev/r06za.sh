#!/bin/bash
# Config #3's deep tier 0 with its lanes spread over every resident wave (fewer lanes per wave)
# against 64 lanes per wave (KETO_DEEP_SPREAD=0), in one process (decisions compared), then the
# items / deep parity suites.
o=gpurun_out/r06za
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u tools/deep_sweep.py "" "KETO_DEEP_SPREAD=0" "" "KETO_DEEP_SPREAD=0" > $o/sweep.log 2> $o/sweep.err || { tail -20 $o/sweep.err; exit 1; }
cat $o/sweep.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_items.py tests/test_gpu_configs_full.py -m gpu > $o/pytest.log 2>&1; rc=$?
tail -3 $o/pytest.log
exit $rc
