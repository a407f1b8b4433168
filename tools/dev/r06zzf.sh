#!/bin/bash
# The in-tree library with migrate.hip also scheduled for memory clauses (keto_amd/build.py
# SOURCE_FLAGS): smoke, the parity / synth / comm / migrate suites and config #4's full-scale parts.
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
bash tools/gpu_steps.sh r06zzf \
  "smoke|180|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "suites|400|$T tests/test_gpu_parity.py tests/test_gpu_synth.py tests/test_gpu_comm.py tests/test_gpu_migrate.py" \
  "parts|420|$T --durations=5 tests/test_gpu_config4_parts.py"
