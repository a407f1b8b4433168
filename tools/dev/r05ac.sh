set -o pipefail
o=gpurun_out/r05ac; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== expand parity $(date +%T)"
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_synth.py tests/test_gpu_configs_full.py -m gpu -k "expand or config" > $o/pytest_exp.log 2>&1 || { tail -30 $o/pytest_exp.log; exit 1; }
tail -2 $o/pytest_exp.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks -o p -- python -u tools/dev/expand_prof.py --reps 10 --check 3000 > $o/ks.log 2>&1 || { tail -20 $o/ks.log; exit 1; }
tail -2 $o/ks.log
cut -c1-150 $o/ks/p_kernel_stats.csv | grep -v "closure_pass\|sig_pass\|scatter_unit\|rocclr" | head -10
