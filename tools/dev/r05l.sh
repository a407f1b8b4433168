set -o pipefail
o=gpurun_out/r05l; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== expand trace $(date +%T)"
KETO_EXPAND_TRACE=1 timeout -k 10 240 python -u tools/dev/expand_prof.py --reps 5 > $o/trace.log 2>&1 || { tail -20 $o/trace.log; exit 1; }
tail -12 $o/trace.log
echo "== expand kernel stats $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks -o p -- python -u tools/dev/expand_prof.py --reps 10 > $o/ks.log 2>&1 || { tail -20 $o/ks.log; exit 1; }
f=$(ls $o/ks/*/p_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(ls $o/ks/p_kernel_stats.csv); cut -c1-200 $f | head -20
