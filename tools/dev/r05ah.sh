set -o pipefail
o=gpurun_out/r05ah; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for rep in 1 2; do
for v in main sp2 ; do
  if [ $v = main ]; then L=""; S=1; else L=keto_amd/variants/lib_sp4w.so; S=2; fi
  echo "== $v rep $rep $(date +%T)"
  KETO_LIB=$L KETO_EXPAND_SPREAD=$S timeout -k 10 200 python -u tools/dev/expand_prof.py --reps 8 --check 2000 > $o/${v}_$rep.log 2>&1 || { tail -20 $o/${v}_$rep.log; exit 1; }
  tail -2 $o/${v}_$rep.log
done
done
KETO_LIB=keto_amd/variants/lib_sp4w.so KETO_EXPAND_SPREAD=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks -o p -- python -u tools/dev/expand_prof.py --reps 10 > $o/ks.log 2>&1 || { tail -20 $o/ks.log; exit 1; }
cut -c1-150 $o/ks/p_kernel_stats.csv | grep "expand_kernel<2\|gather\|copy_lane" | head -5
