set -o pipefail
o=gpurun_out/r05m; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== probe busy $(date +%T)"
timeout -k 10 300 tools/dev/latency_probe busy > $o/probe_busy.log 2>&1 || { tail -20 $o/probe_busy.log; exit 1; }
cat $o/probe_busy.log
for v in "" 64; do
  echo "== expand contig='$v' $(date +%T)"
  KETO_CONTIG_MIB=$v timeout -k 10 240 python -u tools/dev/expand_prof.py --reps 8 --check 2000 > $o/exp_$v.log 2>&1 || { tail -20 $o/exp_$v.log; exit 1; }
  tail -4 $o/exp_$v.log
  echo "== chain contig='$v' $(date +%T)"
  KETO_CONTIG_MIB=$v timeout -k 10 200 python -u tools/dev/chain_probe.py --batch-only > $o/c3_$v.log 2>&1 || { tail -20 $o/c3_$v.log; exit 1; }
  tail -1 $o/c3_$v.log
done
echo "== expand kernel stats $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks -o p -- python -u tools/dev/expand_prof.py --reps 10 > $o/ks.log 2>&1 || { tail -20 $o/ks.log; exit 1; }
cut -c1-200 $o/ks/p_kernel_stats.csv | head -16
for v in "" 64; do
  echo "== tier0 contig='$v' $(date +%T)"
  KETO_CONTIG_MIB=$v timeout -k 10 400 python -u bench.py --no-work --no-cpu-baseline --e2e-steps 0 --string-steps 0 --steps 20 --warmup 3 > $o/t0_$v.log 2>&1 || { tail -20 $o/t0_$v.log; exit 1; }
  tail -1 $o/t0_$v.log | cut -c1-400
done
