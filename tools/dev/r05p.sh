set -o pipefail
o=gpurun_out/r05p; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for sp in 1 2 4; do
  echo "== spread $sp $(date +%T)"
  KETO_EXPAND_SPREAD=$sp timeout -k 10 200 python -u tools/dev/expand_prof.py --reps 8 --check 3000 > $o/s$sp.log 2>&1 || { tail -20 $o/s$sp.log; exit 1; }
  tail -3 $o/s$sp.log
  KETO_EXPAND_SPREAD=$sp KETO_EXPAND_CLOCKS=1 timeout -k 10 200 python -u tools/dev/expand_prof.py --reps 2 > $o/c$sp.log 2>&1 || { tail -20 $o/c$sp.log; exit 1; }
  grep "expand clocks\] accesses\|walk us" $o/c$sp.log | tail -2
done
