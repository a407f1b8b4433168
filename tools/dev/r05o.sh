set -o pipefail
o=gpurun_out/r05o; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for k in 0 2 4; do
  echo "== scale $k $(date +%T)"
  timeout -k 10 200 python -u tools/dev/expand_prof.py --reps 6 --scale $k > $o/s$k.log 2>&1 || { tail -20 $o/s$k.log; exit 1; }
  tail -2 $o/s$k.log
  KETO_EXPAND_CLOCKS=1 timeout -k 10 200 python -u tools/dev/expand_prof.py --reps 2 --scale $k > $o/c$k.log 2>&1 || { tail -20 $o/c$k.log; exit 1; }
  grep "expand clocks\] accesses\|walk us" $o/c$k.log | tail -2
done
