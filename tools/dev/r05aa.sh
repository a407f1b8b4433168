set -o pipefail
o=gpurun_out/r05aa; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for rep in 1 2; do
for v in default s262144 s1048576 s2097152 w6; do
  case $v in default) E="";; w6) E="KETO_T0_W8=0";; s*) E="KETO_SLOTS=${v#s}";; esac
  echo "== $v rep $rep $(date +%T)"
  env $E timeout -k 10 200 python -u tools/bench_configs.py --configs 2 --no-parity > $o/c2_${v}_$rep.log 2>&1 || { tail -20 $o/c2_${v}_$rep.log; exit 1; }
  grep '^{' $o/c2_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['gpu']['tier_ms'], d['gpu']['wall_ms'])"
done
done
