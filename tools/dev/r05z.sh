set -o pipefail
o=gpurun_out/r05z; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for rep in 1 2; do
for v in main nq1w6 nq1w7 nq1w8; do
  if [ $v = main ]; then L=""; else L=keto_amd/variants/lib_$v.so; fi
  echo "== $v rep $rep $(date +%T)"
  KETO_LIB=$L timeout -k 10 300 python -u bench.py --no-work --no-cpu-baseline --e2e-steps 3 --string-steps 0 --steps 30 --warmup 5 > $o/b_${v}_$rep.log 2>&1 || { tail -20 $o/b_${v}_$rep.log; exit 1; }
  tail -1 $o/b_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value']/1e9, d['ms_per_step'], d['detail']['tier0_ms'], d['end_to_end']['value']/1e9, d['end_to_end']['ms_per_batch'])"
done
done
