set -o pipefail
o=gpurun_out/r05ai; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for rep in 1 2; do
for v in main ckw4 ckw6; do
  if [ $v = main ]; then L=""; else L=keto_amd/variants/lib_$v.so; fi
  echo "== $v rep $rep $(date +%T)"
  KETO_LIB=$L timeout -k 10 200 python -u tools/dev/chain_probe.py --batch-only > $o/${v}_$rep.log 2>&1 || { tail -20 $o/${v}_$rep.log; exit 1; }
  tail -1 $o/${v}_$rep.log | cut -c1-200
done
done
