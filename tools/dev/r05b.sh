set -o pipefail
o=gpurun_out/r05b; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== prefix build under the deterministic test (expected to fail) $(date +%T)"
KETO_LIB=keto_amd/variants/lib_prefix_slack.so timeout -k 10 200 python -u -m pytest -v --timeout 100 --timeout-method thread tests/test_gpu_comm.py -k "never_read_stale" > $o/prefix.log 2>&1; echo "prefix exit $?"
grep -E "PASSED|FAILED|^E .*assert" $o/prefix.log | head -8
echo "== current build $(date +%T)"
timeout -k 10 200 python -u -m pytest -v --timeout 100 --timeout-method thread tests/test_gpu_comm.py -k "never_read_stale" > $o/current.log 2>&1 || { tail -30 $o/current.log; exit 1; }
tail -2 $o/current.log
echo "== config 2 A/B (w8 dispatch on / off) $(date +%T)"
for k in 1 2; do
  timeout -k 10 200 python -u tools/bench_configs.py --configs 2 --no-parity > $o/c2_w8_$k.log 2>&1 || { tail -20 $o/c2_w8_$k.log; exit 1; }
  KETO_T0_W8=0 timeout -k 10 200 python -u tools/bench_configs.py --configs 2 --no-parity > $o/c2_w6_$k.log 2>&1 || { tail -20 $o/c2_w6_$k.log; exit 1; }
done
grep -ho '"kernel_ms": [0-9.]*' $o/c2_*.log
echo "== chain probe $(date +%T)"
timeout -k 10 400 python -u tools/dev/chain_probe.py > $o/chain.log 2>&1 || { tail -20 $o/chain.log; exit 1; }
tail -1 $o/chain.log
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES"; do
  i=$((i+1))
  echo "== pmc pass $i $(date +%T)"
  timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d $o/p$i -o p -- python -u tools/dev/chain_probe.py --top 2 --reps 2 > $o/p$i.log 2>&1 || { tail -20 $o/p$i.log; exit 1; }
done
python tools/pmc_sum.py $o check_kernel > $o/pmc_check_kernel.txt; cat $o/pmc_check_kernel.txt | head -60
