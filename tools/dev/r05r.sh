set -o pipefail
o=gpurun_out/r05r; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1)); echo "== config3 pmc $i $(date +%T)"
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $o/c$i -o p -- python -u tools/bench_configs.py --configs 3 --no-parity > $o/c$i.log 2>&1 || { tail -20 $o/c$i.log; exit 1; }
done
mkdir -p $o/all && for j in 1 2 3 4; do cp -r $o/c$j $o/all/p$j; done
python tools/pmc_sum.py $o/all check_kernel > $o/c3_pmc.txt; cat $o/c3_pmc.txt
python tools/pmc_sum.py $o/all pretest > $o/c3_pretest_pmc.txt; head -20 $o/c3_pretest_pmc.txt
