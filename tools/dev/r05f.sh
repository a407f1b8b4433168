set -o pipefail
o=gpurun_out/r05f; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== stream tests $(date +%T)"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_stream.py -m gpu > $o/pytest_stream.log 2>&1 || { tail -30 $o/pytest_stream.log; exit 1; }
tail -2 $o/pytest_stream.log
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1)); echo "== expand pmc $i $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $o/e$i -o p -- python -u tools/dev/expand_prof.py --reps 3 > $o/e$i.log 2>&1 || { tail -20 $o/e$i.log; exit 1; }
done
mkdir -p $o/exp && cp -r $o/e1 $o/exp/p1 && cp -r $o/e2 $o/exp/p2 && cp -r $o/e3 $o/exp/p3 && cp -r $o/e4 $o/exp/p4
python tools/pmc_sum.py $o/exp expand > $o/expand_pmc.txt; cat $o/expand_pmc.txt | grep -v "^$" | head -40
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH" "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS"; do
  i=$((i+1)); echo "== tier-0 pmc $i $(date +%T)"
  timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d $o/t$i -o p -- python -u bench.py --no-work --no-cpu-baseline --e2e-steps 0 --string-steps 0 --steps 5 --warmup 2 > $o/t$i.log 2>&1 || { tail -20 $o/t$i.log; exit 1; }
done
mkdir -p $o/t0 && cp -r $o/t1 $o/t0/p1 && cp -r $o/t2 $o/t0/p2
python tools/pmc_sum.py $o/t0 check_wave_kernel 16777216 > $o/tier0_pmc.txt; cat $o/tier0_pmc.txt
