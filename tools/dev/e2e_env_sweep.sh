set -o pipefail
mkdir -p gpurun_out/r03h
for env in "X=0" "GPU_FORCE_BLIT_COPY_SIZE=0" "ROC_ENABLE_LARGE_BAR=0" "GPU_BLIT_ENGINE_TYPE=2"; do
  echo "== $env" >> gpurun_out/r03h/e2e_env.log
  env $env timeout -k 10 200 python -u tools/e2e_sweep.py --reps 5 --settings "KETO_CHUNK=4194304" >> gpurun_out/r03h/e2e_env.log 2>&1 || exit 1
done
