# Two ranks at full scale (1B tuples each) sharing the box's one GPU over gloo: the per-rank host
# resources (peak RSS, CPU seconds) of the driver's multi-GPU run, which every rank pays alike.
set -o pipefail
mkdir -p gpurun_out/r03f
export KETO_BENCH_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --no-work --e2e-steps 2 --steps 5 --warmup 2 \
  > gpurun_out/r03f/world2_full.log 2> gpurun_out/r03f/world2_full.err
