set -o pipefail
o=gpurun_out/r05ag; mkdir -p $o
echo "== world 2 rehearsal (gloo, one GPU, 1/16 scale) $(date +%T)"
export KETO_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --scale 0.0625 --steps 5 --warmup 2 > $o/world2.log 2> $o/world2.err || { tail -30 $o/world2.err; exit 1; }
tail -1 $o/world2.log | cut -c1-600
