set -e
export KETO_BENCH_BACKEND=gloo
timeout -k 10 300 python -u bench.py --partitioned --part-mode migrate --scale 0.03125 --batch 1048576 --steps 3 --warmup 1 --check-parity > gpurun_out/r02ap_mig_world1.log 2> gpurun_out/r02ap_mig_world1.err
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --partitioned --part-mode migrate --hot-mb 20 --scale 0.03125 --batch 1048576 --steps 3 --warmup 1 --check-parity > gpurun_out/r02ap_mig_world2.log 2> gpurun_out/r02ap_mig_world2.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --partitioned --scale 0.03125 --batch 1048576 --steps 3 --warmup 1 --check-parity > gpurun_out/r02ap_shared_world2.log 2> gpurun_out/r02ap_shared_world2.err
