set -o pipefail
export RSGPU_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 3 --no-cpu > gpurun_out/b_2rank.json 2> gpurun_out/b_2rank.err || { tail -30 gpurun_out/b_2rank.err; exit 1; }
cat gpurun_out/b_2rank.json | head -c 1500
