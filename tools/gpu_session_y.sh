# 2-rank rehearsal of bench.py's N>1 path on one GPU (gloo host reducer instead of RCCL)
set -o pipefail
mkdir -p gpurun_out
export MI_BA_BENCH_BACKEND=gloo
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/y_bench2.json 2> gpurun_out/y_bench2.err
