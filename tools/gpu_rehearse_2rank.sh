#!/bin/bash
# 2-rank rehearsal of bench.py's N>1 path on ONE GPU (both ranks on device 0,
# the LM's reductions through the gloo host reducer instead of RCCL, which
# needs one GPU per rank): strong scaling (C5 = C4 point-sharded), iterative
# LM.  Usage: bash tools/gpu_rehearse_2rank.sh <tag>
set -o pipefail
T=${1:-rehearse}
mkdir -p gpurun_out
export MI_BA_BENCH_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --lm-iters 3 --no-cpu-baseline \
  > gpurun_out/${T}_2rank.json 2> gpurun_out/${T}_2rank.err || { echo "2-rank failed"; tail -20 gpurun_out/${T}_2rank.err; exit 1; }
grep '^{' gpurun_out/${T}_2rank.json | tail -c 1500
