set -o pipefail
# Kernel trace of a 3-iteration C4 LM solve (bench.py), for the idle-gap count
export TMPDIR=/tmp MI_BA_LIB=product
mkdir -p gpurun_out/r5lm2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5lm2/lm -o run -- python3 bench.py --steps 2 --warmup 1 --lm-iters 3 --no-cpu-baseline > gpurun_out/r5lm2/lm.log 2>&1
