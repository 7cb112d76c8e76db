set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5f
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5f/lm -o run -- python3 bench.py --steps 2 --warmup 1 --lm-iters 3 --no-cpu-baseline > gpurun_out/r5f/lm.log 2>&1
