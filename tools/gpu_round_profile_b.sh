set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MI_BA_LIB=product
mkdir -p gpurun_out/r5fin
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5fin/lm -o run -- python3 bench.py --steps 2 --warmup 1 --lm-iters 3 --no-cpu-baseline > gpurun_out/r5fin/lm.log 2>&1 || exit 1
echo "lm trace done"
timeout -k 10 900 bash tools/pmc_semantic.sh gpurun_out/r5fin/pmcs || exit 1
