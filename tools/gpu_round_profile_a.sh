set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MI_BA_LIB=product
mkdir -p gpurun_out/r5fin
timeout -k 10 600 python -u bench.py > gpurun_out/r5fin/bench.json 2> gpurun_out/r5fin/bench.err || { echo "bench failed"; exit 1; }
tail -c 300 gpurun_out/r5fin/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5fin/bench_trace -o run -- python3 bench.py > gpurun_out/r5fin/bench_trace.log 2>&1 || { echo "bench trace failed"; exit 1; }
timeout -k 10 900 bash tools/profile.sh gpurun_out/r5fin/prof C4 || exit 1
