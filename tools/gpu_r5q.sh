set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5q
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -k "semantic or flat or label" tests > gpurun_out/r5q/tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5q/trace -o run -- python3 bench.py --steps 10 --warmup 2 --lm-iters 0 --no-cpu-baseline > gpurun_out/r5q/trace.log 2>&1 &&
timeout -k 10 400 python -u tools/semantic_regime_counts.py > gpurun_out/r5q/regimes.log 2>&1
