# multi-rank tests (banded S all-reduce, multi-rank PCG), then the Cholesky kernel timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_multirank.py tests/test_gpu_parity.py > gpurun_out/mr.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chol_tl -o run -- python3 tools/chol_timeline.py > gpurun_out/chol_tl.log 2>&1 || exit 1
f=$(find gpurun_out/chol_tl -name "*kernel_trace.csv" | sort | tail -n 1)
python3 tools/chol_timeline.py --analyze "$f" > gpurun_out/chol_tl_summary.txt 2>&1
