# re-entry check of HEAD: full GPU tests, default bench (C4 + CPU baseline)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/h_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/h_bench.json 2> gpurun_out/h_bench.err || exit 1
