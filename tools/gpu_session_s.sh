# round-2 measurement of HEAD: full GPU tests, default bench (C4 + CPU baseline),
# rocprofv3 kernel trace + PMC passes, semantic PMC passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/s_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err || exit 1
timeout -k 10 900 bash tools/profile.sh gpurun_out/prof_s C4 > gpurun_out/prof_s.log 2>&1 || exit 1
bash tools/pmc_semantic.sh gpurun_out/pmcs_s > gpurun_out/pmcs_s.log 2>&1
