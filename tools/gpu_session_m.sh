# measurement after the semantic two-pass default: full GPU tests, bench (C4 + CPU baseline),
# rocprofv3 kernel trace + PMC passes, semantic PMC
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/m_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/m_bench.json 2> gpurun_out/m_bench.err || exit 1
timeout -k 10 900 bash tools/profile.sh gpurun_out/prof_m C4 > gpurun_out/prof_m.log 2>&1 || exit 1
bash tools/pmc_semantic.sh gpurun_out/pmcs_m > gpurun_out/pmcs_m.log 2>&1
