# final check of HEAD: full GPU tests, default bench, smoke
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/f2_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/f2_bench.json 2> gpurun_out/f2_bench.err || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f2_smoke.log 2>&1
