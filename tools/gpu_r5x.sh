set -o pipefail
mkdir -p gpurun_out/r5z
timeout -k 10 1100 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r5z/tests.log 2>&1 &&
MI_BA_LIB=ab timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cholesky.py > gpurun_out/r5z/tests_chol_ab.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5z/bench.json 2> gpurun_out/r5z/bench.err
