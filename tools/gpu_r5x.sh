set -o pipefail
mkdir -p gpurun_out/r5af
timeout -k 10 1100 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r5af/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5af/bench.json 2> gpurun_out/r5af/bench.err
