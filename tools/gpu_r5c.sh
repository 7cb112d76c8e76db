set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5c
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_facade.py -x \
  > gpurun_out/r5c/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5c/bench.log 2>&1
