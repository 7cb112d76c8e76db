set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5b
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_facade.py \
  -s > gpurun_out/r5b/tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5b/bench.log 2>&1
