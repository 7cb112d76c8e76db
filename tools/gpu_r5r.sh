set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5r
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gsba.py tests/test_determinism.py > gpurun_out/r5r/tests.log 2>&1
