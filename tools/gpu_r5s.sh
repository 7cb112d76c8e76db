set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5s
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_determinism.py tests/test_cholesky.py tests/test_comm.py > gpurun_out/r5s/tests.log 2>&1
