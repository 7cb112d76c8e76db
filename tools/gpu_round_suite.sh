set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5z
timeout -k 10 1100 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r5z/tests.log 2>&1
echo "tests rc $?"
tail -3 gpurun_out/r5z/tests.log
