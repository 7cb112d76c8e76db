set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5m
MI_BA_LIB=ab timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread -m gpu tests/test_cholesky.py::test_lm_schur_pair_orders > gpurun_out/r5m/test.log 2>&1 &&
timeout -k 10 700 python -u tools/ab_schur.py schur_pairs_variant=4,8,9,6,4,8,9 > gpurun_out/r5m/ab.log 2>&1
