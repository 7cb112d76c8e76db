# Cholesky tests (incl. one-launch panel factor), LM parity suite, then the C4 A/B of own_diag 2 vs 6
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_cholesky.py > gpurun_out/chol6.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_multirank.py tests/test_gpu_scale.py > gpurun_out/parity_b.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_schur.py cholesky_own_diag=2,6 > gpurun_out/ab_own6.jsonl 2> gpurun_out/ab_own6.err
