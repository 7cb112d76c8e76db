# split panel launch (own_diag 8): Cholesky tests, C4 LM A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cholesky.py > gpurun_out/z_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/ab_schur.py cholesky_own_diag=6,8 cholesky_panel_rows=1,2 > gpurun_out/ab_own8.jsonl 2> gpurun_out/ab_own8.err
