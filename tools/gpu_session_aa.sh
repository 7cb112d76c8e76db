# relaxed flag polling + one acquire fence: Cholesky tests, C4 LM phases
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cholesky.py > gpurun_out/aa_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/ab_schur.py cholesky_own_diag=6,2 > gpurun_out/ab_poll.jsonl 2> gpurun_out/ab_poll.err
