# Cholesky tests (lower-triangle-only input), own_diag 6 at C4, semantic-kernel PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_cholesky.py tests/test_pba_reference.py > gpurun_out/chol6c.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_schur.py cholesky_own_diag=6 > gpurun_out/ab_own6c.jsonl 2> gpurun_out/ab_own6c.err || exit 1
bash tools/pmc_semantic.sh gpurun_out/pmcs > gpurun_out/pmcs.log 2>&1
