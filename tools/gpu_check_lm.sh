set -o pipefail
# The LM / Cholesky / determinism GPU tests, then the LM kernel trace
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_lm_semantics.py tests/test_cholesky.py tests/test_determinism.py > gpurun_out/r5lm_tests.log 2>&1
