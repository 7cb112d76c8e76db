set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mixed_models.py tests/test_facade.py tests/test_gpu_parity.py > gpurun_out/mixed.log 2>&1
