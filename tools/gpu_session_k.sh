# semantic flat test (variant 5) A/B + parity tests (semantic variants, batch, parity)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_semantic.py --variants 6,4,1 > gpurun_out/ab_sem_k.jsonl 2> gpurun_out/ab_sem_k.err || exit 1
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_batch.py > gpurun_out/k_tests.log 2>&1
