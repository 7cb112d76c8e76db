# camera-major Z fused into fblock_dense: LM parity tests, C4 LM phases
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_multirank.py tests/test_batch.py > gpurun_out/w_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/ab_schur.py schur_pairs_variant=0 > gpurun_out/ab_zcm.jsonl 2> gpurun_out/ab_zcm.err
