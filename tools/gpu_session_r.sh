# single-pass Jacobian slab as production: A/B, Jacobian parity tests, quick bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_jacobian.py --variants 0,2,4 > gpurun_out/ab_jac_r.jsonl 2> gpurun_out/ab_jac_r.err || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_mixed_models.py tests/test_gpu_scale.py > gpurun_out/r_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --lm-iters 0 --no-cpu-baseline > gpurun_out/r_bench.json 2> gpurun_out/r_bench.err || exit 1
timeout -k 10 500 python -u tools/ab_schur.py cholesky_own_diag=6,7 > gpurun_out/ab_own7.jsonl 2> gpurun_out/ab_own7.err
