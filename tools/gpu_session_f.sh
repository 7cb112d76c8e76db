# semantic kernel restructure: parity tests + A/B timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "semantic" > gpurun_out/sem_par.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_semantic.py --rounds 3 > gpurun_out/ab_sem2.log 2>&1
