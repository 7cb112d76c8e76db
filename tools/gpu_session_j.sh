# batched semantic stencil as default: GPU parity tests (all), semantic A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/j_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_semantic.py --variants 4,3,1 > gpurun_out/ab_sem_j.jsonl 2> gpurun_out/ab_sem_j.err
