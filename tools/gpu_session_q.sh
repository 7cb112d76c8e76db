# measurement with the closed-form Jacobian: A/B of the Jacobian layout variants, full GPU tests, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_jacobian.py --variants 0,1,4,24,25,26,27,30,31,35 > gpurun_out/ab_jac_q.jsonl 2> gpurun_out/ab_jac_q.err || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/q_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || exit 1
