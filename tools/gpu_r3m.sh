#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cholesky.py > gpurun_out/r3m_tests.log 2>&1
echo "tests rc $?"
tail -3 gpurun_out/r3m_tests.log
timeout -k 10 600 python -u bench.py --lm-iters 3 > gpurun_out/r3m_bench.json 2> gpurun_out/r3m_bench.err || { echo "bench failed"; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r3m_bench.json'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value']/1e9, d['ms_per_step'], d['kernels_ms'], d['ba_iteration_ms'])
"
timeout -k 10 500 python -u tools/ab_schur.py schur_pairs_variant=4,5 cholesky_bwd_pairs=1,0 > gpurun_out/r3m_order.jsonl 2>&1 || { echo "ab failed"; exit 1; }
cat gpurun_out/r3m_order.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3m_trace -o run -- python3 bench.py --steps 10 --warmup 2 --lm-iters 0 --no-cpu-baseline > gpurun_out/r3m_trace.log 2>&1
echo "trace rc $?"
