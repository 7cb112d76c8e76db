#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r3n_tests.log 2>&1
echo "tests rc $?"
tail -3 gpurun_out/r3n_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3n_bench.json 2> gpurun_out/r3n_bench.err || { echo "bench failed"; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r3n_bench.json'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value']/1e9, d['ms_per_step'], d['kernels_ms'], d['ba_iteration_ms'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n_trace -o run -- python3 bench.py --steps 10 --warmup 2 --lm-iters 0 --no-cpu-baseline > gpurun_out/r3n_trace.log 2>&1
echo "trace rc $?"
timeout -k 10 700 bash tools/gpu_rehearse_2rank.sh r3n || exit 1
