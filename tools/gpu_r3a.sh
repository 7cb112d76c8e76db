#!/bin/bash
# round 3 checkpoint: dgemm solution sweep, full GPU suite, default bench line, C4 linearization profile + LM kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 tools/probes/dgemm_solutions.bin > gpurun_out/r3a_dgemm_solutions.txt 2>&1
echo "dgemm sweep rc $?"
timeout -k 10 120 tools/probes/dgemm_probe.bin > gpurun_out/r3a_dgemm_probe.txt 2>&1
echo "dgemm probe rc $?"
cat gpurun_out/r3a_dgemm_probe.txt
timeout -k 10 300 python -u tools/ab_chol_keys.py "rest_update=3" "rest_update=4" > gpurun_out/r3a_ab_rest.jsonl 2>&1
echo "ab rest rc $?"
cat gpurun_out/r3a_ab_rest.jsonl
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r3a_tests.log 2>&1
echo "tests rc $?"
tail -3 gpurun_out/r3a_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err || { echo "bench failed"; exit 1; }
tail -c 600 gpurun_out/r3a_bench.json
timeout -k 10 900 bash tools/profile.sh gpurun_out/r3a_prof C4 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3a_lm -o run -- python3 bench.py --steps 2 --warmup 1 --lm-iters 3 --no-cpu-baseline > gpurun_out/r3a_lm.log 2>&1
echo "lm trace rc $?"
