#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r3af_tests.log 2>&1
echo "tests rc $?"
tail -3 gpurun_out/r3af_tests.log
timeout -k 10 300 python -u tools/ab_schur.py > gpurun_out/r3af_lm.jsonl 2>&1 || { echo "lm failed"; exit 1; }
cat gpurun_out/r3af_lm.jsonl
AB_SOLVER=iterative timeout -k 10 400 python -u tools/ab_schur.py > gpurun_out/r3af_pcg.jsonl 2>&1 || { echo "pcg failed"; exit 1; }
cat gpurun_out/r3af_pcg.jsonl
AB_SOLVER=iterative timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3af_trace -o run -- python3 tools/ab_schur.py > gpurun_out/r3af_trace.log 2>&1
echo "trace rc $?"
