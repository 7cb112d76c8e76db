#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SOLVER=iterative timeout -k 10 400 python -u tools/ab_schur.py > gpurun_out/r3y_pcg.jsonl 2>&1 || { echo "pcg failed"; exit 1; }
cat gpurun_out/r3y_pcg.jsonl
AB_SOLVER=iterative timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3y_trace -o run -- python3 tools/ab_schur.py > gpurun_out/r3y_trace.log 2>&1
echo "trace rc $?"
