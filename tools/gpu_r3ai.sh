#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r3ai_tests.log 2>&1
echo "tests rc $?"
tail -1 gpurun_out/r3ai_tests.log
timeout -k 10 300 python -u tools/ab_schur.py > gpurun_out/r3ai_lm.jsonl 2>&1 || { echo "lm failed"; exit 1; }
timeout -k 10 300 python -u tools/ab_schur.py >> gpurun_out/r3ai_lm.jsonl 2>&1 || { echo "lm failed"; exit 1; }
cat gpurun_out/r3ai_lm.jsonl
