#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r3aa_tests.log 2>&1
echo "tests rc $?"
tail -1 gpurun_out/r3aa_tests.log
timeout -k 10 500 python -u tools/ab_schur.py cholesky_panel_cus=0,64,128,192,32 > gpurun_out/r3aa_cus.jsonl 2>&1 || { echo "cus ab failed"; tail -5 gpurun_out/r3aa_cus.jsonl; exit 1; }
cat gpurun_out/r3aa_cus.jsonl
