#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_pcg_constants.py > gpurun_out/r3ac_diag.jsonl 2>&1 || { echo "diag failed"; tail -5 gpurun_out/r3ac_diag.jsonl; exit 1; }
MI_BA_LIB=ab timeout -k 10 300 python -u tools/diag_pcg_constants.py >> gpurun_out/r3ac_diag.jsonl 2>&1 || { echo "diag ab failed"; tail -5 gpurun_out/r3ac_diag.jsonl; exit 1; }
cat gpurun_out/r3ac_diag.jsonl
