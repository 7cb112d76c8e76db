#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
AB_SOLVER=iterative timeout -k 10 500 python -u tools/ab_schur.py pcg_jcm=2,3,2,3 > gpurun_out/r3ag_jcm_fill.jsonl 2>&1 || { echo "ab failed"; tail -5 gpurun_out/r3ag_jcm_fill.jsonl; exit 1; }
cat gpurun_out/r3ag_jcm_fill.jsonl
