#!/bin/bash
# GPU suite + LM phase timings at C4 (tools/ab_schur.py grid from the arguments, e.g. fblock_variant=0,1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/lmchk_tests.log 2>&1
echo "tests rc $?"
tail -3 gpurun_out/lmchk_tests.log
timeout -k 10 400 python -u tools/ab_schur.py "$@" > gpurun_out/lmchk_lm.jsonl 2>&1 || { echo "lm failed"; exit 1; }
cat gpurun_out/lmchk_lm.jsonl
if [ -n "$AB2" ]; then
  timeout -k 10 400 python -u tools/ab_schur.py $AB2 > gpurun_out/lmchk_lm2.jsonl 2>&1 || { echo "lm2 failed"; exit 1; }
  cat gpurun_out/lmchk_lm2.jsonl
fi
