#!/bin/bash
# GPU checkpoint: full GPU suite + default bench line, counter list, in-step vs back-to-back Jacobian PMC
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/chk_tests.log 2>&1
echo "tests rc $?"
tail -3 gpurun_out/chk_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/chk_bench.json 2> gpurun_out/chk_bench.err || { echo "bench failed"; exit 1; }
tail -c 300 gpurun_out/chk_bench.json
timeout -k 10 60 rocprofv3 -L > gpurun_out/chk_counters.txt 2>&1; echo "list rc $?"
timeout -k 10 300 python -u tools/jac_context.py b2b 10 > gpurun_out/chk_jac_b2b.json 2>&1 && timeout -k 10 300 python -u tools/jac_context.py step 10 > gpurun_out/chk_jac_step.json 2>&1 || exit 1
cat gpurun_out/chk_jac_b2b.json gpurun_out/chk_jac_step.json
timeout -k 10 900 bash tools/pmc_jac_context.sh gpurun_out/chk_pmcctx || exit 1
