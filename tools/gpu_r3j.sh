#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "overlap or semantic" > gpurun_out/r3j_tests.log 2>&1
echo "tests rc $?"
tail -3 gpurun_out/r3j_tests.log
timeout -k 10 400 python -u tools/ab_overlap.py > gpurun_out/r3j_overlap.jsonl 2>&1 || { echo "overlap failed"; exit 1; }
cat gpurun_out/r3j_overlap.jsonl
timeout -k 10 400 python -u tools/ab_schur.py schur_block_images=2,4,8 > gpurun_out/r3j_block.jsonl 2>&1 || { echo "ab failed"; exit 1; }
cat gpurun_out/r3j_block.jsonl
timeout -s KILL 300 rocprofv3 --kernel-include-regex "Cijk|panel_factor|schur_pairs" --pmc GRBM_COUNT --output-format csv -d gpurun_out/r3j_clk -o run -- python3 tools/ab_cholesky.py 0 > gpurun_out/r3j_clk.log 2>&1 || { echo "clk failed"; exit 1; }
echo clk_done
