#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r3i_tests.log 2>&1
echo "tests rc $?"
tail -3 gpurun_out/r3i_tests.log
timeout -k 10 400 python -u tools/ab_overlap.py > gpurun_out/r3i_overlap.jsonl 2>&1 || { echo "overlap failed"; exit 1; }
cat gpurun_out/r3i_overlap.jsonl
timeout -k 10 500 python -u tools/ab_schur.py schur_block_images=8,16,32,64,128 > gpurun_out/r3i_block.jsonl 2>&1 || { echo "ab failed"; exit 1; }
cat gpurun_out/r3i_block.jsonl
timeout -k 10 600 python -u tools/ab_schur.py cholesky_panel_rows_per_group=1,2,4 cholesky_panel_group_min_rows=3000,7000 > gpurun_out/r3i_groups.jsonl 2>&1 || { echo "ab groups failed"; exit 1; }
cat gpurun_out/r3i_groups.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3i_gsba_span -o run -- python3 tools/bench_gsba.py 40 12 1080 1920 > gpurun_out/r3i_gsba_span.json 2>gpurun_out/r3i_gsba_span.err || { echo "gsba span failed"; exit 1; }
MI_BA_LIB=ab MI_BA_GSBA_VARIANT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3i_gsba_pixel -o run -- python3 tools/bench_gsba.py 40 12 1080 1920 > gpurun_out/r3i_gsba_pixel.json 2>gpurun_out/r3i_gsba_pixel.err || { echo "gsba pixel failed"; exit 1; }
echo gsba_done
