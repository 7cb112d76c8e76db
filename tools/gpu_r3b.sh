#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/probes/panel_probe.bin 12000 2 1 0 > gpurun_out/r3b_panel_alone.txt 2>&1; echo "probe rc $?"
timeout -k 10 60 tools/probes/panel_probe.bin 12000 2 1 1 > gpurun_out/r3b_panel_busy.txt 2>&1; echo "probe busy rc $?"
grep "rep 2" gpurun_out/r3b_panel_alone.txt gpurun_out/r3b_panel_busy.txt
awk '/rep 2/{g=1} g' gpurun_out/r3b_panel_busy.txt | head -12
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cholesky.py -m gpu -k "schur_pair_orders" > gpurun_out/r3b_t.txt 2>&1; echo "test rc $?"; tail -2 gpurun_out/r3b_t.txt
timeout -k 10 400 python -u tools/ab_schur.py schur_pairs_variant=0,4 schur_block_images=16,32,64 > gpurun_out/r3b_ab_schur.jsonl 2>&1
echo "ab rc $?"
cat gpurun_out/r3b_ab_schur.jsonl
