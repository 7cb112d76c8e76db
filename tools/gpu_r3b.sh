#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/probes/panel_probe.bin 12000 2 1 0 > gpurun_out/r3b_panel_alone.txt 2>&1; echo "probe rc $?"
timeout -k 10 60 tools/probes/panel_probe.bin 12000 2 1 1 > gpurun_out/r3b_panel_busy.txt 2>&1; echo "probe busy rc $?"
grep "rep 2" gpurun_out/r3b_panel_alone.txt gpurun_out/r3b_panel_busy.txt
awk '/rep 2/{g=1} g' gpurun_out/r3b_panel_busy.txt | head -12
