#!/bin/bash
# Cholesky panel session: tile + panel probes, Cholesky tests, C4 A/B of the tile factor
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/probes/tile_probe.bin > gpurun_out/tile_probe.txt 2>&1 &&
timeout -k 10 60 tools/probes/panel_probe.bin 12000 2 1 > gpurun_out/panel_probe.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cholesky.py tests/test_callbacks.py -m gpu > gpurun_out/test_chol.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_chol_keys.py "tile_factor=2" "tile_factor=1" "write_through=0" > gpurun_out/ab_tile.jsonl 2>&1
