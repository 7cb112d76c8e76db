set -o pipefail
mkdir -p gpurun_out/r5aa
export MI_BA_LIB=ab
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cholesky.py -k "handoff or factor_at_c4 or panel_kernel or lookahead_bitwise or not_positive" > gpurun_out/r5aa/tests.log 2>&1 &&
timeout -k 10 60 tools/probes/panel_probe.bin 12000 3 1 0 3 > gpurun_out/r5aa/probe_fv3_wm3.txt 2>&1 &&
timeout -k 10 60 tools/probes/panel_probe.bin 12000 3 1 1 3 > gpurun_out/r5aa/probe_fv3_wm3_busy.txt 2>&1 &&
timeout -k 10 60 tools/probes/panel_probe.bin 4096 3 1 0 2 > gpurun_out/r5aa/probe_4096_wm2.txt 2>&1 &&
timeout -k 10 60 tools/probes/panel_probe.bin 4096 3 1 0 3 > gpurun_out/r5aa/probe_4096_wm3.txt 2>&1 &&
timeout -k 10 600 python -u tools/ab_chol_keys.py "" "panel_wait=3" "" "panel_wait=3" > gpurun_out/r5aa/ab.jsonl 2> gpurun_out/r5aa/ab.err
