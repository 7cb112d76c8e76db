set -o pipefail
mkdir -p gpurun_out/r5ac
timeout -k 10 60 tools/probes/panel_probe.bin 12000 3 1 0 2 > gpurun_out/r5ac/probe_fv3_wm2.txt 2>&1 &&
timeout -k 10 60 tools/probes/panel_probe.bin 12000 3 1 0 0 > gpurun_out/r5ac/probe_fv3_wm0.txt 2>&1 &&
MI_BA_LIB=ab timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cholesky.py > gpurun_out/r5ac/tests_chol_ab.log 2>&1
