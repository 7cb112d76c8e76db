# panel factor rows-per-workgroup A/B: probes, Cholesky tests, C4 LM A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/panel_probe.bin 12000 1 > gpurun_out/panel_probe_r1.txt 2>&1 || exit 1
timeout -k 10 60 ./tools/panel_probe.bin 12000 2 > gpurun_out/panel_probe_r2.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_cholesky.py > gpurun_out/chol6d.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/ab_schur.py cholesky_panel_rows=1,2,4 > gpurun_out/ab_rows.jsonl 2> gpurun_out/ab_rows.err
