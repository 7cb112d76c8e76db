# blocked panel factor: probe, Cholesky tests, C4 A/B own_diag 2 vs 6
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/panel_probe.bin > gpurun_out/panel_probe3.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_cholesky.py > gpurun_out/chol6d.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_schur.py cholesky_own_diag=2,6 > gpurun_out/ab_own6d.jsonl 2> gpurun_out/ab_own6d.err
