set -o pipefail
# Round-end check on one MI355X: the GPU test suite, smoke() and the bench
# line, product library only (bash tools/gpu_round_final.sh).
mkdir -p gpurun_out/r5final4
timeout -k 10 1100 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r5final4/tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5final4/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5final4/bench.json 2> gpurun_out/r5final4/bench.err
