# round 3 session 1: tile probe, full GPU suite with the new tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/probes/tile_probe.bin > gpurun_out/s1_tile_probe.txt 2>&1 || echo "tile probe rc $?"
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/s1_tests.log 2>&1
echo "tests rc $?"
tail -5 gpurun_out/s1_tests.log
