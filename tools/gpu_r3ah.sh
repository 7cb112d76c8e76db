#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r3ah_tests.log 2>&1
echo "tests rc $?"
tail -1 gpurun_out/r3ah_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3ah_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r3ah_smoke.log; exit 1; }
tail -1 gpurun_out/r3ah_smoke.log
