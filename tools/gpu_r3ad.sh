#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_scale.py -k "chunks or iterative" > gpurun_out/r3ad_tests.log 2>&1
echo "tests rc $?"
tail -1 gpurun_out/r3ad_tests.log
