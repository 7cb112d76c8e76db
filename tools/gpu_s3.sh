#!/bin/bash
# Cholesky timeline at nf = 12 000 under the default factorisation
set -o pipefail
mkdir -p gpurun_out/tl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 tools/chol_timeline.py 6 > gpurun_out/tl_run.txt 2>&1 &&
python3 tools/chol_timeline.py --analyze $(find gpurun_out/tl -name '*kernel_trace.csv' | head -1) --seq > gpurun_out/chol_timeline.txt 2>&1
