#!/bin/bash
# Round measurement of HEAD: GPU suite, default bench line, C4 linearization
# trace + PMC (tools/profile.sh), LM kernel trace, Schur-pair PMC passes
# (tools/pmc_lm.sh), semantic-kernel PMC passes (tools/pmc_semantic.sh).
# Usage: bash tools/gpu_profile_round.sh <tag>
set -o pipefail
T=${1:-r3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/${T}_tests.log 2>&1
echo "tests rc $?"
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; exit 1; }
tail -c 400 gpurun_out/${T}_bench.json
timeout -k 10 900 bash tools/profile.sh gpurun_out/${T}_prof C4 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_lm -o run -- python3 bench.py --steps 2 --warmup 1 --lm-iters 3 --no-cpu-baseline > gpurun_out/${T}_lm.log 2>&1 || exit 1
echo "lm trace done"
timeout -k 10 900 bash tools/pmc_lm.sh gpurun_out/${T}_pmclm schur_pairs || exit 1
timeout -k 10 900 bash tools/pmc_semantic.sh gpurun_out/${T}_pmcs || exit 1
