#!/bin/bash
# One GPU session of measurements / tests; steps chained, each under its own limit.
set -o pipefail
T=${1:-r4a}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/test_comm.py} > gpurun_out/$T/comm_tests.log 2>&1
rc=$?; echo "comm tests rc $rc"
tail -3 gpurun_out/$T/comm_tests.log
# test failures (1) do not stop the session; a crash, abort or timeout does
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/ab_jacobian.py --step --variants 0,11,12 --rounds 5 --reps 5 > gpurun_out/$T/ab_step.jsonl 2> gpurun_out/$T/ab_step.err || exit 1
timeout -k 10 300 python -u tools/ab_jacobian.py --variants 0,11,12 --rounds 5 --reps 5 > gpurun_out/$T/ab_b2b.jsonl 2> gpurun_out/$T/ab_b2b.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/bench_trace -o run -- python3 bench.py --lm-iters 0 --no-cpu-baseline > gpurun_out/$T/bench_trace.log 2>&1 || exit 1
echo done
