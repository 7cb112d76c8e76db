#!/bin/bash
# rocprofv3 kernel trace + separate PMC passes of the C4 linearization.
# Usage: bash tools/profile.sh <outdir> [config]
set -e
OUT=${1:-gpurun_out/prof}
CFG=${2:-C4}
export TMPDIR=/tmp
mkdir -p "$OUT"
ARGS="bench.py --config $CFG --steps 20 --warmup 30 --lm-iters 0 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 $ARGS > "$OUT/pmc_write.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/pmc_sq" -o run -- python3 $ARGS > "$OUT/pmc_sq.log" 2>&1
echo profile_done
