#!/bin/bash
# PMC passes over the LM's explicit Schur build and Cholesky kernels at C4
# (tools/ab_cholesky.py, production variant).  Usage: bash tools/pmc_lm.sh <outdir> <kernel regex>
OUT=${1:-gpurun_out/pmclm}
RE=${2:-schur_pairs}
export TMPDIR=/tmp
mkdir -p "$OUT"
ARGS="tools/ab_cholesky.py 0"
run() { timeout -s KILL 300 rocprofv3 --kernel-include-regex "$RE" --pmc $2 --output-format csv -d "$OUT/$1" -o run -- python3 $ARGS > "$OUT/$1.log" 2>&1; }
run tcc "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" &&
run fetch "FETCH_SIZE" &&
run sq "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F64" &&
run tcp "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" &&
echo pmc_done
