#!/bin/bash
# PMC passes over the reproj_jacobian kernel alone (tools/ab_jacobian.py, C4).
# Usage: bash tools/pmc_jacobian.sh <outdir> [variant]
OUT=${1:-gpurun_out/pmcj}
V=${2:-0}
export TMPDIR=/tmp
mkdir -p "$OUT"
ARGS="tools/ab_jacobian.py --variants $V --rounds 1 --reps 3"
run() { timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o run -- python3 $ARGS > "$OUT/$1.log" 2>&1; }
run sqa "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" &&
run sqb "SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM" &&
run tc "TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES TCC_EA0_WRREQ_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL GRBM_GUI_ACTIVE GRBM_COUNT" &&
echo pmc_done
