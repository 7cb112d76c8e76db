#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over tools/ab_jacobian.py,
# for diagnosing the Jacobian kernel's memory pipeline.
# Usage: bash tools/pmc_jac.sh <outdir> <variants>
set -e
OUT=${1:-gpurun_out/pmcj}
VAR=${2:-0,10}
export TMPDIR=/tmp
mkdir -p "$OUT"
ARGS="tools/ab_jacobian.py --variants $VAR --rounds 1 --reps 2"
n=0
while read -r grp; do
  [ -z "$grp" ] && continue
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$n" -o run -- python3 $ARGS > "$OUT/pmc$n.log" 2>&1
done <<'GROUPS'
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum
TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_STALL_sum
TCC_REQ_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_BUSY_sum
TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
GRBM_GUI_ACTIVE GRBM_TA_BUSY SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64
GROUPS
echo pmc_done
