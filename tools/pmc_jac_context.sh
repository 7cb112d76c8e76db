#!/bin/bash
# PMC passes of reproj_jacobian back-to-back vs inside the linearization step (C4).
# Usage: bash tools/pmc_jac_context.sh <outdir>
OUT=${1:-gpurun_out/pmcctx}
export TMPDIR=/tmp
mkdir -p "$OUT"
run() { timeout -s KILL 150 rocprofv3 --pmc $3 --output-format csv -d "$OUT/$1_$2" -o run -- python3 tools/jac_context.py $2 6 > "$OUT/$1_$2.log" 2>&1; }
for m in b2b step; do
  run time $m "GRBM_GUI_ACTIVE GRBM_COUNT" &&
  run wr $m "TCC_EA0_WRREQ_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL TA_DATA_STALLED_BY_TC_CYCLES TA_TA_BUSY" &&
  run sq $m "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_VMEM_WR_TA_DATA_FIFO_FULL" || exit 1
done
echo pmc_ctx_done
