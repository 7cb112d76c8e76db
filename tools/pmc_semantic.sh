#!/bin/bash
# PMC passes over the semantic linearization kernel alone (tools/ab_semantic.py, C4):
# instruction mix (FP64 op counts for the FP64 roofline), issue/wait, HBM bytes.
# Usage: bash tools/pmc_semantic.sh <outdir>
OUT=${1:-gpurun_out/pmcs}
export TMPDIR=/tmp
# variant 6 is the product default: the product library (no A/B build needed)
export MI_BA_LIB=product
mkdir -p "$OUT"
ARGS="tools/ab_semantic.py --rounds 1 --reps 2 --variants 6"
run() { timeout -s KILL 180 rocprofv3 --kernel-include-regex 'semantic_(linearize|flat|deferred)' --pmc $2 --output-format csv -d "$OUT/$1" -o run -- python3 $ARGS > "$OUT/$1.log" 2>&1; }
run f64 "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD" &&
run sq "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" &&
run fetch "FETCH_SIZE" &&
run write "WRITE_SIZE" &&
run tcc "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" &&
echo pmc_done
