set -o pipefail
cd $GRAFT_REPO_ROOT
export MI_BA_LIB=product
timeout -k 10 900 bash tools/pmc_lm.sh gpurun_out/r5j_pmclm "schur_pairs_kernel"
