set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5o
MI_BA_LIB=product timeout -k 10 500 python -u tools/ab_chol_keys.py "" "gemm_solution=-624952238" "" "gemm_solution=-624952238" "gemm_solution=-624952234" > gpurun_out/r5o/ab.log 2>&1
