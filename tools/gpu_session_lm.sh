# kernel trace of the C4 exact-Schur LM (3 iterations, production settings)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lm -o run -- python3 tools/ab_schur.py cholesky_own_diag=6 > gpurun_out/prof_lm.log 2>&1
