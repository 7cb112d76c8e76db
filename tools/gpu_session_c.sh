# Cholesky timeline with the one-launch panel factor (own_diag 6) and the A/B of the semantic fast route
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chol_tl6 -o run -- python3 tools/chol_timeline.py 6 > gpurun_out/chol_tl6.log 2>&1 || exit 1
f=$(find gpurun_out/chol_tl6 -name "*kernel_trace.csv" | sort | tail -n 1)
python3 tools/chol_timeline.py --analyze "$f" > gpurun_out/chol_tl6_summary.txt 2>&1
timeout -k 10 300 python -u tools/ab_semantic.py --rounds 3 > gpurun_out/ab_sem.log 2>&1
