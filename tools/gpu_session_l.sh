# semantic two-pass variant: A/B + kernel trace of variant 6
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_semantic.py --variants 6,4 > gpurun_out/ab_sem_m.jsonl 2> gpurun_out/ab_sem_m.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sem6 -o run -- python3 tools/ab_semantic.py --variants 6 --rounds 2 > gpurun_out/prof_sem6.log 2>&1
