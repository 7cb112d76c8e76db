# semantic batched-stencil A/B (C4, 5.0M samples): variants 1 (per-point) vs 2/3/4 (batched NB 1/2/4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_semantic.py --variants 1,2,3,4,0 > gpurun_out/ab_sem_batched.jsonl 2> gpurun_out/ab_sem_batched.err
