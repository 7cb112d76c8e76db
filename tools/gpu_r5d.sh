set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5d
timeout -k 10 500 python -u tools/ab_jacobian.py --step --rounds 6 --reps 5 --variants 0,43,0:linearize_warm_inputs=0,43:linearize_warm_inputs=0 > gpurun_out/r5d/ab_jac.log 2>&1
