set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5l
timeout -k 10 600 python -u tools/ab_lm_semantic_context.py > gpurun_out/r5l/ab.log 2>&1
