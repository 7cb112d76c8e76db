set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5n
timeout -k 10 400 python -u tools/semantic_regime_counts.py > gpurun_out/r5n/regimes.log 2>&1
