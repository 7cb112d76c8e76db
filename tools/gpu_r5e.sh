set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 bash tools/profile.sh gpurun_out/r5e_prof C4
