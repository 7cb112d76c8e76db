set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5g
MI_BA_LIB=product timeout -k 10 800 python -u tools/ab_chol_keys.py "" "rest_streams=1" "rest_update=4,rest_streams=1" "rest_update=4,rest_streams=1,batch_tile=512" "rest_update=4,rest_streams=1,batch_tile=2048" "" "rest_update=4,rest_streams=1" > gpurun_out/r5g/ab.log 2>&1
