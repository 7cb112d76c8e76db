# usage: bash tools/gpu_quick.sh <log name> <pytest args...>
set -o pipefail
mkdir -p gpurun_out
name=$1; shift
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$name.log 2>&1
