set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5h
python3 -c "
import ctypes; h=ctypes.CDLL('libamdhip64.so'); a=ctypes.c_int(); b=ctypes.c_int(); print('priority range', h.hipDeviceGetStreamPriorityRange(ctypes.byref(a), ctypes.byref(b)), a.value, b.value)" > gpurun_out/r5h/ab.log 2>&1
MI_BA_LIB=product timeout -k 10 500 python -u tools/ab_chol_keys.py "" "rest_priority=2" "" "rest_priority=2" >> gpurun_out/r5h/ab.log 2>&1 &&
MI_BA_LIB=product timeout -k 10 500 python -u tools/ab_chol_keys.py --bench-like "" "rest_priority=2" "" "rest_priority=2" >> gpurun_out/r5h/ab.log 2>&1
