set -o pipefail
mkdir -p gpurun_out/r5ah
export MI_BA_LIB=ab
timeout -k 10 700 python -u tools/ab_chol_keys.py "" "split_tail_cols=6144,split_tail_rest=1" "split_tail_cols=12000,split_tail_rest=1" "" "split_tail_cols=6144,split_tail_rest=1" "split_tail_cols=4096,split_tail_rest=1" > gpurun_out/r5ah/ab.jsonl 2> gpurun_out/r5ah/ab.err &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cholesky.py -k "split_tail" > gpurun_out/r5ah/tests.log 2>&1
