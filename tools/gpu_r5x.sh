set -o pipefail
mkdir -p gpurun_out/r5ag
export MI_BA_LIB=ab
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cholesky.py -k "split_tail or handoff or factor_at_c4 or lookahead" > gpurun_out/r5ag/tests.log 2>&1 &&
timeout -k 10 700 python -u tools/ab_chol_keys.py "" "split_tail_cols=4096" "split_tail_cols=6144" "split_tail_cols=8192" "" "split_tail_cols=6144" "split_tail_cols=12000" > gpurun_out/r5ag/ab.jsonl 2> gpurun_out/r5ag/ab.err
