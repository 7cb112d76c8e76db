set -o pipefail
mkdir -p gpurun_out/r5ab
export MI_BA_LIB=ab
timeout -k 10 900 python -u tools/ab_chol_keys.py "" "panel_rows_per_group=2,panel_group_min_rows=6000" "panel_rows_per_group=2" "head_panel=1024,head_cols=4096" "tail_panel=256,tail_cols=4096" "" "panel_rows_per_group=2,panel_group_min_rows=6000" "head_panel=1024,head_cols=4096" > gpurun_out/r5ab/ab.jsonl 2> gpurun_out/r5ab/ab.err
