"""Per-launch PMC summary of the semantic linearization kernel from the
rocprofv3 --pmc passes of tools/pmc_semantic.sh, for bench.py's
roofline_semantic:
    python tools/summarize_pmc_semantic.py gpurun_out/pmcs profiles/r2_c4_semantic_pmc.json
FP64 operations = 64 lanes x (ADD + MUL + TRANS + 2 FMA) wave instructions
(an upper bound: lanes masked off by divergence are counted); HBM bytes =
FETCH_SIZE x 2 (gfx950 reports half the bytes of coalesced reads,
MI355X_MICROARCH.md) + WRITE_SIZE, KB units x 1024."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src, dst = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
dur = []
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "semantic_linearize" not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
avg = {k: sum(v) / len(v) for k, v in vals.items()}
f64 = 64 * (avg.get("SQ_INSTS_VALU_ADD_F64", 0) + avg.get("SQ_INSTS_VALU_MUL_F64", 0) +
            avg.get("SQ_INSTS_VALU_TRANS_F64", 0) + 2 * avg.get("SQ_INSTS_VALU_FMA_F64", 0))
out = {"kernel": "semantic_linearize_kernel", "launches_sampled": {k: len(v) for k, v in vals.items()},
       "counters_avg_per_launch": avg,
       "fp64_ops_per_launch": f64,
       "hbm_bytes_per_launch": 1024 * (2 * avg.get("FETCH_SIZE", 0) + avg.get("WRITE_SIZE", 0))
       if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg else None,
       "note": "PMC passes under rocprofv3 (kernel serialised); FP64 ops count every lane of each wave instruction"}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
