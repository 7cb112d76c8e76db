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
# one linearization = one launch of each semantic kernel family present
# (semantic_linearize_kernel, or semantic_flat_kernel + semantic_deferred_kernel):
# per-family averages per launch, summed over the families
fams = ("semantic_linearize", "semantic_flat", "semantic_deferred")
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        fam = next((x for x in fams if x in r["Kernel_Name"]), None)
        if fam is None:
            continue
        vals[r["Counter_Name"]][fam].append(float(r["Counter_Value"]))
# the two-pass route when present (tools/ab_semantic.py may also launch the
# one-kernel variants for its bitwise check)
for per in vals.values():
    if "semantic_flat" in per:
        per.pop("semantic_linearize", None)
avg = {k: sum(sum(v) / len(v) for v in per.values()) for k, per in vals.items()}
f64 = 64 * (avg.get("SQ_INSTS_VALU_ADD_F64", 0) + avg.get("SQ_INSTS_VALU_MUL_F64", 0) +
            avg.get("SQ_INSTS_VALU_TRANS_F64", 0) + 2 * avg.get("SQ_INSTS_VALU_FMA_F64", 0))
out = {"kernel": "+".join(sorted({f for per in vals.values() for f in per})),
       "launches_sampled": {k: {f: len(v) for f, v in per.items()} for k, per in vals.items()},
       "counters_avg_per_launch": avg,
       "counters_avg_per_launch_by_kernel": {f: {k: sum(per[f]) / len(per[f]) for k, per in vals.items() if f in per}
                                             for f in sorted({f for per in vals.values() for f in per})},
       "fp64_ops_per_launch": f64,
       "hbm_bytes_per_launch": 1024 * (2 * avg.get("FETCH_SIZE", 0) + avg.get("WRITE_SIZE", 0))
       if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg else None,
       "note": "PMC passes under rocprofv3 (kernel serialised); FP64 ops count every lane of each wave instruction"}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
