"""Print per-kernel PMC averages from a tools/pmc_jac.sh output directory."""
import csv
import os
import re
import sys
from collections import defaultdict

src = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for sub in sorted(os.listdir(src)):
    p = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    with open(p) as f:
        for r in csv.DictReader(f):
            m = re.search(r"(\w+_kernel)(<[^>(]*>)?", r["Kernel_Name"])
            k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:60]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "reproj_jacobian" not in k:
        continue
    print(k)
    for c in sorted(d):
        v = d[c]
        print(f"  {c:42s} {sum(v) / len(v):16.4g}  (n={len(v)})")
