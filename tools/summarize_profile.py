"""Condense a tools/profile.sh output directory into a committed summary.

    python tools/summarize_profile.py gpurun_out/prof profiles/r1_c4 [--config C4]

Writes <prefix>.md (kernel-trace stats + per-dispatch PMC averages) and
<prefix>_traffic.json (HBM bytes per launch of each kernel, read by bench.py
for the `roofline.traffic` field).  HBM bytes follow MI355X_MICROARCH.md
§HBM: FETCH_SIZE (KiB) is doubled on gfx950, WRITE_SIZE (KiB) taken as is;
both come from separate --pmc passes.
"""
import argparse
import csv
import json
import os
import re
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+_kernel)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def read_stats(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((short(r["Name"]), int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["Percentage"]),
                         float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
    return rows


def read_pmc(path):
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = (int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]), int(r["SGPR_Count"]),
                       int(r["LDS_Block_Size"]), int(r["Grid_Size"]), int(r["Workgroup_Size"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("prefix")
    ap.add_argument("--config", default="C4")
    args = ap.parse_args()
    stats = read_stats(os.path.join(args.src, "trace", "run_kernel_stats.csv"))
    pmc, meta = {}, {}
    for sub in sorted(os.listdir(args.src)):
        p = os.path.join(args.src, sub, "run_counter_collection.csv")
        if sub.startswith("pmc") and os.path.exists(p):
            d, m = read_pmc(p)
            meta.update(m)
            for k, v in d.items():
                pmc.setdefault(k, {}).update(v)
    lines = [f"# rocprofv3 summary — {os.path.basename(args.prefix)} ({args.config})", "",
             f"Source: `bash tools/profile.sh {args.src} {args.config}` on one MI355X "
             "(kernel trace + separate PMC passes).", "",
             "## Kernel trace (--kernel-trace --stats)", "",
             "| kernel | calls | avg µs | min µs | max µs | % time |", "|---|---|---|---|---|---|"]
    for n, c, a, pct, mn, mx in stats:
        lines.append(f"| `{n}` | {c} | {a:.1f} | {mn:.1f} | {mx:.1f} | {pct:.2f} |")
    lines += ["", "## PMC per dispatch (averaged over dispatches)", "",
              "HBM read = 2 × FETCH_SIZE (gfx950 correction), write = WRITE_SIZE; KiB → bytes.", "",
              "| kernel | VGPR | LDS B | HBM read MB | HBM write MB | VALU/wave | VMEM rd/wave | VMEM wr/wave "
              "| active % | wait-issue % | parked % |",
              "|---|---|---|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for n in sorted(pmc, key=lambda k: -pmc[k].get("FETCH_SIZE", 0)):
        v = pmc[n]
        if "FETCH_SIZE" not in v and "SQ_WAVES" not in v:
            continue
        rd = 2 * v.get("FETCH_SIZE", 0) * 1024
        wr = v.get("WRITE_SIZE", 0) * 1024
        waves = max(v.get("SQ_WAVES", 0), 1)
        cyc = max(v.get("SQ_WAVE_CYCLES", 0), 1)
        vg, ag, sg, lds, grid, wg = meta.get(n, (0, 0, 0, 0, 0, 0))
        lines.append(
            f"| `{n}` | {vg} | {lds} | {rd / 1e6:.1f} | {wr / 1e6:.1f} | {v.get('SQ_INSTS_VALU', 0) / waves:.0f} | "
            f"{v.get('SQ_INSTS_VMEM_RD', 0) / waves:.1f} | {v.get('SQ_INSTS_VMEM_WR', 0) / waves:.1f} | "
            f"{100 * v.get('SQ_ACTIVE_INST_ANY', 0) / cyc:.0f} | {100 * v.get('SQ_WAIT_INST_ANY', 0) / cyc:.0f} | "
            f"{100 * v.get('SQ_WAIT_ANY', 0) / cyc:.0f} |")
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            traffic[n] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr}
    with open(args.prefix + ".md", "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(args.prefix + "_traffic.json", "w") as f:
        json.dump({"config": args.config, "kernels": traffic}, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
