"""GSBA throughput: one linearization (every block's 1 + 2 * params IoU
evaluations) of a synthetic workload on the GPU vs the CPU oracle (OpenMP,
all host threads) on the same blocks.  Prints one JSON line.

The wall time of mi_ba_gsba_evaluate includes its context setup and mask
upload; the kernel time comes from a rocprofv3 kernel trace of this run:
    rocprofv3 --kernel-trace --stats --output-format csv -d out -o run -- python3 tools/bench_gsba.py > line.json
    python3 tools/bench_gsba.py --merge line.json out/<host>/run_kernel_stats.csv
adds gpu_kernel_ms_per_linearization (gsba_* kernels / linearizations) and
its ratio to the CPU time."""
import csv
import json
import re
import os
import sys
import time

if len(sys.argv) > 1 and sys.argv[1] == "--merge":
    line = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
    ns = 0.0
    per = {}
    for r in csv.DictReader(open(sys.argv[3])):
        if "gsba" in r["Name"]:
            ns += float(r["TotalDurationNs"])
            m = re.search(r"(\w+_kernel)", r["Name"])
            per[m.group(1) if m else r["Name"][:40]] = float(r["TotalDurationNs"]) / 1e6
    runs = line["linearizations_timed"] + 1  # + the warm-up
    line["gpu_kernel_ms_per_linearization"] = round(ns / 1e6 / runs, 3)
    line["gpu_kernel_ms_by_kernel"] = {k: round(v / runs, 3) for k, v in per.items()}
    line["cpu_over_gpu_kernel"] = round(line["cpu_ms"] / line["gpu_kernel_ms_per_linearization"], 1)
    line["note"] = ("gpu_kernel_ms = sum of the gsba_* kernels (rocprofv3 kernel trace) per linearization; "
                    "gpu_ms_per_linearization = mi_ba_gsba_evaluate wall time incl. context setup + upload")
    print(json.dumps(line))
    sys.exit(0)

sys.path[:0] = ["semantic-bundle-adjustment-colmap_amd", "oracle"]
import numpy as np  # noqa: E402
import mi_ba  # noqa: E402
import oracle  # noqa: E402

I = int(sys.argv[1]) if len(sys.argv) > 1 else 40
N = int(sys.argv[2]) if len(sys.argv) > 2 else 12
H, W = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1080, 1920)
sc, cyl = mi_ba.gsba_scene(I, N, H, W, seed=0)
masks = oracle.gsba_render(sc, cyl, H, W)
rng = np.random.default_rng(1)
init = cyl.copy()
init[:, 4:6] += rng.uniform(-0.05, 0.05, (N, 2))
init[:, 7] *= 1.1
g = mi_ba.GsbaInput(masks, init)
sc = sc.gauge()
o = mi_ba.default_options()
mi_ba.gsba_evaluate(o, sc, g)  # warm-up (code objects, allocations)
reps = 5
t = time.perf_counter()
for _ in range(reps):
    ids, r, J = mi_ba.gsba_evaluate(o, sc, g)
gpu_s = (time.perf_counter() - t) / reps
t = time.perf_counter()
ids_o, r_o, J_o = oracle.gsba_evaluate(o, sc, g)
cpu_s = time.perf_counter() - t
nb = len(ids)
evals = int(sum(1 + 2 * (9 if i == 0 else 16) for i in ids[:, 0]))
same = float(np.mean(np.concatenate([(r == r_o)[:, None], J == J_o], axis=1)))
print(json.dumps({"workload": "GSBA %d images x %d cylinders, %dx%d trunk masks" % (I, N, H, W), "blocks": nb,
                  "linearizations_timed": reps,
                  "iou_evaluations": evals, "gpu_ms_per_linearization": round(1e3 * gpu_s, 3),
                  "gpu_evals_per_s": round(evals / gpu_s, 1), "cpu_ms": round(1e3 * cpu_s, 1),
                  "cpu_threads": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count())), "bitwise_equal_fraction": same,
                  "note": "gpu time = mi_ba_gsba_evaluate wall time incl. context setup + upload"}), flush=True)
