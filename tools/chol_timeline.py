"""Kernel timeline of one C4-size (nf = 12 000) factorisation through
mi_ba_dense_cholesky_ex, for rocprofv3 --kernel-trace:
    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/chol_timeline.py [own_diag]
then python3 tools/chol_timeline.py --analyze OUT/.../run_kernel_trace.csv"""
import sys
import time

import numpy as np


def analyze(path):
    import csv
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last factorisation: from the last diag-panel kernel run backwards to the previous gap > 50 ms
    ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?")) for r in rows]
    starts = [t[0] for t in ts]
    cut = 0
    for i in range(1, len(ts)):
        if ts[i][0] - ts[i - 1][1] > 50e6:
            cut = i
    ts = ts[cut:]
    t0 = ts[0][0]
    t1 = max(t[1] for t in ts)
    print(f"kernels {len(ts)} wall {(t1 - t0) / 1e6:.3f} ms")
    fam = {}
    for s, e, n, q in ts:
        k = "dgemm" if n.startswith("Cijk") else n.split("(")[0].replace("void ", "")[-40:]
        a = fam.setdefault((k, q), [0.0, 0])
        a[0] += (e - s) / 1e6
        a[1] += 1
    for (k, q), (t, c) in sorted(fam.items(), key=lambda x: -x[1][0]):
        print(f"  q{q} {t:8.3f} ms {c:5d}  {k}")
    # sequence: every kernel (start, duration) relative to t0, grouped by queue
    if "--seq" in sys.argv:
        for s_, e_, n_, q_ in ts:
            k = "dgemm" if n_.startswith("Cijk") else n_.split("(")[0].replace("void ", "")[-32:]
            print(f"  q{q_} {(s_ - t0) / 1e3:9.1f} us +{(e_ - s_) / 1e3:8.1f} us  {k}")
    # busy union per queue
    for q in sorted(set(t[3] for t in ts)):
        iv = sorted((s, e) for s, e, n, qq in ts if qq == q)
        busy, cs, ce = 0, None, None
        for s, e in iv:
            if ce is None or s > ce:
                if ce is not None:
                    busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        print(f"  queue {q}: busy {busy / 1e6:.3f} ms")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
        sys.exit(0)
    sys.path.insert(0, "semantic-bundle-adjustment-colmap_amd")
    import mi_ba
    n = 12000
    rng = np.random.default_rng(0)
    A = rng.uniform(-1.0, 1.0, (n, n))
    A = (A + A.T) / 2 + np.diag(np.full(n, 2.0 * n))
    own = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    for k in range(2):
        t = time.perf_counter()
        L, _, info = mi_ba.dense_cholesky(A, own_diag=own)
        print(f"call {k}: {time.perf_counter() - t:.3f} s info {info}", flush=True)
    time.sleep(0.2)
