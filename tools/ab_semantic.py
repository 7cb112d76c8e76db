"""Times the semantic linearization kernel alone at C4 (5.0M samples, HIP
events on the context stream) and checks its samples against a reference
download.    python tools/ab_semantic.py [--rounds 5]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import os as _os
_os.environ.setdefault("MI_BA_LIB", "ab")  # A/B variants: the tools-only build (make ab)
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--variants", default="0,1", help="semantic_variant values (0 reference-order fast route, 1 FMA)")
args = ap.parse_args()
cfg = bench.CONFIGS["C4"]
sc, sem = bench.build_shard(cfg, 0, 1)
sc.obs_xy, sc.obs_image, sc.obs_point = sc.obs_xy[:0], sc.obs_image[:0], sc.obs_point[:0]
ctx = mi_ba.Context(mi_ba.default_options(), sc, sem)
_, _, ns = ctx.dims()
ctx.evaluate_semantic()
px, st, r, J = ctx.download_semantic()
for v in [int(x) for x in args.variants.split(",")]:
    ctx.set_tuning("semantic_variant", v)
    ctx.evaluate_semantic()
    _, st_v, r_v, J_v = ctx.download_semantic()
    same = bool(np.array_equal(st, st_v) and np.array_equal(r, r_v) and np.array_equal(J, J_v))
    ts = []
    for rnd in range(args.rounds):
        ctx.set_timing(True)
        ctx.reset_kernel_times()
        for _ in range(args.reps):
            ctx.linearize()
        ms, n = ctx.kernel_time("semantic_jacobian")
        ctx.set_timing(False)
        ts.append(ms / n)
    deferred = None
    if v in (5, 6):
        ctx.set_tuning("semantic_diag", 1)
        ctx.evaluate_semantic()
        _, st_d, _, _ = ctx.download_semantic()
        deferred = int((st_d >= 0x800).sum())
        ctx.set_tuning("semantic_diag", 0)
    print(json.dumps({"variant": v, "deferred": deferred, "samples": ns, "median_ms": float(np.median(ts)), "min_ms": float(np.min(ts)),
                      "bitwise_equal_to_variant0": same,
                      "valid": int((st_v == mi_ba.VALID).sum()), "nonzero_J_rows": int((np.abs(J_v).sum(1) > 0).sum()),
                      "checksum_J": float(np.abs(J_v).sum()), "checksum_r": float(r_v.sum())}), flush=True)
ctx.close()
