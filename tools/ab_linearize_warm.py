"""The C4 linearization step (as bench.py) with the reprojection kernel's
inputs read into the memory-side cache right before it
("linearize_warm_inputs": range mask, default 1 = the observations) and the
flat pass's coarse box ("semantic_flat_coarse"): step wall time, the kernels'
times (HIP events) and the warm-up's over interleaved rounds; the step's cost,
r and J checked equal.
    python tools/ab_linearize_warm.py [--rounds 6] [--reps 10]"""
import argparse
import json
import os
import sys
import time

import numpy as np

if "--overlap" in sys.argv or "--ab" in sys.argv or "--conc" in sys.argv:
    os.environ.setdefault("MI_BA_LIB", "ab")  # linearize_overlap: the tools-only build (make ab)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--overlap", action="store_true",
                help="the semantic pass on a second stream beside the reprojection kernel (1) or only its "
                     "deferred pass (2), with the warm-up (tools build)")
ap.add_argument("--ab", action="store_true", help="the tools build (semantic_deferred_variant)")
ap.add_argument("--conc", action="store_true",
                help="the warm-up on a side stream beside the semantic deferred pass (linearize_warm_concurrent "
                     "range mask, tools build) instead of serially before the reprojection kernel")
args = ap.parse_args()
sc, sem = bench.build_shard(bench.CONFIGS["C4"], 0, 1)
ctx = mi_ba.Context(mi_ba.default_options(), sc, sem)
# (linearize_warm_inputs: range mask read right before the reprojection
#  kernel, 1 observations, 2 image ids, 4 point ids, 8 points; 0 off;
#  semantic_flat_coarse)
# (..., semantic_deferred_compact, warm_workgroups, semantic_deferred_grid)
# (..., semantic_deferred_compact, warm_workgroups, semantic_deferred_grid, semantic_prep_early)
# (..., linearize_order: 1 the semantic pass first)
# (..., warm_unroll, semantic_deferred_variant)
CONFIGS = [(15, 2, 0, 1, 2048, 24, 0, 0, 4, v) for v in range(5)] if args.ab else \
    [(15, 2, 0), (15, 2, 0, 1, 2048, 24, 0, 0, 8)]
if args.overlap:
    CONFIGS = [(15, 2, 0), (15, 2, 1), (15, 2, 2), (0, 2, 1)]
if args.conc:  # cfg[2] is the concurrent range mask here
    CONFIGS = [(15, 2, 0), (0, 2, 15), (0, 2, 1), (14, 2, 1), (0, 2, 7)]


def apply(cfg):
    ctx.set_tuning("linearize_warm_inputs", cfg[0])
    ctx.set_tuning("semantic_flat_coarse", cfg[1])
    ctx.set_tuning("semantic_deferred_compact", cfg[3] if len(cfg) > 3 else 1)
    ctx.set_tuning("warm_workgroups", cfg[4] if len(cfg) > 4 else 2048)
    ctx.set_tuning("semantic_deferred_grid", cfg[5] if len(cfg) > 5 else 24)
    ctx.set_tuning("semantic_prep_early", cfg[6] if len(cfg) > 6 else 0)
    ctx.set_tuning("linearize_order", cfg[7] if len(cfg) > 7 else 0)
    ctx.set_tuning("warm_unroll", cfg[8] if len(cfg) > 8 else 4)
    if len(cfg) > 9:
        ctx.set_tuning("semantic_deferred_variant", cfg[9])
    if args.overlap:
        ctx.set_tuning("linearize_overlap", cfg[2])
    if args.conc:
        ctx.set_tuning("linearize_warm_concurrent", cfg[2])


costs, same = {}, {}
ref = None
for cfg in CONFIGS:
    apply(cfg)
    ctx.linearize()
    costs[cfg] = ctx.cost()
    _, r, J = ctx.download_jacobian()
    ctx.evaluate_semantic()  # the samples re-evaluated with write_samples
    _, sst, sr, sJ = ctx.download_semantic()
    if ref is None:
        ref = (r, J, sst, sr, sJ)
    same[cfg] = bool(np.array_equal(r, ref[0]) and np.array_equal(J, ref[1]) and np.array_equal(sst, ref[2])
                     and np.array_equal(sr, ref[3]) and np.array_equal(sJ, ref[4]))
    del r, J, sst, sr, sJ
ref = None
res = {c: [] for c in CONFIGS}
for rnd in range(args.rounds):
    for cfg in CONFIGS:
        apply(cfg)
        for _ in range(3):
            ctx.linearize()
        ctx.synchronize()
        ctx.set_timing(True)
        ctx.reset_kernel_times()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            ctx.linearize()
        ctx.synchronize()
        wall = (time.perf_counter() - t0) / args.reps * 1e3
        sj = ctx.kernel_time("semantic_jacobian")
        rj = ctx.kernel_time("reproj_jacobian")
        wj = ctx.kernel_time("input_warm")
        ctx.set_timing(False)
        res[cfg].append((sj[0] / sj[1], rj[0] / rj[1], wall, wj[0] / max(1, wj[1])))
for cfg in CONFIGS:
    a = np.array(res[cfg])
    print(json.dumps({"linearize_warm_inputs": cfg[0], "semantic_flat_coarse": cfg[1], "linearize_overlap": cfg[2],
                      "semantic_deferred_compact": cfg[3] if len(cfg) > 3 else 1,
                      "warm_workgroups": cfg[4] if len(cfg) > 4 else 2048,
                      "semantic_deferred_grid": cfg[5] if len(cfg) > 5 else 24,
                      "semantic_prep_early": cfg[6] if len(cfg) > 6 else 0,
                      "linearize_order": cfg[7] if len(cfg) > 7 else 0,
                      "warm_unroll": cfg[8] if len(cfg) > 8 else 4,
                      "semantic_deferred_variant": cfg[9] if len(cfg) > 9 else 0, "cost": costs[cfg], "cost_equal": costs[cfg] == costs[CONFIGS[0]], "r_J_equal": same[cfg],
                      "semantic_ms_median": float(np.median(a[:, 0])), "reproj_ms_median": float(np.median(a[:, 1])),
                      "step_wall_ms_median": float(np.median(a[:, 2])),
                      "input_warm_ms_median": float(np.median(a[:, 3])), "rounds": args.rounds, "reps": args.reps}),
          flush=True)
ctx.close()
