"""The flat pass with and without the rasters' 3x3 window summaries
("semantic_window_summary") or the label planes ("semantic_label_planes"), and the deferred pass with and without the
once-read 3x3 box ("semantic_deferred_box"), inside the C4 linearization
step (as bench.py):
semantic / reprojection kernel times (HIP events) and step wall time over
interleaved rounds; samples checked bitwise against the raster-only route.
    python tools/ab_semantic_ws.py [--rounds 6] [--reps 10]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()
sc, sem = bench.build_shard(bench.CONFIGS["C4"], 0, 1)
ctx = mi_ba.Context(mi_ba.default_options(), sc, sem)
# (window summaries, deferred box, label planes, coarse flat box form)
CONFIGS = [(0, 0, 0, 0), (0, 0, 1, 0), (0, 0, 1, 1), (0, 0, 1, 2), (0, 0, 1, 3)]


def apply(cfg):
    ctx.set_tuning("semantic_window_summary", cfg[0])
    ctx.set_tuning("semantic_deferred_box", cfg[1])
    ctx.set_tuning("semantic_label_planes", cfg[2])
    ctx.set_tuning("semantic_flat_coarse", cfg[3])


def decode(st):
    """semantic_diag 2 marks: +0x1000 deferred, +0x4000 settled without the
    rasters, +0x10000 a deferred sample redone per point"""
    redo = st >= 0xC000
    st = np.where(redo, st - 0x10000, st)
    ws = st >= 0x2800
    st = np.where(ws, st - 0x4000, st)
    d = st >= 0x800
    return np.where(d, st - 0x1000, st), d, ws, redo


ref = None
for cfg in CONFIGS:
    apply(cfg)
    ctx.set_tuning("semantic_diag", 2)
    ctx.evaluate_semantic()
    out = ctx.download_semantic()
    ctx.set_tuning("semantic_diag", 0)
    st, d, ws, redo = decode(out[1])
    out = (out[0], st) + tuple(out[2:])
    if ref is None:
        ref = out
    same = all(np.array_equal(a, b) for a, b in zip(ref[1:], out[1:]))
    n = len(st)
    print(json.dumps({"window_summary": cfg[0], "deferred_box": cfg[1], "label_planes": cfg[2], "flat_coarse": cfg[3],
                      "bitwise_equal": bool(same),
                      "samples": n, "deferred": int(d.sum()), "deferred_redone_per_point": int(redo.sum()),
                      "window_decided": int(ws.sum()),
                      "window_decided_valid": int((ws & (st == mi_ba.VALID)).sum()),
                      "status_valid": int((st == mi_ba.VALID).sum()),
                      "status_invalid_depth": int((st == mi_ba.INVALID_DEPTH).sum()),
                      "status_other": int(((st != mi_ba.VALID) & (st != mi_ba.INVALID_DEPTH)).sum())}), flush=True)
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
        ctx.set_timing(False)
        res[cfg].append((sj[0] / sj[1], rj[0] / rj[1], wall))
for cfg in CONFIGS:
    a = np.array(res[cfg])
    print(json.dumps({"window_summary": cfg[0], "deferred_box": cfg[1], "label_planes": cfg[2], "flat_coarse": cfg[3], "semantic_ms_median": float(np.median(a[:, 0])),
                      "reproj_ms_median": float(np.median(a[:, 1])), "step_wall_ms_median": float(np.median(a[:, 2])),
                      "rounds": args.rounds, "reps": args.reps}), flush=True)
ctx.close()
