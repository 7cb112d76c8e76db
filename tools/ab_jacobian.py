"""Times the reproj_jacobian kernel alone on a BASELINE config (HIP events on
the context stream, interleaved rounds) and reports GB/s vs the 8 TB/s peak.
    python tools/ab_jacobian.py [--config C4] [--rounds 5] [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C4")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
cfg = dict(bench.CONFIGS[args.config])
c = mi_ba.synth_config(cfg["model"], cfg["images"], cfg["points"], track_length=cfg["track"], rotation_range=0.05,
                       extra=cfg["extra"])
sc = mi_ba.generate_scene(c).gauge()
ctx = mi_ba.Context(mi_ba.default_options(), sc)
nb, W, _ = ctx.dims()
bpb = bench.bytes_per_block(cfg["model"], cfg["track"])
ctx.evaluate_jacobian()
ctx.synchronize()
_, r, J = ctx.download_jacobian()
checksum = (float(np.abs(r).sum()), float(np.abs(J).sum()))
del r, J
res = []
for rnd in range(args.rounds):
    ctx.set_timing(True)
    ctx.reset_kernel_times()
    for _ in range(args.reps):
        ctx.evaluate_jacobian()
    ms, n = ctx.kernel_time("reproj_jacobian")
    ctx.set_timing(False)
    res.append(ms / n)
med = float(np.median(res))
print(json.dumps({"config": args.config, "blocks": nb, "bytes_per_block": bpb, "median_ms": med,
                  "min_ms": float(np.min(res)), "GBps": bpb * nb / (med * 1e-3) / 1e9,
                  "frac_of_8TBps": bpb * nb / (med * 1e-3) / 8e12, "checksum": checksum}))
ctx.close()
