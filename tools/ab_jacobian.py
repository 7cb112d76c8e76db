"""Times the reproj_jacobian kernel alone on a BASELINE config (HIP events on
the context stream, interleaved rounds) and reports GB/s vs the 8 TB/s peak.
    python tools/ab_jacobian.py [--config C4] [--rounds 5] [--reps 5] [--variants 0,13,0:linearize_warm_inputs=0]
A variant is a jacobian_variant number, optionally with tuning keys set for
it alone ("0:linearize_warm_inputs=0:linearize_order=1"; reset to the product
defaults afterwards).
"""
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
ap.add_argument("--config", default="C4")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--variants", default="0")
ap.add_argument("--step", action="store_true",
                help="time the kernel inside the full C4 linearization step (after the semantic pass, as bench.py)")
args = ap.parse_args()
cfg = dict(bench.CONFIGS[args.config])
c = mi_ba.synth_config(cfg["model"], cfg["images"], cfg["points"], track_length=cfg["track"], rotation_range=0.05,
                       extra=cfg["extra"])
if args.step:
    sc, sem = bench.build_shard(cfg, 0, 1)
    ctx = mi_ba.Context(mi_ba.default_options(), sc, sem)
else:
    sc = mi_ba.generate_scene(c).gauge()
    ctx = mi_ba.Context(mi_ba.default_options(), sc)
nb, W, _ = ctx.dims()
bpb = bench.bytes_per_block(cfg["model"], cfg["track"])
variants = args.variants.split(",")


# the product defaults the keys return to after a variant that set them
DEFAULTS = {"linearize_order": 0, "linearize_warm_inputs": 15, "warm_workgroups": 2048}


def apply(spec, on=True):
    parts = spec.split(":")
    if on:
        ctx.set_tuning("jacobian_variant", int(parts[0]))
    for kv in parts[1:]:
        k, val = kv.split("=")
        ctx.set_tuning(k, int(val) if on else DEFAULTS.get(k, 0))


ref = None
ok = {}
for v in variants:
    apply(v)
    ctx.evaluate_jacobian()
    ctx.synchronize()
    _, r, J = ctx.download_jacobian()
    if ref is None:
        ref = (r.copy(), J.copy())
    ok[v] = bool(np.array_equal(r, ref[0]) and np.array_equal(J, ref[1]))
    ok[v] = (ok[v], float(np.abs(J - ref[1]).max() / max(1.0, float(np.abs(ref[1]).max()))))
    apply(v, False)
    del r, J
res = {v: [] for v in variants}
for rnd in range(args.rounds):
    for v in variants:
        apply(v)
        ctx.evaluate_jacobian()
        ctx.set_timing(True)
        ctx.reset_kernel_times()
        for _ in range(args.reps):
            ctx.linearize() if args.step else ctx.evaluate_jacobian()
        ms, n = ctx.kernel_time("reproj_jacobian")
        ctx.set_timing(False)
        apply(v, False)
        res[v].append(ms / n)
for v in variants:
    med = float(np.median(res[v]))
    print(json.dumps({"config": args.config, "variant": v, "identical_to_first": ok[v][0], "max_rel_dJ_vs_first": ok[v][1], "blocks": nb,
                      "bytes_per_block": bpb, "median_ms": med, "min_ms": float(np.min(res[v])),
                      "GBps": bpb * nb / (med * 1e-3) / 1e9, "frac_of_8TBps": bpb * nb / (med * 1e-3) / 8e12}))
ctx.close()
