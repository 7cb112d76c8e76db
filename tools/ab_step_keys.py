"""A/B of the bench's C4 linearization step over tuning keys (full key names):
    python tools/ab_step_keys.py "semantic_label_nibbles=1" "semantic_label_nibbles=0"
One context (bench.py's C4 scene with its semantic samples); every round
sets each variant's keys (list every key in every variant), warms up, times 20 steps by wall clock and 10 more by the per-kernel HIP
events.  Rounds interleave the variants."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

variants = [dict(kv.split("=") for kv in arg.split(",") if kv) for arg in (sys.argv[1:] or [""])]
sc, sem = bench.build_shard(bench.CONFIGS["C4"], 0, 1)
ctx = mi_ba.Context(mi_ba.default_options(), sc, sem)
nb, _, ns = ctx.dims()
for rnd in range(3):
    for keys in variants:
        for k, v in keys.items():
            ctx.set_tuning(k, int(v))
        for _ in range(3):
            ctx.linearize()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            ctx.linearize()
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / 20
        ctx.set_timing(True)
        ctx.reset_kernel_times()
        for _ in range(10):
            ctx.linearize()
        t = {k: ctx.kernel_time(k) for k in ("reproj_jacobian", "semantic_jacobian", "input_warm")}
        ctx.set_timing(False)
        print(json.dumps({"round": rnd, "keys": keys, "step_ms": round(1e3 * dt, 4),
                          "value": (nb + ns) / dt,
                          **{k + "_ms": round(v[0] / max(1, v[1]), 4) for k, v in t.items()}}), flush=True)
ctx.close()
