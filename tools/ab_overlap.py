"""C4 linearization step with the semantic kernel on the context stream after
the reprojection kernel (linearize_overlap 0) or on a second stream beside it
(1): step wall time and per-kernel HIP-event times.
    python tools/ab_overlap.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import os as _os
_os.environ.setdefault("MI_BA_LIB", "ab")  # A/B variants: the tools-only build (make ab)
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

cfg = bench.CONFIGS["C4"]
sc, sem = bench.build_shard(cfg, 0, 1)
ctx = mi_ba.Context(mi_ba.default_options(), sc, sem)
nb, _, ns = ctx.dims()
for rnd in range(2):
    for ov in (0, 2, 1):
        ctx.set_tuning("linearize_overlap", ov)
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
        j = ctx.kernel_time("reproj_jacobian")
        s = ctx.kernel_time("semantic_jacobian")
        ctx.set_timing(False)
        print(json.dumps({"overlap": ov, "step_ms": 1e3 * dt, "value": (nb + ns) / dt,
                          "reproj_ms": j[0] / j[1], "semantic_ms": s[0] / s[1]}), flush=True)
ctx.close()
