"""reproj_jacobian in two contexts at C4, for PMC passes (one context per process):
    python tools/jac_context.py b2b    # evaluate_jacobian back-to-back
    python tools/jac_context.py step   # full linearization steps (semantic pass + reprojection)
Prints the kernel's mean time (HIP events) over the timed launches."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "step"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
sc, sem = bench.build_shard(bench.CONFIGS["C4"], 0, 1)
with mi_ba.Context(mi_ba.default_options(), sc, sem) as ctx:
    fn = ctx.evaluate_jacobian if mode == "b2b" else ctx.linearize
    for _ in range(3):
        fn()
    ctx.synchronize()
    ctx.set_timing(True)
    ctx.reset_kernel_times()
    for _ in range(reps):
        fn()
    ctx.synchronize()
    j = ctx.kernel_time("reproj_jacobian")
    print(json.dumps({"mode": mode, "reps": reps, "reproj_ms": j[0] / max(1, j[1])}), flush=True)
