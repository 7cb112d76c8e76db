"""Jacobian-kernel time in different step contexts at C4 (HIP events on the
context stream): back-to-back evaluate_jacobian, the full linearization step
(reprojection + semantic), and the linearization of a geometric-only context.
    python tools/ab_step_context.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import os as _os
_os.environ.setdefault("MI_BA_LIB", "ab")  # A/B variants: the tools-only build (make ab)
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

cfg = bench.CONFIGS["C4"]
sc, sem = bench.build_shard(cfg, 0, 1)


def timed(ctx, fn, reps=10):
    for _ in range(3):
        fn()
    ctx.set_timing(True)
    ctx.reset_kernel_times()
    for _ in range(reps):
        fn()
    j = ctx.kernel_time("reproj_jacobian")
    s = ctx.kernel_time("semantic_jacobian")
    ctx.set_timing(False)
    return j[0] / max(1, j[1]), (s[0] / s[1] if s[1] else None)


with mi_ba.Context(mi_ba.default_options(), sc.copy(), sem) as ctx:
    for rnd in range(2):
        print(json.dumps({"context": "semantic ctx", "mode": "evaluate_jacobian x10",
                          "reproj_ms": timed(ctx, ctx.evaluate_jacobian)[0]}), flush=True)
        for v in (6,):
            ctx.set_tuning("semantic_variant", v)
            j, s = timed(ctx, ctx.linearize)
            print(json.dumps({"context": "semantic ctx", "mode": "linearize x10", "semantic_variant": v,
                              "reproj_ms": j, "semantic_ms": s}), flush=True)
        ctx.set_tuning("semantic_variant", 6)
    # the step with an idle gap after the semantic pass (clocks / power vs cache / TLB state)
    import time

    def lin_gap():
        ctx.linearize()
        ctx.synchronize()
        time.sleep(0.002)
    j, s = timed(ctx, lin_gap)
    print(json.dumps({"context": "semantic ctx", "mode": "linearize + sync + 2 ms idle x10", "reproj_ms": j,
                      "semantic_ms": s}), flush=True)

    def sem_then_jac():
        ctx.evaluate_semantic()
        ctx.evaluate_jacobian()
    j, s = timed(ctx, sem_then_jac)
    print(json.dumps({"context": "semantic ctx", "mode": "evaluate_semantic(write) + evaluate_jacobian x10",
                      "reproj_ms": j, "semantic_ms": s}), flush=True)
with mi_ba.Context(mi_ba.default_options(), sc.copy()) as ctx:
    for rnd in range(2):
        j, _ = timed(ctx, ctx.linearize)
        print(json.dumps({"context": "geometric ctx", "mode": "linearize x10", "reproj_ms": j}), flush=True)
