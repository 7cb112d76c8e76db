"""LM-phase timings of the C4 exact-Schur LM with and without the semantic
term on the same scene (bench.py's shard), to separate the semantic
context's effect on the geometric phases.
    python tools/ab_lm_semantic_context.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

cfg = bench.CONFIGS["C4"]
sc, sem = bench.build_shard(cfg, 0, 1)
w = mi_ba.generate_scene(mi_ba.synth_config(cfg["model"], 30, 300, track_length=5, rotation_range=0.05,
                                            extra=cfg["extra"])).gauge()
with mi_ba.Context(mi_ba.default_options(max_num_iterations=2), w) as x:
    x.solve()
for label, s_in in (("semantic", sem), ("geometric", None), ("semantic", sem), ("geometric", None)):
    with mi_ba.Context(mi_ba.default_options(max_num_iterations=3), sc.copy(), s_in) as ctx:
        ctx.set_timing(True)
        s = ctx.solve()
        its = s.num_successful_steps + s.num_unsuccessful_steps
        ph = {k: ctx.kernel_time(k) for k in ("cholesky", "schur_build", "fblock", "backsub", "reproj_jacobian")}
        print(json.dumps(dict(case=label, ba_ms=round(1e3 * s.total_time_in_seconds / its, 3),
                              **{k: [round(t[0], 3), t[1]] for k, t in ph.items()})), flush=True)
