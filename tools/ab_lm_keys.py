"""A/B of the C4 LM phase timings over arbitrary tuning keys (full key names):
    python tools/ab_lm_keys.py "" "schur_pairs_variant=6" "cholesky_tail_panel=256,cholesky_tail_cols=6144"
Each argument is one variant (comma-separated key=value); every variant runs a
3-iteration exact-Schur C4 solve (bench.py's C4 scene with its semantic
samples) twice, interleaved, and the second run of each is reported."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

sc, sem = bench.build_shard(bench.CONFIGS["C4"], 0, 1)
w = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 30, 300, track_length=5, rotation_range=0.05,
                                            extra=(-0.1, 0.01, 1e-4, -1e-4))).gauge()
with mi_ba.Context(mi_ba.default_options(max_num_iterations=2), w) as x:
    x.solve()
PH = ("cholesky", "cholesky_solve", "schur_build", "fblock", "backsub", "point_prepare", "trial_cost", "s_zero")
variants = sys.argv[1:] or [""]
for rep in range(2):
    for arg in variants:
        keys = dict(kv.split("=") for kv in arg.split(",") if kv)
        with mi_ba.Context(mi_ba.default_options(max_num_iterations=3), sc.copy(), sem) as ctx:
            for k, v in keys.items():
                ctx.set_tuning(k, int(v))
            ctx.set_timing(True)
            s = ctx.solve()
            its = s.num_successful_steps + s.num_unsuccessful_steps
            ph = {k: ctx.kernel_time(k) for k in PH}
        if rep == 1:
            print(json.dumps(dict(keys=keys, ba_ms=round(1e3 * s.total_time_in_seconds / its, 3), final=s.final_cost,
                                  steps=(s.num_successful_steps, s.num_unsuccessful_steps),
                                  **{k: round(t[0] / max(1, t[1]), 3) for k, t in ph.items()})), flush=True)
