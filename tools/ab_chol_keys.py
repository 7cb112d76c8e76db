"""A/B of the C4 LM-phase timings over arbitrary cholesky_* tuning keys.
    python tools/ab_chol_keys.py "tile_factor=0,write_through=0" "tile_factor=1,write_through=1" ...
Each argument is one variant (comma-separated key=value, keys without the
cholesky_ prefix); every variant runs a 3-iteration C4 solve twice (the second
is reported)."""
import json
import sys

sys.path.insert(0, 'semantic-bundle-adjustment-colmap_amd')
import os as _os
_os.environ.setdefault("MI_BA_LIB", "ab")  # A/B variants: the tools-only build (make ab)
import mi_ba  # noqa: E402

c = mi_ba.synth_config(mi_ba.OPENCV, 1000, 1_000_000, track_length=10, rotation_range=0.05,
                       extra=(-0.1, 0.01, 1e-4, -1e-4))
sc = mi_ba.generate_scene(c).gauge()
w = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 30, 300, track_length=5, rotation_range=0.05,
                                            extra=(-0.1, 0.01, 1e-4, -1e-4))).gauge()
with mi_ba.Context(mi_ba.default_options(max_num_iterations=2), w) as x:
    x.solve()
# --bench-like: bench.py's linearization context (its streams and memory) alive
# and stepped beside the LM contexts, as in the bench's BA-iteration leg
# --bench-like-closed: the same context stepped and then closed before the LM runs
argv = [a for a in sys.argv[1:] if a not in ("--bench-like", "--bench-like-closed")]
lin = None
if "--bench-like" in sys.argv or "--bench-like-closed" in sys.argv:
    sys.path.insert(0, ".")
    import bench  # noqa: E402
    bsc, bsem = bench.build_shard(bench.CONFIGS["C4"], 0, 1)
    lin = mi_ba.Context(mi_ba.default_options(), bsc, bsem)
    for _ in range(5):
        lin.linearize()
    lin.synchronize()
    if "--bench-like-closed" in sys.argv:
        lin.close()
        lin = None
for arg in argv or [""]:
    keys = dict(kv.split("=") for kv in arg.split(",") if kv)
    for rep in range(2):
        with mi_ba.Context(mi_ba.default_options(max_num_iterations=3), sc.copy()) as ctx:
            for k, v in keys.items():
                ctx.set_tuning("cholesky_" + k, int(v))
            ctx.set_timing(True)
            s = ctx.solve()
            its = s.num_successful_steps + s.num_unsuccessful_steps
            ph = {k: ctx.kernel_time(k) for k in ("cholesky", "cholesky_solve", "schur_build", "fblock", "backsub")}
        if rep == 1:
            print(json.dumps(dict(keys=keys, ba_ms=round(1e3 * s.total_time_in_seconds / its, 3), final=s.final_cost,
                                  steps=(s.num_successful_steps, s.num_unsuccessful_steps),
                                  **{k: round(t[0] / max(1, t[1]), 3) for k, t in ph.items()})), flush=True)
