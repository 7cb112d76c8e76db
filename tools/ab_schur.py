"""A/B of LM tuning keys at C4: LM-phase timings of a 3-iteration exact-Schur
LM per combination of the given keys.
    python tools/ab_schur.py schur_pairs_variant=0,1 cholesky_rest_update=0,1,2,3"""
import json
import os
import sys

import os as _os
_os.environ.setdefault("MI_BA_LIB", "ab")  # A/B variants: the tools-only build (make ab)
sys.path.insert(0, 'semantic-bundle-adjustment-colmap_amd')
import mi_ba  # noqa: E402

c = mi_ba.synth_config(mi_ba.OPENCV, 1000, 1_000_000, track_length=10, rotation_range=0.05,
                       extra=(-0.1, 0.01, 1e-4, -1e-4))
sc = mi_ba.generate_scene(c).gauge()
w = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 30, 300, track_length=5, rotation_range=0.05,
                                            extra=(-0.1, 0.01, 1e-4, -1e-4))).gauge()
with mi_ba.Context(mi_ba.default_options(max_num_iterations=2), w) as x:
    x.solve()
# argv: comma lists of tuning-key assignments, e.g. schur_pairs_variant=0 cholesky_rest_update=0,1,2
grid = [[]]
for arg in sys.argv[1:]:
    key, vals = arg.split("=")
    grid = [g + [(key, int(v))] for g in grid for v in vals.split(",")]
# AB_SOLVER=iterative: the implicit-Schur PCG LM (the N > 1 default) instead of the exact one
solver = mi_ba.SOLVER_ITERATIVE_SCHUR if os.environ.get("AB_SOLVER") == "iterative" else mi_ba.SOLVER_DENSE_SCHUR
for tun in grid:
    with mi_ba.Context(mi_ba.default_options(max_num_iterations=3, linear_solver_type=solver), sc.copy()) as ctx:
        for key, val in tun:
            ctx.set_tuning(key, val)
        ctx.set_timing(True)
        s = ctx.solve()
        its = s.num_successful_steps + s.num_unsuccessful_steps
        ph = {k: ctx.kernel_time(k) for k in ("cholesky", "cholesky_solve", "schur_build", "fblock", "backsub", "pcg")}
        print(json.dumps(dict(tun, ba_ms=1e3 * s.total_time_in_seconds / its,
                              final=s.final_cost, steps=(s.num_successful_steps, s.num_unsuccessful_steps),
                              **{k: round(t[0] / max(1, t[1]), 3) for k, t in ph.items()})), flush=True)
