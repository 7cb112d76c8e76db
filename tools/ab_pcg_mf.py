"""ITERATIVE_SCHUR (implicit-Schur PCG) at C4 with the stored-J Schur product
(pcg_matrix_free 0: point pass on J, camera pass on the camera-major copy)
and the matrix-free one (1: both passes recompute the Jacobian rows):
3-iteration LM on the C4 scene (+ semantic samples), BA-iteration time, PCG
time per CG product, final costs.
    python tools/ab_pcg_mf.py [--iters 3] [--reps 2]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--config", default="C4")
args = ap.parse_args()
sc, sem = bench.build_shard(bench.CONFIGS[args.config], 0, 1)
w = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 30, 300, track_length=5, rotation_range=0.05,
                                            extra=(-0.1, 0.01, 1e-4, -1e-4))).gauge()
with mi_ba.Context(mi_ba.default_options(max_num_iterations=2, linear_solver_type=mi_ba.SOLVER_ITERATIVE_SCHUR),
                   w) as x:
    x.set_tuning("pcg_matrix_free", 1)
    x.solve()
for rep in range(args.reps):
    for mf in (0, 1):
        opts = mi_ba.default_options(max_num_iterations=args.iters, linear_solver_type=mi_ba.SOLVER_ITERATIVE_SCHUR)
        with mi_ba.Context(opts, sc.copy(), sem) as ctx:
            ctx.set_tuning("pcg_matrix_free", mf)
            ctx.set_timing(True)
            s = ctx.solve()
            its = s.num_successful_steps + s.num_unsuccessful_steps
            ph = {k: ctx.kernel_time(k) for k in ("pcg", "fblock", "permute_rows", "gather_cm", "backsub",
                                                   "point_prepare", "trial_cost")}
        print(json.dumps({"config": args.config, "rep": rep, "pcg_matrix_free": mf,
                          "ba_iteration_ms": round(1e3 * s.total_time_in_seconds / max(1, its), 3),
                          "cg_products": s.num_linear_solver_iterations,
                          "pcg_ms_per_iteration": round(ph["pcg"][0] / max(1, ph["pcg"][1]), 3),
                          "pcg_ms_per_product": round(ph["pcg"][0] / max(1, s.num_linear_solver_iterations), 4),
                          "final_cost": s.final_cost, "steps": [s.num_successful_steps, s.num_unsuccessful_steps],
                          **{k: [round(v[0], 3), v[1]] for k, v in ph.items()}}), flush=True)
