"""Diagnostic: step counts / final cost of the 'constants' PCG parity case
under the oracle, the exact GPU solve and the PCG GPU solve (with the A/B
build: each PCG pass variant toggled).  python tools/diag_pcg_constants.py"""
import os, sys, json
sys.path.insert(0, 'semantic-bundle-adjustment-colmap_amd'); sys.path.insert(0, 'oracle')
import numpy as np, mi_ba, oracle
sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 30, 2000, track_length=6, rotation_range=0.05,
                                             extra=(-0.1, 0.01, 1e-4, -1e-4), seed=11)).gauge()
rng = np.random.default_rng(3)
sc.point_config = np.where(rng.uniform(size=sc.num_points) < 0.3, 2, 1).astype(np.uint8)
sc.camera_constant = (np.arange(sc.num_cameras) % 3 == 0).astype(np.uint8)
sc.image_constant_pose[5] = 1
def show(tag, s):
    print(json.dumps({"run": tag, "steps": [s.num_successful_steps, s.num_unsuccessful_steps],
                      "final": s.final_cost, "cg": s.num_linear_solver_iterations}), flush=True)
ref = mi_ba.default_options(max_num_iterations=8, eta=1e-12)
if os.environ.get("MI_BA_LIB") != "ab":
    show("oracle", oracle.solve(ref, sc.copy(), None))
    show("gpu_dense", mi_ba.solve(mi_ba.default_options(max_num_iterations=8, eta=1e-12), sc.copy(), None))
opts = mi_ba.default_options(max_num_iterations=8, eta=1e-12, max_linear_solver_iterations=1000,
                             linear_solver_type=mi_ba.SOLVER_ITERATIVE_SCHUR)
keys = [dict()] if os.environ.get("MI_BA_LIB") != "ab" else [
    dict(), dict(pcg_jcm=0), dict(pcg_point_chunks=0), dict(point_normal_chunks=0), dict(fblock_variant=2),
    dict(pcg_jcm=0, pcg_point_chunks=0, point_normal_chunks=0, fblock_variant=2)]
for kv in keys:
    with mi_ba.Context(opts, sc.copy()) as ctx:
        for k, v in kv.items():
            ctx.set_tuning(k, v)
        show("pcg " + json.dumps(kv), ctx.solve())
