"""CPU BA-iteration time of the oracle's LM (dense Schur, the 'port' CPU
restatement, not Ceres) on a BASELINE config, beside the GPU solver's on the
same problem; one JSON line.  The oracle runs with OMP_NUM_THREADS threads
(the job's CPU share on the GPU boxes).
    python tools/cpu_ba_iteration.py [--config C4] [--iters 1] [--no-gpu]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import oracle  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C4")
ap.add_argument("--iters", type=int, default=1)
ap.add_argument("--no-gpu", action="store_true")
args = ap.parse_args()
c = bench.CONFIGS[args.config]
sc = mi_ba.generate_scene(mi_ba.synth_config(c["model"], c["images"], c["points"], track_length=c["track"],
                                             rotation_range=0.05, extra=c["extra"])).gauge()
opts = mi_ba.default_options(max_num_iterations=args.iters)
t0 = time.perf_counter()
oracle.solve(mi_ba.default_options(max_num_iterations=0), sc.copy())
t_setup = time.perf_counter() - t0
t0 = time.perf_counter()
s = oracle.solve(opts, sc.copy())
wall = time.perf_counter() - t0 - t_setup
its = max(1, s.num_successful_steps + s.num_unsuccessful_steps)
out = {"workload": f"{args.config}: {c['desc']} (geometric part), exact dense-Schur LM", "iterations": its,
       "cpu_ms_per_iteration": 1e3 * wall / its, "cpu_threads": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count())),
       "cpu_kind": "port (oracle/ C++/OpenMP dense-Schur LM, not Ceres)", "cpu_final_cost": s.final_cost}
if not args.no_gpu:
    with mi_ba.Context(opts, sc.copy()) as ctx:
        g = ctx.solve()
    out.update({"gpu_ms_per_iteration": 1e3 * g.total_time_in_seconds / max(1, g.num_successful_steps +
                                                                             g.num_unsuccessful_steps),
                "gpu_final_cost": g.final_cost})
print(json.dumps(out), flush=True)
