"""CPU BA-iteration time of the oracle's LM (dense Schur, the 'port' CPU
restatement, not Ceres) on a BASELINE config — the bench's BA-iteration
workload, semantic term included — beside the GPU solver's on the same
problem; one JSON line.  The oracle runs with OMP_NUM_THREADS threads
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
ap.add_argument("--geometric-only", action="store_true",
                help="drop the config's semantic term (default: the bench's workload, semantic term included)")
args = ap.parse_args()
c = bench.CONFIGS[args.config]
# the bench's own scene and semantic input (bench.build_shard), so the CPU and
# GPU iterations run the BA-iteration figure's workload
sc, sem = bench.build_shard(c, 0, 1)
if args.geometric_only:
    sem = None
opts = mi_ba.default_options(max_num_iterations=args.iters)
oracle.use_lapack_factor(True)  # the oracle's own O(n^3) Cholesky takes minutes at nf ~ 12 000
t0 = time.perf_counter()
oracle.solve(mi_ba.default_options(max_num_iterations=0), sc.copy(), sem)
t_setup = time.perf_counter() - t0
t0 = time.perf_counter()
s = oracle.solve(opts, sc.copy(), sem)
wall = time.perf_counter() - t0 - t_setup
its = max(1, s.num_successful_steps + s.num_unsuccessful_steps)
out = {"workload": f"{args.config}: {c['desc']}" + (" (geometric part)" if sem is None else "") +
                   ", exact dense-Schur LM (the bench's BA-iteration workload)", "iterations": its,
       "cpu_ms_per_iteration": 1e3 * wall / its, "cpu_threads": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count())),
       "cpu_kind": "port (oracle/ C++/OpenMP dense-Schur LM, its S factored by LAPACK dpotrf; not Ceres)",
       "cpu_setup_s": t_setup, "cpu_final_cost": s.final_cost,
       "num_semantic_residuals": int(s.num_semantic_residuals)}
if not args.no_gpu:
    # the GPU solve twice, the second reported: the first pays the lazy
    # code-object loads of every LM kernel (bench.py warms them on a small scene)
    for _ in range(2):
        with mi_ba.Context(opts, sc.copy(), sem) as ctx:
            g = ctx.solve()
    out.update({"gpu_ms_per_iteration": 1e3 * g.total_time_in_seconds / max(1, g.num_successful_steps +
                                                                             g.num_unsuccessful_steps),
                "gpu_final_cost": g.final_cost})
print(json.dumps(out), flush=True)
