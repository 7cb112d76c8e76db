"""One rank of the full-size C5 rehearsal (tests/test_c5_rehearsal.py): the
C4 scene (bench.build_shard, seed 0) point- and pair-sharded across `world`
ranks that share the one GPU, the LM's sums through gloo
(mi_ba_context_set_host_reducer), the solver bench.py runs at N > 1
(ITERATIVE_SCHUR + SCHUR_JACOBI at the default eta).  world = 1 (no
torch.distributed) is the unsharded reference run.  Writes its summary as
JSON."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
import multirank_cases as mc  # noqa: E402
import bench  # noqa: E402

mi_ba = mc.mi_ba


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dist = None
    if a.world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank, world_size=a.world)
    sc, sem = bench.build_shard(bench.CONFIGS["C4"], a.rank, a.world, "strong")
    opts = mi_ba.default_options(max_num_iterations=a.iters, linear_solver_type=mi_ba.SOLVER_ITERATIVE_SCHUR)
    with mi_ba.Context(opts, sc, sem) as ctx:
        if dist is not None:
            ctx.set_host_reducer(a.rank, a.world, mc.gloo_reducer())
        t0 = time.perf_counter()
        s = ctx.solve()
        solve_s = time.perf_counter() - t0
        ctx.writeback()
    with open(a.out, "w") as f:
        json.dump({"rank": a.rank, "world": a.world, "eta": opts.eta, "initial_cost": s.initial_cost,
                   "final_cost": s.final_cost, "successful": s.num_successful_steps,
                   "unsuccessful": s.num_unsuccessful_steps, "cg_iterations": s.num_linear_solver_iterations, "solve_s": solve_s,
                   "qvec0": sc.qvec[:50].tolist(), "tvec0": sc.tvec[:50].tolist()}, f)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
