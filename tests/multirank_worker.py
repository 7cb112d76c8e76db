"""One rank of the multi-rank LM test: solves its shard (mi_ba.shard_scene)
with the sums of the reduced camera system and of the LM scalars going
through gloo (mi_ba_context_set_host_reducer); writes its result as JSON."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import multirank_cases as mc  # noqa: E402

import torch.distributed as dist  # noqa: E402

mi_ba = mc.mi_ba


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--case", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank, world_size=a.world)
    sc, sem, opts = mc.make_case(a.case)
    sh, shsem = mi_ba.shard_scene(sc, a.rank, a.world, sem)
    with mi_ba.Context(opts, sh, shsem) as ctx:
        ctx.set_host_reducer(a.rank, a.world, mc.gloo_reducer())
        s = ctx.solve()
        ctx.writeback()
    P = sc.num_points
    p0, p1 = P * a.rank // a.world, P * (a.rank + 1) // a.world
    with open(a.out, "w") as f:
        json.dump({"rank": a.rank, "initial_cost": s.initial_cost, "final_cost": s.final_cost,
                   "successful": s.num_successful_steps, "unsuccessful": s.num_unsuccessful_steps,
                   "qvec": sh.qvec.tolist(), "tvec": sh.tvec.tolist(), "camera_params": sh.camera_params.tolist(),
                   "points": [p0, p1], "xyz": sh.xyz[p0:p1].tolist()}, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
