"""Repeats tests/test_batch.py's batch-vs-solo comparison (12 local problems,
6 concurrent workers on recycled contexts) and counts mismatching problems.
    python tools/stress_batch.py [--rounds 10]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mi_ba  # noqa: E402
from test_batch import local_problem, options  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=10)
args = ap.parse_args()
scenes = [local_problem(100 + k) for k in range(12)]
solo = []
for sc in scenes:
    a = sc.copy()
    solo.append((mi_ba.solve(options(), a), a))
bad_total = 0
for rnd in range(args.rounds):
    batch = [sc.copy() for sc in scenes]
    st, sums = mi_ba.solve_batch(options(), batch, max_concurrent=6)
    bad = []
    for k, ((s_o, a), s_b, b) in enumerate(zip(solo, sums, batch)):
        same = ((s_b.num_successful_steps, s_b.num_unsuccessful_steps) ==
                (s_o.num_successful_steps, s_o.num_unsuccessful_steps) and
                abs(s_b.final_cost - s_o.final_cost) <= 1e-9 * s_o.final_cost and
                np.abs(b.xyz - a.xyz).max() <= 1e-8)
        if not same:
            bad.append((k, s_b.num_successful_steps, s_b.num_unsuccessful_steps, s_o.num_successful_steps,
                        s_o.num_unsuccessful_steps, s_b.final_cost, s_o.final_cost))
    bad_total += len(bad)
    print(json.dumps({"round": rnd, "statuses": list(st), "mismatches": bad}), flush=True)
print(json.dumps({"rounds": args.rounds, "mismatching_problems": bad_total}), flush=True)
