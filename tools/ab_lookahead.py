"""A/B of the look-ahead Cholesky (tuning key cholesky_lookahead) on a 3-iteration C4 LM run:
final cost and wall time with the side-stream factor on and off.   python tools/ab_lookahead.py
"""
import sys, json, time
import os as _os
_os.environ.setdefault("MI_BA_LIB", "ab")  # A/B variants: the tools-only build (make ab)
sys.path.insert(0, "semantic-bundle-adjustment-colmap_amd"); sys.path.insert(0, ".")
import mi_ba, bench
cfg = dict(bench.CONFIGS["C4"])
c = mi_ba.synth_config(cfg["model"], cfg["images"], cfg["points"], track_length=cfg["track"], rotation_range=0.05, extra=cfg["extra"])
sc = mi_ba.generate_scene(c).gauge()
for la in (1, 0):
    with mi_ba.Context(mi_ba.default_options(max_num_iterations=3), sc.copy()) as ctx:
        ctx.set_tuning("cholesky_lookahead", la)
        t = time.time(); s = ctx.solve(); dt = time.time() - t
        print(json.dumps({"lookahead": la, "final_cost": repr(s.final_cost), "succ": s.num_successful_steps, "unsucc": s.num_unsuccessful_steps, "s": dt}), flush=True)
