"""A/B of the LM-phase timings at C4 over Cholesky tuning keys (own_diag, lookahead, panel, solve).
    python tools/ab_cholesky.py [comma list of variant indices; 0 = production]"""
import sys, time, json
import os as _os
_os.environ.setdefault("MI_BA_LIB", "ab")  # A/B variants: the tools-only build (make ab)
sys.path.insert(0,'semantic-bundle-adjustment-colmap_amd')
import numpy as np, mi_ba
c = mi_ba.synth_config(mi_ba.OPENCV, 1000, 1_000_000, track_length=10, rotation_range=0.05, extra=(-0.1, 0.01, 1e-4, -1e-4))
sc = mi_ba.generate_scene(c).gauge()
# warm
w = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 30, 300, track_length=5, rotation_range=0.05, extra=(-0.1, 0.01, 1e-4, -1e-4))).gauge()
with mi_ba.Context(mi_ba.default_options(max_num_iterations=2), w) as x: x.solve()
import os
# index 0: the production configuration (one-launch panel factor, sync-free sweeps)
variants = [dict(own=6, la=1, panel=512, solve=2),
            dict(own=1, la=1, panel=512, solve=1), dict(own=2, la=1, panel=512, solve=1),
            dict(own=2, la=1, panel=1024, solve=1), dict(own=3, la=1, panel=512, solve=1),
            dict(own=0, la=1, panel=512, solve=1), dict(own=4, la=1, panel=512, solve=1),
            dict(own=5, la=1, panel=512, solve=1),
            dict(own=1, la=0, panel=512, solve=1), dict(own=1, la=1, panel=1024, solve=1),
            dict(own=1, la=1, panel=256, solve=1)]
if len(sys.argv) > 1:
    variants = [variants[int(k)] for k in sys.argv[1].split(",")]
for v in variants:
    with mi_ba.Context(mi_ba.default_options(max_num_iterations=3), sc.copy()) as ctx:
        ctx.set_tuning("cholesky_own_diag", v["own"]); ctx.set_tuning("cholesky_lookahead", v["la"]); ctx.set_tuning("cholesky_panel", v["panel"]); ctx.set_tuning("cholesky_solve", v["solve"])
        ctx.set_timing(True)
        s = ctx.solve()
        its = s.num_successful_steps + s.num_unsuccessful_steps
        ph = {k: ctx.kernel_time(k) for k in ("cholesky", "cholesky_solve", "schur_build", "fblock", "backsub")}
        print(json.dumps(dict(v, ba_ms=1e3*s.total_time_in_seconds/its, final=s.final_cost, steps=(s.num_successful_steps, s.num_unsuccessful_steps),
                              **{k: round(t[0]/max(1,t[1]),3) for k,t in ph.items()})), flush=True)
