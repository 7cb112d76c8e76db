"""Mismatch counts of every semantic kernel variant against the oracle for
other Ceres relative steps / distortion (diagnostic for the flat test).
    python tools/check_semantic_regimes.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import os as _os
_os.environ.setdefault("MI_BA_LIB", "ab")  # A/B variants: the tools-only build (make ab)
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mi_ba  # noqa: E402
import oracle  # noqa: E402
from test_gpu_parity import semantic_scene  # noqa: E402

for rel, extra in [(1e-2, None), (3e-3, None), (1e-3, None), (1e-5, None), (1e-3, (-0.6, 0.3, 0.01, -0.01))]:
    sc, sem = semantic_scene(mi_ba.OPENCV, images=4, size=160, step=3, seed=7)
    if extra is not None:
        sc.camera_params[:, 4:8] = extra
    sem.numeric_relative_step_size = rel
    opts = mi_ba.default_options()
    px_o, st_o, r_o, J_o = oracle.semantic_eval(opts, sc, sem)
    out = {"rel_step": rel, "extra": extra, "samples": len(st_o)}
    for v in (0, 1, 4, 5, 6):
        with mi_ba.Context(opts, sc.copy(), sem) as ctx:
            ctx.set_tuning("semantic_variant", v)
            ctx.set_tuning("semantic_diag", 1)
            ctx.evaluate_semantic()
            px_g, st_g, r_g, J_g = ctx.download_semantic()
        d = st_g >= 0x800
        st_g = np.where(d, st_g - 0x1000, st_g)
        bad = ~((st_g == st_o) & (r_g == r_o) & np.all(J_g == J_o, axis=1))
        out[f"v{v}"] = {"bad": int(bad.sum()), "bad_status": int((st_g != st_o).sum()), "bad_r": int((r_g != r_o).sum()),
                        "deferred": int(d.sum()), "bad_nondeferred": int((bad & ~d).sum())}
    print(json.dumps(out), flush=True)
