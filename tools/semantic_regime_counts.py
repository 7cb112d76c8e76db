"""How the C4 semantic samples are decided by the flat pass (bench.py's
shard): cleared without a raster read (label planes), cleared after the
raster read, deferred to the full stencil.
    python tools/semantic_regime_counts.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
sys.path.insert(0, ROOT)
import mi_ba  # noqa: E402
import bench  # noqa: E402

sc, sem = bench.build_shard(bench.CONFIGS["C4"], 0, 1)
with mi_ba.Context(mi_ba.default_options(), sc, sem) as ctx:
    ctx.set_tuning("semantic_diag", 2)
    ctx.evaluate_semantic()
    px, st, r, J = ctx.download_semantic()
st = st.astype(np.int64)
flags = np.full(st.shape, -1, np.int64)
base = np.zeros(st.shape, np.int64)
for b in (10, -1, -2):  # status + 0x1000 (deferred) + 0x4000 (decided without the raster)
    m = np.isin(st - b, [0, 0x1000, 0x4000, 0x5000]) & (flags < 0)
    flags[m] = st[m] - b
    base[m] = b
if (flags < 0).any():
    u, c = np.unique(st[flags < 0], return_counts=True)
    print("unmatched statuses", dict(zip(u.tolist()[:20], c.tolist()[:20])))
    flags[flags < 0] = 0
deferred = (flags & 0x1000) != 0
decided = (flags & 0x4000) != 0
n = len(st)
print(json.dumps({"samples": n, "deferred": float(deferred.mean()), "decided_without_raster": float(decided.mean()),
                  "raster_read_not_deferred": float((~decided & ~deferred).mean()),
                  "status_valid": float((base == 10).mean()), "out_of_bounds": float((base == -1).mean()), "invalid_depth": float((base == -2).mean()), "nonzero_residual": float((r != 0).mean())}))
