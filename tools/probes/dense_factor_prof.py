"""Factor + solve a random SPD matrix twice through mi_ba_dense_cholesky (run under rocprofv3).
    python tools/probes/dense_factor_prof.py N"""
import sys
sys.path.insert(0,'semantic-bundle-adjustment-colmap_amd')
import numpy as np, mi_ba
n = int(sys.argv[1])
rng = np.random.default_rng(0)
G = rng.standard_normal((n, 64))
A = G @ G.T / 64 + np.eye(n)
b = rng.standard_normal(n)
for _ in range(2):
    L, x, info = mi_ba.dense_cholesky(A, b)
print("info", info, "resid", np.abs(A @ x - b).max())
