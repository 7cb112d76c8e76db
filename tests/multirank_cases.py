"""Shared cases of the multi-rank LM tests (tests/test_multirank.py and its
worker tests/multirank_worker.py): deterministic scenes, and the gloo host
reducer the ranks plug into mi_ba_context_set_host_reducer."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)
import mi_ba  # noqa: E402

OPENCV_EXTRA = (-0.1, 0.01, 1e-4, -1e-4)


def make_case(name):
    """(scene, semantic or None, options) of a named case."""
    if name == "geo":
        sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 12, 600, track_length=4, rotation_range=0.05,
                                                     extra=OPENCV_EXTRA, seed=7)).gauge()
        return sc, None, mi_ba.default_options(max_num_iterations=15)
    if name == "sem":
        I, size = 4, 120
        sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, I, 50, track_length=I, image_size=size,
                                                     rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=2)).gauge()
        depth, label = mi_ba.render_semantic(sc, size, size, plane_z=1.0, cell=0.5)
        pairs = np.array([(i, j) for i in range(I) for j in range(I) if i != j], np.int32)
        sem = mi_ba.SemanticInput(depth, label, pairs, pixel_step=6)
        rng = np.random.default_rng(2)
        sc.tvec[2:] += rng.uniform(-0.02, 0.02, sc.tvec[2:].shape)
        return sc, sem, mi_ba.default_options(max_num_iterations=10, semantic_weight=0.01, eta=1e-12)
    if name in ("c2", "c2_pcg"):
        # C2 (200 SIMPLE_RADIAL cameras, 50k points, 500k observations) with a
        # semantic term: pairs (i, i + 1), (i, i + 2) sampled every 25 pixels
        # of the 1000 x 1000 maps (640k samples), 5 LM iterations; exact Schur
        # (nf = 1593, S summed in bands) or ITERATIVE_SCHUR at the bench's
        # N > 1 settings (eta 0.1)
        I = 200
        sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, I, 50_000, track_length=10,
                                                     rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=0)).gauge()
        depth, label = mi_ba.render_semantic(sc, 1000, 1000, plane_z=1.0, cell=0.1)
        pairs = np.array([(i, (i + d) % I) for i in range(I) for d in (1, 2)], np.int32)
        sem = mi_ba.SemanticInput(depth, label, pairs, pixel_step=25)
        opts = mi_ba.default_options(max_num_iterations=5)
        if name == "c2_pcg":
            opts.linear_solver_type = mi_ba.SOLVER_ITERATIVE_SCHUR
        return sc, sem, opts
    if name in ("geo_pcg", "sem_pcg"):
        # ITERATIVE_SCHUR: one nf-vector all-reduce per Schur product; eta small
        # so the linear solves are exact to rounding
        sc, sem, opts = make_case(name[:3])
        opts.linear_solver_type = mi_ba.SOLVER_ITERATIVE_SCHUR
        opts.eta = 1e-12
        opts.max_linear_solver_iterations = 500
        return sc, sem, opts
    raise KeyError(name)


def gloo_reducer():
    """In-place sum of a float64 numpy array over the default torch.distributed group."""
    import torch
    import torch.distributed as dist

    def reduce_inplace(a):
        t = torch.from_numpy(a)  # shares the library's host buffer
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return reduce_inplace
