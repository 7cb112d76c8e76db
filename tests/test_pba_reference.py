"""Cross-check against the REFERENCE CODE itself: the reference's PBA CPU
double-precision solver (lib/PBA, ParallelBundleAdjuster's CPU device,
src/optim/bundle_adjustment.cc:559-663), compiled from the reference's own
sources by oracle/Makefile.ref into oracle/_ref/libpba_ref.so.

PBA stores cameras, points and observations as float32, so the scenes are
rounded to float32 first (both solvers then see identical data).  PBA has no
gauge fixing and refines every pose (ParallelBundleAdjuster rejects constant
poses), so the compared problems hold every pose variable; the minimum cost
does not depend on the gauge.

Checks (SIMPLE_RADIAL, one camera per image, focal + k refined):
  * initial cost: the reference's MSE-derived cost vs ours, within 1e-7
    relative (PBA reports its MSE as float32) — every reprojection residual
    of the scene through reference code;
  * converged cost: ours <= PBA's * (1 + 1e-9) and within 1e-5 relative (PBA
    stops on its own delta / gradient thresholds a little above the minimum;
    our cost evaluated at PBA's solution is also >= our minimum).
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
import mi_ba  # noqa: E402
import oracle  # noqa: E402

needs_ref = pytest.mark.skipif(not oracle.ref_available(),
                               reason="oracle/_ref/libpba_ref.so not built (needs /root/reference; parity unpinned)")


def pba_scene(images, points, track, seed):
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, images, points, track_length=track,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=seed))
    for a in ("xyz", "obs_xy", "tvec", "camera_params"):
        setattr(sc, a, getattr(sc, a).astype(np.float32).astype(np.float64))
    sc.image_constant_pose = np.zeros(sc.num_images, np.uint8)
    if sc.image_constant_tvec is not None:
        sc.image_constant_tvec = np.zeros_like(sc.image_constant_tvec)
    return sc


CASES = [(10, 500, 6, 3), (30, 3000, 8, 4)]


@needs_ref
@pytest.mark.parametrize("images,points,track,seed", CASES)
def test_oracle_matches_reference_pba(images, points, track, seed):
    sc = pba_scene(images, points, track, seed)
    ref = sc.copy()
    ic, fc, _ = oracle.pba_ref_solve(ref, max_iterations=300, threads=4)
    s = oracle.solve(mi_ba.default_options(max_num_iterations=200), sc.copy())
    assert abs(s.initial_cost - ic) <= 1e-7 * ic, (s.initial_cost, ic)
    assert s.final_cost <= fc * (1 + 1e-9), (s.final_cost, fc)
    assert (fc - s.final_cost) <= 1e-5 * fc, (s.final_cost, fc)
    at_ref = oracle.solve(mi_ba.default_options(max_num_iterations=0), ref.copy()).initial_cost
    assert at_ref >= s.final_cost * (1 - 1e-12)


@needs_ref
@pytest.mark.gpu
@pytest.mark.parametrize("images,points,track,seed", CASES + [(200, 20000, 10, 5)])
def test_gpu_solver_matches_reference_pba(gpu, images, points, track, seed):
    """The GPU LM (the ParallelBundleAdjuster replacement's solver) against
    the reference PBA on the same float32-rounded problem."""
    sc = pba_scene(images, points, track, seed)
    ref = sc.copy()
    ic, fc, _ = oracle.pba_ref_solve(ref, max_iterations=300, threads=8)
    g = sc.copy()
    s = mi_ba.solve(mi_ba.default_options(max_num_iterations=200), g)
    assert abs(s.initial_cost - ic) <= 1e-7 * ic, (s.initial_cost, ic)
    assert s.final_cost <= fc * (1 + 1e-9), (s.final_cost, fc)
    assert (fc - s.final_cost) <= 1e-5 * fc, (s.final_cost, fc)
