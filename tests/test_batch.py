"""Many independent problems at once (mi_ba_solve_batch): the incremental
mapper's local bundle adjustments (src/sfm/incremental_mapper.cc:560-666
AdjustLocalBundle: a handful of images, some poses constant, SOFT_L1 loss,
points whose tracks leave the local set held constant by SetUp) solved
concurrently on their own contexts and streams.

Pass: every problem reaches the result of solving it alone with mi_ba_solve
(same successful / unsuccessful step counts, final cost within 1e-9
relative, parameters within 1e-8), and a problem without residuals reports
MI_BA_ERR_NO_RESIDUALS without disturbing the others.
"""
import numpy as np
import pytest

import mi_ba

pytestmark = pytest.mark.gpu


def local_problem(seed):
    rng = np.random.default_rng(seed)
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 16, 1200, track_length=5, rotation_range=0.05,
                                                 extra=(0.05, 0, 0, 0), noise=2.0, seed=seed))
    I = sc.num_images
    local = rng.choice(I, 6, replace=False)
    sc.image_in_config = np.zeros(I, np.uint8)
    sc.image_in_config[local] = 1
    sc.image_constant_pose = np.zeros(I, np.uint8)
    sc.image_constant_pose[local[:2]] = 1          # the mapper fixes some poses of the local set
    sc.camera_constant = np.zeros(sc.num_cameras, np.uint8)
    sc.camera_constant[local[2]] = 1
    return sc


def options():
    return mi_ba.default_options(loss_function_type=mi_ba.LOSS_SOFT_L1, loss_function_scale=1.0,
                                 max_num_iterations=25)


def test_batch_matches_one_by_one(gpu):
    scenes = [local_problem(100 + k) for k in range(12)]
    solo = []
    for sc in scenes:
        a = sc.copy()
        solo.append((mi_ba.solve(options(), a), a))
    batch = [sc.copy() for sc in scenes]
    st, sums = mi_ba.solve_batch(options(), batch, max_concurrent=6)
    assert all(s == 0 for s in st), st
    for (s_o, a), s_b, b in zip(solo, sums, batch):
        assert (s_b.num_successful_steps, s_b.num_unsuccessful_steps) == \
            (s_o.num_successful_steps, s_o.num_unsuccessful_steps)
        assert abs(s_b.final_cost - s_o.final_cost) <= 1e-9 * s_o.final_cost
        assert s_b.final_cost < s_b.initial_cost
        assert np.abs(b.xyz - a.xyz).max() <= 1e-8
        assert np.abs(b.qvec - a.qvec).max() <= 1e-8
        assert np.abs(b.camera_params - a.camera_params).max() <= 1e-8 * np.abs(a.camera_params).max()


def test_batch_reports_per_problem_status(gpu):
    scenes = [local_problem(200 + k) for k in range(4)]
    empty = scenes[2]
    empty.obs_xy, empty.obs_image, empty.obs_point = empty.obs_xy[:0], empty.obs_image[:0], empty.obs_point[:0]
    st, sums = mi_ba.solve_batch([options()] * 4, scenes, max_concurrent=4)
    assert st[2] == mi_ba.ERR_NO_RESIDUALS
    assert [st[k] for k in (0, 1, 3)] == [0, 0, 0]
    assert all(sums[k].final_cost < sums[k].initial_cost for k in (0, 1, 3))


def test_arena_sequence_matches_fresh_solves(gpu):
    """mi_ba_solve_in on one recycled context over problems that grow and
    shrink (device arrays re-used in place) and switch between the exact and
    the iterative solver: each result equals a fresh mi_ba_solve."""
    probs = [local_problem(300), local_problem(301)]
    big = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 30, 4000, track_length=6, rotation_range=0.05,
                                                  extra=(-0.1, 0.01, 1e-4, -1e-4), seed=302)).gauge()
    probs = [probs[0], big, probs[1], big]
    opts = [options(), mi_ba.default_options(max_num_iterations=10), options(),
            mi_ba.default_options(max_num_iterations=10, linear_solver_type=mi_ba.SOLVER_ITERATIVE_SCHUR,
                                  eta=1e-12, max_linear_solver_iterations=1000)]
    with mi_ba.Arena() as arena:
        for o, sc in zip(opts, probs):
            a, b = sc.copy(), sc.copy()
            s_f = mi_ba.solve(o, a)
            s_a = arena.solve(o, b)
            assert (s_a.num_successful_steps, s_a.num_unsuccessful_steps) == \
                (s_f.num_successful_steps, s_f.num_unsuccessful_steps)
            assert abs(s_a.final_cost - s_f.final_cost) <= 1e-9 * s_f.final_cost
            assert np.abs(b.xyz - a.xyz).max() <= 1e-8
