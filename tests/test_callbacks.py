"""Iteration callbacks, the stop flag, and the Cholesky flag-wait timeout at
the C-ABI (mi_ba_options.iteration_callback / stop_flag, ABI 3).

Reference: the controllers install a ceres::IterationCallback that blocks
while the thread is paused and returns SOLVER_TERMINATE_SUCCESSFULLY once it
is stopped (src/controllers/bundle_adjustment.cc:43-61,87-88); SBA / GSBA run
per-iteration snapshot callbacks with update_state_every_iteration
(src/optim/semantic_bundle_adjustment.h:129, .cc:1086-1123).  Ceres 2.1
semantics restated: callbacks run after iteration 0 and after every later
iteration; TERMINATE_SUCCESSFULLY ends with USER_SUCCESS and the state is
written back, ABORT ends with USER_FAILURE and the caller's parameters are
not updated (unless update_state_every_iteration wrote them).

Pass criteria: a solve stopped by a callback at iteration k equals the
max_num_iterations = k solve (same step counts; parameters within 1e-9
relative and costs within 1e-12 relative — the normal-equation reductions use
float atomics, so repeated runs may differ in the last bits); snapshots taken
in the callback equal the k-iteration solves; ABORT leaves the caller's
arrays exactly as they were; a flag wait that runs out
(cholesky_spin_log2 = 0) makes the solve return MI_BA_ERR_HIP.
"""
import threading

import numpy as np
import pytest

import mi_ba

pytestmark = pytest.mark.gpu


def small_scene(seed=0, images=20, points=2000):
    return mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, images, points, track_length=6,
                                                   rotation_range=0.05, extra=(0.05, 0, 0, 0),
                                                   seed=seed)).gauge()


def params(sc):
    return np.concatenate([sc.qvec.ravel(), sc.tvec.ravel(), sc.xyz.ravel(), sc.camera_params.ravel()])


def same(a, b, rel=1e-9):
    return np.abs(a - b).max() <= rel * max(1.0, np.abs(b).max())


def same_cost(a, b, rel=1e-12):
    return abs(a - b) <= rel * abs(b)


@pytest.mark.parametrize("k", [0, 1, 4])
@pytest.mark.parametrize("solver", [mi_ba.SOLVER_DENSE_SCHUR, mi_ba.SOLVER_ITERATIVE_SCHUR])
def test_terminate_at_k_equals_max_iterations_k(gpu, k, solver):
    sc = small_scene()
    ref = sc.copy()
    s_ref = mi_ba.solve(mi_ba.default_options(max_num_iterations=k, linear_solver_type=solver), ref)
    assert s_ref.termination_type == mi_ba.NO_CONVERGENCE
    seen = []

    def cb(it):
        seen.append((it.iteration, it.cost, it.step_is_successful))
        return mi_ba.SOLVER_TERMINATE_SUCCESSFULLY if it.iteration == k else mi_ba.SOLVER_CONTINUE

    got = sc.copy()
    o = mi_ba.default_options(linear_solver_type=solver).set_callback(cb)
    s = mi_ba.solve(o, got)
    assert s.termination_type == mi_ba.USER_SUCCESS
    assert [x[0] for x in seen] == list(range(k + 1))
    assert same(params(got), params(ref))
    assert same_cost(s.final_cost, s_ref.final_cost)
    assert (s.num_successful_steps, s.num_unsuccessful_steps) == (s_ref.num_successful_steps,
                                                                  s_ref.num_unsuccessful_steps)
    # the summary's cost is the cost at the accepted point: iteration 0 = initial
    assert seen[0][1] == s.initial_cost
    assert seen[-1][1] == s.final_cost


def test_abort_keeps_caller_parameters(gpu):
    sc = small_scene(1)
    orig = sc.copy()
    o = mi_ba.default_options().set_callback(
        lambda it: mi_ba.SOLVER_ABORT if it.iteration == 2 else mi_ba.SOLVER_CONTINUE)
    s = mi_ba.solve(o, sc)
    assert s.termination_type == mi_ba.USER_FAILURE
    # SetUp normalises the config qvecs in place (identity-rotation-free scene:
    # compare against the normalised originals)
    q = orig.qvec / np.linalg.norm(orig.qvec, axis=1, keepdims=True)
    assert np.allclose(sc.qvec, q, rtol=0, atol=1e-15)
    assert np.array_equal(sc.tvec, orig.tvec) and np.array_equal(sc.xyz, orig.xyz)
    assert np.array_equal(sc.camera_params, orig.camera_params)


def test_update_state_every_iteration_snapshots(gpu):
    """SBA snapshot semantics: in the callback the caller's arrays hold the
    current point — the max_num_iterations = i solve at iteration i."""
    sc = small_scene(2)
    snaps = []
    o = mi_ba.default_options(max_num_iterations=3)
    got = sc.copy()

    def cb(it):
        snaps.append(params(got).copy())

    o.set_callback(cb, update_state_every_iteration=True)
    mi_ba.solve(o, got)
    assert len(snaps) == 4  # iterations 0..3 (the callback runs before the max-iteration check)
    for i in range(4):
        ref = sc.copy()
        mi_ba.solve(mi_ba.default_options(max_num_iterations=i), ref)
        assert same(snaps[i], params(ref)), i
    assert np.array_equal(snaps[3], params(got))


def test_semantic_snapshot_callback(gpu):
    """The SBA callback path (pose-only semantic problem) with snapshots."""
    sc = small_scene(3, images=8, points=500)
    sc.camera_constant = np.ones(sc.num_images, np.uint8)
    depth, label = mi_ba.render_semantic(sc, 160, 160, plane_z=1.0, cell=0.1)
    pairs = np.array([(i, (i + 1) % 8) for i in range(8)], np.int32)
    sem = mi_ba.SemanticInput(depth, label, pairs, pixel_step=4)
    got = sc.copy()
    costs = []
    poses = []

    def cb(it):
        costs.append(it.cost)
        poses.append(got.qvec.copy())
        return mi_ba.SOLVER_TERMINATE_SUCCESSFULLY if it.iteration == 2 else mi_ba.SOLVER_CONTINUE

    s = mi_ba.solve(mi_ba.default_options().set_callback(cb, update_state_every_iteration=True), got, sem)
    assert s.termination_type == mi_ba.USER_SUCCESS
    assert len(costs) == 3 and costs[0] == s.initial_cost and costs[-1] == s.final_cost
    ref = sc.copy()
    mi_ba.solve(mi_ba.default_options(max_num_iterations=2), ref, sem)
    assert same(poses[-1], ref.qvec)
    assert np.array_equal(got.qvec, poses[-1])


def test_stop_flag(gpu):
    """Thread::Stop through the stop flag: set before the solve, the LM stops
    after iteration 0 with USER_SUCCESS; set from another thread during a
    solve, it stops at an iteration boundary."""
    sc = small_scene(4)
    flag = np.array([mi_ba.SOLVER_TERMINATE_SUCCESSFULLY], np.int32)
    s = mi_ba.solve(mi_ba.default_options().set_stop_flag(flag), sc.copy())
    assert s.termination_type == mi_ba.USER_SUCCESS
    assert s.num_successful_steps + s.num_unsuccessful_steps == 0
    flag[0] = mi_ba.SOLVER_ABORT
    s = mi_ba.solve(mi_ba.default_options().set_stop_flag(flag), sc.copy())
    assert s.termination_type == mi_ba.USER_FAILURE
    # from another thread, released by the callback of iteration 3
    flag[0] = 0
    go = threading.Event()
    done = threading.Event()

    def stopper():
        go.wait(30)
        flag[0] = mi_ba.SOLVER_TERMINATE_SUCCESSFULLY
        done.set()

    t = threading.Thread(target=stopper)
    t.start()

    def cb(it):
        if it.iteration == 3:
            go.set()
            done.wait(30)

    o = mi_ba.default_options(max_num_iterations=50).set_stop_flag(flag).set_callback(cb)
    s = mi_ba.solve(o, sc.copy())
    t.join()
    assert s.termination_type == mi_ba.USER_SUCCESS
    assert s.num_successful_steps + s.num_unsuccessful_steps == 4  # the flag is read before iteration 4's callback


def test_cholesky_wait_timeout_is_an_error(gpu):
    """A flag wait of the one-launch panel factor / sync-free sweeps that runs
    out is reported (MI_BA_ERR_HIP), never used as a factor: with no polling
    (cholesky_spin_log2 = 0) every wait whose flag is not already set runs
    out.  The next solve on a fresh context is unaffected."""
    sc = small_scene(5, images=40)  # nf = 40 * 8 - 7 = 313: 5 tiles, 5 sweep blocks
    o = mi_ba.default_options(linear_solver_type=mi_ba.SOLVER_DENSE_SCHUR, max_num_iterations=3)
    with mi_ba.Context(o, sc.copy()) as ctx:
        ctx.set_tuning("cholesky_spin_log2", 0)
        with pytest.raises(mi_ba.MiBaError) as e:
            ctx.solve()
        assert e.value.status == mi_ba.ERR_HIP
    with mi_ba.Context(o, sc.copy()) as ctx:
        s = ctx.solve()
        assert s.num_successful_steps >= 1 and s.final_cost < s.initial_cost


def test_positive_depth_matches_restatement(gpu):
    """mi_ba_positive_depth (FilterObservationsWithNegativeDepth's test,
    reconstruction.cc:647-665 / projection.cc:191-195) against a numpy
    restatement: points pushed behind some cameras, unregistered images
    kept.  The reference's known answers run in tests/cpp/controllers_test.cc."""
    sc = small_scene(6)
    rng = np.random.default_rng(0)
    pts = rng.choice(sc.num_points, 200, replace=False)
    sc.xyz[pts, 2] = -10.0 - rng.uniform(0.0, 1.0, 200) + rng.choice([0.0, 2.0], 200)
    mask = np.ones(sc.num_images, np.uint8)
    mask[3] = 0
    keep, neg = mi_ba.positive_depth(sc, mask)
    q = sc.qvec / np.linalg.norm(sc.qvec, axis=1, keepdims=True)
    w, x, y, z = q.T
    R2 = np.stack([2 * x * z - 2 * y * w, 2 * y * z + 2 * x * w, 1 - (2 * x * x + 2 * y * y)], 1)
    d = np.einsum("ij,ij->i", R2[sc.obs_image], sc.xyz[sc.obs_point]) + sc.tvec[sc.obs_image, 2]
    want = (d >= np.finfo(float).eps) | (mask[sc.obs_image] == 0)
    assert np.array_equal(keep, want)
    assert neg == int((~want).sum()) and neg > 0
