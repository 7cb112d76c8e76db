"""GPU parity tests: libmi_ba.so (HIP, gfx950) against the CPU oracle.

Tolerances (f64 throughout):
  * reprojection residuals: |dr| <= 1e-9 px (residuals are O(1) px
    differences of O(1e3) px quantities; 1e-9 is ~5e3 ulp of 1e3)
  * reprojection Jacobian: max|dJ| <= 1e-10 * max(1, max|J|) per block (the
    GPU's analytic derivatives vs the oracle's dual numbers)
  * semantic samples: status, residual and Jacobian bitwise identical on
    >= 99.99% of samples, both built without FMA
  * end-to-end LM: final cost within 1e-6 relative of the oracle's dense-Schur
    LM (BASELINE.json north_star tolerance), parameters within 1e-5 relative
"""
import numpy as np
import pytest

import mi_ba
import oracle

pytestmark = pytest.mark.gpu

MODEL_EXTRA = {
    mi_ba.SIMPLE_PINHOLE: (0, 0, 0, 0),
    mi_ba.PINHOLE: (0, 0, 0, 0),
    mi_ba.SIMPLE_RADIAL: (0.05, 0, 0, 0),
    mi_ba.RADIAL: (0.05, -0.01, 0, 0),
    mi_ba.OPENCV: (-0.1, 0.01, 1e-4, -1e-4),
}


def scene(model, images=6, points=300, track=4, seed=0, rot=0.05):
    sc = mi_ba.generate_scene(mi_ba.synth_config(model, images, points, track_length=track, rotation_range=rot,
                                                 extra=MODEL_EXTRA[model], seed=seed))
    return sc.gauge()


def compare_jacobians(opts, sc):
    bo_o, r_o, J_o = oracle.reproj_eval(opts, sc)
    with mi_ba.Context(opts, sc.copy()) as ctx:
        ctx.linearize()
        bo_g, r_g, J_g = ctx.download_jacobian()
    # oracle has every program block; product keeps the reduced ones
    idx = {int(k): i for i, k in enumerate(bo_o)}
    sel = np.array([idx[int(k)] for k in bo_g])
    assert len(bo_g) > 0
    dr = np.abs(r_g - r_o[sel]).max()
    assert dr <= 1e-9, dr
    Jo = J_o[sel]
    scale = np.maximum(1.0, np.abs(Jo).reshape(len(sel), -1).max(axis=1))
    dj = (np.abs(J_g - Jo).reshape(len(sel), -1).max(axis=1) / scale).max()
    assert dj <= 1e-10, dj
    return len(bo_g)


@pytest.mark.parametrize("model", [mi_ba.SIMPLE_PINHOLE, mi_ba.PINHOLE, mi_ba.SIMPLE_RADIAL, mi_ba.RADIAL,
                                   mi_ba.OPENCV])
def test_reproj_jacobian_parity_models(gpu, model):
    sc = scene(model)
    compare_jacobians(mi_ba.default_options(), sc)
    compare_jacobians(mi_ba.default_options(refine_principal_point=1), sc)


@pytest.mark.parametrize("model", [mi_ba.SIMPLE_RADIAL, mi_ba.OPENCV])
def test_reproj_jacobian_non_unit_quaternions(gpu, model):
    """Poses whose quaternion is not normalised (|q| = 0.98 .. 1.03): the
    rotation columns take the general Dq * PlusJacobian product there (the
    closed form -2[RX]x holds for unit quaternions only), as AutoDiff does."""
    sc = scene(model, images=6, points=300, track=4, seed=4)
    scale = np.array([1.0, 1.0, 1.03, 0.98, 1.0 + 1e-9, 1.01])
    sc.qvec = sc.qvec * scale[:, None]
    compare_jacobians(mi_ba.default_options(), sc)


def test_reproj_jacobian_parity_flags(gpu):
    rng = np.random.default_rng(3)
    for trial in range(6):
        sc = scene(mi_ba.OPENCV, images=7, points=200, track=3, seed=10 + trial)
        I = sc.num_images
        sc.image_in_config = (rng.random(I) < 0.8).astype(np.uint8)
        sc.image_constant_pose = (rng.random(I) < 0.3).astype(np.uint8)
        sc.image_constant_tvec = np.where(sc.image_constant_pose == 0, rng.integers(0, 8, I), 0).astype(np.uint8)
        sc.camera_constant = (rng.random(I) < 0.3).astype(np.uint8)
        sc.point_config = rng.integers(0, 3, sc.num_points).astype(np.uint8)
        opts = mi_ba.default_options(refine_focal_length=int(rng.integers(0, 2)),
                                     refine_extra_params=int(rng.integers(0, 2)),
                                     loss_function_type=int(trial % 3), loss_function_scale=2.0)
        try:
            compare_jacobians(opts, sc)
        except mi_ba.MiBaError as e:
            assert e.status == mi_ba.ERR_NO_RESIDUALS


def test_linearize_cost_matches_oracle(gpu):
    sc = scene(mi_ba.SIMPLE_RADIAL, images=10, points=2000, track=5)
    for loss in (mi_ba.LOSS_TRIVIAL, mi_ba.LOSS_SOFT_L1, mi_ba.LOSS_CAUCHY):
        opts = mi_ba.default_options(loss_function_type=loss, loss_function_scale=1.5, max_num_iterations=0)
        s_o = oracle.solve(opts, sc.copy())
        with mi_ba.Context(opts, sc.copy()) as ctx:
            c = ctx.cost()
        assert abs(c - s_o.initial_cost) <= 1e-12 * abs(s_o.initial_cost)


def assert_solve_parity(opts, sc, semantic=None, rel=1e-6):
    a, b = sc.copy(), sc.copy()
    s_o = oracle.solve(opts, a, semantic)
    s_g = mi_ba.solve(opts, b, semantic)
    assert s_g.num_residuals_reduced == s_o.num_residuals_reduced
    assert s_g.num_effective_parameters_reduced == s_o.num_effective_parameters_reduced
    assert abs(s_g.initial_cost - s_o.initial_cost) <= 1e-12 * s_o.initial_cost
    assert abs(s_g.final_cost - s_o.final_cost) <= rel * s_o.final_cost, (s_g.final_cost, s_o.final_cost)
    return s_o, s_g, a, b


@pytest.mark.parametrize("model", [mi_ba.SIMPLE_PINHOLE, mi_ba.SIMPLE_RADIAL, mi_ba.OPENCV])
def test_solve_parity(gpu, model):
    sc = scene(model, images=8, points=400, track=4)
    opts = mi_ba.default_options(max_num_iterations=100)
    s_o, s_g, a, b = assert_solve_parity(opts, sc)
    # The north-star criterion is the final cost (above).  Parameters are
    # compared at the scale of the scene (unit cube): the two LM runs reduce
    # in different orders (GPU atomics vs a serial CPU loop), so near-flat
    # directions of the OPENCV problem (focal vs distortion vs depth) settle
    # ~1e-6 apart.
    dx = np.abs(b.xyz - a.xyz).max()
    assert dx <= 1e-5, dx
    dk = (np.abs(b.camera_params - a.camera_params) / np.maximum(1.0, np.abs(a.camera_params))).max()
    assert dk <= 1e-6, dk


def test_solve_parity_constant_points(gpu):
    """Points the config holds constant (AddConstantPoint) next to variable
    ones: the back substitution / model-cost pass covers the variable points,
    the blocks of constant points enter the model cost without a point step."""
    sc = scene(mi_ba.SIMPLE_RADIAL, images=8, points=400, track=4)
    rng = np.random.default_rng(3)
    sc.point_config = np.where(rng.uniform(size=sc.num_points) < 0.3, 2, 1).astype(np.uint8)
    opts = mi_ba.default_options(max_num_iterations=50)
    s_o, s_g, a, b = assert_solve_parity(opts, sc)
    const = sc.point_config == 2
    assert np.array_equal(b.xyz[const], sc.xyz[const])
    assert np.abs(b.xyz - a.xyz).max() <= 1e-5


def test_solve_parity_c1_reference_generator(gpu):
    """Config C1 shape: 20-image SIMPLE_PINHOLE scene, every point in every image."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_PINHOLE, 20, 200)).gauge()
    assert_solve_parity(mi_ba.default_options(), sc)


@pytest.mark.parametrize("loss", [mi_ba.LOSS_SOFT_L1, mi_ba.LOSS_CAUCHY])
def test_solve_parity_robust_loss(gpu, loss):
    sc = scene(mi_ba.SIMPLE_RADIAL, images=6, points=300, track=4, seed=5)
    assert_solve_parity(mi_ba.default_options(loss_function_type=loss, loss_function_scale=1.0), sc)


def test_reference_two_view_behaviour(gpu):
    """TestTwoView (bundle_adjustment_test.cc:210-245) on the GPU solver."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 2, 100)).gauge()
    orig = sc.copy()
    s = mi_ba.solve(mi_ba.default_options(), sc)
    assert s.num_residuals_reduced == 400 and s.num_effective_parameters_reduced == 309
    assert s.final_cost < s.initial_cost
    assert np.array_equal(sc.qvec[0], orig.qvec[0]) and np.array_equal(sc.tvec[0], orig.tvec[0])
    assert sc.tvec[1][0] == orig.tvec[1][0]
    assert not np.array_equal(sc.tvec[1], orig.tvec[1]) and not np.array_equal(sc.qvec[1], orig.qvec[1])
    for c in range(2):
        assert sc.camera_params[c][0] != orig.camera_params[c][0]   # focal refined
        assert sc.camera_params[c][3] != orig.camera_params[c][3]   # radial refined
        assert np.array_equal(sc.camera_params[c][1:3], orig.camera_params[c][1:3])
    assert np.all(np.any(sc.xyz != orig.xyz, axis=1))


def test_reference_partially_contained_tracks(gpu):
    """TestPartiallyContainedTracks (bundle_adjustment_test.cc:281-326)."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 3, 100))
    keep = ~((sc.obs_image == 2) & (sc.obs_point == 0))
    sc.obs_xy, sc.obs_image, sc.obs_point = sc.obs_xy[keep], sc.obs_image[keep], sc.obs_point[keep]
    sc.image_in_config = np.array([1, 1, 0], np.uint8)
    sc.image_constant_pose = np.array([1, 1, 0], np.uint8)
    orig = sc.copy()
    s = mi_ba.solve(mi_ba.default_options(), sc)
    assert s.num_residuals_reduced == 400 and s.num_effective_parameters_reduced == 7
    assert not np.array_equal(sc.xyz[0], orig.xyz[0])
    assert np.array_equal(sc.xyz[1:], orig.xyz[1:])
    assert np.array_equal(sc.camera_params[2], orig.camera_params[2])
    assert not np.array_equal(sc.camera_params[0], orig.camera_params[0])


def test_no_residuals_status(gpu):
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 2, 10))
    sc.image_in_config = np.zeros(2, np.uint8)
    with pytest.raises(mi_ba.MiBaError) as e:
        mi_ba.solve(mi_ba.default_options(), sc)
    assert e.value.status == mi_ba.ERR_NO_RESIDUALS


def test_empty_and_single_observation(gpu):
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 2, 1)).gauge()
    compare_jacobians(mi_ba.default_options(), sc)


# ---------------------------------------------------------------------------
# Semantic term
# ---------------------------------------------------------------------------
def semantic_scene(model=mi_ba.SIMPLE_PINHOLE, images=4, size=160, step=4, seed=2):
    sc = mi_ba.generate_scene(mi_ba.synth_config(model, images, 50, track_length=images, image_size=size,
                                                 rotation_range=0.05, extra=MODEL_EXTRA[model], seed=seed))
    sc.gauge()
    sc.camera_constant = np.ones(images, np.uint8)  # SemanticBundleAdjustmentController: constant intrinsics
    depth, label = mi_ba.render_semantic(sc, size, size, plane_z=1.0, cell=0.5)
    pairs = np.array([(i, j) for i in range(images) for j in range(images) if i != j], np.int32)
    sem = mi_ba.SemanticInput(depth, label, pairs, pixel_step=step)
    # perturb poses so that residuals and boundary-crossing Jacobians appear
    rng = np.random.default_rng(seed)
    sc.tvec[2:] += rng.uniform(-0.02, 0.02, sc.tvec[2:].shape)
    return sc, sem


@pytest.mark.parametrize("model", [mi_ba.SIMPLE_PINHOLE, mi_ba.OPENCV])
def test_semantic_parity_bitwise(gpu, model):
    sc, sem = semantic_scene(model)
    opts = mi_ba.default_options()
    px_o, st_o, r_o, J_o = oracle.semantic_eval(opts, sc, sem)
    with mi_ba.Context(opts, sc.copy(), sem) as ctx:
        ctx.evaluate_semantic()
        px_g, st_g, r_g, J_g = ctx.download_semantic()
    assert np.array_equal(px_g, px_o)
    n = len(st_o)
    assert n > 1000
    same = (st_g == st_o) & (r_g == r_o) & np.all(J_g == J_o, axis=1)
    assert same.mean() >= 0.9999, (n, int((~same).sum()))
    assert (st_o == mi_ba.VALID).sum() > 0 and (np.abs(J_o).sum(axis=1) > 0).sum() > 0


@pytest.mark.parametrize("model", [mi_ba.SIMPLE_PINHOLE, mi_ba.SIMPLE_RADIAL, mi_ba.OPENCV])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6])
def test_semantic_kernel_variants_bitwise(gpu, model, variant):
    """Every semantic kernel variant (0 uncontracted per-point route, 1 FMA
    per-point route, 2-4 batched stencil with 1/2/4 parameters per step,
    5 flat test + batched stencil on the gathered samples, 6 flat pass +
    deferred-sample pass)
    reproduces the oracle's samples bit for bit, constant first/second poses
    and a constant tvec component included (gauge)."""
    if variant != 6 and not mi_ba.ab_build():
        pytest.skip("one-kernel A/B route: tools build only (MI_BA_LIB=ab)")
    sc, sem = semantic_scene(model, images=4, size=160, step=3, seed=5)
    opts = mi_ba.default_options()
    px_o, st_o, r_o, J_o = oracle.semantic_eval(opts, sc, sem)
    with mi_ba.Context(opts, sc.copy(), sem) as ctx:
        ctx.set_tuning("semantic_variant", variant)
        ctx.evaluate_semantic()
        px_g, st_g, r_g, J_g = ctx.download_semantic()
    assert np.array_equal(px_g, px_o)
    same = (st_g == st_o) & (r_g == r_o) & np.all(J_g == J_o, axis=1)
    assert same.mean() >= 0.9999, (len(st_o), int((~same).sum()))
    assert (np.abs(J_o).sum(axis=1) > 0).sum() > 0


@pytest.mark.parametrize("rel_step,extra", [(1e-2, None), (1e-5, None), (1e-3, (-0.6, 0.3, 0.01, -0.01))])
def test_semantic_flat_test_regimes(gpu, rel_step, extra):
    """The two-pass route's flat test under other stencil sizes (Ceres
    relative step 1e-2 / 1e-5: wide and tiny perturbation boxes) and strong
    OPENCV distortion (the curvature guard): samples bitwise equal to the
    oracle's whatever share the flat test clears."""
    sc, sem = semantic_scene(mi_ba.OPENCV, images=4, size=160, step=3, seed=7)
    if extra is not None:
        sc.camera_params[:, 4:8] = extra
    sem.numeric_relative_step_size = rel_step
    opts = mi_ba.default_options()
    px_o, st_o, r_o, J_o = oracle.semantic_eval(opts, sc, sem)
    with mi_ba.Context(opts, sc.copy(), sem) as ctx:
        ctx.set_tuning("semantic_variant", 6)
        ctx.set_tuning("semantic_diag", 1)
        ctx.evaluate_semantic()
        px_g, st_g, r_g, J_g = ctx.download_semantic()
    deferred = st_g >= 0x800           # semantic_diag: +0x1000 on deferred samples
    st_g = np.where(deferred, st_g - 0x1000, st_g)
    assert np.array_equal(px_g, px_o)
    same = (st_g == st_o) & (r_g == r_o) & np.all(J_g == J_o, axis=1)
    assert same.mean() >= 0.9999, (len(st_o), int((~same).sum()))
    # every sample with a nonzero Jacobian went through the full stencil
    assert np.all(deferred[np.abs(J_o).sum(axis=1) > 0])


def test_semantic_solve_parity(gpu):
    """Semantic BA (pose-only, constant intrinsics) through both LMs."""
    sc, sem = semantic_scene(mi_ba.SIMPLE_PINHOLE, images=3, size=120, step=4)
    sc.obs_xy = sc.obs_xy[:0]
    sc.obs_image = sc.obs_image[:0]
    sc.obs_point = sc.obs_point[:0]
    opts = mi_ba.default_options(max_num_iterations=20, eta=1e-12)  # exact linear solves: discrete cost
    s_o, s_g, a, b = assert_solve_parity(opts, sc, sem, rel=1e-6)
    assert s_g.num_semantic_residuals == s_o.num_semantic_residuals > 0


def test_combined_geometric_semantic_solve(gpu):
    sc, sem = semantic_scene(mi_ba.SIMPLE_RADIAL, images=4, size=120, step=6)
    sc.camera_constant = None
    opts = mi_ba.default_options(max_num_iterations=30, semantic_weight=0.01, eta=1e-12)
    assert_solve_parity(opts, sc, sem, rel=1e-6)


@pytest.mark.parametrize("loss", [mi_ba.LOSS_SOFT_L1, mi_ba.LOSS_CAUCHY])
def test_semantic_solve_parity_robust_loss(gpu, loss):
    """Robust losses on the semantic residuals (ScaledLoss + the loss's
    Corrector in the pair blocks, semantic.hip) as well as the reprojection
    residuals: the LM against the oracle's."""
    sc, sem = semantic_scene(mi_ba.SIMPLE_RADIAL, images=4, size=120, step=6, seed=4)
    sc.camera_constant = None
    opts = mi_ba.default_options(max_num_iterations=20, semantic_weight=0.05, eta=1e-12,
                                 loss_function_type=loss, loss_function_scale=1.0)
    assert_solve_parity(opts, sc, sem, rel=1e-6)


# ---------------------------------------------------------------------------
# Full-size properties (BASELINE configs) — size-independent checks
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("cfg", ["C2", "C4"])
def test_large_scene_properties(gpu, cfg):
    if cfg == "C2":
        c = mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 200, 50_000, track_length=10, rotation_range=0.05,
                               extra=MODEL_EXTRA[mi_ba.SIMPLE_RADIAL])
    else:
        c = mi_ba.synth_config(mi_ba.OPENCV, 1000, 1_000_000, track_length=10, rotation_range=0.05,
                               extra=MODEL_EXTRA[mi_ba.OPENCV])
    sc = mi_ba.generate_scene(c).gauge()
    opts = mi_ba.default_options()
    with mi_ba.Context(opts, sc) as ctx:
        ctx.linearize()
        bo, r, J = ctx.download_jacobian()
        cost = ctx.cost()
    # every observation becomes exactly one block, point-major
    assert np.array_equal(np.sort(bo), np.arange(sc.num_obs))
    assert np.all(np.diff(sc.obs_point[bo]) >= 0)
    # cost == 0.5 * sum r^2 (TRIVIAL) — a checksum of the residual array
    assert abs(cost - 0.5 * np.sum(r * r)) <= 1e-9 * cost
    # sampled rows against the oracle (sub-problem of the sampled points)
    rng = np.random.default_rng(0)
    pts = np.unique(rng.choice(sc.num_points, 200, replace=False))
    mask = np.isin(sc.obs_point, pts)
    sub = sc.copy()
    sub.obs_xy, sub.obs_image, sub.obs_point = sc.obs_xy[mask], sc.obs_image[mask], sc.obs_point[mask]
    bo_o, r_o, J_o = oracle.reproj_eval(opts, sub)
    obs_idx = np.nonzero(mask)[0][bo_o]
    pos = {int(k): i for i, k in enumerate(bo)}
    sel = np.array([pos[int(k)] for k in obs_idx])
    assert np.abs(r[sel] - r_o).max() <= 1e-9
    scale = np.maximum(1.0, np.abs(J_o).reshape(len(sel), -1).max(axis=1))
    assert (np.abs(J[sel] - J_o).reshape(len(sel), -1).max(axis=1) / scale).max() <= 1e-10


@pytest.mark.parametrize("images", [70, 121])
def test_own_diagonal_cholesky_matches_rocsolver(gpu, images):
    """The hand-written diagonal-block factor (cholesky.cpp diag_panel_kernel /
    diag_update_kernel) against rocsolver_dpotrf inside the same LM run, on
    reduced camera systems spanning several 64-wide sub-panels and (121
    images) two 512-wide panels, with ragged last sub-panels (SIMPLE_RADIAL
    with the gauge: nf = 8 * images - 7).  Tolerance: final cost within 1e-9
    relative, same step counts."""
    sc = scene(mi_ba.SIMPLE_RADIAL, images=images, points=2000, track=6, seed=3)
    opts = mi_ba.default_options(max_num_iterations=8)
    out = []
    for own in (1, 0):
        with mi_ba.Context(opts, sc.copy()) as ctx:
            ctx.set_tuning("cholesky_own_diag", own)
            out.append(ctx.solve())
    a, b = out
    assert a.num_successful_steps == b.num_successful_steps
    assert a.num_unsuccessful_steps == b.num_unsuccessful_steps
    assert abs(a.final_cost - b.final_cost) <= 1e-9 * b.final_cost, (a.final_cost, b.final_cost)
    assert a.final_cost < a.initial_cost


def test_linearize_overlap_modes_agree(gpu):
    """The linearization step's stream layouts — all on one stream (0), the
    semantic kernels beside the reprojection kernel (1), the flat pass first
    and the deferred-sample pass beside the reprojection kernel (2) — give the
    same cost and drive the same LM (pair blocks are atomic sums: order-only
    differences)."""
    if not mi_ba.ab_build():
        pytest.skip("stream layouts 1 / 2 (measured slower): tools build only (MI_BA_LIB=ab)")
    sc, sem = semantic_scene(mi_ba.SIMPLE_RADIAL, images=6, size=160, step=3, seed=9)
    sc.camera_constant = None
    opts = mi_ba.default_options(max_num_iterations=10, semantic_weight=0.01, eta=1e-12)
    res = []
    for ov in (0, 1, 2):
        with mi_ba.Context(opts, sc.copy(), sem) as ctx:
            ctx.set_tuning("linearize_overlap", ov)
            ctx.linearize()
            res.append(ctx.solve())
    for s in res[1:]:
        assert abs(s.initial_cost - res[0].initial_cost) <= 1e-12 * res[0].initial_cost
        assert (s.num_successful_steps, s.num_unsuccessful_steps) == (res[0].num_successful_steps,
                                                                      res[0].num_unsuccessful_steps)
        assert abs(s.final_cost - res[0].final_cost) <= 1e-9 * res[0].final_cost
    assert res[0].final_cost < res[0].initial_cost
