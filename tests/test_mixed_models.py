"""Per-camera camera models (SURVEY 8b model_id[C]; the reference dispatches
the model per camera: camera_models.h:117-141, bundle_adjustment.cc:396-406).

CPU (no GPU needed): the product's host problem assembly against the
oracle's for mixed reconstructions (reduced counts, effective parameters,
camera tangent width).  GPU: residuals / Jacobians of every block against
the oracle's dual numbers (the same tolerances as test_gpu_parity.py),
end-to-end LM parity, semantic samples of pairs whose cameras differ in
model bitwise, and camera_model_ids with a single model bitwise equal to the
camera_model path.
"""
import numpy as np
import pytest

import mi_ba
import oracle

ALL = [mi_ba.SIMPLE_PINHOLE, mi_ba.PINHOLE, mi_ba.SIMPLE_RADIAL, mi_ba.RADIAL, mi_ba.OPENCV]


def mixed_scene(models=ALL, images=10, points=600, track=5, seed=0):
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, images, points, track_length=track,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=seed))
    return mi_ba.convert_cameras(sc, models).gauge()


@pytest.mark.parametrize("flags", [dict(), dict(refine_principal_point=1), dict(refine_extra_params=0),
                                   dict(refine_focal_length=0, refine_extra_params=0)])
def test_setup_counts_match_oracle(flags):
    sc = mixed_scene()
    sc.camera_constant = np.zeros(sc.num_cameras, np.uint8)
    sc.camera_constant[3] = 1
    opts = mi_ba.default_options(**flags)
    a = mi_ba.setup_stats(opts, sc.copy())
    b = oracle.setup_stats(opts, sc.copy())
    for f in ("num_residual_blocks", "num_residuals_reduced", "num_effective_parameters_reduced",
              "num_variable_cameras", "camera_tangent_size"):
        assert getattr(a, f) == getattr(b, f), f
    # widest refined-intrinsics set: OPENCV (8 params) under these flags
    expect = {(): 6, ("refine_principal_point",): 8, ("refine_extra_params",): 2,
              ("refine_extra_params", "refine_focal_length"): 0}[tuple(sorted(flags))]
    assert a.camera_tangent_size == expect


def test_unknown_model_id_rejected():
    sc = mixed_scene()
    sc.camera_models[2] = 11  # FULL_OPENCV: not in this build
    with pytest.raises(mi_ba.MiBaError) as e:
        mi_ba.setup_stats(mi_ba.default_options(), sc)
    assert e.value.status == mi_ba.ERR_UNSUPPORTED


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [dict(), dict(refine_principal_point=1),
                                   dict(loss_function_type=mi_ba.LOSS_CAUCHY, loss_function_scale=2.0)])
def test_mixed_jacobian_parity(gpu, flags):
    from test_gpu_parity import compare_jacobians
    sc = mixed_scene(seed=1)
    assert compare_jacobians(mi_ba.default_options(**flags), sc) > 1000


@pytest.mark.gpu
def test_mixed_lm_parity(gpu):
    from test_gpu_parity import assert_solve_parity
    sc = mixed_scene(images=12, points=1500, seed=2)
    # the descent (12 iterations): every accept / reject decision equal
    s_o, s_g, a, b = assert_solve_parity(mi_ba.default_options(max_num_iterations=12), sc)
    assert (s_g.num_successful_steps, s_g.num_unsuccessful_steps) == \
        (s_o.num_successful_steps, s_o.num_unsuccessful_steps)
    assert s_g.final_cost < s_g.initial_cost
    assert np.abs(b.camera_params - a.camera_params).max() <= 1e-5 * np.abs(a.camera_params).max()
    # converged (20 iterations): decisions compare cost changes at the rounding
    # level of the sum (as test_c2_converged_lm_parity), so the cost only
    assert_solve_parity(mi_ba.default_options(max_num_iterations=20), sc)


@pytest.mark.gpu
def test_single_model_ids_bitwise_equal(gpu):
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 8, 800, track_length=5, rotation_range=0.05,
                                                 extra=(-0.1, 0.01, 1e-4, -1e-4), seed=3)).gauge()
    ids = sc.copy()
    ids.camera_models = np.full(sc.num_cameras, mi_ba.OPENCV, np.int32)
    ids.camera_params = ids.camera_params.reshape(-1)
    out = []
    for s in (sc, ids):
        with mi_ba.Context(mi_ba.default_options(), s.copy()) as ctx:
            ctx.linearize()
            out.append(ctx.download_jacobian())
    for x, y in zip(*out):
        assert np.array_equal(x, y)


@pytest.mark.gpu
def test_mixed_semantic_bitwise(gpu):
    from test_gpu_scale import semantic_input
    sc = mixed_scene(images=10, points=200, seed=4)
    sc.obs_xy, sc.obs_image, sc.obs_point = sc.obs_xy[:0], sc.obs_image[:0], sc.obs_point[:0]
    sc.camera_constant = np.ones(sc.num_cameras, np.uint8)
    sem = semantic_input(sc, step=6, pairs_per_image=2, size=120, cell=0.5)
    opts = mi_ba.default_options()
    with mi_ba.Context(opts, sc.copy(), sem) as ctx:
        ctx.evaluate_semantic()
        px_g, st_g, r_g, J_g = ctx.download_semantic()
    px_o, st_o, r_o, J_o = oracle.semantic_eval(opts, sc, sem)
    assert np.array_equal(px_g, px_o)
    same = (st_g == st_o) & (r_g == r_o) & np.all(J_g == J_o, axis=1)
    assert same.mean() >= 0.9999, int((~same).sum())
    assert (st_o == mi_ba.VALID).sum() > 500
    # the semantic LM over mixed-model pairs
    opts = mi_ba.default_options(max_num_iterations=10, eta=1e-12)
    a, b = sc.copy(), sc.copy()
    s_o = oracle.solve(opts, a, sem)
    s_g = mi_ba.solve(opts, b, sem)
    assert abs(s_g.final_cost - s_o.final_cost) <= 1e-6 * s_o.final_cost
