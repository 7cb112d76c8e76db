"""CPU tests: the oracle (and the product's host-side problem assembly) against
the reference's own known answers (tests/golden/reference_known_answers.json,
transcribed from the reference's unit tests; see make_reference_vectors.py).

Mirrors src/base/cost_functions_test.cc, src/base/projection_test.cc,
src/base/camera_models_test.cc and the structural assertions of
src/optim/bundle_adjustment_test.cc.
"""
import json
import os

import numpy as np
import pytest

import mi_ba
import oracle

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_known_answers.json")))


def test_cost_function_known_answers():
    g = GOLD["cost_function"]
    for case in g["cases"]:
        r = oracle.reproj_residual(mi_ba.SIMPLE_PINHOLE, g["qvec"], g["tvec"], case["point3D"], case["camera"],
                                   g["observed"])
        # BOOST_CHECK_EQUAL: exact
        assert r.tolist() == [float(v) for v in case["residual"]], case


def test_projection_known_answer():
    g = GOLD["projection"]
    rng = np.random.default_rng(0)
    X = np.abs(rng.uniform(-1, 1, 3))
    xy = X[:2] / X[2]
    e1 = oracle.squared_reprojection_error(mi_ba.SIMPLE_PINHOLE, g["camera"], xy, X, g["qvec"], g["tvec"])
    assert e1 == 0.0
    e3 = oracle.squared_reprojection_error(mi_ba.SIMPLE_PINHOLE, g["camera"], xy + 1, X, g["qvec"], g["tvec"])
    assert abs(e3 - g["shift_error"]) <= g["close_tol_percent"] / 100 * g["shift_error"]
    # cheirality sentinel (projection.cc:120-123)
    e4 = oracle.squared_reprojection_error(mi_ba.SIMPLE_PINHOLE, g["camera"], xy, -X, g["qvec"], g["tvec"])
    assert e4 == np.finfo(np.float64).max


@pytest.mark.parametrize("name", ["SIMPLE_PINHOLE", "PINHOLE", "SIMPLE_RADIAL", "RADIAL", "OPENCV"])
def test_camera_model_round_trips(name):
    g = GOLD["camera_models"]
    model = mi_ba.MODEL_NAMES[name]
    wg, ig = g["world_grid"], g["image_grid"]
    for params in g["models"][name]:
        for u in np.arange(wg["start"], wg["stop"] + 1e-9, wg["step"]):
            for v in np.arange(wg["start"], wg["stop"] + 1e-9, wg["step"]):
                x, y = oracle.world_to_image(model, params, u, v)
                uu, vv = oracle.image_to_world(model, params, x, y)
                assert abs(uu - u) < wg["tol"] and abs(vv - v) < wg["tol"]
        for x in range(ig["start"], ig["stop"] + 1, ig["step"]):
            for y in range(ig["start"], ig["stop"] + 1, ig["step"]):
                u, v = oracle.image_to_world(model, params, x, y)
                xx, yy = oracle.world_to_image(model, params, u, v)
                assert abs(xx - x) < ig["tol"] and abs(yy - y) < ig["tol"]


def build_case(case):
    """GenerateReconstruction + the case's BundleAdjustmentConfig as a Scene."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, case["images"], case["points"]))
    I, P = case["images"], case["points"]
    if "delete_observation" in case:
        img, p2d = case["delete_observation"]
        keep = ~((sc.obs_image == img) & (sc.obs_point == p2d))
        sc.obs_xy, sc.obs_image, sc.obs_point = sc.obs_xy[keep], sc.obs_image[keep], sc.obs_point[keep]
    cfg = np.zeros(I, np.uint8)
    cfg[case.get("config_images", [])] = 1
    sc.image_in_config = cfg
    sc.image_constant_pose = np.zeros(I, np.uint8)
    sc.image_constant_pose[case.get("constant_pose", [])] = 1
    sc.image_constant_tvec = np.zeros(I, np.uint8)
    for k, idxs in case.get("constant_tvec", {}).items():
        sc.image_constant_tvec[int(k)] = sum(1 << i for i in idxs)
    sc.camera_constant = np.zeros(I, np.uint8)
    sc.camera_constant[case.get("constant_cameras", [])] = 1
    pc = np.zeros(P, np.uint8)
    for pid in case.get("constant_points", []):
        pc[pid - 1] = 2  # point3D_t ids are 1-based in COLMAP
    if "add_variable_point_of" in case:
        pc[case["add_variable_point_of"][1]] = 1
    if "add_constant_point_of" in case:
        pc[case["add_constant_point_of"][1]] = 2
    sc.point_config = pc
    opts = mi_ba.default_options(**case.get("options", {}))
    return sc, opts


@pytest.mark.parametrize("case", [c for c in GOLD["bundle_adjustment"]["cases"] if "steps" not in c],
                         ids=lambda c: c["name"])
@pytest.mark.parametrize("impl", ["oracle", "product_setup"])
def test_bundle_adjustment_counts(case, impl):
    sc, opts = build_case(case)
    info = oracle.setup_stats(opts, sc) if impl == "oracle" else mi_ba.setup_stats(opts, sc)
    assert info.num_residuals_reduced == case["num_residuals_reduced"]
    assert info.num_effective_parameters_reduced == case["num_effective_parameters_reduced"]


@pytest.mark.parametrize("impl", ["oracle", "product_setup"])
def test_config_num_observations(impl):
    """TestConfigNumObservations: NumResiduals = 2 * (image obs + out-of-set track obs of config points)."""
    case = [c for c in GOLD["bundle_adjustment"]["cases"] if c["name"] == "TestConfigNumObservations"][0]
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, case["images"], case["points"]))
    cfg = np.zeros(case["images"], np.uint8)
    pc = np.zeros(case["points"], np.uint8)
    for step in case["steps"]:
        cfg[step.get("add_images", [])] = 1
        for pid in step.get("add_variable_points", []):
            pc[pid - 1] = 1
        for pid in step.get("add_constant_points", []):
            pc[pid - 1] = 2
        s = sc.copy()
        s.image_in_config = cfg.copy()
        s.point_config = pc.copy()
        # every camera variable, no constant poses: all residual blocks reduced
        opts = mi_ba.default_options()
        info = oracle.setup_stats(opts, s) if impl == "oracle" else mi_ba.setup_stats(opts, s)
        assert 2 * info.num_residual_blocks == step["num_residuals"]


def test_product_setup_matches_oracle_random_configs():
    rng = np.random.default_rng(1)
    for trial in range(20):
        I = int(rng.integers(2, 6))
        sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, I, 40, track_length=int(rng.integers(2, I + 1)),
                                                     rotation_range=0.05, seed=trial))
        sc.image_in_config = (rng.random(I) < 0.7).astype(np.uint8)
        sc.image_constant_pose = (rng.random(I) < 0.3).astype(np.uint8)
        sc.image_constant_tvec = np.where(sc.image_constant_pose == 0, rng.integers(0, 8, I), 0).astype(np.uint8)
        sc.camera_constant = (rng.random(I) < 0.3).astype(np.uint8)
        sc.point_config = rng.integers(0, 3, 40).astype(np.uint8)
        opts = mi_ba.default_options(refine_focal_length=int(rng.integers(0, 2)),
                                     refine_principal_point=int(rng.integers(0, 2)),
                                     refine_extra_params=int(rng.integers(0, 2)),
                                     refine_extrinsics=int(rng.random() < 0.8))
        a = oracle.setup_stats(opts, sc)
        b = mi_ba.setup_stats(opts, sc)
        for f, _ in mi_ba.SetupInfo._fields_:
            assert getattr(a, f) == getattr(b, f), (trial, f)


def test_oracle_jacobian_matches_finite_differences():
    """The oracle's dual-number Jacobian vs central differences of its residual."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 3, 20, track_length=3, rotation_range=0.1,
                                                 extra=(-0.1, 0.01, 1e-4, -1e-4)))
    sc.gauge()
    opts = mi_ba.default_options(refine_principal_point=1)
    bo, r, J = oracle.reproj_eval(opts, sc)
    h = 1e-6
    for b in range(0, len(bo), 7):
        k = bo[b]
        img, pt = sc.obs_image[k], sc.obs_point[k]
        cam = sc.image_camera[img]
        if sc.image_constant_pose[img]:
            continue
        # point columns
        for c in range(3):
            Xp = sc.xyz[pt].copy(); Xp[c] += h
            Xm = sc.xyz[pt].copy(); Xm[c] -= h
            rp = oracle.reproj_residual(sc.camera_model, sc.qvec[img], sc.tvec[img], Xp, sc.camera_params[cam],
                                        sc.obs_xy[k])
            rm = oracle.reproj_residual(sc.camera_model, sc.qvec[img], sc.tvec[img], Xm, sc.camera_params[cam],
                                        sc.obs_xy[k])
            fd = (rp - rm) / (2 * h)
            assert np.allclose(fd, J[b, :, 6 + c], rtol=1e-5, atol=1e-4)
        # rotation tangent: q' = Plus(q, d)
        q = sc.qvec[img] / np.linalg.norm(sc.qvec[img])
        for c in range(3):
            d = np.zeros(3); d[c] = h
            def plus(dd):
                n = np.linalg.norm(dd)
                a = np.concatenate([[np.cos(n)], np.sin(n) / n * dd])
                w0, x0, y0, z0 = a
                w1, x1, y1, z1 = q
                return np.array([w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1, w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
                                 w0 * y1 - x0 * z1 + y0 * w1 + z0 * x1, w0 * z1 + x0 * y1 - y0 * x1 + z0 * w1])
            rp = oracle.reproj_residual(sc.camera_model, plus(d), sc.tvec[img], sc.xyz[pt], sc.camera_params[cam],
                                        sc.obs_xy[k])
            rm = oracle.reproj_residual(sc.camera_model, plus(-d), sc.tvec[img], sc.xyz[pt],
                                        sc.camera_params[cam], sc.obs_xy[k])
            fd = (rp - rm) / (2 * h)
            assert np.allclose(fd, J[b, :, c], rtol=1e-5, atol=1e-3)


def test_oracle_solve_reduces_cost_and_respects_constants():
    """TestTwoView / TestVariableImage behaviour on the oracle LM (CheckConstant*/CheckVariable*)."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 3, 100))
    sc.gauge()
    orig = sc.copy()
    s = oracle.solve(mi_ba.default_options(max_num_iterations=30), sc)
    assert s.final_cost < s.initial_cost
    assert s.num_residuals_reduced == 600 and s.num_effective_parameters_reduced == 317
    assert np.array_equal(sc.qvec[0], orig.qvec[0]) and np.array_equal(sc.tvec[0], orig.tvec[0])
    assert sc.tvec[1][0] == orig.tvec[1][0] and not np.array_equal(sc.tvec[1], orig.tvec[1])
    assert not np.array_equal(sc.qvec[2], orig.qvec[2])
    assert not np.array_equal(sc.camera_params[0], orig.camera_params[0])
    assert np.all(sc.camera_params[:, 1:3] == orig.camera_params[:, 1:3])  # principal point constant
    assert np.all(np.any(sc.xyz != orig.xyz, axis=1))
