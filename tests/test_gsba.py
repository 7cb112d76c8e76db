"""Geometric-semantic BA (GSBA): cylinder IoU residuals.

Reference: GeometricSemanticBundleAdjuster<Cylinder> and
<CylinderBy2Points> (src/optim/geometric_semantic_bundle_adjustment.cc:
481-1010,1160-1232; src/util/cylinder_by_2_points.h:26-155; functors
geometric_semantic_cost_functions.h:167-348),
Cylinder::ComputeSemanticIoU (src/util/cylinder.h:270-540), drawQuadrilateral
(:21-117), the GSBA cost functions (src/base/geometric_semantic_cost_functions.h:
33-165).  The reference has no GSBA tests or data: parity unpinned beyond
the known answers below (oracle/oracle_gsba.h restates the algorithm).

CPU: known answers of the restatement — a cylinder against a mask drawn from
itself has IoU 1; a camera inside the (infinite) cylinder or a quadrilateral
behind the camera gives IoU 0 (the reference catches the exception and
returns 0); block counts per variant; the oracle LM reduces the cost.
GPU (libmi_ba.so vs oracle): residuals and ambient CENTRAL Jacobians of every
block bitwise equal on >= 99.9 % of entries (both built without FMA; only a
libm ulp in acos/sin/cos could move a pixel decision); LM: the same
successful / unsuccessful steps over the descent, final cost within 1e-6,
cylinders within 1e-6; the landmark term (include_landmark_error) included.
"""
import numpy as np
import pytest

import mi_ba
import oracle

H, W = 240, 320


BY2 = mi_ba.CYLINDER_BY_2_POINTS


def workload(seed=0, images=10, cylinders=5, points=0, shift=0.08, tilt=0.0):
    sc, cyl = mi_ba.gsba_scene(images, cylinders, H, W, seed=seed, points=points)
    masks = oracle.gsba_render(sc, cyl, H, W)
    rng = np.random.default_rng(seed + 100)
    init = cyl.copy()
    init[:, 4:6] += rng.uniform(-shift, shift, (cylinders, 2))
    init[:, 7] *= rng.uniform(0.85, 1.15, cylinders)
    init[:, 8] *= rng.uniform(0.9, 1.1, cylinders)
    if tilt:
        # lean the initial cylinders (by 2 points: tvec_2 leaves the vertical)
        for c in range(cylinders):
            a = rng.uniform(-tilt, tilt, 2)
            q = np.array([1.0, a[0] / 2, a[1] / 2, 0.0])
            init[c, :4] = q / np.linalg.norm(q)
    sc = sc.gauge()
    sc.tvec[2:] += rng.uniform(-0.02, 0.02, sc.tvec[2:].shape)  # pose noise on the free images
    return sc, mi_ba.GsbaInput(masks, init), cyl


def test_iou_known_answers():
    sc, cyl = mi_ba.gsba_scene(6, 3, H, W, seed=1)
    for c in range(3):
        own = oracle.gsba_render(sc, cyl[c:c + 1], H, W)
        for i in range(sc.num_images):
            if own[i].sum() == 0:
                continue
            assert oracle.gsba_iou(sc.qvec[i], sc.tvec[i], sc.camera_params[i], cyl[c], own[i]) == 1.0
    # camera centre inside the infinite cylinder: GetEdgePoints throws -> IoU 0
    wide = cyl[0].copy()
    wide[7] = 50.0
    assert oracle.gsba_iou(sc.qvec[0], sc.tvec[0], sc.camera_params[0], wide, np.ones((H, W), np.uint8)) == 0.0
    # cylinder behind the camera: simplePinholeProject throws -> IoU 0
    R = mi_ba.quat_to_rot(sc.qvec[0])
    centre = -R.T @ sc.tvec[0]
    behind = cyl[0].copy()
    behind[4:7] = centre - 5.0 * R[2] - [0, 0, 2.0]
    assert oracle.gsba_iou(sc.qvec[0], sc.tvec[0], sc.camera_params[0], behind, np.ones((H, W), np.uint8)) == 0.0


def test_block_variants_and_oracle_descent():
    sc, g, _ = workload(seed=2)
    ids, r, J = oracle.gsba_evaluate(mi_ba.default_options(), sc, g)
    assert len(ids) == sc.num_images * 5
    const = ids[:, 0] == 0  # image 0: constant pose -> ConstantPoseGSBACostFunction
    assert np.all(J[const][:, :7] == 0) and np.abs(J[const][:, 7:]).sum() > 0
    assert np.abs(J[~const][:, :7]).sum() > 0
    # refine_geometry = 0: ConstantCylinderGSBACostFunction, constant-pose images dropped
    g2 = g.copy()
    g2.refine_geometry = 0
    ids2, _, J2 = oracle.gsba_evaluate(mi_ba.default_options(), sc, g2)
    assert len(ids2) == (sc.num_images - 1) * 5 and np.all(J2[:, 7:] == 0)
    a = g.copy()
    s = oracle.gsba_solve(mi_ba.default_options(max_num_iterations=10), sc.copy(), a)
    assert s.final_cost < s.initial_cost
    assert s.num_residuals_reduced == sc.num_images * 5


def test_assert_rejections():
    sc, g, _ = workload(seed=3)
    with pytest.raises(RuntimeError):
        oracle.gsba_solve(mi_ba.default_options(loss_function_type=mi_ba.LOSS_CAUCHY), sc.copy(), g.copy())
    bad = sc.copy()
    bad.camera_constant = np.zeros(bad.num_images, np.uint8)
    with pytest.raises(RuntimeError):
        oracle.gsba_solve(mi_ba.default_options(), bad, g.copy())


@pytest.mark.gpu
@pytest.mark.parametrize("refine_geometry", [1, 0])
def test_gsba_evaluate_bitwise(gpu, refine_geometry):
    sc, g, _ = workload(seed=4)
    g.refine_geometry = refine_geometry
    o = mi_ba.default_options()
    ids_o, r_o, J_o = oracle.gsba_evaluate(o, sc, g)
    ids_g, r_g, J_g = mi_ba.gsba_evaluate(o, sc, g)
    assert np.array_equal(ids_g, ids_o)
    same = np.concatenate([(r_g == r_o)[:, None], J_g == J_o], axis=1)
    assert same.mean() >= 0.999, int((~same).sum())
    assert np.abs(J_o).sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["full", "constant_geometry", "landmarks"])
def test_gsba_solve_parity(gpu, case):
    sc, g, gt = workload(seed=5, points=200 if case == "landmarks" else 0)
    if case == "constant_geometry":
        g.refine_geometry = 0
    if case == "landmarks":
        g.include_landmark_error = 1
        g.landmark_error_weight = 0.5
    o = mi_ba.default_options(max_num_iterations=8)
    a, b = g.copy(), g.copy()
    s_o = oracle.gsba_solve(o, sc.copy(), a)
    s_g = mi_ba.gsba_solve(o, sc.copy(), b)
    assert s_g.num_residuals_reduced == s_o.num_residuals_reduced
    assert s_g.num_effective_parameters_reduced == s_o.num_effective_parameters_reduced
    assert abs(s_g.initial_cost - s_o.initial_cost) <= 1e-12 * s_o.initial_cost
    assert (s_g.num_successful_steps, s_g.num_unsuccessful_steps) == \
        (s_o.num_successful_steps, s_o.num_unsuccessful_steps)
    assert abs(s_g.final_cost - s_o.final_cost) <= 1e-6 * s_o.final_cost
    assert np.abs(b.cylinders - a.cylinders).max() <= 1e-6
    assert s_g.final_cost < s_g.initial_cost


@pytest.mark.gpu
def test_gsba_facade_workflow_from_files(gpu, tmp_path):
    """The GeometricSemanticBundleAdjuster workflow through the C++ facade
    (colmap_amd/geometric_semantic_bundle_adjustment.h): COLMAP text model,
    depth_tiff / semantic_tiff float32 maps (trunk class 250), cylinder text
    file in and out; same result as mi_ba.gsba_solve on the arrays."""
    import os
    import subprocess
    from PIL import Image
    from test_model_io import write_text_model
    sc, g, _ = workload(seed=6)
    sc.image_constant_tvec = None  # the workflow fixes the first pose only
    write_text_model(sc, str(tmp_path / "model"))
    (tmp_path / "data" / "depth_tiff").mkdir(parents=True)
    (tmp_path / "data" / "semantic_tiff").mkdir()
    for i in range(sc.num_images):
        Image.fromarray(np.full((H, W), 5.0, np.float32), mode="F").save(
            tmp_path / "data" / "depth_tiff" / ("img%d_depth.tiff" % i))
        Image.fromarray(np.where(g.masks[i] > 0, 250.0, 3.0).astype(np.float32), mode="F").save(
            tmp_path / "data" / "semantic_tiff" / ("img%d_semantic.tiff" % i), compression="tiff_lzw")
    with open(tmp_path / "cyl.txt", "w") as f:
        for c in g.cylinders:
            f.write("q %r %r %r %r t %r %r %r r %r h %r\n" % tuple(float(v) for v in c))
    exe = os.path.join(os.path.dirname(__file__), "cpp", "model_io_test")
    subprocess.run(["make", "-s", "-C", os.path.dirname(exe), "model_io_test"], check=True)
    r = subprocess.run([exe, "gsba", str(tmp_path / "model"), str(tmp_path / "data"), str(tmp_path / "cyl.txt"),
                        str(tmp_path / "out.txt"), "8"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    c0, c1, ns, nu = r.stdout.split()
    ref = g.copy()
    s = mi_ba.gsba_solve(mi_ba.default_options(max_num_iterations=8), sc.copy(), ref)
    assert abs(float(c0) - s.initial_cost) <= 1e-12 * s.initial_cost
    assert abs(float(c1) - s.final_cost) <= 1e-6 * s.final_cost
    assert (int(ns), int(nu)) == (s.num_successful_steps, s.num_unsuccessful_steps)
    out = []
    for line in open(tmp_path / "out.txt"):
        t = line.split()
        out.append([float(v) for v in t[1:5] + t[6:9] + [t[10], t[12]]])
    assert np.abs(np.array(out) - ref.cylinders).max() <= 1e-6


# ---------------------------------------------------------------------------
# CylinderBy2Points (cylinder_parametrization = "by_2_points")
# ---------------------------------------------------------------------------
def test_by2_block_variants_and_oracle_descent():
    """Blocks as for Cylinder; the cylinder columns are tvec_1, tvec_2, radius
    (GSBACostFunctionBy2Points / ConstantPose..., 7 parameters, no manifold);
    7 effective parameters per refined cylinder; the oracle LM descends."""
    sc, g, _ = workload(seed=12, tilt=0.1)
    g.cylinder_parametrization = BY2
    ids, r, J = oracle.gsba_evaluate(mi_ba.default_options(), sc, g)
    assert len(ids) == sc.num_images * 5
    assert np.all(J[:, 14:] == 0) and np.abs(J[:, 7:14]).sum() > 0
    const = ids[:, 0] == 0
    assert np.all(J[const][:, :7] == 0)
    a = g.copy()
    s = oracle.gsba_solve(mi_ba.default_options(max_num_iterations=10), sc.copy(), a)
    assert s.final_cost < s.initial_cost
    b = g.copy()
    b.cylinder_parametrization = mi_ba.CYLINDER_DEFAULT
    s8 = oracle.gsba_solve(mi_ba.default_options(max_num_iterations=0), sc.copy(), b)
    assert s.num_effective_parameters_reduced == s8.num_effective_parameters_reduced - 5  # 7 vs 8 per cylinder
    # the cylinders leave as ToCylinder(): unit quaternions, radius >= 0
    assert np.allclose(np.linalg.norm(a.cylinders[:, :4], axis=1), 1.0, atol=1e-12)
    assert np.all(a.cylinders[:, 7] >= 0)


def test_by2_round_trip_keeps_the_cylinder():
    """CylinderBy2Points(Cylinder) -> ToCylinder keeps the lower centre, the
    radius, the height and the axis (a rotation about the axis is not kept:
    the reference writes the canonical z -> axis rotation); a vertical
    cylinder comes back exactly.  Checked through a zero-iteration oracle
    solve (the cylinders are written back through ToCylinder)."""
    sc, g, gt = workload(seed=13, tilt=0.3)
    g.cylinder_parametrization = BY2
    out = g.copy()
    oracle.gsba_solve(mi_ba.default_options(max_num_iterations=0), sc.copy(), out)
    assert np.allclose(out.cylinders[:, 4:9], g.cylinders[:, 4:9], rtol=0, atol=1e-12)
    for c in range(len(g.cylinders)):
        axis_in = mi_ba.quat_to_rot(g.cylinders[c, :4])[:, 2]
        axis_out = mi_ba.quat_to_rot(out.cylinders[c, :4])[:, 2]
        assert np.abs(axis_in - axis_out).max() <= 1e-12
    vert = g.copy()
    vert.cylinders = gt.copy()
    o2 = vert.copy()
    oracle.gsba_solve(mi_ba.default_options(max_num_iterations=0), sc.copy(), o2)
    assert np.array_equal(o2.cylinders, gt)


@pytest.mark.gpu
@pytest.mark.parametrize("refine_geometry", [1, 0])
def test_by2_evaluate_bitwise(gpu, refine_geometry):
    sc, g, _ = workload(seed=14, tilt=0.1)
    g.cylinder_parametrization = BY2
    g.refine_geometry = refine_geometry
    o = mi_ba.default_options()
    ids_o, r_o, J_o = oracle.gsba_evaluate(o, sc, g)
    ids_g, r_g, J_g = mi_ba.gsba_evaluate(o, sc, g)
    assert np.array_equal(ids_g, ids_o)
    same = np.concatenate([(r_g == r_o)[:, None], J_g == J_o], axis=1)
    assert same.mean() >= 0.999, int((~same).sum())
    assert np.abs(J_o).sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["full", "constant_geometry", "landmarks"])
def test_by2_solve_parity(gpu, case):
    sc, g, _ = workload(seed=15, points=200 if case == "landmarks" else 0, tilt=0.1)
    g.cylinder_parametrization = BY2
    if case == "constant_geometry":
        g.refine_geometry = 0
    if case == "landmarks":
        g.include_landmark_error = 1
        g.landmark_error_weight = 0.5
    o = mi_ba.default_options(max_num_iterations=8)
    a, b = g.copy(), g.copy()
    s_o = oracle.gsba_solve(o, sc.copy(), a)
    s_g = mi_ba.gsba_solve(o, sc.copy(), b)
    assert s_g.num_residuals_reduced == s_o.num_residuals_reduced
    assert s_g.num_effective_parameters_reduced == s_o.num_effective_parameters_reduced
    assert abs(s_g.initial_cost - s_o.initial_cost) <= 1e-12 * s_o.initial_cost
    assert (s_g.num_successful_steps, s_g.num_unsuccessful_steps) == \
        (s_o.num_successful_steps, s_o.num_unsuccessful_steps)
    assert abs(s_g.final_cost - s_o.final_cost) <= 1e-6 * s_o.final_cost
    assert np.abs(b.cylinders - a.cylinders).max() <= 1e-6
    assert s_g.final_cost <= s_g.initial_cost


@pytest.mark.gpu
def test_by2_facade_option(gpu, tmp_path):
    """cylinder_parametrization = "by_2_points" through the facade equals the
    array solve; an unknown name throws (GetCylinderParametrization)."""
    import os
    import subprocess
    from PIL import Image
    from test_model_io import write_text_model
    sc, g, _ = workload(seed=16, tilt=0.1)
    sc.image_constant_tvec = None
    write_text_model(sc, str(tmp_path / "model"))
    (tmp_path / "data" / "depth_tiff").mkdir(parents=True)
    (tmp_path / "data" / "semantic_tiff").mkdir()
    for i in range(sc.num_images):
        Image.fromarray(np.full((H, W), 5.0, np.float32), mode="F").save(
            tmp_path / "data" / "depth_tiff" / ("img%d_depth.tiff" % i))
        Image.fromarray(np.where(g.masks[i] > 0, 250.0, 3.0).astype(np.float32), mode="F").save(
            tmp_path / "data" / "semantic_tiff" / ("img%d_semantic.tiff" % i))
    with open(tmp_path / "cyl.txt", "w") as f:
        for c in g.cylinders:
            f.write("q %r %r %r %r t %r %r %r r %r h %r\n" % tuple(float(v) for v in c))
    exe = os.path.join(os.path.dirname(__file__), "cpp", "model_io_test")
    subprocess.run(["make", "-s", "-C", os.path.dirname(exe), "model_io_test"], check=True)
    args = [exe, "gsba", str(tmp_path / "model"), str(tmp_path / "data"), str(tmp_path / "cyl.txt"),
            str(tmp_path / "out.txt"), "6"]
    r = subprocess.run(args + ["by_2_points"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    c0, c1, ns, nu = r.stdout.split()
    ref = g.copy()
    ref.cylinder_parametrization = BY2
    s = mi_ba.gsba_solve(mi_ba.default_options(max_num_iterations=6), sc.copy(), ref)
    assert abs(float(c1) - s.final_cost) <= 1e-6 * s.final_cost
    assert (int(ns), int(nu)) == (s.num_successful_steps, s.num_unsuccessful_steps)
    bad = subprocess.run(args + ["by_3_points"], capture_output=True, text=True)
    assert bad.returncode == 3 and "not a valid cylinder parametrization" in bad.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("by2", [0, 1])
def test_gsba_span_kernel_tilted_wide(gpu, by2):
    """The IoU by row spans over bit-packed masks (gsba_iou_span_kernel: per
    edge a binary search with the per-pixel predicate) on wide rows (1000
    pixels: 16 mask words per row) with tilted cylinders (slanted edges, every
    edge search live) and a shift that pushes quadrilaterals over the image
    borders: residuals and Jacobians against the oracle's per-pixel scan."""
    h, w = 360, 1000
    sc, cyl = mi_ba.gsba_scene(8, 4, h, w, seed=11)
    masks = oracle.gsba_render(sc, cyl, h, w)
    rng = np.random.default_rng(12)
    init = cyl.copy()
    init[:, 4:6] += rng.uniform(-0.3, 0.3, (4, 2))
    init[:, 7] *= rng.uniform(0.7, 1.4, 4)
    for c in range(4):
        a = rng.uniform(-0.5, 0.5, 2)
        q = np.array([1.0, a[0] / 2, a[1] / 2, 0.0])
        init[c, :4] = q / np.linalg.norm(q)
    sc = sc.gauge()
    g = mi_ba.GsbaInput(masks, init)
    if by2:
        g.cylinder_parametrization = BY2
    o = mi_ba.default_options()
    ids_o, r_o, J_o = oracle.gsba_evaluate(o, sc, g)
    ids_g, r_g, J_g = mi_ba.gsba_evaluate(o, sc, g)
    assert np.array_equal(ids_g, ids_o)
    same = np.concatenate([(r_g == r_o)[:, None], J_g == J_o], axis=1)
    assert same.mean() >= 0.999, int((~same).sum())
    assert np.abs(J_o).sum() > 0 and (r_o != 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("solver", [mi_ba.SOLVER_DENSE_SCHUR, mi_ba.SOLVER_ITERATIVE_SCHUR])
@pytest.mark.parametrize("case", ["full", "landmarks"])
def test_gsba_solve_bitwise_reproducible(gpu, case, solver):
    """The cylinder terms are summed per owner (image, cylinder) in block
    order, not by float atomics: two GSBA solves give the same bits (cost,
    poses, cylinders), on the exact and the iterative path."""
    sc, g, gt = workload(seed=5, points=200 if case == "landmarks" else 0)
    if case == "landmarks":
        g.include_landmark_error = 1
        g.landmark_error_weight = 0.5
    o = mi_ba.default_options(max_num_iterations=8, linear_solver_type=solver)
    runs = []
    for _ in range(2):
        x, gg = sc.copy(), g.copy()
        s = mi_ba.gsba_solve(o, x, gg)
        runs.append((s, x, gg))
    (s1, x1, g1), (s2, x2, g2) = runs
    assert s1.final_cost == s2.final_cost
    assert (s1.num_successful_steps, s1.num_unsuccessful_steps) == (s2.num_successful_steps, s2.num_unsuccessful_steps)
    assert np.array_equal(x1.qvec, x2.qvec) and np.array_equal(x1.tvec, x2.tvec)
    assert np.array_equal(g1.cylinders, g2.cylinders)
