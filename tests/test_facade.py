"""The reference's BundleAdjuster tests (src/optim/bundle_adjustment_test.cc)
rerun in C++ through the colmap_amd facade (include/colmap_amd/) on
libmi_ba.so: structural counts on the host, full Solve on the MI355X.  Also
the controllers / iteration callbacks / Reconstruction filters
(tests/cpp/controllers_test.cc: reconstruction_test.cc:415-434,510-531 known
answers, controllers/bundle_adjustment.cc:43-103 callback semantics)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def build(name="bundle_adjustment_test"):
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    return os.path.join(CPP, name)


def run(mode, name="bundle_adjustment_test"):
    exe = build(name)
    out = subprocess.run([exe, mode], capture_output=True, text=True, timeout=600)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failure(s)" in out.stdout
    return out.stdout


def test_facade_counts_cpu():
    out = run("counts")
    assert out.count("PASS") == 16


@pytest.mark.gpu
def test_facade_solve_gpu(gpu):
    out = run("solve")
    assert out.count("PASS") == 16


def test_controllers_host():
    out = run("host", "controllers_test")
    assert out.count("PASS") == 3


@pytest.mark.gpu
def test_controllers_gpu(gpu):
    out = run("gpu", "controllers_test")
    assert out.count("PASS") == 11


def test_sba_reference_signature_host():
    """SemanticBundleAdjuster(options, config) with options.data_path
    (semantic_bundle_adjustment.h:219-225): the TIFF maps read back bitwise,
    a missing map file raised as ReadDepthAndSemanticMaps does, a camera model
    other than SIMPLE_PINHOLE refused with the reference's runtime_error
    (semantic_bundle_adjustment.cc:619-631)."""
    out = run("host", "sba_reference_test")
    assert out.count("PASS") == 3


@pytest.mark.gpu
def test_sba_reference_signature_gpu(gpu):
    """The reference controller's construction + Solve
    (controllers/semantic_bundle_adjustment.cc:100-119) from TIFF files equals
    the in-memory-maps solve bitwise."""
    out = run("gpu", "sba_reference_test")
    assert out.count("PASS") == 4


@pytest.mark.gpu
def test_sba_mixed_sizes_match_oracle(gpu, tmp_path):
    """The reference controller's SBA from TIFF maps of three different sizes
    (60 x 60, 48 x 72, 66 x 54) through the two-argument facade, against the
    oracle's LM on the problem the facade flattened (each image sampled on its
    own grid, the reprojected pixel bounds-checked against the second image's
    own size: semantic_bundle_adjustment.cc:792-799, semantic_cost_functions.h:
    163).  The semantic samples of the initial and the final point are bitwise
    equal (status, residual, Jacobian); the LMs take the same steps to the same
    final cost."""
    import numpy as np
    import mi_ba
    import oracle
    exe = build("sba_reference_test")
    out = subprocess.run([exe, "export", str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0 and "0 failure(s)" in out.stdout, out.stdout + out.stderr
    ld = lambda n, t: np.fromfile(tmp_path / n, t)
    meta = dict(l.split() for l in (tmp_path / "summary.txt").read_text().splitlines())
    I = len(ld("image_camera.i32", np.int32))
    sc = mi_ba.Scene(mi_ba.SIMPLE_PINHOLE, ld("camera_params.f64", np.float64).reshape(-1, 3),
                     ld("qvec.f64", np.float64).reshape(I, 4), ld("tvec.f64", np.float64).reshape(I, 3),
                     ld("image_camera.i32", np.int32), np.zeros((0, 3)), np.zeros((0, 2)), np.zeros(0, np.int32),
                     np.zeros(0, np.int32), camera_constant=ld("camera_constant.u8", np.uint8),
                     image_in_config=ld("image_in_config.u8", np.uint8),
                     image_constant_pose=ld("image_constant_pose.u8", np.uint8),
                     image_constant_tvec=ld("image_constant_tvec.u8", np.uint8))
    h, w = ld("image_height.i32", np.int32), ld("image_width.i32", np.int32)
    assert sorted(zip(h.tolist(), w.tolist())) == [(48, 72), (60, 60), (66, 54)]
    off = np.concatenate([[0], np.cumsum(h.astype(np.int64) * w)])
    dep, lab = ld("depth.f32", np.float32), ld("label.f32", np.float32)
    depth = [dep[off[i]:off[i + 1]].reshape(h[i], w[i]) for i in range(I)]
    label = [lab[off[i]:off[i + 1]].reshape(h[i], w[i]) for i in range(I)]
    sem = mi_ba.SemanticInput(depth, label, ld("pairs.i32", np.int32).reshape(-1, 2),
                              pixel_step=int(meta["pixel_step"]),
                              depth_error_threshold=float(meta["depth_error_threshold"]),
                              numeric_relative_step_size=float(meta["numeric_relative_step_size"]))
    opts = mi_ba.default_options(max_num_iterations=int(meta["max_num_iterations"]),
                                 function_tolerance=float(meta["function_tolerance"]),
                                 gradient_tolerance=float(meta["gradient_tolerance"]),
                                 parameter_tolerance=float(meta["parameter_tolerance"]))
    fq, ft = ld("final_qvec.f64", np.float64).reshape(I, 4), ld("final_tvec.f64", np.float64).reshape(I, 3)
    # the samples at the initial point and at the facade's final point, bitwise
    for q, t in ((sc.qvec, sc.tvec), (fq, ft)):
        at = sc.copy()
        at.qvec[:], at.tvec[:] = q, t
        with mi_ba.Context(opts, at.copy(), sem) as ctx:
            ctx.evaluate_semantic()
            px_g, st_g, r_g, J_g = ctx.download_semantic()
        px_o, st_o, r_o, J_o = oracle.semantic_eval(opts, at, sem)
        assert len(st_g) == len(st_o) > 0
        assert np.array_equal(px_g, px_o) and np.array_equal(st_g, st_o)
        assert np.array_equal(r_g, r_o) and np.array_equal(J_g, J_o)
        # every image's grid on its own size: pair (i, j) has image i's H_i x W_i grid
        pairs = sem.pairs
        for k, (i, j) in enumerate(pairs):
            if i == j:
                continue
            sel = px_o[:, 0] == k
            assert px_o[sel, 1].max() < w[i] and px_o[sel, 2].max() < h[i]
    s_o = oracle.solve(opts, sc.copy(), sem)
    assert s_o.num_residuals_reduced == int(meta["num_residuals_reduced"])
    assert (s_o.num_successful_steps, s_o.num_unsuccessful_steps) == \
        (int(meta["num_successful_steps"]), int(meta["num_unsuccessful_steps"]))
    assert s_o.termination_type == int(meta["termination_type"])
    assert s_o.initial_cost == float(meta["initial_cost"])
    assert abs(s_o.final_cost - float(meta["final_cost"])) <= 1e-6 * max(1.0, s_o.final_cost)
