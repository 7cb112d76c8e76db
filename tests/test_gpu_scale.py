"""Parity at BASELINE.json's full sizes (GPU LM / kernels vs the CPU oracle).

  * C2 (200 cams / 50k points / 500k obs, SIMPLE_RADIAL): GPU LM vs
    oracle.solve, exact Schur solve (nf = 1593: four 512-wide look-ahead
    panels of the hand-written diagonal factor).  Descent (8 iterations):
    same successful / unsuccessful step counts, final cost within 1e-6
    relative (north-star tolerance); converged (100-iteration cap): final
    cost within 1e-6.  bundle_adjustment.cc:258-320 (BundleAdjuster::Solve).
  * C3 (C2 + 4.0M semantic samples, pairs (i, i+1), (i, i+2), step 10 at
    1000 x 1000): GPU LM vs oracle.solve.  Same pass criteria.
    semantic_cost_functions.h:87-208, semantic_bundle_adjustment.cc:699-906.
  * C4 semantic (1000 OPENCV cameras, 5.0M samples, step 20): every sample of
    the GPU evaluation downloaded; 20 pairs spread over the pair list compared
    with the oracle's evaluation of the same pairs, status / residual /
    Jacobian bitwise (>= 99.99 % of samples).
  * ITERATIVE_SCHUR (implicit-Schur PCG with SCHUR_JACOBI, the solver
    bundle_adjustment.cc:283-285 selects above 1000 images): GPU LM vs the
    oracle's exact LM with eta = 1e-12 so every CG solve is exact.  Pass:
    final cost within 1e-6 relative, same step counts.
  * ITERATIVE_SCHUR at the settings bench.py uses at N > 1 (default eta 0.1,
    200 CG iterations per solve), C2 size, run to the 100-iteration cap
    against the oracle's exact LM: the inexact steps take another path; the
    converged cost (1e-6 relative) is compared, and the parameter difference
    is shown to lie along the problem's near-null direction (tests/valley.py).
    Step-for-step against the oracle's own PCG: tests/test_lm_semantics.py.
  * C4 LM: the first iteration against the oracle live; the bench's three
    iterations against the oracle's committed trajectory
    (tests/golden/c4_lm3.json).
"""
import os

import numpy as np
import pytest

import mi_ba
import oracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

OPENCV_EXTRA = (-0.1, 0.01, 1e-4, -1e-4)


def c2_scene(seed=0):
    return mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 200, 50_000, track_length=10,
                                                   rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=seed)).gauge()


def semantic_input(sc, step, pairs_per_image, size=1000, cell=0.1):
    I = sc.num_images
    depth, label = mi_ba.render_semantic(sc, size, size, plane_z=1.0, cell=cell)
    pairs = np.array([(i, (i + d) % I) for i in range(I) for d in range(1, pairs_per_image + 1)], np.int32)
    return mi_ba.SemanticInput(depth, label, pairs, pixel_step=step)


def assert_lm_parity(opts, sc, sem=None, rel=1e-6):
    a, b = sc.copy(), sc.copy()
    s_o = oracle.solve(opts, a, sem)
    s_g = mi_ba.solve(opts, b, sem)
    assert s_g.num_residuals_reduced == s_o.num_residuals_reduced
    assert s_g.num_effective_parameters_reduced == s_o.num_effective_parameters_reduced
    assert abs(s_g.initial_cost - s_o.initial_cost) <= 1e-12 * s_o.initial_cost
    assert (s_g.num_successful_steps, s_g.num_unsuccessful_steps) == \
        (s_o.num_successful_steps, s_o.num_unsuccessful_steps)
    assert abs(s_g.final_cost - s_o.final_cost) <= rel * s_o.final_cost, (s_g.final_cost, s_o.final_cost)
    assert s_g.final_cost < s_g.initial_cost
    return s_o, s_g, a, b


def test_c2_full_lm_parity(gpu):
    sc = c2_scene()
    # the descent: every accept/reject decision equal, same final cost
    s_o, s_g, a, b = assert_lm_parity(mi_ba.default_options(max_num_iterations=8), sc)
    assert s_g.num_successful_steps >= 6
    # points at the scene's scale (unit cube)
    assert np.abs(b.xyz - a.xyz).max() <= 1e-5


def test_c2_converged_lm_parity(gpu):
    """Run to the reference's 100-iteration default cap.  Once converged, the
    accept/reject decisions compare cost changes at the rounding level of a
    1M-term sum (both solvers stop on Ceres' function tolerance 0 when a
    candidate's cost equals the current cost exactly), so only the converged
    cost is compared (north-star criterion, 1e-6 relative)."""
    sc = c2_scene()
    opts = mi_ba.default_options(max_num_iterations=100)
    a, b = sc.copy(), sc.copy()
    s_o = oracle.solve(opts, a)
    s_g = mi_ba.solve(opts, b)
    assert abs(s_g.final_cost - s_o.final_cost) <= 1e-6 * s_o.final_cost, (s_g.final_cost, s_o.final_cost)
    assert np.abs(b.xyz - a.xyz).max() <= 1e-5


def test_c3_semantic_lm_parity(gpu):
    sc = c2_scene()
    sem = semantic_input(sc, step=10, pairs_per_image=2)
    opts = mi_ba.default_options(max_num_iterations=8)
    s_o, s_g, _, _ = assert_lm_parity(opts, sc, sem)
    assert s_g.num_semantic_residuals == s_o.num_semantic_residuals
    assert 3_500_000 <= s_g.num_semantic_residuals <= 4_000_000


def test_c4_semantic_sampled_pairs_bitwise(gpu):
    c = mi_ba.synth_config(mi_ba.OPENCV, 1000, 1_000_000, track_length=10, rotation_range=0.05,
                           extra=OPENCV_EXTRA)
    sc = mi_ba.generate_scene(c).gauge()
    # the semantic term alone (the reprojection blocks are covered elsewhere)
    sc.obs_xy, sc.obs_image, sc.obs_point = sc.obs_xy[:0], sc.obs_image[:0], sc.obs_point[:0]
    sc.camera_constant = np.ones(sc.num_images, np.uint8)
    sem = semantic_input(sc, step=20, pairs_per_image=2)
    opts = mi_ba.default_options()
    with mi_ba.Context(opts, sc.copy(), sem) as ctx:
        ctx.evaluate_semantic()
        px_g, st_g, r_g, J_g = ctx.download_semantic()
    assert len(st_g) >= 4_500_000
    K = len(sem.pairs)
    pick = np.linspace(0, K - 1, 20).astype(np.int64)
    sub = mi_ba.SemanticInput(sem.depth, sem.label, sem.pairs[pick], pixel_step=20)
    px_o, st_o, r_o, J_o = oracle.semantic_eval(opts, sc, sub)
    # GPU samples of the picked pairs, in the same (pair, y, x) order
    sel = np.concatenate([np.nonzero(px_g[:, 0] == k)[0] for k in pick])
    assert np.array_equal(px_g[sel, 1:], px_o[:, 1:])
    assert np.array_equal(pick[px_o[:, 0]], px_g[sel, 0])
    same = (st_g[sel] == st_o) & (r_g[sel] == r_o) & np.all(J_g[sel] == J_o, axis=1)
    assert same.mean() >= 0.9999, int((~same).sum())
    assert (st_o == mi_ba.VALID).mean() > 0.5 and (np.abs(J_o).sum(axis=1) > 0).sum() > 100


@pytest.mark.parametrize("mf", [0, 1])
@pytest.mark.parametrize("case", ["geo", "sem"])
def test_iterative_schur_parity(gpu, case, mf):
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 30, 2000, track_length=6,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=9)).gauge()
    sem = None
    if case == "sem":
        sem = semantic_input(sc, step=6, pairs_per_image=2, size=120, cell=0.5)
    opts = mi_ba.default_options(max_num_iterations=12, eta=1e-12, max_linear_solver_iterations=1000,
                                 semantic_weight=0.01)
    ref = mi_ba.default_options(max_num_iterations=12, eta=1e-12, semantic_weight=0.01)
    a, b = sc.copy(), sc.copy()
    s_o = oracle.solve(ref, a, sem)
    opts.linear_solver_type = mi_ba.SOLVER_ITERATIVE_SCHUR
    with mi_ba.Context(opts, b, sem) as ctx:  # mf 1: the matrix-free Schur product
        ctx.set_tuning("pcg_matrix_free", mf)
        s_g = ctx.solve()
        ctx.writeback()
    assert s_g.num_linear_solver_iterations > s_g.num_successful_steps  # the CG path ran
    assert (s_g.num_successful_steps, s_g.num_unsuccessful_steps) == \
        (s_o.num_successful_steps, s_o.num_unsuccessful_steps)
    assert abs(s_g.final_cost - s_o.final_cost) <= 1e-6 * s_o.final_cost, (s_g.final_cost, s_o.final_cost)


def test_c2_iterative_schur_default_eta_converges_to_oracle(gpu):
    """ITERATIVE_SCHUR at bench.py's N > 1 settings (eta 0.1, 200 CG
    iterations per solve) run to the 100-iteration cap against the oracle's
    exact-Schur LM: the converged cost within 1e-6 relative, and the
    parameters checked against the problem's flat valley (round 4 deleted
    that check after a 3.5e-4 point difference; the step-for-step PCG parity
    is tests/test_lm_semantics.py).  At the exact solution the Jacobi-scaled
    reduced camera system has a near-null direction (focal length against
    point depth); the camera-side difference of the two solutions must lie
    along it: >= 99.9 % of its energy in the two smallest-eigenvalue
    eigenvectors, whose eigenvalues are < 1e-5 of the median (measured:
    lambda 7.6e-7 and 5.2e-6 against a median of 0.81; 99.45 % of the energy
    on the first, 99.9995 % on the two; tests/valley.py)."""
    import valley
    sc = c2_scene()
    ref = mi_ba.default_options(max_num_iterations=100)
    opts = mi_ba.default_options(max_num_iterations=100, linear_solver_type=mi_ba.SOLVER_ITERATIVE_SCHUR)
    assert opts.eta == 0.1 and opts.max_linear_solver_iterations == 200
    a, b = sc.copy(), sc.copy()
    s_o = oracle.solve(ref, a)
    s_g = mi_ba.solve(opts, b)
    assert s_g.num_linear_solver_iterations > s_g.num_successful_steps  # the CG path ran
    assert abs(s_g.final_cost - s_o.final_cost) <= 1e-6 * s_o.final_cost, (s_g.final_cost, s_o.final_cost)
    rep = valley.valley_report(mi_ba.default_options(), a, b)
    print("valley: lambda", rep["lam"][:4], "median", np.median(rep["lam"]), "energy", rep["energy"][:4],
          "|d|", rep["norm"], "xyz diff", np.abs(a.xyz - b.xyz).max())
    assert rep["lam"][1] < 1e-5 * np.median(rep["lam"])
    assert rep["energy"][1] >= 0.999, rep["energy"][:4]


@pytest.mark.parametrize("mf", [0, 1])
@pytest.mark.parametrize("case", ["constants", "long_tracks", "soft_l1"])
def test_iterative_schur_parity_chunks(gpu, case, mf):
    """The PCG path's chunked point passes and camera-major J copy against the
    oracle: constant points (camera-major slots without a point term),
    constant cameras and poses (skipped f-slots), or every point observed by
    70 images (each point chunk a single point of more than 64 blocks: the
    carried multi-pass sums)."""
    if case == "constants":
        sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 30, 2000, track_length=6, rotation_range=0.05,
                                                     extra=(-0.1, 0.01, 1e-4, -1e-4), seed=11)).gauge()
        rng = np.random.default_rng(3)
        sc.point_config = np.where(rng.uniform(size=sc.num_points) < 0.3, 2, 1).astype(np.uint8)
        sc.camera_constant = (np.arange(sc.num_cameras) % 3 == 0).astype(np.uint8)
        sc.image_constant_pose[5] = 1
    elif case == "long_tracks":
        sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 80, 300, track_length=70,
                                                     rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=12)).gauge()
    else:  # robust loss: the Corrector's sqrt(rho') on the recomputed rows
        sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 30, 2000, track_length=6, rotation_range=0.05,
                                                     extra=(-0.1, 0.01, 1e-4, -1e-4), seed=13)).gauge()
    loss = dict(loss_function_type=mi_ba.LOSS_SOFT_L1, loss_function_scale=1.0) if case == "soft_l1" else {}
    # 3 iterations: same accept/reject decisions; 8: converged to the same
    # cost.  (Once converged, steps are decided at the rounding floor, where
    # the oracle and even the exact GPU solve differ: 'constants' reaches
    # 13157.18092343093 with (6, 2) oracle steps, (8, 0) exact GPU steps,
    # (6, 1) PCG steps — tools/diag_pcg_constants.py.)
    for iters in (3, 8):
        ref = mi_ba.default_options(max_num_iterations=iters, eta=1e-12, **loss)
        opts = mi_ba.default_options(max_num_iterations=iters, eta=1e-12, max_linear_solver_iterations=1000,
                                     linear_solver_type=mi_ba.SOLVER_ITERATIVE_SCHUR, **loss)
        a, b = sc.copy(), sc.copy()
        s_o = oracle.solve(ref, a, None)
        with mi_ba.Context(opts, b) as ctx:
            ctx.set_tuning("pcg_matrix_free", mf)
            s_g = ctx.solve()
        assert s_g.num_linear_solver_iterations > s_g.num_successful_steps  # the CG path ran
        if iters == 3:
            assert (s_g.num_successful_steps, s_g.num_unsuccessful_steps) == \
                (s_o.num_successful_steps, s_o.num_unsuccessful_steps)
        assert abs(s_g.final_cost - s_o.final_cost) <= 1e-6 * s_o.final_cost, (iters, s_g.final_cost, s_o.final_cost)


def test_c4_lm_first_iteration_matches_oracle(gpu):
    """The C4 exact-Schur LM the bench times (1000 OPENCV cameras, 1M points,
    10M observations + 5.0M semantic samples; nf = 11 993, dense S) against
    the oracle's LM on the same scene: one full LM iteration (Jacobi scaling,
    damped point blocks, explicit S, the 24-panel factor, back-substitution,
    trial cost, acceptance).  The oracle factors its S with LAPACK dpotrf
    (oracle.use_lapack_factor: its own O(n^3) Cholesky takes minutes at this
    size); its LM takes ~1 minute of host time per iteration, so the pinned
    trajectory is the first iteration — the C2 / C3 tests above pin full
    trajectories.  Pass: same step counts, initial cost within 1e-12, final
    cost within 1e-6 relative (north-star tolerance), and every parameter's
    change within 1e-6 of the oracle's change (relative to the largest
    change of its block type)."""
    import bench
    sc, sem = bench.build_shard(bench.CONFIGS["C4"], 0, 1)
    opts = mi_ba.default_options(max_num_iterations=1)
    g = sc.copy()
    s_g = mi_ba.solve(opts, g, sem)
    oracle.use_lapack_factor(True)
    try:
        o = sc.copy()
        s_o = oracle.solve(opts, o, sem)
    finally:
        oracle.use_lapack_factor(False)
    assert s_g.num_residuals_reduced == s_o.num_residuals_reduced
    assert abs(s_g.initial_cost - s_o.initial_cost) <= 1e-12 * s_o.initial_cost
    assert (s_g.num_successful_steps, s_g.num_unsuccessful_steps) == (1, 0)
    assert (s_o.num_successful_steps, s_o.num_unsuccessful_steps) == (1, 0)
    assert abs(s_g.final_cost - s_o.final_cost) <= 1e-6 * s_o.final_cost, (s_g.final_cost, s_o.final_cost)
    assert s_g.final_cost < s_g.initial_cost
    q0 = sc.qvec / np.linalg.norm(sc.qvec, axis=1, keepdims=True)
    for name, x0 in (("qvec", q0), ("tvec", sc.tvec), ("xyz", sc.xyz), ("camera_params", sc.camera_params)):
        dg, do = getattr(g, name) - x0, getattr(o, name) - x0
        assert np.abs(dg - do).max() <= 1e-6 * max(np.abs(do).max(), 1e-300), name


def test_c4_lm_three_iterations_match_fixture(gpu):
    """The bench's BA-iteration leg itself — 3 exact-Schur LM iterations on
    C4 with the 5.0M-sample semantic term — against the oracle's trajectory
    on the same scene, committed as tests/golden/c4_lm3.json (written in the
    container by tests/golden/make_c4_lm_fixture.py; the oracle's C4 LM takes
    minutes of host time per iteration, too long for a GPU test).  Pass: the
    same accept / reject sequence, initial cost within 1e-12, final cost
    within 1e-6 relative (north-star tolerance), per parameter block type the
    largest change within 1e-6 relative and every sampled parameter's change
    within 1e-6 of that block type's largest change."""
    import json
    import bench
    fx = json.load(open(os.path.join(HERE, "golden", "c4_lm3.json")))
    sc, sem = bench.build_shard(bench.CONFIGS["C4"], 0, 1)
    rec = {}
    opts = mi_ba.default_options(max_num_iterations=fx["options"]["max_num_iterations"])
    opts.set_callback(lambda it: rec.__setitem__(it.iteration, (it.step_is_valid, it.step_is_successful)))
    g = sc.copy()
    with mi_ba.Context(opts, g, sem) as ctx:
        s = ctx.solve()
        ctx.writeback()
    assert s.num_residuals_reduced == fx["num_residuals_reduced"]
    assert s.num_semantic_residuals == fx["num_semantic_residuals"]
    assert (s.num_successful_steps, s.num_unsuccessful_steps) == \
        (fx["num_successful_steps"], fx["num_unsuccessful_steps"])
    for k, (valid, succ, _) in enumerate(fx["trace"], start=1):
        assert rec[k] == (valid, succ), (k, rec[k])
    assert abs(s.initial_cost - fx["initial_cost"]) <= 1e-12 * fx["initial_cost"]
    assert abs(s.final_cost - fx["final_cost"]) <= 1e-6 * fx["final_cost"], (s.final_cost, fx["final_cost"])
    q0 = sc.qvec / np.linalg.norm(sc.qvec, axis=1, keepdims=True)
    d = {"qvec": g.qvec - q0, "tvec": g.tvec - sc.tvec, "xyz": g.xyz - sc.xyz,
         "camera_params": g.camera_params - sc.camera_params}
    smp = fx["sample"]
    idx = {"qvec": smp["images"], "tvec": smp["images"], "xyz": smp["points"], "camera_params": smp["cameras"]}
    for name, v in d.items():
        m = fx["max_change"][name]
        assert abs(np.abs(v).max() - m) <= 1e-6 * m, (name, np.abs(v).max(), m)
        assert np.abs(v[idx[name]] - np.asarray(smp[name])).max() <= 1e-6 * m, name


def test_c3_window_summary_flat_pass_bitwise(gpu):
    """The flat pass deciding samples from the rasters' 3x3 window summaries
    (semantic_window_summary 1) or from the label planes (8-bit label indices
    + tile depth ranges, semantic_label_planes 1), the coarse box
    (semantic_flat_coarse 1: same values, a superset of the deferrals) and
    the deferred pass taking its stencil
    pixels from the once-read 3x3 box (semantic_deferred_box 1) against the
    raster-only passes at C3 size (4.0M samples): status, residual and
    Jacobian of every sample bitwise, and the same samples deferred to the
    full stencil."""
    sc = c2_scene()
    sem = semantic_input(sc, step=10, pairs_per_image=2)
    sc.tvec[5:] += 0.002  # pose errors: some samples change label between pixels
    out = []
    with mi_ba.Context(mi_ba.default_options(), sc.copy(), sem) as ctx:
        ctx.set_tuning("semantic_diag", 1)
        for ws, box, lp, coarse in ((0, 0, 0, 0), (1, 0, 0, 0), (1, 1, 0, 0), (0, 1, 0, 0), (0, 0, 1, 0), (1, 1, 1, 0),
                                    (0, 0, 1, 1), (0, 0, 1, 2), (0, 0, 1, 3), (1, 0, 0, 1), (0, 0, 0, 1)):
            ctx.set_tuning("semantic_window_summary", ws)
            ctx.set_tuning("semantic_deferred_box", box)
            ctx.set_tuning("semantic_label_planes", lp)
            ctx.set_tuning("semantic_flat_coarse", coarse)
            ctx.evaluate_semantic()
            out.append(ctx.download_semantic())
    for k, o in enumerate(out[1:]):
        for m, (a, b) in enumerate(zip(out[0], o)):
            if k >= 5 and m == 1:  # the coarse boxes defer a few more samples: statuses sans the mark
                a, b = np.where(a >= 0x800, a - 0x1000, a), np.where(b >= 0x800, b - 0x1000, b)
            assert np.array_equal(a, b)
    st = out[0][1]
    deferred = st >= 0x800  # semantic_diag: deferred samples' status offset by +0x1000
    assert deferred.sum() > 0 and (np.where(deferred, st - 0x1000, st) == mi_ba.VALID).mean() > 0.5
