"""Bitwise run-to-run reproducibility of the GPU LM.

Every camera-side sum of the solver is flushed in a fixed order instead of by
float atomics: the tile passes' per-tile partials summed per image / camera
(kernels.hip owner_flush_kernel: S's image blocks, b, diag(U), the
Schur-Jacobi blocks, every implicit Schur product, the gradient), the
explicit Schur pair tiles written once or summed per S block in tile order
(schur_pairs_flush_kernel when no camera is shared between images, else
per (pose | camera) owner pair from every tile's partial), the semantic
term's deferred samples listed in sample order and its pair blocks summed in
chunk order, then per image / S block in pair order (semantic.hip
deferred_order_kernel, pair_reduce_kernel and the owner kernels).  So two
solves of one problem take the same steps with the same bits, on the exact
(DENSE_SCHUR) and the iterative (ITERATIVE_SCHUR) path, with and without the
semantic term.  "deterministic_sums" 0 restores the atomic flushes (same
steps, costs equal to rounding).
"""
import numpy as np
import pytest

import mi_ba

pytestmark = pytest.mark.gpu


def scene(seed=5):
    return mi_ba.generate_scene(mi_ba.synth_config(mi_ba.OPENCV, 60, 8000, track_length=8, rotation_range=0.05,
                                                   extra=(-0.1, 0.01, 1e-4, -1e-4), seed=seed)).gauge()


def shared(sc, ncam):
    """The same scene with image i on camera i % ncam (the generator gives
    every camera the same intrinsics, so the observations stay consistent)."""
    sc = sc.copy()
    sc.image_camera = (np.arange(sc.num_images) % ncam).astype(np.int32)
    sc.camera_params = sc.camera_params[:ncam].copy()
    if sc.camera_constant is not None:
        sc.camera_constant = sc.camera_constant[:ncam].copy()
    return sc


def semantic(sc):
    depth, label = mi_ba.render_semantic(sc, 200, 200, plane_z=1.0, cell=0.2)
    I = sc.num_images
    pairs = np.array([(i, (i + d) % I) for i in range(I) for d in (1, 2)], np.int32)
    return mi_ba.SemanticInput(depth, label, pairs, pixel_step=5)


def run(sc, sem, solver, det=1):
    opts = mi_ba.default_options(max_num_iterations=6, linear_solver_type=solver, semantic_weight=0.1)
    b = sc.copy()
    with mi_ba.Context(opts, b, sem) as ctx:
        ctx.set_tuning("deterministic_sums", det)
        s = ctx.solve()
        ctx.writeback()
    return s, b


@pytest.mark.parametrize("solver", [mi_ba.SOLVER_DENSE_SCHUR, mi_ba.SOLVER_ITERATIVE_SCHUR])
@pytest.mark.parametrize("case", ["geo", "sem", "shared4", "shared1"])
def test_lm_bitwise_reproducible(gpu, case, solver):
    """shared4 / shared1: cameras shared by several images (4 cameras, one
    camera): the Schur pair blocks are summed per (pose | camera) owner pair
    from every tile's partial (schur_owner_chunk / schur_owner_flush)."""
    sc = scene()
    if case.startswith("shared"):
        sc = shared(sc, int(case[-1]))
    sem = semantic(sc) if case == "sem" else None
    s0, a = run(sc, sem, solver)
    s1, b = run(sc, sem, solver)
    assert s0.num_successful_steps >= 3
    assert (s1.num_successful_steps, s1.num_unsuccessful_steps, s1.num_linear_solver_iterations) == \
        (s0.num_successful_steps, s0.num_unsuccessful_steps, s0.num_linear_solver_iterations)
    assert s1.initial_cost == s0.initial_cost and s1.final_cost == s0.final_cost
    for key in ("qvec", "tvec", "xyz", "camera_params"):
        assert np.array_equal(getattr(a, key), getattr(b, key)), key


@pytest.mark.parametrize("solver", [mi_ba.SOLVER_DENSE_SCHUR, mi_ba.SOLVER_ITERATIVE_SCHUR])
@pytest.mark.parametrize("ncam", [0, 4, 1])
def test_atomic_flush_takes_the_same_steps(gpu, solver, ncam):
    """The float-atomic flushes (deterministic_sums 0) sum the same terms in
    another order: the same steps, costs equal to rounding (one camera per
    image, or ncam cameras shared by the images)."""
    sc = scene(seed=6)
    if ncam:
        sc = shared(sc, ncam)
    sem = semantic(sc)
    s0, _ = run(sc, sem, solver, det=1)
    s1, _ = run(sc, sem, solver, det=0)
    assert (s1.num_successful_steps, s1.num_unsuccessful_steps) == (s0.num_successful_steps, s0.num_unsuccessful_steps)
    assert abs(s1.final_cost - s0.final_cost) <= 1e-10 * s0.final_cost


@pytest.mark.parametrize("ncam", [4, 1])
def test_shared_camera_lm_matches_oracle(gpu, ncam):
    """The owner-pair flush builds the same S as the oracle's dense Schur
    solve: shared cameras, exact LM, the oracle's steps and cost."""
    import oracle
    sc = shared(scene(seed=7), ncam)
    opts = mi_ba.default_options(max_num_iterations=6)
    s_o = oracle.solve(opts, sc.copy())
    s_g, _ = run(sc, None, mi_ba.SOLVER_DENSE_SCHUR)
    assert (s_g.num_successful_steps, s_g.num_unsuccessful_steps) == (s_o.num_successful_steps, s_o.num_unsuccessful_steps)
    assert abs(s_g.final_cost - s_o.final_cost) <= 1e-9 * s_o.final_cost


@pytest.mark.parametrize("key,default", [("schur_z_image_order", 0), ("schur_self_one_load", 1)])
@pytest.mark.parametrize("case", ["sem", "shared4", "const"])
def test_schur_build_variants_bitwise(gpu, case, key, default):
    """Two forms of the explicit Schur build that take the same products in
    the same order drive a bitwise equal exact LM: the Schur factors Z in
    image order (schur_z_image_order 1: row k is the block at camera-major
    position k, the pair list in positions) or block order (0, default); the
    pair kernel's self tiles with one Z load per pair (schur_self_one_load 1,
    default) or two (0).  const: every fourth point held constant (zero Z
    rows).  Tools build only (the non-default values measured slower)."""
    if not mi_ba.ab_build():
        pytest.skip(key + " != default: tools build (MI_BA_LIB=ab)")
    sc = scene(seed=8)
    if case == "shared4":
        sc = shared(sc, 4)
    if case == "const":
        sc.point_config = np.where(np.arange(sc.num_points) % 4 == 0, 2, 1).astype(np.uint8)
    sem = semantic(sc) if case == "sem" else None
    out = []
    for v in (default, 1 - default):
        opts = mi_ba.default_options(max_num_iterations=6, semantic_weight=0.1)
        b = sc.copy()
        with mi_ba.Context(opts, b, sem) as ctx:
            ctx.set_tuning(key, v)
            s = ctx.solve()
            ctx.writeback()
        out.append((s, b))
    (s0, a), (s1, b) = out
    assert s0.num_successful_steps >= 2
    assert (s1.num_successful_steps, s1.num_unsuccessful_steps) == (s0.num_successful_steps, s0.num_unsuccessful_steps)
    assert s1.final_cost == s0.final_cost
    for key_ in ("qvec", "tvec", "xyz", "camera_params"):
        assert np.array_equal(getattr(a, key_), getattr(b, key_)), key_
