"""Per-image raster sizes (ABI 4): each image's depth / semantic maps (SBA)
and trunk masks (GSBA) on their own size.

Reference: SemanticBundleAdjuster::AddImagePairToProblem samples image 1 on
its own map size (semantic_bundle_adjustment.cc:792-799) and
compute_semantic_error bounds-checks the reprojected pixel against image 2's
own depth map (semantic_cost_functions.h:163); the GSBA IoU is rasterised on
each image's own semantic map (Cylinder::ComputeSemanticIoU, cylinder.h:
496-504; geometric_semantic_bundle_adjustment.cc:1530-1531).

The maps here are crops of maps rendered at one size (top-left origin, so
the cameras' geometry is unchanged): a pixel outside an image's crop is
OUT_OF_BOUNDS for that image only.

CPU: the oracle with a list of equal-size maps equals its one-size form
bitwise; with mixed sizes its samples lie on each first image's own grid and
OUT_OF_BOUNDS is exactly "outside the second image's own size" (its export
rows give the rounded pixel); GSBA block residuals are 1 - IoU on each
image's own mask.  GPU: the product against the oracle bitwise (semantic
samples on every flat-pass route, export rows, GSBA blocks) and the LMs
(same steps, final cost within 1e-6).
"""
import numpy as np
import pytest

import mi_ba
import oracle

SIZES = [(160, 160), (120, 160), (160, 100), (90, 130)]  # (H, W) of images 0..3


def crop(maps, sizes):
    return [np.ascontiguousarray(m[:h, :w]) for m, (h, w) in zip(maps, sizes)]


def semantic_scene(model=mi_ba.SIMPLE_PINHOLE, images=4, size=160, step=4, seed=2):
    extra = {mi_ba.SIMPLE_PINHOLE: (), mi_ba.SIMPLE_RADIAL: (0.05, 0, 0, 0),
             mi_ba.OPENCV: (-0.1, 0.01, 1e-4, -1e-4)}[model]
    sc = mi_ba.generate_scene(mi_ba.synth_config(model, images, 50, track_length=images, image_size=size,
                                                 rotation_range=0.05, extra=extra, seed=seed))
    sc.gauge()
    sc.camera_constant = np.ones(images, np.uint8)
    depth, label = mi_ba.render_semantic(sc, size, size, plane_z=1.0, cell=0.5)
    pairs = np.array([(i, j) for i in range(images) for j in range(images) if i != j], np.int32)
    rng = np.random.default_rng(seed)
    sc.tvec[2:] += rng.uniform(-0.02, 0.02, sc.tvec[2:].shape)
    sizes = [SIZES[i % len(SIZES)] for i in range(images)]
    mixed = mi_ba.SemanticInput(crop(depth, sizes), crop(label, sizes), pairs, pixel_step=step)
    return sc, mi_ba.SemanticInput(depth, label, pairs, pixel_step=step), mixed, sizes


def test_oracle_equal_size_list_equals_array():
    sc, sem, _, _ = semantic_scene(step=5)
    listed = mi_ba.SemanticInput(list(sem.depth), list(sem.label), sem.pairs, pixel_step=5)
    opts = mi_ba.default_options()
    a = oracle.semantic_eval(opts, sc, sem)
    b = oracle.semantic_eval(opts, sc, listed)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_oracle_mixed_sizes_grid_and_bounds():
    sc, _, mixed, sizes = semantic_scene(step=3)
    opts = mi_ba.default_options()
    px, st, r, J = oracle.semantic_eval(opts, sc, mixed)
    for k, (i, j) in enumerate(mixed.pairs):
        sel = px[:, 0] == k
        h, w = sizes[i]
        # image i's own grid: every pixel with depth >= 1e-4 on (y, x) steps of 3
        d = mixed.depth[i]
        ys, xs = np.meshgrid(np.arange(0, h, 3), np.arange(0, w, 3), indexing="ij")
        keep = d[ys, xs] >= 1e-4
        assert sel.sum() == keep.sum()
        assert np.array_equal(px[sel, 1], xs[keep]) and np.array_equal(px[sel, 2], ys[keep])
    n_oob = 0
    for i in range(sc.num_images):
        for j in range(sc.num_images):
            if i == j:
                continue
            pix, status, err, world = oracle.semantic_export(opts, sc, mixed, i, j)
            h, w = sizes[j]
            out = (pix[:, 2] < 0) | (pix[:, 2] >= w) | (pix[:, 3] < 0) | (pix[:, 3] >= h)
            assert np.array_equal(status == mi_ba.OUT_OF_BOUNDS, out)
            assert np.all(pix[:, 0] < sizes[i][1]) and np.all(pix[:, 1] < sizes[i][0])
            n_oob += int(out.sum())
    assert n_oob > 0
    # the one-size maps sample more pixels of image 1 than the crops
    _, full, _, _ = semantic_scene(step=3)
    assert len(oracle.semantic_eval(opts, sc, full)[1]) > len(st)


def gsba_mixed(seed=4, images=8, cylinders=4):
    H, W = 240, 320
    sc, cyl = mi_ba.gsba_scene(images, cylinders, H, W, seed=seed)
    masks = oracle.gsba_render(sc, cyl, H, W)
    sizes = [(H - 40 * (i % 3), W - 56 * (i % 4)) for i in range(images)]
    rng = np.random.default_rng(seed + 100)
    init = cyl.copy()
    init[:, 4:6] += rng.uniform(-0.08, 0.08, (cylinders, 2))
    init[:, 7] *= rng.uniform(0.85, 1.15, cylinders)
    sc = sc.gauge()
    sc.tvec[2:] += rng.uniform(-0.02, 0.02, sc.tvec[2:].shape)
    return sc, mi_ba.GsbaInput(crop(masks, sizes), init), mi_ba.GsbaInput(masks, init.copy()), sizes


def test_oracle_gsba_mixed_sizes_iou_on_own_mask():
    sc, g, full, sizes = gsba_mixed()
    ids, r, J = oracle.gsba_evaluate(mi_ba.default_options(), sc, g)
    ids_f, r_f, _ = oracle.gsba_evaluate(mi_ba.default_options(), sc, full)
    assert np.array_equal(ids, ids_f)
    for k, (i, c) in enumerate(ids):
        iou = oracle.gsba_iou(sc.qvec[i], sc.tvec[i], sc.camera_params[i], g.cylinders[c], g.masks[i])
        assert r[k] == 1.0 - iou
    assert np.any(r != r_f)  # the crops cut some quadrilaterals


# ---------------------------------------------------------------------------
# GPU against the oracle
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("model", [mi_ba.SIMPLE_PINHOLE, mi_ba.OPENCV])
def test_semantic_mixed_sizes_bitwise(gpu, model):
    sc, _, mixed, _ = semantic_scene(model, step=3, seed=5)
    sc.obs_xy, sc.obs_image, sc.obs_point = sc.obs_xy[:0], sc.obs_image[:0], sc.obs_point[:0]  # cost: the term alone
    opts = mi_ba.default_options()
    px_o, st_o, r_o, J_o = oracle.semantic_eval(opts, sc, mixed)
    assert (st_o == mi_ba.OUT_OF_BOUNDS).sum() > 0 and (np.abs(J_o).sum(axis=1) > 0).sum() > 0
    with mi_ba.Context(opts, sc.copy(), mixed) as ctx:
        # the flat pass's routes: label planes (default), window summaries, rasters only
        for lp, ws in ((1, 0), (0, 1), (0, 0)):
            ctx.set_tuning("semantic_label_planes", lp)
            ctx.set_tuning("semantic_window_summary", ws)
            ctx.evaluate_semantic()
            px_g, st_g, r_g, J_g = ctx.download_semantic()
            assert np.array_equal(px_g, px_o)
            assert np.array_equal(st_g, st_o) and np.array_equal(r_g, r_o) and np.array_equal(J_g, J_o)
        c_g = ctx.cost()
    assert c_g == pytest.approx(0.5 * float((r_o * r_o).sum()), rel=1e-15, abs=0)


@pytest.mark.gpu
def test_semantic_mixed_sizes_export_rows(gpu):
    sc, _, mixed, _ = semantic_scene(step=4, seed=6)
    opts = mi_ba.default_options()
    with mi_ba.Context(opts, sc.copy(), mixed) as ctx:
        for i, j in ((0, 1), (1, 3), (3, 2), (2, 0)):
            g = ctx.semantic_export(i, j)
            o = oracle.semantic_export(opts, sc, mixed, i, j)
            for a, b in zip(g, o):
                assert np.array_equal(a, b)


@pytest.mark.gpu
def test_semantic_mixed_sizes_solve_parity(gpu):
    sc, _, mixed, _ = semantic_scene(images=4, step=4, seed=2)
    sc.obs_xy, sc.obs_image, sc.obs_point = sc.obs_xy[:0], sc.obs_image[:0], sc.obs_point[:0]
    opts = mi_ba.default_options(max_num_iterations=20, eta=1e-12)
    a, b = sc.copy(), sc.copy()
    s_o = oracle.solve(opts, a, mixed)
    s_g = mi_ba.solve(opts, b, mixed)
    assert s_g.num_semantic_residuals == s_o.num_semantic_residuals > 0
    assert s_g.initial_cost == s_o.initial_cost
    assert (s_g.num_successful_steps, s_g.num_unsuccessful_steps) == \
        (s_o.num_successful_steps, s_o.num_unsuccessful_steps)
    assert abs(s_g.final_cost - s_o.final_cost) <= 1e-6 * max(1.0, s_o.final_cost)
    assert np.abs(b.tvec - a.tvec).max() <= 1e-7


@pytest.mark.gpu
def test_gsba_mixed_sizes_bitwise_and_solve(gpu):
    sc, g, _, _ = gsba_mixed(seed=7)
    o = mi_ba.default_options()
    ids_o, r_o, J_o = oracle.gsba_evaluate(o, sc, g)
    ids_g, r_g, J_g = mi_ba.gsba_evaluate(o, sc, g)
    assert np.array_equal(ids_g, ids_o)
    same = np.concatenate([(r_g == r_o)[:, None], J_g == J_o], axis=1)
    assert same.mean() >= 0.999, int((~same).sum())
    o = mi_ba.default_options(max_num_iterations=8)
    a, b = g.copy(), g.copy()
    s_o = oracle.gsba_solve(o, sc.copy(), a)
    s_g = mi_ba.gsba_solve(o, sc.copy(), b)
    assert (s_g.num_successful_steps, s_g.num_unsuccessful_steps) == \
        (s_o.num_successful_steps, s_o.num_unsuccessful_steps)
    assert abs(s_g.final_cost - s_o.final_cost) <= 1e-6 * s_o.final_cost
    assert np.abs(b.cylinders - a.cylinders).max() <= 1e-6
