"""ExportSemanticErrorToCSV rows on the GPU (mi_ba_semantic_export) against
the oracle's restatement of compute_semantic_error
(semantic_bundle_adjustment.cc:908-1019, semantic_cost_functions.h:87-208):
every pixel of image 1's grid, zero-depth pixels included, status / error /
the rounded pixel in image 2 bitwise, the world point bitwise; and the rows
of the problem's own samples equal the solver's semantic evaluation.  Semantic
parity is unpinned by reference fixtures (the reference holds none): the
oracle is the literal restatement.  The facade's CSV files and per-iteration
snapshots are checked in tests/cpp/bundle_adjustment_test.cc
(TestSemanticBundleAdjusterSnapshots)."""
import numpy as np
import pytest

import mi_ba
import oracle

pytestmark = pytest.mark.gpu


def scene(model, extra=(0, 0, 0, 0)):
    sc = mi_ba.generate_scene(mi_ba.synth_config(model, 3, 10, track_length=3, image_size=96, rotation_range=0.05,
                                                 extra=extra)).gauge()
    sc.camera_constant = np.ones(3, np.uint8)
    depth, label = mi_ba.render_semantic(sc, 96, 96, cell=0.5)
    depth[0, :12, :] = 0.0  # a zero-depth band: exported, but not a sample of the problem
    sem = mi_ba.SemanticInput(depth, label, np.array([(0, 1), (1, 2), (2, 0)], np.int32), pixel_step=4)
    sc.tvec[2] += 0.01
    return sc, sem


@pytest.mark.parametrize("model", ["SIMPLE_PINHOLE", "SIMPLE_RADIAL", "OPENCV"])
def test_export_matches_oracle(gpu, model):
    m = mi_ba.MODEL_NAMES[model]
    extra = {"SIMPLE_PINHOLE": (0, 0, 0, 0), "SIMPLE_RADIAL": (0.05, 0, 0, 0),
             "OPENCV": (-0.1, 0.01, 1e-4, -1e-4)}[model]
    sc, sem = scene(m, extra)
    opts = mi_ba.default_options()
    with mi_ba.Context(opts, sc.copy(), sem) as ctx:
        for (i, j) in [(0, 1), (1, 0), (2, 1)]:
            pix, st, err, world = ctx.semantic_export(i, j)
            pix_o, st_o, err_o, world_o = oracle.semantic_export(opts, sc, sem, i, j)
            assert len(st) == 24 * 24
            assert np.array_equal(pix, pix_o)
            assert np.array_equal(st, st_o)
            assert np.array_equal(err, err_o)
            assert np.array_equal(world, world_o)
        # the configured pair (0, 1): its samples are the grid rows with depth
        ctx.evaluate_semantic()
        px_s, st_s, r_s, _ = ctx.download_semantic()
        pix, st, err, _ = ctx.semantic_export(0, 1)
        sel = px_s[:, 0] == 0
        grid = {(int(x), int(y)): k for k, (x, y) in enumerate(pix[:, :2])}
        rows = np.array([grid[(int(x), int(y))] for x, y in px_s[sel, 1:]])
        assert len(rows) <= 24 * 21  # the 12-pixel zero-depth band: 3 grid rows are no samples
        assert np.array_equal(st[rows], st_s[sel]) and np.array_equal(err[rows], r_s[sel])
        assert (st == mi_ba.VALID).sum() > 100 and err.sum() > 0


def test_export_needs_resident_rasters(gpu):
    sc, sem = scene(mi_ba.SIMPLE_PINHOLE)
    # pairs (0, 1), (1, 2): images 1 and 2 are some pair's second image, so
    # only their rasters are on the device; the export needs both images'
    only = mi_ba.SemanticInput(sem.depth, sem.label, np.array([(0, 1), (1, 2)], np.int32), pixel_step=4)
    with mi_ba.Context(mi_ba.default_options(), sc.copy(), only) as ctx:
        ctx.semantic_export(1, 2)
        ctx.semantic_export(2, 1)
        for i, j in ((0, 1), (1, 0)):
            with pytest.raises(mi_ba.MiBaError) as e:
                ctx.semantic_export(i, j)  # image 0 is no pair's second image: no raster on the device
            assert e.value.status == mi_ba.ERR_UNSUPPORTED
        with pytest.raises(mi_ba.MiBaError):
            ctx.semantic_export(1, 1)
