"""The flat pass's label planes (semantic_label_planes): an 8-bit index plane
into the rasters' distinct label bit patterns and 8 x 8 tile depth ranges
(extended by the 2 pixels a 3 x 3 box can reach past the tile) settle most
samples of the flat test without the float rasters.  The test is the same
per-pixel outcome comparison as the raster route (semantic_cost_functions.h:
141-205; the range bound: |d - z| is convex in d), so every sample's status,
residual, Jacobian and deferral must be bitwise those of the raster route —
with few labels (the planes used), labels that differ only in sign of zero or
NaN payload, and more than 256 distinct labels (the palette overflows and the
flat pass reads the rasters).  Semantic parity is unpinned by reference
fixtures; the raster route is the one pinned bitwise against the oracle."""
import numpy as np
import pytest

import mi_ba

pytestmark = pytest.mark.gpu


def scene(seed=0):
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 8, 200, track_length=3, image_size=160,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=seed)).gauge()
    depth, label = mi_ba.render_semantic(sc, 160, 160, cell=0.5)
    sc.tvec[3:] += 0.003
    return sc, depth, label


def run(sc, sem, lp):
    with mi_ba.Context(mi_ba.default_options(), sc.copy(), sem) as ctx:
        ctx.set_tuning("semantic_window_summary", 0)
        ctx.set_tuning("semantic_label_planes", lp)
        ctx.set_tuning("semantic_diag", 2)
        ctx.evaluate_semantic()
        return ctx.download_semantic()


def decode(st):
    st = np.where(st >= 0xC000, st - 0x10000, st)  # +0x10000: a deferred sample redone per point
    return st >= 0x2800  # +0x4000: decided without the float rasters


@pytest.mark.parametrize("labels", ["few", "signed_zero_nan", "many"])
def test_label_planes_bitwise(gpu, labels):
    sc, depth, label = scene()
    rng = np.random.default_rng(1)
    if labels == "signed_zero_nan":
        label = label.copy()
        label[label == 0] = -0.0
        label[:, ::7, ::5] = 0.0
        label[:, ::11, ::3] = np.float32(np.nan)
    elif labels == "many":
        label = (label + rng.integers(0, 600, size=label.shape)).astype(np.float32)
    depth = depth.copy()
    depth[:, 40:44, :] *= 1.5  # depth steps: tiles that cannot settle the depth test
    pairs = np.array([(i, (i + 1) % 8) for i in range(8)] + [(i, (i + 3) % 8) for i in range(8)], np.int32)
    sem = mi_ba.SemanticInput(depth, label, pairs, pixel_step=3)
    a, b = run(sc, sem, 0), run(sc, sem, 1)
    for k, (x, y) in enumerate(zip(a, b)):
        if k != 1:  # the status is compared below, without the diagnostic mark
            assert np.array_equal(x, y)
    st_a, st_b = a[1], b[1]
    plain = lambda st: np.where(decode(st), st - 0x4000, st) % 0x10000  # noqa: E731
    assert np.array_equal(plain(st_a), plain(st_b))
    # a box wholly outside the raster is decided without it in every mode
    # (every stencil point OUT_OF_BOUNDS); the planes decide the rest
    outside_a = decode(st_a) & (plain(st_a) == 0xFFFF)
    assert outside_a.sum() > 0
    assert np.array_equal(outside_a, decode(st_b) & (plain(st_b) == 0xFFFF))
    settled_b = (decode(st_b) & ~outside_a).sum()
    assert (decode(st_a) & ~outside_a).sum() == 0  # neither summary in use
    if labels == "many":
        assert settled_b == 0  # > 256 labels: no planes
    else:
        assert settled_b > 0.1 * len(st_b)
