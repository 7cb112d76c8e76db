"""Property test of the semantic flat test (csrc/semantic.hip flat_box /
flat_check; derivation in DESIGN.md §4).

The two-pass semantic linearization clears most samples without evaluating
their Ceres CENTRAL stencil (NumericDiffCostFunction<..., CENTRAL, 1, 4, 3,
4, 3>, semantic_cost_functions.h:247-258): it proves that every stencil point
reprojects to a pixel (and depth) with the centre's outcome, so every CENTRAL
difference is +0.0.  Here the oracle restates that test with its own
arithmetic (oracle.cc FlatClears) and checks it against the full stencil of
every sample (the reference's compute_semantic_error, :87-208, 29 / 15
evaluations): a cleared sample whose stencil values are not all equal to its
centre residual is a counterexample.  Pass: zero counterexamples over
>= 1e7 samples spanning the three models of the configs, Ceres relative step
sizes 1e-2 .. 1e-6, strong distortion, projections at and beyond the image
border, fine label cells and depths near the threshold.  (The GPU parity
tests then check that the product's flat pass clears exactly such samples:
tests/test_gpu_parity.py test_semantic_flat_test_regimes.)
"""
import numpy as np
import pytest

import mi_ba
import oracle

SIZE = 400
EXTRA = {
    mi_ba.SIMPLE_PINHOLE: (0, 0, 0, 0),
    mi_ba.SIMPLE_RADIAL: (0.05, 0, 0, 0),
    mi_ba.OPENCV: (-0.1, 0.01, 1e-4, -1e-4),
}


def scene(model, extra, rel_step, seed, rot=0.05, tnoise=0.02, cell=0.05, depth_noise=0.0, threshold=2.0, step=2):
    sc = mi_ba.generate_scene(mi_ba.synth_config(model, 6, 50, track_length=6, image_size=SIZE,
                                                 rotation_range=rot, extra=extra, seed=seed))
    sc.gauge()
    sc.camera_constant = np.ones(6, np.uint8)
    depth, label = mi_ba.render_semantic(sc, SIZE, SIZE, plane_z=1.0, cell=cell)
    rng = np.random.default_rng(seed)
    if depth_noise:
        depth = (depth * (1.0 + rng.uniform(-depth_noise, depth_noise, depth.shape))).astype(np.float32)
    pairs = np.array([(i, j) for i in range(6) for j in range(6) if i != j], np.int32)
    sem = mi_ba.SemanticInput(depth, label, pairs, pixel_step=step, depth_error_threshold=threshold,
                              numeric_relative_step_size=rel_step)
    sc.tvec[1:] += rng.uniform(-tnoise, tnoise, sc.tvec[1:].shape)
    return sc, sem


CASES = [
    # model, extra, relative step, seed, keyword overrides
    (mi_ba.SIMPLE_PINHOLE, EXTRA[mi_ba.SIMPLE_PINHOLE], 1e-3, 1, {}),
    (mi_ba.SIMPLE_RADIAL, EXTRA[mi_ba.SIMPLE_RADIAL], 1e-2, 2, {}),
    (mi_ba.SIMPLE_RADIAL, (0.4, 0, 0, 0), 1e-3, 3, {}),                      # strong radial distortion
    (mi_ba.OPENCV, EXTRA[mi_ba.OPENCV], 1e-4, 4, {}),
    (mi_ba.OPENCV, (-0.6, 0.3, 0.01, -0.01), 1e-3, 5, {}),                   # strong OPENCV distortion
    (mi_ba.OPENCV, (-0.6, 0.3, 0.01, -0.01), 1e-2, 6, {}),
    (mi_ba.OPENCV, EXTRA[mi_ba.OPENCV], 1e-6, 7, {}),
    (mi_ba.SIMPLE_PINHOLE, EXTRA[mi_ba.SIMPLE_PINHOLE], 1e-5, 8,
     dict(depth_noise=0.05, threshold=0.3)),                                 # depths near the threshold
    (mi_ba.OPENCV, EXTRA[mi_ba.OPENCV], 1e-3, 9, dict(rot=0.2, tnoise=0.5)),  # projections across the border
    (mi_ba.SIMPLE_RADIAL, EXTRA[mi_ba.SIMPLE_RADIAL], 1e-3, 10, dict(cell=0.01, step=1)),  # fine labels, every pixel
]


@pytest.mark.parametrize("coarse", [0, 1, 2, 3])
def test_flat_test_never_clears_a_non_flat_stencil(coarse):
    """coarse 1 / 2 / 3: the forms with the stencil classes gathered into a
    rotation and a translation group (semantic_flat_coarse, csrc/semantic.hip
    flat_box_coarse; 1 bounds |A| from the radius, 2 keeps the camera model's
    exact A, 3 bounds the two groups apart)."""
    total = cleared = nonzero = 0
    rows = []
    for model, extra, rel, seed, kw in CASES:
        sc, sem = scene(model, extra, rel, seed, **kw)
        c = oracle.semantic_flat_property(mi_ba.default_options(), sc, sem, coarse=coarse)
        rows.append((model, rel, seed, c))
        assert c["cleared_not_flat"] == 0, (model, extra, rel, seed, kw, c)
        total += c["samples"]
        cleared += c["cleared"]
        nonzero += c["nonzero_jacobian"]
    for r in rows:
        print(r)
    assert total >= 10_000_000, total
    # the test is useful (clears most samples) and the cases exercise real boundaries
    assert cleared >= 0.5 * total, (cleared, total)
    assert nonzero >= 10_000, nonzero


def test_property_check_catches_an_unsound_bound():
    """Negative control: with the pixel bound shrunk to 30 % the restated test
    clears samples whose stencil is not flat, and the check reports them."""
    sc, sem = scene(mi_ba.OPENCV, (-0.6, 0.3, 0.01, -0.01), 1e-2, 6)
    c = oracle.semantic_flat_property(mi_ba.default_options(), sc, sem, bound_scale=0.3)
    assert c["cleared_not_flat"] > 0, c
    c = oracle.semantic_flat_property(mi_ba.default_options(), sc, sem, bound_scale=0.3, coarse=1)
    assert c["cleared_not_flat"] > 0, c
