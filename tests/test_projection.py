"""Reprojection errors and the post-BA track filter on the GPU
(mi_ba_squared_reprojection_errors, mi_ba_filter_points3d) against the
oracle: CalculateSquaredReprojectionError (src/base/projection.cc:111-128,
pinned by projection_test.cc:95-124 in test_oracle_golden.py) and
FilterPoints3DWithLargeReprojectionError (src/base/reconstruction.cc:
1472-1525, restated in oracle.filter_points3d).

Tolerances: squared errors within 1e-12 relative (+1e-12 px^2 absolute),
DBL_MAX bitwise for points behind the camera; keep masks and the filtered
count exactly equal; point errors within 1e-12 relative.
"""
import numpy as np
import pytest

import mi_ba
import oracle
from test_mixed_models import mixed_scene

pytestmark = pytest.mark.gpu

DBL_MAX = np.finfo(np.float64).max


def scene_with_outliers(seed=0):
    sc = mixed_scene(images=8, points=400, track=4, seed=seed)
    rng = np.random.default_rng(seed)
    # outliers of various sizes, a few points behind every camera, a
    # single-observation track, unnormalised quaternions
    bad = rng.choice(sc.num_obs, sc.num_obs // 10, replace=False)
    sc.obs_xy[bad] += rng.normal(0, 8, (len(bad), 2))
    sc.xyz[:3, 2] = -50.0
    keep = np.ones(sc.num_obs, bool)
    lone = int(sc.obs_point[0])
    idx = np.nonzero(sc.obs_point == lone)[0]
    keep[idx[1:]] = False
    for name in ("obs_xy", "obs_image", "obs_point"):
        setattr(sc, name, getattr(sc, name)[keep])
    sc.qvec *= 1.5
    return sc


def test_squared_errors_match_oracle(gpu):
    sc = scene_with_outliers()
    g = mi_ba.squared_reprojection_errors(sc)
    o = oracle.scene_squared_reprojection_errors(sc)
    behind = o == DBL_MAX
    assert behind.sum() > 0 and np.array_equal(g == DBL_MAX, behind)
    assert np.all(np.abs(g[~behind] - o[~behind]) <= 1e-12 * np.abs(o[~behind]) + 1e-12)


@pytest.mark.parametrize("max_err", [0.5, 2.0, 4.0, 1e9])
def test_filter_points_match_oracle(gpu, max_err):
    sc = scene_with_outliers(seed=1)
    sq = oracle.scene_squared_reprojection_errors(sc)
    prior = np.full(sc.num_points, -1.0)
    ok_o, pk_o, err_o, nf_o = oracle.filter_points3d(sc, max_err, point_error=prior, sq=sq)
    ok_g, pk_g, err_g, nf_g = mi_ba.filter_points3d(sc, max_err, point_error=prior)
    assert nf_g == nf_o and np.array_equal(ok_g, ok_o) and np.array_equal(pk_g, pk_o)
    assert np.all(np.abs(err_g - err_o) <= 1e-12 * np.abs(err_o))
    assert (not pk_o.all()) and (max_err > 100 or nf_o > 0)


def test_filter_points_mask_and_empty(gpu):
    sc = scene_with_outliers(seed=2)
    mask = np.zeros(sc.num_points, np.uint8)
    mask[::3] = 1
    ok_o, pk_o, err_o, nf_o = oracle.filter_points3d(sc, 2.0, point_mask=mask)
    ok_g, pk_g, err_g, nf_g = mi_ba.filter_points3d(sc, 2.0, point_mask=mask)
    assert nf_g == nf_o and np.array_equal(ok_g, ok_o) and np.array_equal(pk_g, pk_o)
    assert np.all(np.abs(err_g - err_o) <= 1e-12 * np.abs(err_o))
    assert pk_g[mask == 0].all()
    empty = sc.copy()
    for name in ("obs_xy", "obs_image", "obs_point"):
        setattr(empty, name, getattr(empty, name)[:0])
    ok, pk, _, nf = mi_ba.filter_points3d(empty, 2.0)
    assert nf == 0 and len(ok) == 0 and not pk.any()  # every track empty: deleted, nothing filtered
    assert len(mi_ba.squared_reprojection_errors(empty)) == 0


def test_c4_size_properties(gpu):
    """C4 size (10M observations): errors of the synthetic scene are the
    generator's noise (bounded), and the filter at a 4 px threshold keeps
    every observation whose error is below it."""
    c = mi_ba.synth_config(mi_ba.OPENCV, 1000, 1_000_000, track_length=10, rotation_range=0.05,
                           extra=(-0.1, 0.01, 1e-4, -1e-4))
    sc = mi_ba.generate_scene(c)
    g = mi_ba.squared_reprojection_errors(sc)
    assert len(g) == 10_000_000 and np.all(g < 4.0 * 4.0 * 2)
    ok, pk, err, nf = mi_ba.filter_points3d(sc, 4.0)
    assert nf == 0 and ok.all() and pk.all()
    # 1 px: the decision rule restated over whole arrays
    ok, pk, err, nf = mi_ba.filter_points3d(sc, 1.0)
    bad = g > 1.0
    P = sc.num_points
    nbad = np.bincount(sc.obs_point, weights=bad, minlength=P).astype(np.int64)
    tl = np.bincount(sc.obs_point, minlength=P)
    deleted = (tl < 2) | (nbad >= tl - 1)
    assert nf == int(tl[deleted].sum() + nbad[~deleted].sum())
    assert np.array_equal(pk, ~deleted)
    assert np.array_equal(ok, ~bad & ~deleted[sc.obs_point])
    mean = np.bincount(sc.obs_point, weights=np.where(bad, 0.0, np.sqrt(g)), minlength=P) / np.maximum(tl - nbad, 1)
    assert np.allclose(err[~deleted], mean[~deleted], rtol=1e-12, atol=0)
    sample = np.random.default_rng(0).choice(sc.num_obs, 2000, replace=False)
    sub = sc.copy()
    for name in ("obs_xy", "obs_image", "obs_point"):
        setattr(sub, name, getattr(sub, name)[sample])
    o = oracle.scene_squared_reprojection_errors(sub)
    assert np.all(np.abs(g[sample] - o) <= 1e-12 * np.abs(o) + 1e-12)
