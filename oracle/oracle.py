"""ctypes binding of liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference hot path (see oracle.cc).  Imported only
by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as
the checker, never as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.join(os.path.dirname(_HERE), "semantic-bundle-adjustment-colmap_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)
import mi_ba  # noqa: E402  (struct layouts of the boundary)

LIB_PATH = os.path.join(_HERE, "liboracle.so")
_dp = C.POINTER(C.c_double)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    lib.oracle_world_to_image.argtypes = [C.c_int, _dp, C.c_double, C.c_double, _dp, _dp]
    lib.oracle_image_to_world.argtypes = [C.c_int, _dp, C.c_double, C.c_double, _dp, _dp]
    lib.oracle_reproj_residual.argtypes = [C.c_int, _dp, _dp, _dp, _dp, C.c_double, C.c_double, _dp]
    lib.oracle_squared_reprojection_error.restype = C.c_double
    lib.oracle_squared_reprojection_error.argtypes = [C.c_int, _dp, _dp, _dp, _dp, _dp]
    lib.oracle_setup_stats.argtypes = [C.POINTER(mi_ba.Options), C.POINTER(mi_ba.Problem),
                                       C.POINTER(mi_ba.SetupInfo)]
    lib.oracle_reproj_eval.restype = C.c_int64
    lib.oracle_reproj_eval.argtypes = [C.POINTER(mi_ba.Options), C.POINTER(mi_ba.Problem), _i64p, _dp, _dp,
                                       C.c_int64]
    lib.oracle_reproj_throughput.restype = C.c_double
    lib.oracle_reproj_throughput.argtypes = [C.POINTER(mi_ba.Options), C.POINTER(mi_ba.Problem), C.c_int64,
                                             C.c_int, C.c_int, _i64p]
    lib.oracle_semantic_export.restype = C.c_int64
    lib.oracle_semantic_export.argtypes = [C.POINTER(mi_ba.Options), C.POINTER(mi_ba.Problem),
                                           C.POINTER(mi_ba.Semantic), C.c_int32, C.c_int32, _i32p, _i32p,
                                           _dp, _dp, C.c_int64]
    lib.oracle_semantic_eval.restype = C.c_int64
    lib.oracle_semantic_eval.argtypes = [C.POINTER(mi_ba.Options), C.POINTER(mi_ba.Problem),
                                         C.POINTER(mi_ba.Semantic), _i32p, _i32p, _dp, _dp, C.c_int64]
    lib.oracle_semantic_throughput.restype = C.c_double
    lib.oracle_semantic_throughput.argtypes = [C.POINTER(mi_ba.Options), C.POINTER(mi_ba.Problem),
                                               C.POINTER(mi_ba.Semantic), C.c_int64, C.c_int, _i64p]
    lib.oracle_solve.argtypes = [C.POINTER(mi_ba.Options), C.POINTER(mi_ba.Problem), C.POINTER(mi_ba.Semantic),
                                 C.POINTER(mi_ba.Summary)]
    lib.oracle_gsba_render.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
    lib.oracle_gsba_evaluate.restype = C.c_int64
    lib.oracle_gsba_evaluate.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                         C.c_void_p]
    lib.oracle_gsba_solve.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.oracle_gsba_iou.restype = C.c_double
    lib.oracle_gsba_iou.argtypes = [_dp, _dp, _dp, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    lib.oracle_cholesky.restype = C.c_int
    lib.oracle_cholesky.argtypes = [_dp, C.c_int]
    lib.oracle_semantic_flat_property.argtypes = [C.POINTER(mi_ba.Options), C.POINTER(mi_ba.Problem),
                                                  C.POINTER(mi_ba.Semantic), _i64p]
    lib.oracle_set_flat_bound_scale.argtypes = [C.c_double]
    lib.oracle_set_flat_bound_scale.restype = None
    lib.oracle_set_flat_coarse.argtypes = [C.c_int]
    lib.oracle_set_flat_coarse.restype = None
    lib.oracle_set_dense_factor.argtypes = [DENSE_FACTOR_FN]
    lib.oracle_set_dense_factor.restype = None
    lib.oracle_set_trace.argtypes = [_i32p, C.c_int]
    lib.oracle_set_trace.restype = None
    lib.oracle_set_trace_values.argtypes = [_dp]
    lib.oracle_set_trace_values.restype = None
    _lib = lib
    return lib


# int (*)(double* A, int n): row-major lower factor in place, 0 or failing column
DENSE_FACTOR_FN = C.CFUNCTYPE(C.c_int, _dp, C.c_int)


def _lapack_factor(ptr, n):
    """LAPACK dpotrf on the oracle's row-major lower triangle: the same bytes
    read column-major are the upper triangle, and dpotrf(lower=0) leaves U
    with U'U = A there, i.e. L = U' row-major."""
    from scipy.linalg import lapack
    A = np.ctypeslib.as_array(ptr, shape=(n, n))
    F = A.T  # column-major view, no copy
    c, info = lapack.dpotrf(F, lower=0, clean=0, overwrite_a=1)
    if not np.shares_memory(c, A):
        F[...] = c
    return int(info)


_lapack_thunk = DENSE_FACTOR_FN(_lapack_factor)


def use_lapack_factor(enable: bool = True):
    """Route the oracle LM's reduced-camera-system factorisation through
    LAPACK dpotrf (multi-threaded; for C4-sized systems, nf ~ 12 000) instead
    of the oracle's own blocked Cholesky.  Test infrastructure only."""
    load().oracle_set_dense_factor(_lapack_thunk if enable else DENSE_FACTOR_FN())


def _a(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    return x, x.ctypes.data_as(_dp)


def world_to_image(model, params, u, v):
    p, pp = _a(params)
    x, y = C.c_double(), C.c_double()
    load().oracle_world_to_image(model, pp, u, v, C.byref(x), C.byref(y))
    return x.value, y.value


def image_to_world(model, params, x, y):
    p, pp = _a(params)
    u, v = C.c_double(), C.c_double()
    load().oracle_image_to_world(model, pp, x, y, C.byref(u), C.byref(v))
    return u.value, v.value


def reproj_residual(model, q, t, X, cam, obs):
    arrs = [_a(a) for a in (q, t, X, cam)]
    r = np.zeros(2)
    load().oracle_reproj_residual(model, arrs[0][1], arrs[1][1], arrs[2][1], arrs[3][1], float(obs[0]),
                                  float(obs[1]), r.ctypes.data_as(_dp))
    return r


def squared_reprojection_error(model, params, xy, X, q, t):
    arrs = [_a(a) for a in (params, xy, X, q, t)]
    return load().oracle_squared_reprojection_error(model, *[a[1] for a in arrs])


def scene_squared_reprojection_errors(scene):
    """CalculateSquaredReprojectionError (projection.cc:111-128) of every
    observation of a flattened scene (per-camera models)."""
    off = scene.camera_param_offsets()
    out = np.zeros(scene.num_obs)
    for k in range(scene.num_obs):
        i, p = int(scene.obs_image[k]), int(scene.obs_point[k])
        c = int(scene.image_camera[i])
        model = int(scene.camera_models[c]) if scene.camera_models is not None else scene.camera_model
        out[k] = squared_reprojection_error(model, scene.camera_params.reshape(-1)[off[c]:off[c + 1]],
                                            scene.obs_xy[k], scene.xyz[p], scene.qvec[i], scene.tvec[i])
    return out


def filter_points3d(scene, max_reproj_error, point_mask=None, point_error=None, sq=None):
    """Reconstruction::FilterPoints3DWithLargeReprojectionError
    (reconstruction.cc:1472-1525) over every point with point_mask[p] != 0;
    a point's track elements in observation order.  Returns (obs_keep,
    point_keep, point_error, num_filtered)."""
    sq = scene_squared_reprojection_errors(scene) if sq is None else sq
    max_sq = max_reproj_error * max_reproj_error
    P = scene.num_points
    obs_keep = np.ones(scene.num_obs, bool)
    point_keep = np.ones(P, bool)
    err = np.zeros(P) if point_error is None else np.array(point_error, np.float64)
    order = np.argsort(scene.obs_point, kind="stable")
    bounds = np.searchsorted(scene.obs_point[order], np.arange(P + 1))
    num_filtered = 0
    for p in range(P):
        if point_mask is not None and not point_mask[p]:
            continue
        track = order[bounds[p]:bounds[p + 1]]
        if len(track) < 2:                                   # :1486-1490
            num_filtered += len(track)
            point_keep[p] = False
            obs_keep[track] = False
            continue
        bad = [k for k in track if sq[k] > max_sq]           # :1496-1504
        s = 0.0
        for k in track:
            if not sq[k] > max_sq:
                s += float(np.sqrt(sq[k]))
        if len(bad) >= len(track) - 1:                       # :1507-1509
            num_filtered += len(track)
            point_keep[p] = False
            obs_keep[track] = False
        else:                                                # :1510-1516
            num_filtered += len(bad)
            obs_keep[bad] = False
            err[p] = s / (len(track) - len(bad))
    return obs_keep, point_keep, err, num_filtered


def gsba_render(scene, cylinders, height, width):
    """Trunk masks [I][H][W] uint8: the union of the cylinders' projected
    quadrilaterals (drawQuadrilateral) per image."""
    lib = load()
    n = len(cylinders)
    arr = (mi_ba.Cylinder * max(1, n))()
    for k in range(n):
        arr[k].qvec[:] = list(cylinders[k][:4])
        arr[k].tvec[:] = list(cylinders[k][4:7])
        arr[k].radius = float(cylinders[k][7])
        arr[k].height = float(cylinders[k][8])
    out = np.zeros((scene.num_images, height, width), np.uint8)
    p = scene.problem()
    lib.oracle_gsba_render(C.byref(p), arr, n, height, width, out.ctypes.data_as(C.c_void_p))
    return out


def gsba_evaluate(options, scene, gsba):
    lib = load()
    p = scene.problem()
    g, arr = gsba.struct()
    n = lib.oracle_gsba_evaluate(C.byref(options), C.byref(p), C.byref(g), 0, None, None, None)
    if n < 0:
        raise RuntimeError("oracle_gsba_evaluate status %d" % -n)
    ids = np.zeros((n, 2), np.int32)
    r = np.zeros(n)
    J = np.zeros((n, 16))
    lib.oracle_gsba_evaluate(C.byref(options), C.byref(p), C.byref(g), n, ids.ctypes.data_as(C.c_void_p),
                             r.ctypes.data_as(C.c_void_p), J.ctypes.data_as(C.c_void_p))
    return ids, r, J


def gsba_solve(options, scene, gsba):
    lib = load()
    s = mi_ba.Summary()
    p = scene.problem()
    g, arr = gsba.struct()
    st = lib.oracle_gsba_solve(C.byref(options), C.byref(p), C.byref(g), C.byref(s))
    if st != 0:
        raise RuntimeError("oracle_gsba_solve status %d" % st)
    gsba.read_back(arr)
    return s


def gsba_iou(cq, ct, K, cylinder, mask):
    lib = load()
    y = mi_ba.Cylinder()
    y.qvec[:] = list(cylinder[:4])
    y.tvec[:] = list(cylinder[4:7])
    y.radius = float(cylinder[7])
    y.height = float(cylinder[8])
    m = np.ascontiguousarray(mask, np.uint8)
    return lib.oracle_gsba_iou(_a(cq)[1], _a(ct)[1], _a(K)[1], C.byref(y), m.ctypes.data_as(C.c_void_p),
                               m.shape[0], m.shape[1])


def setup_stats(options, scene) -> "mi_ba.SetupInfo":
    info = mi_ba.SetupInfo()
    sc = scene.copy()  # SetUp normalises qvecs in place
    p = sc.problem()
    st = load().oracle_setup_stats(C.byref(options), C.byref(p), C.byref(info))
    if st != 0:
        raise RuntimeError(f"oracle_setup_stats status {st}")
    return info


def reproj_eval(options, scene):
    """Residual + tangent Jacobian of every program block (program order)."""
    sc = scene.copy()
    p = sc.problem()
    lib = load()
    n = lib.oracle_reproj_eval(C.byref(options), C.byref(p), None, None, None, 0)
    if n < 0:
        raise RuntimeError(f"oracle_reproj_eval status {-n}")
    info = setup_stats(options, scene)
    w = 9 + info.camera_tangent_size
    bo = np.empty(n, np.int64)
    r = np.empty((n, 2))
    J = np.empty((n, 2, w))
    sc = scene.copy()
    p = sc.problem()
    lib.oracle_reproj_eval(C.byref(options), C.byref(p), bo.ctypes.data_as(_i64p), r.ctypes.data_as(_dp),
                           J.ctypes.data_as(_dp), n)
    return bo, r, J


def semantic_eval(options, scene, semantic):
    sc = scene.copy()
    p = sc.problem()
    s = semantic.struct()
    lib = load()
    n = lib.oracle_semantic_eval(C.byref(options), C.byref(p), C.byref(s), None, None, None, None, 0)
    if n < 0:
        raise RuntimeError(f"oracle_semantic_eval status {-n}")
    px = np.empty((n, 3), np.int32)
    st = np.empty(n, np.int32)
    r = np.empty(n)
    J = np.empty((n, 12))
    sc = scene.copy()
    p = sc.problem()
    lib.oracle_semantic_eval(C.byref(options), C.byref(p), C.byref(s), px.ctypes.data_as(_i32p),
                             st.ctypes.data_as(_i32p), r.ctypes.data_as(_dp), J.ctypes.data_as(_dp), n)
    return px, st, r, J


def semantic_export(options, scene, semantic, image1, image2):
    """ExportSemanticErrorToCSV rows of (image1, image2) at the scene's
    parameters: (pixels [n][4], status [n], error [n], world [n][3])."""
    s = semantic.struct()
    sc = scene.copy()
    p = sc.problem()
    lib = load()
    n = lib.oracle_semantic_export(C.byref(options), C.byref(p), C.byref(s), image1, image2, None, None, None, None, 0)
    if n < 0:
        raise RuntimeError(f"oracle_semantic_export status {-n}")
    pix = np.empty((n, 4), np.int32)
    st = np.empty(n, np.int32)
    err = np.empty(n)
    world = np.empty((n, 3))
    sc = scene.copy()
    p = sc.problem()
    lib.oracle_semantic_export(C.byref(options), C.byref(p), C.byref(s), image1, image2, pix.ctypes.data_as(_i32p),
                               st.ctypes.data_as(_i32p), err.ctypes.data_as(_dp), world.ctypes.data_as(_dp), n)
    return pix, st, err, world


def semantic_flat_property(options, scene, semantic, bound_scale=1.0, coarse=False):
    """The product's semantic flat test (restated) vs the full CENTRAL
    stencil over every sample: dict(samples, cleared, cleared_not_flat,
    nonzero_jacobian, flat_deferred).  cleared_not_flat must be 0.
    bound_scale < 1 shrinks the pixel bound (negative control); coarse 1 / 2:
    the forms with the classes' componentwise maxima (semantic_flat_coarse;
    1 bounds |A| from the radius, 2 keeps it exact)."""
    sc = scene.copy()
    p = sc.problem()
    s = semantic.struct()
    counts = np.zeros(5, np.int64)
    lib = load()
    lib.oracle_set_flat_bound_scale(bound_scale)
    lib.oracle_set_flat_coarse(int(coarse))
    try:
        st = lib.oracle_semantic_flat_property(C.byref(options), C.byref(p), C.byref(s), counts.ctypes.data_as(_i64p))
    finally:
        lib.oracle_set_flat_bound_scale(1.0)
        lib.oracle_set_flat_coarse(0)
    if st != 0:
        raise RuntimeError(f"oracle_semantic_flat_property status {st}")
    return dict(zip(("samples", "cleared", "cleared_not_flat", "nonzero_jacobian", "flat_deferred"),
                    (int(v) for v in counts)))


def cholesky(A):
    """Lower Cholesky factor of a symmetric matrix (the oracle's DENSE_SCHUR
    factorisation).  Returns (L, info)."""
    M = np.ascontiguousarray(A, dtype=np.float64).copy()
    info = load().oracle_cholesky(M.ctypes.data_as(_dp), M.shape[0])
    return np.tril(M), info


def solve(options, scene, semantic=None):
    """CPU LM + dense Schur; updates scene arrays in place."""
    s = mi_ba.Summary()
    p = scene.problem()
    sem = semantic.struct() if semantic is not None else None
    st = load().oracle_solve(C.byref(options), C.byref(p), C.byref(sem) if sem is not None else None, C.byref(s))
    if st != 0:
        raise RuntimeError(f"oracle_solve status {st}")
    return s


def solve_traced(options, scene, semantic=None, return_values=False):
    """oracle.solve plus the per-iteration LM trace: an int32 array
    [iterations][4] = (step valid, step successful, linear solver iterations,
    1 on the iteration that ended the solve), rows of iterations that did not
    run are -1; with return_values also a float array [iterations][4] =
    (step norm, the parameter tolerance's bound, cost change, model cost
    change) of each valid step (NaN elsewhere)."""
    cap = max(1, int(options.max_num_iterations))
    buf = np.full((cap, 4), -1, np.int32)
    vals = np.full((cap, 4), np.nan)
    lib = load()
    lib.oracle_set_trace(buf.ctypes.data_as(_i32p), cap)
    lib.oracle_set_trace_values(vals.ctypes.data_as(_dp))
    try:
        s = solve(options, scene, semantic)
    finally:
        lib.oracle_set_trace(None, 0)
        lib.oracle_set_trace_values(None)
    if return_values:
        return s, buf, vals
    return s, buf


def reproj_throughput(options, scene, max_blocks, repeats=1, threads=1):
    sc = scene.copy()
    p = sc.problem()
    done = C.c_int64()
    sec = load().oracle_reproj_throughput(C.byref(options), C.byref(p), max_blocks, repeats, threads,
                                          C.byref(done))
    return sec, done.value


def semantic_throughput(options, scene, semantic, max_samples, threads=1):
    sc = scene.copy()
    p = sc.problem()
    s = semantic.struct()
    done = C.c_int64()
    sec = load().oracle_semantic_throughput(C.byref(options), C.byref(p), C.byref(s), max_samples, threads,
                                            C.byref(done))
    return sec, done.value


# ---------------------------------------------------------------------------
# oracle/_ref: the reference's own PBA CPU double solver (built from the
# reference's lib/PBA sources by oracle/Makefile.ref when /root/reference is
# present; the built .so travels with the tree).  Cross-check of converged
# geometric BA for SIMPLE_RADIAL (ParallelBundleAdjuster, bundle_adjustment.cc:559-663).
REF_LIB_PATH = os.path.join(_HERE, "_ref", "libpba_ref.so")
_ref_lib = None


def ref_available():
    return os.path.exists(REF_LIB_PATH)


def load_ref():
    global _ref_lib
    if _ref_lib is None:
        lib = C.CDLL(REF_LIB_PATH)
        lib.pba_ref_solve.argtypes = [C.c_int, _dp, _dp, _dp, C.c_int, _dp, C.c_int, _dp, _i32p, _i32p, C.c_int,
                                      C.c_int, C.c_int, _dp, _dp, _i32p]
        _ref_lib = lib
    return _ref_lib


def pba_ref_solve(scene, max_iterations=50, refine_intrinsics=True, threads=1):
    """Runs the reference PBA (CPU, double) on a SIMPLE_RADIAL scene with one
    camera per image; updates the scene in place; returns (initial_cost,
    final_cost, lm_iterations) as ParallelBundleAdjuster reports them."""
    assert scene.camera_model == mi_ba.SIMPLE_RADIAL
    order = np.argsort(scene.obs_point, kind="stable")
    cam_of_img = np.asarray(scene.image_camera)
    assert len(np.unique(cam_of_img)) == scene.num_images, "PBA: one camera per image"
    params = np.ascontiguousarray(scene.camera_params[cam_of_img], dtype=np.float64).copy()
    q = np.ascontiguousarray(scene.qvec, dtype=np.float64).copy()
    t = np.ascontiguousarray(scene.tvec, dtype=np.float64).copy()
    X = np.ascontiguousarray(scene.xyz, dtype=np.float64).copy()
    xy = np.ascontiguousarray(scene.obs_xy[order], dtype=np.float64)
    oc = np.ascontiguousarray(scene.obs_image[order], dtype=np.int32)
    op = np.ascontiguousarray(scene.obs_point[order], dtype=np.int32)
    ic, fc, it = C.c_double(0), C.c_double(0), C.c_int32(0)
    rc = load_ref().pba_ref_solve(scene.num_images, params.ctypes.data_as(_dp), q.ctypes.data_as(_dp),
                                  t.ctypes.data_as(_dp), scene.num_points, X.ctypes.data_as(_dp), len(op),
                                  xy.ctypes.data_as(_dp), oc.ctypes.data_as(_i32p), op.ctypes.data_as(_i32p),
                                  max_iterations, int(refine_intrinsics), threads, C.byref(ic), C.byref(fc),
                                  C.byref(it))
    if rc != 0:
        raise RuntimeError(f"pba_ref_solve failed: {rc}")
    scene.camera_params[cam_of_img] = params
    scene.qvec[:], scene.tvec[:], scene.xyz[:] = q, t, X
    return ic.value, fc.value, it.value
