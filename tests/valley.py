"""Near-null directions of the reduced camera system (test helper).

Where two LM solves of one problem stop at points that differ by more than
their costs do, the question is whether the difference lies along the
problem's flat valley.  This builds the Jacobi-scaled reduced camera system
S = F'F - F'E (E'E)^-1 E'F at a point from the oracle's tangent Jacobian
(oracle.reproj_eval: the same columns the LM's Schur solve uses, scaled as
its Jacobi scaling does) and decomposes the camera-side difference of two
solutions along S's eigenvectors.  SIMPLE_RADIAL, one camera per image, no
constant points (the synthetic C2-style scenes).  Test infrastructure only.
"""
import numpy as np
import scipy.sparse as sp

import oracle


def _qmul(p, q):
    w1, x1, y1, z1 = p.T
    w2, x2, y2, z2 = q.T
    return np.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], 1)


def reduced_system(options, scene):
    """(S over the variable camera-side columns, their indices, the column
    scaling of the camera side) at the scene's parameters."""
    bo, _, J = oracle.reproj_eval(options, scene)
    I, P, C = scene.num_images, scene.num_points, scene.num_cameras
    nb, _, W = J.shape
    ct = W - 9
    img = scene.obs_image[bo]
    pt = scene.obs_point[bo]
    cam = scene.image_camera[img]
    nf = 6 * I + ct * C
    cols = np.zeros((nb, W), np.int64)
    cols[:, :6] = 6 * img[:, None] + np.arange(6)
    cols[:, 6:9] = nf + 3 * pt[:, None] + np.arange(3)
    cols[:, 9:] = 6 * I + ct * cam[:, None] + np.arange(ct)
    rows = np.repeat(np.arange(2 * nb), W)
    Jm = sp.csr_matrix((J.reshape(-1), (rows, np.broadcast_to(cols[:, None, :], (nb, 2, W)).reshape(-1))),
                       shape=(2 * nb, nf + 3 * P))
    colnorm = np.sqrt(np.asarray(Jm.multiply(Jm).sum(axis=0)).ravel())
    scale = 1.0 / (1.0 + colnorm)  # Ceres' Jacobi scaling
    Js = (Jm @ sp.diags(scale)).tocsc()
    Jf, Je = Js[:, :nf], Js[:, nf:]
    V = (Je.T @ Je).tocsr()
    Vinv = sp.block_diag([np.linalg.inv(V[3 * p:3 * p + 3, 3 * p:3 * p + 3].toarray()) for p in range(P)]).tocsr()
    Wm = (Jf.T @ Je).tocsr()
    S = (Jf.T @ Jf).toarray() - (Wm @ Vinv @ Wm.T).toarray()
    var = np.nonzero(np.diag(S) > 0)[0]
    return S[np.ix_(var, var)], var, scale[:nf]


def camera_difference(a, b):
    """Tangent camera-side difference b - a at a (QuaternionManifold: Plus(q,
    d) = [cos|d|, sin|d| d/|d|] * q, so d ~ vec(q_b q_a^-1); tvec; the
    refined SIMPLE_RADIAL intrinsics f, k), f-vector layout."""
    I, C = a.num_images, a.num_cameras
    qa = a.qvec / np.linalg.norm(a.qvec, axis=1, keepdims=True)
    qb = b.qvec / np.linalg.norm(b.qvec, axis=1, keepdims=True)
    qr = _qmul(qb, qa * np.array([1, -1, -1, -1]))
    qr *= np.sign(qr[:, :1])
    d = np.zeros(6 * I + 2 * C)
    pose = np.arange(6 * I).reshape(I, 6)
    d[pose[:, :3]] = qr[:, 1:]
    d[pose[:, 3:]] = b.tvec - a.tvec
    cp = np.asarray(b.camera_params).reshape(C, -1) - np.asarray(a.camera_params).reshape(C, -1)
    d[6 * I:] = cp[:, [0, 3]].reshape(-1)
    return d


def valley_report(options, a, b):
    """Decompose b's camera-side difference from a along the eigenvectors of
    the scaled reduced camera system at a.  Returns dict(lam: eigenvalues
    ascending, energy: cumulative fraction of |d|^2 in the k smallest
    eigenvectors, rayleigh: d'Sd / d'd, norm: |d| (scaled coordinates))."""
    S, var, scale = reduced_system(options, a)
    lam, U = np.linalg.eigh(S)
    d = (camera_difference(a, b) / scale)[var]
    c = U.T @ d
    e = np.cumsum(c ** 2) / max(np.sum(c ** 2), 1e-300)
    return dict(lam=lam, energy=e, rayleigh=float(d @ S @ d / max(d @ d, 1e-300)), norm=float(np.linalg.norm(d)))
