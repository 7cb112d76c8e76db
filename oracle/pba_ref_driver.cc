// pba_ref_driver.cc — TEST INFRASTRUCTURE ONLY (never linked by the product).
//
// Runs the reference's own PBA CPU double-precision solver (lib/PBA of the
// reference, compiled from its sources where they lie by oracle/Makefile.ref
// into oracle/_ref/libpba_ref.so) on a flattened SIMPLE_RADIAL problem,
// configured exactly as ParallelBundleAdjuster::Solve does
// (src/optim/bundle_adjustment.cc:559-636): BUNDLE_FULL, projection
// distortion, intrinsics fixed iff neither focal nor extra params are refined,
// __lm_delta_threshold and __lm_gradient_threshold / 100, __lm_mse_threshold
// 0, __cg_min_iteration 10; cameras from AddImagesToProblem (:699-741: R as
// QuaternionToRotationMatrix(q), f, k, t), observations shifted by the
// principal point (AddPointsToProblem :743-781, tracks contiguous per point);
// costs from the MSE as in :617-626 (final_cost = MSE * num_residuals / 4).
// Results are written back like TearDown (:639-663).
#include <cmath>
#include <vector>

#include "pba.h"

namespace {

void quat_to_rot(const double* q, double* R) {  // row-major, q = (w, x, y, z), normalised
  const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const double w = q[0] / n, x = q[1] / n, y = q[2] / n, z = q[3] / n;
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w);     R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w);     R[7] = 2 * (y * z + x * w);     R[8] = 1 - 2 * (x * x + y * y);
}

void rot_to_quat(const double* R, double* q) {  // RotationMatrixToQuaternion, w >= 0
  const double tr = R[0] + R[4] + R[8];
  if (tr > 0) {
    const double s = 0.5 / std::sqrt(tr + 1.0);
    q[0] = 0.25 / s; q[1] = (R[7] - R[5]) * s; q[2] = (R[2] - R[6]) * s; q[3] = (R[3] - R[1]) * s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    const double s = 2.0 * std::sqrt(1.0 + R[0] - R[4] - R[8]);
    q[0] = (R[7] - R[5]) / s; q[1] = 0.25 * s; q[2] = (R[1] + R[3]) / s; q[3] = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    const double s = 2.0 * std::sqrt(1.0 + R[4] - R[0] - R[8]);
    q[0] = (R[2] - R[6]) / s; q[1] = (R[1] + R[3]) / s; q[2] = 0.25 * s; q[3] = (R[5] + R[7]) / s;
  } else {
    const double s = 2.0 * std::sqrt(1.0 + R[8] - R[0] - R[4]);
    q[0] = (R[3] - R[1]) / s; q[1] = (R[2] + R[6]) / s; q[2] = (R[5] + R[7]) / s; q[3] = 0.25 * s;
  }
  if (q[0] < 0) for (int k = 0; k < 4; ++k) q[k] = -q[k];
}

}  // namespace

// One image per camera (PBA has no shared intrinsics).  params[ncam][4] =
// SIMPLE_RADIAL (f, cx, cy, k); qvec[ncam][4], tvec[ncam][3]; xyz[npt][3];
// observations sorted by point (obs_pt non-decreasing).  Returns 0 on
// success; parameters are updated in place.
extern "C" int pba_ref_solve(int ncam, double* params, double* qvec, double* tvec, int npt, double* xyz, int nobs,
                             const double* obs_xy, const int* obs_cam, const int* obs_pt, int max_iterations,
                             int refine_intrinsics, int num_threads, double* initial_cost, double* final_cost,
                             int* iterations) {
  std::vector<pba::CameraT> cams(ncam);
  for (int i = 0; i < ncam; ++i) {
    double R[9];
    quat_to_rot(qvec + 4 * i, R);
    cams[i].SetFocalLength(params[4 * i]);
    cams[i].SetProjectionDistortion(params[4 * i + 3]);
    cams[i].SetMatrixRotation(R);
    cams[i].SetTranslation(tvec + 3 * i);
    cams[i].SetVariableCamera();
  }
  std::vector<pba::Point3D> pts(npt);
  for (int p = 0; p < npt; ++p) pts[p].SetPoint(xyz + 3 * p);
  std::vector<pba::Point2D> meas(nobs);
  std::vector<int> cidx(obs_cam, obs_cam + nobs), pidx(obs_pt, obs_pt + nobs);
  for (int o = 0; o < nobs; ++o) {
    const double* K = params + 4 * obs_cam[o];
    meas[o].SetPoint2D(obs_xy[2 * o] - K[1], obs_xy[2 * o + 1] - K[2]);
  }
  pba::ParallelBA ba(pba::ParallelBA::PBA_CPU_DOUBLE, num_threads);
  ba.SetNextBundleMode(pba::ParallelBA::BUNDLE_FULL);
  ba.EnableRadialDistortion(pba::ParallelBA::PBA_PROJECTION_DISTORTION);
  ba.SetFixedIntrinsics(!refine_intrinsics);
  pba::ConfigBA* cfg = ba.GetInternalConfig();
  cfg->__lm_delta_threshold /= 100.0f;
  cfg->__lm_gradient_threshold /= 100.0f;
  cfg->__lm_mse_threshold = 0.0f;
  cfg->__cg_min_iteration = 10;
  cfg->__verbose_level = 0;
  cfg->__lm_max_iteration = max_iterations;
  ba.SetCameraData(cams.size(), cams.data());
  ba.SetPointData(pts.size(), pts.data());
  ba.SetProjection(meas.size(), meas.data(), pidx.data(), cidx.data());
  ba.RunBundleAdjustment();
  const double nres = 2.0 * nobs;
  *initial_cost = cfg->GetInitialMSE() * nres / 4;
  *final_cost = cfg->GetFinalMSE() * nres / 4;
  *iterations = cfg->GetIterationsLM();
  for (int i = 0; i < ncam; ++i) {
    double R[9];
    cams[i].GetMatrixRotation(R);
    rot_to_quat(R, qvec + 4 * i);
    cams[i].GetTranslation(tvec + 3 * i);
    params[4 * i] = cams[i].GetFocalLength();
    params[4 * i + 3] = cams[i].GetProjectionDistortion();
  }
  for (int p = 0; p < npt; ++p) pts[p].GetPoint(xyz + 3 * p);
  return 0;
}
