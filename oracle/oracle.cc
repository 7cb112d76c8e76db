// oracle.cc — TEST INFRASTRUCTURE ONLY (the checker, never the product).
//
// CPU restatement of the reference hot path, exported as a C ABI for ctypes.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
// liboracle.so.  Every function cites the reference file:line it restates
// (AlainSchoebi/semantic-bundle-adjustment-colmap, COLMAP 3.8 fork; Ceres 2.1
// is a third-party dependency that the reference does not vendor — its
// algorithms are restated from its published behaviour and marked so).
//
// Pinning: the known answers of src/base/cost_functions_test.cc:41-99,
// src/base/projection_test.cc:95-124, src/base/camera_models_test.cc:39-218
// and the structural counts of src/optim/bundle_adjustment_test.cc:186-642
// are asserted against this oracle in tests/test_oracle_golden.py.
// The semantic path has no reference tests or data: "parity unpinned" for
// that oracle beyond self-consistency.
#include <algorithm>
#include <array>
#include <cmath>
#include <omp.h>
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <map>
#include <set>
#include <vector>

#include "../include/mi_ba.h"
#include "oracle_math.h"
#include "oracle_gsba.h"

using namespace oracle;

namespace {

constexpr int kJ = 18;  // 4 (q) + 3 (t) + 3 (X) + 8 (max camera params)
typedef Jet<kJ> J18;

// cost_functions.h:57-81 (BundleAdjustmentCostFunction::operator()) and
// :116-142 (BundleAdjustmentConstantPoseCostFunction::operator()).
template <typename T>
void ReprojResidual(int model, const T q[4], const T t[3], const T X[3], const T* cam,
                    double ox, double oy, T r[2]) {
  T projection[3];
  UnitQuaternionRotatePoint(q, X, projection);
  projection[0] += t[0];
  projection[1] += t[1];
  projection[2] += t[2];
  projection[0] /= projection[2];
  projection[1] /= projection[2];
  WorldToImage(model, cam, projection[0], projection[1], &r[0], &r[1]);
  r[0] -= T(ox);
  r[1] -= T(oy);
}

constexpr int kLossScaled = 3;  // internal: ceres::ScaledLoss(nullptr, scale)

// Ceres 2.1 loss functions (restated): rho[0..2] at s = |r|^2.
void LossEvaluate(int type, double scale, double s, double rho[3]) {
  if (type == MI_BA_LOSS_SOFT_L1) {
    const double b = scale * scale, c = 1.0 / b;
    const double sum = 1.0 + s * c;
    const double tmp = std::sqrt(sum);
    rho[0] = 2.0 * b * (tmp - 1.0);
    rho[1] = std::max(std::numeric_limits<double>::min(), 1.0 / tmp);
    rho[2] = -(c * rho[1]) / (2.0 * sum);
  } else if (type == MI_BA_LOSS_CAUCHY) {
    const double b = scale * scale, c = 1.0 / b;
    const double sum = 1.0 + s * c;
    const double inv = 1.0 / sum;
    rho[0] = b * std::log(sum);
    rho[1] = std::max(std::numeric_limits<double>::min(), inv);
    rho[2] = -c * (inv * inv);
  } else if (type == kLossScaled) {  // ScaledLoss(nullptr, a): the GSBA weights
    rho[0] = scale * s; rho[1] = scale; rho[2] = 0.0;
  } else {
    rho[0] = s; rho[1] = 1.0; rho[2] = 0.0;
  }
}

// Ceres 2.1 Corrector (corrector.cc, restated): applied to residuals and
// Jacobian rows of one block.  nres = residual count, ncols = columns.
void ApplyCorrector(const double rho[3], double sq_norm, int nres, double* r, int ncols, double* J) {
  const double sqrt_rho1 = std::sqrt(rho[1]);
  double residual_scaling, alpha_sq_norm;
  if (sq_norm == 0.0 || rho[2] <= 0.0) {
    residual_scaling = sqrt_rho1;
    alpha_sq_norm = 0.0;
  } else {
    const double D = 1.0 + 2.0 * sq_norm * rho[2] / rho[1];
    const double alpha = 1.0 - std::sqrt(D);
    residual_scaling = sqrt_rho1 / (1 - alpha);
    alpha_sq_norm = alpha / sq_norm;
  }
  if (J) {
    if (alpha_sq_norm == 0.0) {
      for (int i = 0; i < nres * ncols; ++i) J[i] *= sqrt_rho1;
    } else {
      for (int c = 0; c < ncols; ++c) {
        double rtJ = 0.0;
        for (int k = 0; k < nres; ++k) rtJ += r[k] * J[k * ncols + c];
        for (int k = 0; k < nres; ++k)
          J[k * ncols + c] = sqrt_rho1 * (J[k * ncols + c] - alpha_sq_norm * r[k] * rtJ);
      }
    }
  }
  for (int k = 0; k < nres; ++k) r[k] *= residual_scaling;
}

// ---------------------------------------------------------------------------
// Problem assembly: BundleAdjuster::SetUp / AddImageToProblem /
// AddPointToProblem / ParameterizeCameras / ParameterizePoints
// (src/optim/bundle_adjustment.cc:326-530) + Ceres reduced program.
// ---------------------------------------------------------------------------
struct Setup {
  int ct = 0;                          // widest camera tangent (Jacobian rows are 9 + ct wide)
  std::vector<int> cam_model;          // model id per camera (camera_models.h:117-141)
  std::vector<int64_t> cam_poff;       // offset of the camera's params in camera_params
  std::vector<std::vector<int>> cam_tangent;  // per camera: refined param indices (SubsetManifold)
  std::vector<int64_t> block_obs;      // blocks in program order
  std::vector<uint8_t> block_const_pose;
  std::vector<double> block_pose;      // [nb][7] baked (q,t) for constant-pose blocks
  std::vector<uint8_t> block_reduced;  // has >= 1 variable parameter block
  std::vector<uint8_t> img_var;        // pose is a variable parameter block
  std::vector<uint8_t> img_tvec_mask;  // constant tvec coords (bitmask)
  std::vector<uint8_t> cam_var;        // camera block variable with tangent > 0
  std::vector<uint8_t> pt_var;
  int64_t num_residuals_reduced = 0;
  int64_t num_effective_parameters_reduced = 0;
};

int BuildSetup(const mi_ba_options* o, mi_ba_problem* p, Setup* s) {
  const int I = p->num_images, C = p->num_cameras;
  if (!p->camera_model_ids && NumParams(p->camera_model) < 0) return MI_BA_ERR_UNSUPPORTED;
  s->cam_model.assign(C, 0);
  s->cam_poff.assign(C + 1, 0);
  for (int c = 0; c < C; ++c) {
    s->cam_model[c] = p->camera_model_ids ? p->camera_model_ids[c] : p->camera_model;
    if (NumParams(s->cam_model[c]) < 0) return MI_BA_ERR_UNSUPPORTED;
    s->cam_poff[c + 1] = s->cam_poff[c] + NumParams(s->cam_model[c]);
  }
  const int64_t P = p->num_points, N = p->num_obs;
  auto in_cfg = [&](int i) { return p->image_in_config ? p->image_in_config[i] != 0 : true; };
  auto const_pose_cfg = [&](int i) { return p->image_constant_pose && p->image_constant_pose[i]; };
  auto tvec_mask = [&](int i) { return p->image_constant_tvec ? p->image_constant_tvec[i] : 0; };
  std::vector<std::vector<int64_t>> obs_of_img(I), obs_of_pt(P);
  for (int64_t k = 0; k < N; ++k) {
    obs_of_img[p->obs_image[k]].push_back(k);
    obs_of_pt[p->obs_point[k]].push_back(k);
  }
  std::set<int> cam_ids;
  std::vector<uint8_t> cam_const_cfg(C, 0);
  for (int c = 0; c < C; ++c) cam_const_cfg[c] = p->camera_constant ? p->camera_constant[c] : 0;
  std::map<int64_t, int64_t> pt_nobs;
  s->img_var.assign(I, 0);
  s->img_tvec_mask.assign(I, 0);
  auto add_block = [&](int64_t k, bool cpose, int img) {
    s->block_obs.push_back(k);
    s->block_const_pose.push_back(cpose ? 1 : 0);
    for (int j = 0; j < 4; ++j) s->block_pose.push_back(p->qvec[img * 4 + j]);
    for (int j = 0; j < 3; ++j) s->block_pose.push_back(p->tvec[img * 3 + j]);
  };
  // AddImageToProblem (:348-427)
  for (int i = 0; i < I; ++i) {
    if (!in_cfg(i)) continue;
    // Image::NormalizeQvec -> NormalizeQuaternion (pose.cc:82-91)
    double* q = &p->qvec[i * 4];
    const double norm = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (norm == 0) { q[0] = 1.0; }
    else { for (int j = 0; j < 4; ++j) q[j] = q[j] / norm; }
    const bool cpose = !o->refine_extrinsics || const_pose_cfg(i);
    int64_t nobs = 0;
    for (int64_t k : obs_of_img[i]) {
      nobs += 1;
      pt_nobs[p->obs_point[k]] += 1;
      add_block(k, cpose, i);
    }
    if (nobs > 0) {
      cam_ids.insert(p->image_camera[i]);
      if (!cpose) {
        s->img_var[i] = 1;
        s->img_tvec_mask[i] = tvec_mask(i);
      }
    }
  }
  // AddPointToProblem (:429-478): variable points first, then constant.
  for (int pass = 1; pass <= 2; ++pass) {
    for (int64_t pt = 0; pt < P; ++pt) {
      if (!p->point_config || p->point_config[pt] != pass) continue;
      const int64_t track_len = (int64_t)obs_of_pt[pt].size();
      if (pt_nobs[pt] == track_len) continue;
      for (int64_t k : obs_of_pt[pt]) {
        const int img = p->obs_image[k];
        if (in_cfg(img)) continue;
        pt_nobs[pt] += 1;
        const int cam = p->image_camera[img];
        if (!cam_ids.count(cam)) { cam_ids.insert(cam); cam_const_cfg[cam] = 1; }
        add_block(k, true, img);
      }
    }
  }
  // ParameterizeCameras (:480-516), per camera model
  s->cam_tangent.assign(C, {});
  s->ct = 0;
  for (int c = 0; c < C; ++c) {
    int f[2], nf, pp[2], npp, ex[4], nex;
    ParamGroups(s->cam_model[c], f, &nf, pp, &npp, ex, &nex);
    std::vector<int> const_idx;
    if (!o->refine_focal_length) const_idx.insert(const_idx.end(), f, f + nf);
    if (!o->refine_principal_point) const_idx.insert(const_idx.end(), pp, pp + npp);
    if (!o->refine_extra_params) const_idx.insert(const_idx.end(), ex, ex + nex);
    for (int k = 0; k < NumParams(s->cam_model[c]); ++k)
      if (std::find(const_idx.begin(), const_idx.end(), k) == const_idx.end()) s->cam_tangent[c].push_back(k);
    s->ct = std::max(s->ct, (int)s->cam_tangent[c].size());
  }
  const bool constant_camera = !o->refine_focal_length && !o->refine_principal_point && !o->refine_extra_params;
  s->cam_var.assign(C, 0);
  for (int cam : cam_ids) {
    if (constant_camera || cam_const_cfg[cam]) continue;
    // Ceres: a SubsetManifold with tangent size 0 makes the block constant.
    if (!s->cam_tangent[cam].empty()) s->cam_var[cam] = 1;
  }
  // ParameterizePoints (:518-530)
  s->pt_var.assign(P, 0);
  for (auto& e : pt_nobs) {
    const int64_t pt = e.first;
    bool constant = (int64_t)obs_of_pt[pt].size() > e.second;
    if (p->point_config && p->point_config[pt] == 2) constant = true;
    s->pt_var[pt] = constant ? 0 : 1;
  }
  // Ceres reduced program: drop residual blocks whose parameter blocks are
  // all constant, then parameter blocks no longer referenced.
  const int64_t nb = (int64_t)s->block_obs.size();
  s->block_reduced.assign(nb, 0);
  std::vector<uint8_t> used_img(I, 0), used_cam(C, 0), used_pt(P, 0);
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t k = s->block_obs[b];
    const int img = p->obs_image[k];
    const int cam = p->image_camera[img];
    const int64_t pt = p->obs_point[k];
    const bool vpose = !s->block_const_pose[b] && s->img_var[img];
    const bool any = vpose || s->cam_var[cam] || s->pt_var[pt];
    if (!any) continue;
    s->block_reduced[b] = 1;
    s->num_residuals_reduced += 2;
    if (vpose) used_img[img] = 1;
    if (s->cam_var[cam]) used_cam[cam] = 1;
    if (s->pt_var[pt]) used_pt[pt] = 1;
  }
  int64_t ne = 0;
  for (int i = 0; i < I; ++i)
    if (used_img[i]) {
      int masked = 0;
      for (int k = 0; k < 3; ++k) masked += (s->img_tvec_mask[i] >> k) & 1;
      ne += 3 + (3 - masked);
    }
  for (int c = 0; c < C; ++c)
    if (used_cam[c]) ne += (int64_t)s->cam_tangent[c].size();
  for (int64_t pt = 0; pt < P; ++pt)
    if (used_pt[pt]) ne += 3;
  s->num_effective_parameters_reduced = ne;
  return MI_BA_OK;
}

// Evaluate one geometric block: residual (2) and tangent Jacobian row-major
// [2][9+c] with column order rot(3) trans(3) point(3) cam(c), via Jets.
void EvalBlock(const Setup& s, const mi_ba_problem* p, int64_t b, double r[2], double* Jt) {
  const int64_t k = s.block_obs[b];
  const int img = p->obs_image[k];
  const int cam = p->image_camera[img];
  const int64_t pt = p->obs_point[k];
  const int np = NumParams(s.cam_model[cam]);
  const bool cpose = s.block_const_pose[b] != 0;
  const double* qv = cpose ? &s.block_pose[b * 7] : &p->qvec[img * 4];
  const double* tv = cpose ? &s.block_pose[b * 7 + 4] : &p->tvec[img * 3];
  J18 q[4], t[3], X[3], params[8], res[2];
  for (int j = 0; j < 4; ++j) q[j] = cpose ? J18(qv[j]) : J18(qv[j], j);
  for (int j = 0; j < 3; ++j) t[j] = cpose ? J18(tv[j]) : J18(tv[j], 4 + j);
  for (int j = 0; j < 3; ++j) X[j] = J18(p->xyz[pt * 3 + j], 7 + j);
  for (int j = 0; j < np; ++j) params[j] = J18(p->camera_params[s.cam_poff[cam] + j], 10 + j);
  ReprojResidual(s.cam_model[cam], q, t, X, params, p->obs_xy[k * 2], p->obs_xy[k * 2 + 1], res);
  r[0] = res[0].a;
  r[1] = res[1].a;
  if (!Jt) return;
  // rows are 9 + s.ct wide; a camera with fewer refined intrinsics leaves
  // the rest of its columns zero
  const int c = (int)s.cam_tangent[cam].size();
  const int w = 9 + s.ct;
  double PJ[12];
  QuaternionPlusJacobian(qv, PJ);
  const bool vpose = !cpose && s.img_var[img];
  for (int row = 0; row < 2; ++row) {
    double* Jr = Jt + row * w;
    const double* d = res[row].v;
    for (int col = 0; col < 3; ++col) {
      double acc = 0.0;
      for (int m = 0; m < 4; ++m) acc += d[m] * PJ[m * 3 + col];
      Jr[col] = vpose ? acc : 0.0;
    }
    for (int col = 0; col < 3; ++col) {
      const bool masked = (s.img_tvec_mask[img] >> col) & 1;
      Jr[3 + col] = (vpose && !masked) ? d[4 + col] : 0.0;
    }
    for (int col = 0; col < 3; ++col) Jr[6 + col] = s.pt_var[pt] ? d[7 + col] : 0.0;
    for (int col = 0; col < s.ct; ++col) Jr[9 + col] = (col < c && s.cam_var[cam]) ? d[10 + s.cam_tangent[cam][col]] : 0.0;
  }
}

// ---------------------------------------------------------------------------
// Semantic residual: BaseSemanticBACostFunction::compute_semantic_error
// (src/base/semantic_cost_functions.h:87-208), with P_c1 precomputed
// (:103-118; pose-independent, so evaluating it once is bitwise identical).
// ---------------------------------------------------------------------------
struct SemSample {
  int32_t pair, x, y;
  double pc1[3];
  float label1;
};

// One image's depth / semantic map (the depth_maps_ / semantic_maps_ entry,
// semantic_bundle_adjustment.cc:1021-1068): its own rows x cols.
struct SemRaster {
  const float* depth;
  const float* label;
  int H, W;
};

// Every image's raster (mi_ba_semantic: one size for all, or per-image sizes
// with the planes back to back in image order).
struct SemPlanes {
  std::vector<SemRaster> img;
  void build(const mi_ba_semantic* sem, int I) {
    img.assign(I, SemRaster{nullptr, nullptr, 0, 0});
    int64_t off = 0;
    for (int i = 0; i < I; ++i) {
      const int H = sem->image_height ? sem->image_height[i] : sem->height;
      const int W = sem->image_width ? sem->image_width[i] : sem->width;
      img[i] = SemRaster{sem->depth + off, sem->label + off, H, W};
      off += (int64_t)H * W;
    }
  }
};

struct SemSetup {
  std::vector<SemSample> samples;
  std::vector<uint8_t> pair_var1, pair_var2;  // pose i / pose j variable
  SemPlanes planes;
};

// semantic_bundle_adjustment.cc:699-906 (AddImagePairToProblem): pixel grid
// of image 1's own size (:792-799), y outer, x inner, step s, skip depth <
// 1e-4, skip both-constant pairs.
void BuildSemSetup(const mi_ba_options* o, const mi_ba_problem* p, const Setup& s,
                   const mi_ba_semantic* sem, SemSetup* ss) {
  const int step = sem->pixel_step;
  ss->planes.build(sem, p->num_images);
  ss->pair_var1.assign(sem->num_pairs, 0);
  ss->pair_var2.assign(sem->num_pairs, 0);
  for (int k = 0; k < sem->num_pairs; ++k) {
    const int i = sem->pairs[2 * k], j = sem->pairs[2 * k + 1];
    if (i == j) continue;
    const bool c1 = !o->refine_extrinsics || (p->image_constant_pose && p->image_constant_pose[i]);
    const bool c2 = !o->refine_extrinsics || (p->image_constant_pose && p->image_constant_pose[j]);
    if (c1 && c2) continue;
    ss->pair_var1[k] = !c1;
    ss->pair_var2[k] = !c2;
    const int cam1 = p->image_camera[i];
    const double* K1 = &p->camera_params[s.cam_poff[cam1]];
    const SemRaster& r1 = ss->planes.img[i];
    const int H = r1.H, W = r1.W;
    const float* depth1 = r1.depth;
    const float* label1 = r1.label;
    for (int y = 0; y < H; y += step) {
      for (int x = 0; x < W; x += step) {
        const float depth = depth1[(int64_t)y * W + x];
        if (depth < 1e-4) continue;
        SemSample smp;
        smp.pair = k; smp.x = x; smp.y = y;
        double u1, v1;
        ImageToWorld(s.cam_model[cam1], K1, (double)x, (double)y, &u1, &v1);
        smp.pc1[0] = u1 * (double)depth;
        smp.pc1[1] = v1 * (double)depth;
        smp.pc1[2] = (double)depth;
        smp.label1 = label1[(int64_t)y * W + x];
        ss->samples.push_back(smp);
      }
    }
  }
}

// compute_semantic_error (semantic_cost_functions.h:87-208) against image j
// (raster r2 = image j's maps); pw_out / pxy_out (nullable): return_point3D /
// return_point2D_2.
double SemanticErrorTo(const mi_ba_problem* p, const Setup& s, const mi_ba_semantic* sem, int j, const SemRaster& r2,
                       const SemSample& smp, const double q1[4], const double t1[3], const double q2[4],
                       const double t2[3], int* status, double* pw_out = nullptr, int* pxy_out = nullptr);

double SemanticError(const mi_ba_problem* p, const Setup& s, const mi_ba_semantic* sem, const SemSetup& ss,
                     const SemSample& smp, const double q1[4], const double t1[3], const double q2[4],
                     const double t2[3], int* status) {
  const int j = sem->pairs[2 * smp.pair + 1];
  return SemanticErrorTo(p, s, sem, j, ss.planes.img[j], smp, q1, t1, q2, t2, status);
}

double SemanticErrorTo(const mi_ba_problem* p, const Setup& s, const mi_ba_semantic* sem, int j, const SemRaster& r2,
                       const SemSample& smp, const double q1[4], const double t1[3], const double q2[4],
                       const double t2[3], int* status, double* pw_out, int* pxy_out) {
  const int cam2 = p->image_camera[j];
  const double* K2 = &p->camera_params[s.cam_poff[cam2]];
  double q1i[4], t1i[3];
  PoseInverse(q1, t1, q1i, t1i);                       // :121-125
  double pw[3];
  PoseTransformPoint(q1i, t1i, smp.pc1, pw);           // :127-128
  if (pw_out) for (int m = 0; m < 3; ++m) pw_out[m] = pw[m];  // :131-133
  double pc2[3];
  PoseTransformPoint(q2, t2, pw, pc2);                 // :136-138
  const double u2 = pc2[0] / pc2[2];                   // :141-144
  const double v2 = pc2[1] / pc2[2];
  const double measured_depth_2 = pc2[2];
  double x2 = 0.0, y2 = 0.0;
  WorldToImage(s.cam_model[cam2], K2, u2, v2, &x2, &y2); // :149-151
  const int px = CastToIntX86(std::round(x2));         // :154-156
  const int py = CastToIntX86(std::round(y2));
  if (pxy_out) {                                       // :159-160
    pxy_out[0] = px;
    pxy_out[1] = py;
  }
  const int H = r2.H, W = r2.W;                        // depth_map_2_ rows / cols (:163)
  if (px < 0 || px >= W || py < 0 || py >= H) {        // :163-177
    *status = MI_BA_OUT_OF_BOUNDS;
    return 0.0;
  }
  const int64_t off = (int64_t)py * W + px;
  const double depth_2 = (double)r2.depth[off];
  if (std::fabs(depth_2 - measured_depth_2) > sem->depth_error_threshold) {  // :180-196
    *status = MI_BA_INVALID_DEPTH;
    return 0.0;
  }
  *status = MI_BA_VALID;                               // :199-205
  return (smp.label1 == r2.label[off]) ? 0.0 : 1.0;
}

// Ceres 2.1 NumericDiffCostFunction<..., CENTRAL, 1, 4,3[,4,3]> (restated):
// delta_j = max(sqrt(eps), |x_j| * relative_step_size);
// J_j = (f(x + delta e_j) - f(x - delta e_j)) * ((1/delta)/2);
// then QuaternionManifold / SubsetManifold PlusJacobian.
void EvalSemantic(const mi_ba_problem* p, const Setup& s, const mi_ba_semantic* sem, const SemSetup& ss,
                  int64_t n, int* status, double* r, double* J) {
  const SemSample& smp = ss.samples[n];
  const int i = sem->pairs[2 * smp.pair], j = sem->pairs[2 * smp.pair + 1];
  double x[14];
  for (int m = 0; m < 4; ++m) x[m] = p->qvec[i * 4 + m];
  for (int m = 0; m < 3; ++m) x[4 + m] = p->tvec[i * 3 + m];
  for (int m = 0; m < 4; ++m) x[7 + m] = p->qvec[j * 4 + m];
  for (int m = 0; m < 3; ++m) x[11 + m] = p->tvec[j * 3 + m];
  int st;
  *r = SemanticError(p, s, sem, ss, smp, &x[0], &x[4], &x[7], &x[11], status);
  double Jamb[14] = {0};
  const bool var[2] = {ss.pair_var1[smp.pair] != 0, ss.pair_var2[smp.pair] != 0};
  const double min_step = std::sqrt(std::numeric_limits<double>::epsilon());
  for (int blk = 0; blk < 2; ++blk) {
    if (!var[blk]) continue;
    for (int m = 0; m < 7; ++m) {
      const int idx = blk * 7 + m;
      const double orig = x[idx];
      const double delta = std::max(min_step, std::fabs(orig) * sem->numeric_relative_step_size);
      x[idx] = orig + delta;
      const double fp = SemanticError(p, s, sem, ss, smp, &x[0], &x[4], &x[7], &x[11], &st);
      x[idx] = orig - delta;
      const double fm = SemanticError(p, s, sem, ss, smp, &x[0], &x[4], &x[7], &x[11], &st);
      x[idx] = orig;
      double one_over_delta = 1.0 / delta;
      one_over_delta /= 2;
      Jamb[idx] = (fp - fm) * one_over_delta;
    }
  }
  for (int blk = 0; blk < 2; ++blk) {
    double* Jb = J + blk * 6;
    const int img = blk == 0 ? i : j;
    if (!var[blk]) { for (int m = 0; m < 6; ++m) Jb[m] = 0.0; continue; }
    double PJ[12];
    QuaternionPlusJacobian(&x[blk * 7], PJ);
    for (int col = 0; col < 3; ++col) {
      double acc = 0.0;
      for (int m = 0; m < 4; ++m) acc += Jamb[blk * 7 + m] * PJ[m * 3 + col];
      Jb[col] = acc;
    }
    for (int col = 0; col < 3; ++col) {
      const bool masked = (s.img_tvec_mask[img] >> col) & 1;
      Jb[3 + col] = masked ? 0.0 : Jamb[blk * 7 + 4 + col];
    }
  }
}

// ---------------------------------------------------------------------------
// The product's semantic flat test (csrc/semantic.hip flat_box / flat_check
// and stencil_bounds; derivation in DESIGN.md §4), restated with the
// oracle's own arithmetic for the property test
// (tests/test_semantic_flat_property.py): a sample it clears must have every
// CENTRAL stencil value equal to its centre residual.
// ---------------------------------------------------------------------------
// Negative control of the property test (oracle_set_flat_bound_scale): the
// pixel bound bx, by is multiplied by this factor (1 = the product's test).
double g_flat_bound_scale = 1.0;
// 1 / 2 / 3: the coarse forms of the product's flat pass
// (semantic_flat_coarse, csrc/semantic.hip flat_box_coarse): the stencil
// classes gathered into a rotation group and a translation group; 1 / 2
// combine the groups' (du, dv) into one bound, |A| from the radius (1) or
// exact (2); 3 bounds the groups apart, |A| from the radius
// (oracle_set_flat_coarse).
int g_flat_coarse = 0;

struct FlatBounds {
  double rho1 = 0, rho2 = 0, dt1[3] = {0, 0, 0}, dt2[3] = {0, 0, 0}, C[9] = {0};
};

// |R(q') - R(q)| <= 2 d_perp / (|q| - d) per quaternion step, translation
// steps d; padded by 1.001.
void FlatStencilBounds(const double* q, const double* t, double rel, double* rho, double dt[3]) {
  const double min_step = std::sqrt(std::numeric_limits<double>::epsilon());
  const double nq2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  const double nq = std::sqrt(nq2);
  double r = 0.0;
  for (int k = 0; k < 4; ++k) {
    const double delta = std::max(min_step, std::fabs(q[k]) * rel);
    const double d = std::max(std::fabs((q[k] + delta) - q[k]), std::fabs(q[k] - (q[k] - delta)));
    const double perp = d * std::sqrt(std::max(0.0, 1.0 - q[k] * q[k] / nq2));
    const double den = nq - d;
    r = std::max(r, den > 0.0 ? 2.0 * perp / den : std::numeric_limits<double>::infinity());
  }
  *rho = r * 1.001;
  for (int k = 0; k < 3; ++k) {
    const double delta = std::max(min_step, std::fabs(t[k]) * rel);
    dt[k] = std::max(std::fabs((t[k] + delta) - t[k]), std::fabs(t[k] - (t[k] - delta))) * 1.001;
  }
}

double FlatDistortionGain(int model, const double* K, double r2) {
  double s = 0.0;
  if (model == MI_BA_SIMPLE_RADIAL || model == MI_BA_RADIAL)
    for (int k = 3; k < NumParams(model); ++k) s += std::fabs(K[k]);
  else if (model == MI_BA_OPENCV)
    for (int k = 4; k < 8; ++k) s += std::fabs(K[k]);
  const double g = 1.0 + r2;
  return 1.0 + s * g * g * g;
}

// Upper bounds of |d(x, y) / d(u, v)| from the radius (semantic.hip
// image_jac_bound; the coarse form)
void FlatImageJacBound(int model, const double* K, double u, double v, double Ah[4]) {
  const double r2 = u * u + v * v, r1 = std::fabs(u) + std::fabs(v);
  if (model == MI_BA_SIMPLE_PINHOLE) {
    Ah[0] = Ah[3] = std::fabs(K[0]);
    Ah[1] = Ah[2] = 0.0;
  } else if (model == MI_BA_PINHOLE) {
    Ah[0] = std::fabs(K[0]);
    Ah[3] = std::fabs(K[1]);
    Ah[1] = Ah[2] = 0.0;
  } else if (model == MI_BA_SIMPLE_RADIAL) {
    const double k = std::fabs(K[3]);
    Ah[0] = Ah[3] = std::fabs(K[0]) * (1.0 + 3.0 * k * r2);
    Ah[1] = Ah[2] = std::fabs(K[0]) * (k * r2);
  } else if (model == MI_BA_RADIAL) {
    const double k1 = std::fabs(K[3]), k2 = std::fabs(K[4]);
    Ah[0] = Ah[3] = std::fabs(K[0]) * (1.0 + 3.0 * k1 * r2 + 5.0 * k2 * r2 * r2);
    Ah[1] = Ah[2] = std::fabs(K[0]) * (k1 * r2 + 2.0 * k2 * r2 * r2);
  } else {
    const double k1 = std::fabs(K[4]), k2 = std::fabs(K[5]), p1 = std::fabs(K[6]), p2 = std::fabs(K[7]);
    const double rad = 3.0 * k1 * r2 + 5.0 * k2 * r2 * r2;
    const double off = k1 * r2 + 2.0 * k2 * r2 * r2 + 2.0 * (p1 + p2) * r1;
    Ah[0] = std::fabs(K[0]) * (1.0 + rad + (2.0 * p1 + 6.0 * p2) * r1);
    Ah[1] = std::fabs(K[0]) * off;
    Ah[2] = std::fabs(K[1]) * off;
    Ah[3] = std::fabs(K[1]) * (1.0 + rad + (6.0 * p1 + 2.0 * p2) * r1);
  }
}

// every second derivative of (u, v) -> u + Du over |(u, v)| <= rho
double FlatSecondDerivativeBound(int model, const double* K, double rho) {
  if (model == MI_BA_SIMPLE_RADIAL) return 6.0 * std::fabs(K[3]) * rho;
  if (model == MI_BA_RADIAL) return 6.0 * std::fabs(K[3]) * rho + 20.0 * std::fabs(K[4]) * rho * rho * rho;
  if (model == MI_BA_OPENCV)
    return 6.0 * std::fabs(K[4]) * rho + 20.0 * std::fabs(K[5]) * rho * rho * rho +
           6.0 * (std::fabs(K[6]) + std::fabs(K[7]));
  return 0.0;
}

bool FlatClears(const mi_ba_problem* p, const Setup& s, const mi_ba_semantic* sem, const SemSetup& ss, const SemSample& smp,
                const FlatBounds& B, bool var1, bool var2, double r_centre) {
  const int i = sem->pairs[2 * smp.pair], j = sem->pairs[2 * smp.pair + 1];
  const double* q1 = &p->qvec[i * 4];
  const double* t1 = &p->tvec[i * 3];
  const double* q2 = &p->qvec[j * 4];
  const double* t2 = &p->tvec[j * 3];
  const int model = s.cam_model[p->image_camera[j]];
  const double* K = &p->camera_params[s.cam_poff[p->image_camera[j]]];
  double q1i[4], t1i[3], pw[3], p2[3];
  PoseInverse(q1, t1, q1i, t1i);
  PoseTransformPoint(q1i, t1i, smp.pc1, pw);
  PoseTransformPoint(q2, t2, pw, p2);
  const double w[3] = {smp.pc1[0] - t1[0], smp.pc1[1] - t1[1], smp.pc1[2] - t1[2]};
  double mag = 0.0;
  for (int m = 0; m < 3; ++m) mag += std::fabs(smp.pc1[m]) + std::fabs(t1[m]) + std::fabs(pw[m]) + std::fabs(t2[m]);
  const double z = p2[2];
  if (!(z > 0.0)) return false;
  const double iz = 1.0 / z;
  double u = p2[0] * iz, v = p2[1] * iz;
  // x, y and A = d(x, y) / d(u, v) by dual numbers
  Jet<2> Kj[8], uj(u, 0), vj(v, 1), xj, yj;
  for (int m = 0; m < NumParams(model); ++m) Kj[m] = Jet<2>(K[m]);
  WorldToImage(model, Kj, uj, vj, &xj, &yj);
  double x = xj.a, y = yj.a;
  double A[4] = {xj.v[0], xj.v[1], yj.v[0], yj.v[1]};
  if (g_flat_coarse == 1 || g_flat_coarse == 3) {
    // the coarse form expands about the reference's own centre pixel and
    // bounds |A| from the radius (semantic.hip image_jac_bound; form 2 keeps
    // the exact A)
    u = p2[0] / p2[2];
    v = p2[1] / p2[2];
    WorldToImage(model, K, u, v, &x, &y);
    FlatImageJacBound(model, K, u, v, A);
  }
  if (!(std::fabs(x) < 1e8 && std::fabs(y) < 1e8 && std::fabs(u) < 1e6 && std::fabs(v) < 1e6)) return false;
  const double dq1 = var1 ? B.rho1 * std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]) * (1.0 + 1e-12) : 0.0;
  const double dq2 = var2 ? B.rho2 * std::sqrt(pw[0] * pw[0] + pw[1] * pw[1] + pw[2] * pw[2]) * (1.0 + 1e-12) : 0.0;
  std::vector<std::array<double, 3>> cls;
  if (var1) {
    cls.push_back({dq1, dq1, dq1});
    for (int k = 0; k < 3; ++k)
      cls.push_back({B.dt1[k] * std::fabs(B.C[k]), B.dt1[k] * std::fabs(B.C[3 + k]), B.dt1[k] * std::fabs(B.C[6 + k])});
  }
  if (var2) {
    cls.push_back({dq2, dq2, dq2});
    cls.push_back({B.dt2[0], 0.0, 0.0});
    cls.push_back({0.0, B.dt2[1], 0.0});
    cls.push_back({0.0, 0.0, B.dt2[2]});
  }
  if (g_flat_coarse && !cls.empty()) {
    // two groups: the rotation classes (isotropic dq) and the translation
    // classes (componentwise maxima)
    std::array<double, 3> rg = {0.0, 0.0, 0.0}, tg = {0.0, 0.0, 0.0};
    for (const auto& c : cls) {
      const bool rot = c[0] == c[1] && c[1] == c[2] && (c[0] == dq1 || c[0] == dq2) && c[0] > 0.0;
      auto& g = rot ? rg : tg;
      for (int k = 0; k < 3; ++k) g[k] = std::max(g[k], c[k]);
    }
    const double dq = std::max(rg[0], std::max(rg[1], rg[2]));
    cls.assign({{dq, dq, dq}, tg});
  }
  double az = 0.0;
  for (const auto& c : cls) az = std::max(az, c[2]);
  if (!(z - az > 0.5 * z)) return false;
  const double iden = 1.0 / (z - az) * (1.0 + 1e-12);
  double gm = 0.0;
  std::vector<std::array<double, 2>> d;
  for (const auto& c : cls) {
    d.push_back({(c[0] + std::fabs(u) * c[2]) * iden, (c[1] + std::fabs(v) * c[2]) * iden});
    gm = std::max(gm, std::max(d.back()[0], d.back()[1]));
  }
  if (g_flat_coarse == 1 || g_flat_coarse == 2) {  // the groups' (du, dv) combined (3 keeps them apart)
    std::array<double, 2> e = {0.0, 0.0};
    for (const auto& x : d) e = {std::max(e[0], x[0]), std::max(e[1], x[1])};
    d.assign(1, e);
  }
  if (!(gm < 0.1)) return false;
  const double ru = std::fabs(u) + gm, rv = std::fabs(v) + gm;
  const double H = FlatSecondDerivativeBound(model, K, std::sqrt(ru * ru + rv * rv) * (1.0 + 1e-12));
  const double fx = std::fabs(K[0]);
  const double fy = (model == MI_BA_PINHOLE || model == MI_BA_OPENCV) ? std::fabs(K[1]) : std::fabs(K[0]);
  double bxm = 0.0, bym = 0.0;
  for (const auto& e : d) {
    const double sk = e[0] + e[1];
    bxm = std::max(bxm, (std::fabs(A[0]) + fx * H * sk) * e[0] + (std::fabs(A[1]) + fx * H * sk) * e[1]);
    bym = std::max(bym, (std::fabs(A[2]) + fy * H * sk) * e[0] + (std::fabs(A[3]) + fy * H * sk) * e[1]);
  }
  const double gain = FlatDistortionGain(model, K, u * u + v * v);
  const double kscale =
      (std::fabs(K[0]) + std::fabs(K[1])) * gain * (1.0 + std::fabs(u) + std::fabs(v)) * (1.0 + mag * std::fabs(iz));
  const double ex = 1e-6 + 1e-11 * (kscale + std::fabs(x) + std::fabs(y));
  const double bx = (bxm * (1.0 + 1e-12) + ex) * g_flat_bound_scale;
  const double by = (bym * (1.0 + 1e-12) + ex) * g_flat_bound_scale;
  const int x0 = (int)std::round(x - bx), y0 = (int)std::round(y - by);
  const int ncol = (int)std::round(x + bx) - x0 + 1, nrow = (int)std::round(y + by) - y0 + 1;
  if (ncol > 3 || nrow > 3) return false;
  const SemRaster& r2 = ss.planes.img[j];
  const int H_ = r2.H, W_ = r2.W;
  for (int py = y0; py < y0 + nrow; ++py)
    for (int px = x0; px < x0 + ncol; ++px) {
      double f = 0.0;
      if (px >= 0 && px < W_ && py >= 0 && py < H_) {
        const int64_t off = (int64_t)py * W_ + px;
        const double sd = (double)r2.depth[off];
        const double dz = std::fabs(sd - z) - sem->depth_error_threshold;
        if (!(std::fabs(dz) > az + 1e-9 * (1.0 + std::fabs(sd) + mag))) return false;
        f = dz > 0.0 ? 0.0 : (smp.label1 == r2.label[off] ? 0.0 : 1.0);
      }
      if (f != r_centre) return false;
    }
  return true;
}

// ---------------------------------------------------------------------------
// Dense LM + Schur elimination (Ceres 2.1 TrustRegionMinimizer +
// LevenbergMarquardtStrategy + DENSE_SCHUR, restated; bundle_adjustment.cc:
// 271-306 selects it for <= 50 images).
// ---------------------------------------------------------------------------
// GSBA term (geometric_semantic_bundle_adjustment.cc:714-909): one block per
// (config image, cylinder) in config-image then cylinder order.
struct GsbaBlock {
  int img, cyl, variant;
};
struct GsbaSetup {
  const mi_ba_gsba* g = nullptr;
  std::vector<GsbaBlock> blocks;
  std::vector<int64_t> sem_total;  // per image: count of the trunk mask
  std::vector<int64_t> mask_off;   // per image: its trunk mask plane (own size, image_height / image_width)
  std::vector<int> mask_h, mask_w;
  double weight = 1.0;             // ScaledLoss(1 / #config images), :721-722
  bool by2 = false;                // MI_BA_CYLINDER_BY_2_POINTS
  std::vector<double> by2p;        // by2: [ncyl][7] tvec_1, tvec_2, radius (the LM's parameters)
  int cw() const { return by2 ? 7 : 8; }
};

// GeometricSemanticBundleAdjuster::Assert (:664-712) + AddImageToProblem
// (:835-909).
int BuildGsbaSetup(const mi_ba_options* o, const mi_ba_problem* p, const Setup& s, const mi_ba_gsba* g,
                   GsbaSetup* gs) {
  gs->g = g;
  const int I = p->num_images;
  auto in_cfg = [&](int i) { return p->image_in_config ? p->image_in_config[i] != 0 : true; };
  int64_t ncfg = 0;
  for (int i = 0; i < I; ++i) {
    if (!in_cfg(i)) continue;
    ++ncfg;
    const int cam = p->image_camera[i];
    if (!(p->camera_constant && p->camera_constant[cam])) return MI_BA_ERR_UNSUPPORTED;
    if (s.cam_model[cam] != MI_BA_SIMPLE_PINHOLE) return MI_BA_ERR_UNSUPPORTED;
  }
  gs->weight = ncfg > 0 ? 1. / (double)ncfg : 1.0;
  if (g->cylinder_parametrization != MI_BA_CYLINDER_DEFAULT && g->cylinder_parametrization != MI_BA_CYLINDER_BY_2_POINTS)
    return MI_BA_ERR_INVALID_ARGUMENT;
  gs->by2 = g->cylinder_parametrization == MI_BA_CYLINDER_BY_2_POINTS;
  if (gs->by2) {
    // pushBackCylindersReadFromText: every Cylinder converted (cylinder_by_2_points.h:145-153)
    gs->by2p.assign(7 * (size_t)g->num_cylinders, 0.0);
    for (int c = 0; c < g->num_cylinders; ++c) {
      const mi_ba_cylinder& y = g->cylinders[c];
      GsbaCylinderToBy2(y.qvec, y.tvec, y.radius, y.height, &gs->by2p[7 * (size_t)c]);
    }
  }
  gs->sem_total.assign(I, 0);
  gs->mask_off.assign(I, 0);
  gs->mask_h.assign(I, 0);
  gs->mask_w.assign(I, 0);
  int64_t off = 0;
  for (int i = 0; i < I; ++i) {
    gs->mask_h[i] = g->image_height ? g->image_height[i] : g->height;
    gs->mask_w[i] = g->image_width ? g->image_width[i] : g->width;
    gs->mask_off[i] = off;
    const int64_t plane = (int64_t)gs->mask_h[i] * gs->mask_w[i];
    int64_t c = 0;
    for (int64_t k = 0; k < plane; ++k) c += g->trunk_mask[off + k] != 0;
    gs->sem_total[i] = c;
    off += plane;
  }
  for (int i = 0; i < I; ++i) {
    if (!in_cfg(i)) continue;
    const bool constant_pose = !o->refine_extrinsics || (p->image_constant_pose && p->image_constant_pose[i]);
    if (constant_pose && !g->refine_geometry) continue;
    for (int c = 0; c < g->num_cylinders; ++c) {
      const int v = constant_pose ? kGsbaConstantPose : g->refine_geometry ? kGsbaFull : kGsbaConstantCylinder;
      gs->blocks.push_back(GsbaBlock{i, c, v});
    }
  }
  return MI_BA_OK;
}

// Poses of GSBA blocks are variable parameter blocks (SetUpManifolds,
// :1205-1232).
void AddGsbaPoses(const mi_ba_problem* p, const GsbaSetup& gs, Setup* s) {
  for (const GsbaBlock& b : gs.blocks) {
    if (b.variant == kGsbaConstantPose || s->img_var[b.img]) continue;
    s->img_var[b.img] = 1;
    s->img_tvec_mask[b.img] = p->image_constant_tvec ? p->image_constant_tvec[b.img] : 0;
    int masked = 0;
    for (int k = 0; k < 3; ++k) masked += (s->img_tvec_mask[b.img] >> k) & 1;
    s->num_effective_parameters_reduced += 6 - masked;
  }
}

// Residual (1 - IoU) and ambient Jacobian of GSBA block b at the current
// parameters.
double GsbaResidual(const mi_ba_problem* p, const Setup& s, const GsbaSetup& gs, const GsbaBlock& b, double* J16) {
  const mi_ba_gsba* g = gs.g;
  const mi_ba_cylinder& y = g->cylinders[b.cyl];
  const double* K = &p->camera_params[s.cam_poff[p->image_camera[b.img]]];
  const uint8_t* mask = g->trunk_mask + gs.mask_off[b.img];
  const int H = gs.mask_h[b.img], W = gs.mask_w[b.img];
  if (gs.by2)
    return GsbaEvalBlock(b.variant, &p->qvec[b.img * 4], &p->tvec[b.img * 3], K, nullptr, &gs.by2p[7 * (size_t)b.cyl],
                         0.0, 0.0, mask, H, W, gs.sem_total[b.img], g->numeric_relative_step_size, J16);
  return GsbaEvalBlock(b.variant, &p->qvec[b.img * 4], &p->tvec[b.img * 3], K, y.qvec, y.tvec, y.radius, y.height,
                       mask, H, W, gs.sem_total[b.img], g->numeric_relative_step_size, J16);
}

struct Layout {
  // f-block (reduced camera system) coordinates
  std::vector<int> img_off;   // -1 if not variable; 6 tangent slots (masked coords skipped)
  std::vector<int> img_cols;  // mapping slot (0..5) -> column or -1
  std::vector<int> cam_off;
  std::vector<int> cyl_off;   // GSBA cylinders: 8 tangent slots (q 3, t 3, radius, height), by 2 points 7
                              // (tvec_1 3, tvec_2 3, radius), or -1
  int nf = 0;
  std::vector<int64_t> pt_off;  // -1 if constant
  int64_t ne = 0;
};

// Poses of semantic pairs are parameter blocks with the quaternion / tvec
// manifolds of SetUpManifolds (semantic_bundle_adjustment.cc:670-693).
void AddSemanticPoses(const mi_ba_problem* p, const mi_ba_semantic* sem, const SemSetup& ss, Setup* s) {
  for (int k = 0; k < sem->num_pairs; ++k) {
    for (int side = 0; side < 2; ++side) {
      if (!(side == 0 ? ss.pair_var1[k] : ss.pair_var2[k])) continue;
      const int img = sem->pairs[2 * k + side];
      if (s->img_var[img]) continue;
      s->img_var[img] = 1;
      s->img_tvec_mask[img] = p->image_constant_tvec ? p->image_constant_tvec[img] : 0;
      int masked = 0;
      for (int b = 0; b < 3; ++b) masked += (s->img_tvec_mask[img] >> b) & 1;
      s->num_effective_parameters_reduced += 6 - masked;
    }
  }
}

void BuildLayout(const Setup& s, const mi_ba_problem* p, Layout* L, const mi_ba_semantic* sem = nullptr,
                 const SemSetup* ss = nullptr, const GsbaSetup* gs = nullptr) {
  const int I = p->num_images, C = p->num_cameras;
  L->img_off.assign(I, -1);
  L->img_cols.assign((size_t)I * 6, -1);
  std::vector<uint8_t> used_img(I, 0), used_cam(C, 0), used_pt(p->num_points, 0);
  if (sem && ss)
    for (int k = 0; k < sem->num_pairs; ++k) {
      if (ss->pair_var1[k]) used_img[sem->pairs[2 * k]] = 1;
      if (ss->pair_var2[k]) used_img[sem->pairs[2 * k + 1]] = 1;
    }
  std::vector<uint8_t> used_cyl(gs && gs->g ? gs->g->num_cylinders : 0, 0);
  if (gs)
    for (const GsbaBlock& b : gs->blocks) {
      if (b.variant != kGsbaConstantPose) used_img[b.img] = 1;
      if (b.variant != kGsbaConstantCylinder) used_cyl[b.cyl] = 1;
    }
  for (size_t b = 0; b < s.block_obs.size(); ++b) {
    if (!s.block_reduced[b]) continue;
    const int64_t k = s.block_obs[b];
    const int img = p->obs_image[k];
    if (!s.block_const_pose[b] && s.img_var[img]) used_img[img] = 1;
    if (s.cam_var[p->image_camera[img]]) used_cam[p->image_camera[img]] = 1;
    if (s.pt_var[p->obs_point[k]]) used_pt[p->obs_point[k]] = 1;
  }
  int nf = 0;
  for (int i = 0; i < I; ++i) {
    if (!used_img[i]) continue;
    L->img_off[i] = nf;
    for (int m = 0; m < 6; ++m) {
      if (m >= 3 && ((s.img_tvec_mask[i] >> (m - 3)) & 1)) continue;
      L->img_cols[(size_t)i * 6 + m] = nf++;
    }
  }
  L->cam_off.assign(C, -1);
  for (int c = 0; c < C; ++c) {
    if (!used_cam[c]) continue;
    L->cam_off[c] = nf;
    nf += (int)s.cam_tangent[c].size();
  }
  L->cyl_off.assign(used_cyl.size(), -1);
  for (size_t c = 0; c < used_cyl.size(); ++c) {
    if (!used_cyl[c]) continue;
    L->cyl_off[c] = nf;
    nf += gs && gs->by2 ? 7 : 8;
  }
  L->nf = nf;
  L->pt_off.assign(p->num_points, -1);
  int64_t ne = 0;
  for (int64_t pt = 0; pt < p->num_points; ++pt)
    if (used_pt[pt]) { L->pt_off[pt] = ne; ne += 3; }
  L->ne = ne;
}

// Dense Cholesky of the reduced camera system (the oracle's restatement of
// the DENSE_SCHUR factorisation): row-major lower triangle in place, right-
// looking blocked by kCholBlock columns — the diagonal block by the column
// algorithm, the rows below it by forward substitution (one thread per row),
// the trailing lower triangle by row axpys against the transposed panel
// (contiguous, no reassociation).  Returns 0, or the 1-based column of the
// first pivot that is not positive.  O(n^3 / 3) flops over all threads: the
// C4 system (n = 11 993) factors in seconds instead of minutes.
constexpr int kCholBlock = 96;
int CholeskyBlocked(double* A, int n) {
  std::vector<double> P;
  for (int k0 = 0; k0 < n; k0 += kCholBlock) {
    const int k1 = std::min(n, k0 + kCholBlock), w = k1 - k0;
    for (int j = k0; j < k1; ++j) {
      double d = A[(size_t)j * n + j];
      for (int k = k0; k < j; ++k) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
      if (!(d > 0.0)) return j + 1;
      d = std::sqrt(d);
      A[(size_t)j * n + j] = d;
      for (int i = j + 1; i < k1; ++i) {
        double v = A[(size_t)i * n + j];
        for (int k = k0; k < j; ++k) v -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
        A[(size_t)i * n + j] = v / d;
      }
    }
    if (k1 == n) break;
#pragma omp parallel for schedule(static)
    for (int i = k1; i < n; ++i) {
      double* r = A + (size_t)i * n;
      for (int j = k0; j < k1; ++j) {
        double v = r[j];
        for (int k = k0; k < j; ++k) v -= r[k] * A[(size_t)j * n + k];
        r[j] = v / A[(size_t)j * n + j];
      }
    }
    P.assign((size_t)w * n, 0.0);
#pragma omp parallel for schedule(static)
    for (int j = k1; j < n; ++j)
      for (int k = 0; k < w; ++k) P[(size_t)k * n + j] = A[(size_t)j * n + k0 + k];
#pragma omp parallel for schedule(dynamic, 8)
    for (int i = k1; i < n; ++i) {
      double* r = A + (size_t)i * n;
      for (int j0 = k1; j0 <= i; j0 += 512) {
        const int j1 = std::min(i + 1, j0 + 512);
        for (int k = 0; k < w; ++k) {
          const double a = r[k0 + k];
          const double* pk = P.data() + (size_t)k * n;
#pragma omp simd
          for (int j = j0; j < j1; ++j) r[j] -= a * pk[j];
        }
      }
    }
  }
  return 0;
}

// Optional external dense factor (test infrastructure: a LAPACK dpotrf
// wrapper registered from Python, oracle.use_lapack_factor) for the C4-sized
// reduced camera systems; same contract as CholeskyBlocked.
typedef int (*DenseFactorFn)(double* A, int n);
DenseFactorFn g_dense_factor = nullptr;

// Optional per-iteration trace of the LM (test infrastructure,
// oracle_set_trace): per iteration k >= 1, entries [4k-4, 4k) = step valid,
// step successful, linear solver iterations, termination marker (1 on the
// iteration that ended the solve).
int32_t* g_trace = nullptr;
int g_trace_cap = 0;
// ... and its values (oracle_set_trace_values): per iteration k >= 1 with a
// valid step, entries [4k-4, 4k) = step_norm (ambient |x - candidate_x|), the
// parameter tolerance's bound tol (|x| + tol), cost change, model cost change
double* g_trace_v = nullptr;

bool Cholesky(std::vector<double>& A, int n) {  // in place, lower
  if (g_dense_factor) return g_dense_factor(A.data(), n) == 0;
  return CholeskyBlocked(A.data(), n) == 0;
}
void CholSolve(const std::vector<double>& L, int n, std::vector<double>& b) {
  for (int i = 0; i < n; ++i) {
    double v = b[i];
    for (int k = 0; k < i; ++k) v -= L[(size_t)i * n + k] * b[k];
    b[i] = v / L[(size_t)i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double v = b[i];
    for (int k = i + 1; k < n; ++k) v -= L[(size_t)k * n + i] * b[k];
    b[i] = v / L[(size_t)i * n + i];
  }
}
bool Inv3(const double A[9], double Ai[9]) {
  const double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8], c02 = A[3] * A[7] - A[4] * A[6];
  const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
  if (!(std::fabs(det) > 0.0)) return false;
  const double id = 1.0 / det;
  Ai[0] = c00 * id; Ai[1] = (A[2] * A[7] - A[1] * A[8]) * id; Ai[2] = (A[1] * A[5] - A[2] * A[4]) * id;
  Ai[3] = c01 * id; Ai[4] = (A[0] * A[8] - A[2] * A[6]) * id; Ai[5] = (A[2] * A[3] - A[0] * A[5]) * id;
  Ai[6] = c02 * id; Ai[7] = (A[1] * A[6] - A[0] * A[7]) * id; Ai[8] = (A[0] * A[4] - A[1] * A[3]) * id;
  return true;
}

// Sparse-row Jacobian of the whole reduced program, flat: row k has fn[k]
// f-block entries (column, value) at [k * kF, ...) and en[k] e-block
// (point) entries at [k * 3, ...).
struct Linearization {
  static constexpr int kF = 16;
  std::vector<double> r;          // residuals (corrected)
  std::vector<int32_t> fcol;
  std::vector<double> fval;
  std::vector<uint8_t> fn;
  std::vector<int64_t> ecol;
  std::vector<double> eval;
  std::vector<uint8_t> en;
  double cost = 0.0;              // 0.5 sum rho (reduced program only)
  size_t rows() const { return r.size(); }
  void resize(size_t n) {
    r.assign(n, 0.0);
    fcol.assign(n * kF, 0);
    fval.assign(n * kF, 0.0);
    fn.assign(n, 0);
    ecol.assign(n * 3, 0);
    eval.assign(n * 3, 0.0);
    en.assign(n, 0);
  }
};

struct Solver {
  const mi_ba_options* o;
  mi_ba_problem* p;
  const mi_ba_semantic* sem;
  Setup s;
  SemSetup ss;
  GsbaSetup gs;                   // GSBA blocks (empty without a GSBA term)
  Layout L;
  std::vector<int64_t> reduced;   // reduced program blocks, program order

  double GsbaCost(size_t k) {
    const double r = GsbaResidual(p, s, gs, gs.blocks[k], nullptr);
    double rho[3];
    LossEvaluate(kLossScaled, gs.weight, r * r, rho);
    return 0.5 * rho[0];
  }

  double BlockCost(int64_t b) {
    double r[2];
    EvalBlock(s, p, b, r, nullptr);
    double rho[3];
    LossEvaluate(o->loss_function_type, o->loss_function_scale, r[0] * r[0] + r[1] * r[1], rho);
    return 0.5 * rho[0];
  }
  double SemCost(int64_t n) {
    const SemSample& smp = ss.samples[n];
    const int i = sem->pairs[2 * smp.pair], j = sem->pairs[2 * smp.pair + 1];
    int st;
    const double r = SemanticError(p, s, sem, ss, smp, &p->qvec[i * 4], &p->tvec[i * 3], &p->qvec[j * 4], &p->tvec[j * 3], &st);
    double rho[3];
    LossEvaluate(o->loss_function_type, o->loss_function_scale, r * r, rho);
    return 0.5 * (o->semantic_weight * rho[0]);  // ScaledLoss(w)
  }
  // Cost of the reduced program (Ceres adds fixed_cost separately).  Terms
  // are evaluated in parallel and summed in program order.
  double Cost() {
    const int64_t nr = (int64_t)reduced.size(), ns = (int64_t)ss.samples.size();
    const int64_t ng = (int64_t)gs.blocks.size();
    std::vector<double> t(nr + (sem ? ns : 0) + ng);
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nr; ++k) t[k] = BlockCost(reduced[k]);
    if (sem) {
#pragma omp parallel for schedule(dynamic, 1024)
      for (int64_t n = 0; n < ns; ++n) t[nr + n] = SemCost(n);
    }
    const int64_t g0 = nr + (sem ? ns : 0);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t k = 0; k < ng; ++k) t[g0 + k] = GsbaCost((size_t)k);
    double c = 0.0;
    for (double v : t) c += v;
    return c;
  }
  void Linearize(Linearization* lin) {
    const int c = s.ct;
    const int64_t nr = (int64_t)reduced.size(), ns = sem ? (int64_t)ss.samples.size() : 0;
    const int64_t ng = (int64_t)gs.blocks.size();
    lin->resize(2 * nr + ns + ng);
    std::vector<double> cost(nr + ns + ng);
#pragma omp parallel
    {
      std::vector<double> J(2 * (9 + c));
#pragma omp for schedule(static)
      for (int64_t k = 0; k < nr; ++k) {
        const int64_t b = reduced[k];
        double r[2];
        EvalBlock(s, p, b, r, J.data());
        double rho[3];
        const double sq = r[0] * r[0] + r[1] * r[1];
        LossEvaluate(o->loss_function_type, o->loss_function_scale, sq, rho);
        cost[k] = 0.5 * rho[0];
        ApplyCorrector(rho, sq, 2, r, 9 + c, J.data());
        const int64_t ob = s.block_obs[b];
        const int img = p->obs_image[ob];
        const int cam = p->image_camera[img];
        const int64_t pt = p->obs_point[ob];
        for (int row = 0; row < 2; ++row) {
          const size_t R = 2 * (size_t)k + row;
          const double* Jr = &J[row * (9 + c)];
          int nf = 0;
          if (!s.block_const_pose[b] && L.img_off[img] >= 0)
            for (int m = 0; m < 6; ++m) {
              const int col = L.img_cols[(size_t)img * 6 + m];
              if (col >= 0) { lin->fcol[R * Linearization::kF + nf] = col; lin->fval[R * Linearization::kF + nf++] = Jr[m]; }
            }
          if (L.cam_off[cam] >= 0)
            for (int m = 0; m < (int)s.cam_tangent[cam].size(); ++m) {
              lin->fcol[R * Linearization::kF + nf] = L.cam_off[cam] + m;
              lin->fval[R * Linearization::kF + nf++] = Jr[9 + m];
            }
          lin->fn[R] = (uint8_t)nf;
          if (L.pt_off[pt] >= 0) {
            for (int m = 0; m < 3; ++m) { lin->ecol[R * 3 + m] = L.pt_off[pt] + m; lin->eval[R * 3 + m] = Jr[6 + m]; }
            lin->en[R] = 3;
          }
          lin->r[R] = r[row];
        }
      }
      if (sem) {
#pragma omp for schedule(dynamic, 1024)
        for (int64_t n = 0; n < ns; ++n) {
          int st; double r; double Js[12];
          EvalSemantic(p, s, sem, ss, n, &st, &r, Js);
          double rho[3];
          LossEvaluate(o->loss_function_type, o->loss_function_scale, r * r, rho);
          for (int m = 0; m < 3; ++m) rho[m] *= o->semantic_weight;  // ScaledLoss
          cost[nr + n] = 0.5 * rho[0];
          ApplyCorrector(rho, r * r, 1, &r, 12, Js);
          const SemSample& smp = ss.samples[n];
          const size_t R = 2 * (size_t)nr + n;
          int nf = 0;
          for (int blk = 0; blk < 2; ++blk) {
            const int img = sem->pairs[2 * smp.pair + blk];
            if (L.img_off[img] < 0) continue;
            for (int m = 0; m < 6; ++m) {
              const int col = L.img_cols[(size_t)img * 6 + m];
              if (col >= 0) { lin->fcol[R * Linearization::kF + nf] = col; lin->fval[R * Linearization::kF + nf++] = Js[blk * 6 + m]; }
            }
          }
          lin->fn[R] = (uint8_t)nf;
          lin->r[R] = r;
        }
      }
      // GSBA rows: tangent columns camera pose (6) + cylinder (8)
#pragma omp for schedule(dynamic, 1)
      for (int64_t k = 0; k < ng; ++k) {
        const GsbaBlock& b = gs.blocks[k];
        double J16[16];
        double r = GsbaResidual(p, s, gs, b, J16);
        double Jt[14];
        double PJ[12];
        QuaternionPlusJacobian(&p->qvec[b.img * 4], PJ);
        for (int col = 0; col < 3; ++col) {
          double acc = 0.0;
          for (int m = 0; m < 4; ++m) acc += J16[m] * PJ[m * 3 + col];
          Jt[col] = acc;
        }
        for (int col = 0; col < 3; ++col) Jt[3 + col] = J16[4 + col];
        if (gs.by2) {
          for (int col = 0; col < 7; ++col) Jt[6 + col] = J16[7 + col];  // Euclidean
          Jt[13] = 0.0;
        } else {
          QuaternionPlusJacobian(gs.g->cylinders[b.cyl].qvec, PJ);
          for (int col = 0; col < 3; ++col) {
            double acc = 0.0;
            for (int m = 0; m < 4; ++m) acc += J16[7 + m] * PJ[m * 3 + col];
            Jt[6 + col] = acc;
          }
          for (int col = 0; col < 5; ++col) Jt[9 + col] = J16[11 + col];
        }
        double rho[3];
        LossEvaluate(kLossScaled, gs.weight, r * r, rho);
        cost[nr + ns + k] = 0.5 * rho[0];
        ApplyCorrector(rho, r * r, 1, &r, 14, Jt);
        const size_t R = 2 * (size_t)nr + ns + k;
        int nf = 0;
        if (b.variant != kGsbaConstantPose && L.img_off[b.img] >= 0)
          for (int m = 0; m < 6; ++m) {
            const int col = L.img_cols[(size_t)b.img * 6 + m];
            if (col >= 0) { lin->fcol[R * Linearization::kF + nf] = col; lin->fval[R * Linearization::kF + nf++] = Jt[m]; }
          }
        if (b.variant != kGsbaConstantCylinder && L.cyl_off[b.cyl] >= 0)
          for (int m = 0; m < gs.cw(); ++m) {
            lin->fcol[R * Linearization::kF + nf] = L.cyl_off[b.cyl] + m;
            lin->fval[R * Linearization::kF + nf++] = Jt[6 + m];
          }
        lin->fn[R] = (uint8_t)nf;
        lin->r[R] = r;
      }
    }
    lin->cost = 0.0;
    for (double v : cost) lin->cost += v;
  }
  // Apply tangent step delta (f then e coordinates) with manifold Plus.
  void Plus(const std::vector<double>& delta) {
    for (int i = 0; i < p->num_images; ++i) {
      if (L.img_off[i] < 0) continue;
      double d[6] = {0, 0, 0, 0, 0, 0};
      for (int m = 0; m < 6; ++m) {
        const int col = L.img_cols[(size_t)i * 6 + m];
        if (col >= 0) d[m] = delta[col];
      }
      double qn[4];
      QuaternionPlus(&p->qvec[i * 4], d, qn);
      for (int m = 0; m < 4; ++m) p->qvec[i * 4 + m] = qn[m];
      for (int m = 0; m < 3; ++m) p->tvec[i * 3 + m] += d[3 + m];
    }
    for (int c = 0; c < p->num_cameras; ++c) {
      if (L.cam_off[c] < 0) continue;
      for (size_t m = 0; m < s.cam_tangent[c].size(); ++m)
        p->camera_params[s.cam_poff[c] + s.cam_tangent[c][m]] += delta[L.cam_off[c] + m];
    }
    for (int64_t pt = 0; pt < p->num_points; ++pt) {
      if (L.pt_off[pt] < 0) continue;
      for (int m = 0; m < 3; ++m) p->xyz[pt * 3 + m] += delta[L.nf + L.pt_off[pt] + m];
    }
    // cylinders: QuaternionManifold on qvec; radius clamped to its lower
    // bound 0 (ParameterBlock::Plus projects onto the bounds)
    for (size_t c = 0; c < L.cyl_off.size(); ++c) {
      if (L.cyl_off[c] < 0) continue;
      if (gs.by2) {  // Euclidean; radius bounded below by 0 (:1185-1213)
        double* y = &gs.by2p[7 * c];
        const double* d = &delta[L.cyl_off[c]];
        for (int m = 0; m < 6; ++m) y[m] += d[m];
        y[6] = std::max(y[6] + d[6], 0.0);
        continue;
      }
      mi_ba_cylinder& y = gs.g->cylinders[c];
      const double* d = &delta[L.cyl_off[c]];
      double qn[4];
      QuaternionPlus(y.qvec, d, qn);
      for (int m = 0; m < 4; ++m) y.qvec[m] = qn[m];
      for (int m = 0; m < 3; ++m) y.tvec[m] += d[3 + m];
      y.radius = std::max(y.radius + d[6], 0.0);
      y.height += d[7];
    }
  }
  // TrustRegionMinimizer's state vector x_: the reduced program's variable
  // parameter blocks in ambient coordinates (qvec 4, tvec 3, the camera's
  // params, X 3, the cylinder's blocks).  |x| and |x - candidate| give Ceres'
  // ParameterToleranceReached (step_norm = |x - candidate_x|).
  void State(std::vector<double>* x) const {
    x->clear();
    for (int i = 0; i < p->num_images; ++i) {
      if (L.img_off[i] < 0) continue;
      x->insert(x->end(), &p->qvec[i * 4], &p->qvec[i * 4] + 4);
      x->insert(x->end(), &p->tvec[i * 3], &p->tvec[i * 3] + 3);
    }
    for (int c = 0; c < p->num_cameras; ++c)
      if (L.cam_off[c] >= 0)
        x->insert(x->end(), &p->camera_params[s.cam_poff[c]], &p->camera_params[s.cam_poff[c + 1]]);
    for (int64_t pt = 0; pt < p->num_points; ++pt)
      if (L.pt_off[pt] >= 0) x->insert(x->end(), &p->xyz[pt * 3], &p->xyz[pt * 3] + 3);
    for (size_t c = 0; c < L.cyl_off.size(); ++c) {
      if (L.cyl_off[c] < 0) continue;
      if (gs.by2) {
        x->insert(x->end(), &gs.by2p[7 * c], &gs.by2p[7 * c] + 7);
      } else {
        const mi_ba_cylinder& y = gs.g->cylinders[c];
        x->insert(x->end(), y.qvec, y.qvec + 4);
        x->insert(x->end(), y.tvec, y.tvec + 3);
        x->push_back(y.radius);
        x->push_back(y.height);
      }
    }
  }
  // |x - Plus(x, -g)|_inf with g = J'f the tangent gradient at the current
  // point (TrustRegionMinimizer::EvaluateGradientAndJacobian: Ceres' gradient
  // max norm, projected through each block's Plus and its bounds — the
  // cylinder radius >= 0).
  double GradientMaxNorm(const Linearization& lin) const {
    constexpr int kF = Linearization::kF;
    const int nf = L.nf;
    std::vector<double> g(nf + L.ne, 0.0);
    for (size_t R = 0; R < lin.rows(); ++R) {
      for (int m = 0; m < lin.fn[R]; ++m) g[lin.fcol[R * kF + m]] += lin.fval[R * kF + m] * lin.r[R];
      for (int m = 0; m < lin.en[R]; ++m) g[nf + lin.ecol[R * 3 + m]] += lin.eval[R * 3 + m] * lin.r[R];
    }
    double mx = 0.0;
    auto euclid = [&](double x, double gc) { mx = std::max(mx, std::fabs(x - (x + -gc))); };
    auto quat = [&](const double* q, const double* gq) {
      const double d[3] = {-gq[0], -gq[1], -gq[2]};
      double qn[4];
      QuaternionPlus(q, d, qn);
      for (int m = 0; m < 4; ++m) mx = std::max(mx, std::fabs(q[m] - qn[m]));
    };
    for (int i = 0; i < p->num_images; ++i) {
      if (L.img_off[i] < 0) continue;
      double gq[3];
      for (int m = 0; m < 3; ++m) gq[m] = g[L.img_cols[(size_t)i * 6 + m]];
      quat(&p->qvec[i * 4], gq);
      for (int m = 3; m < 6; ++m) {
        const int col = L.img_cols[(size_t)i * 6 + m];
        if (col >= 0) euclid(p->tvec[i * 3 + m - 3], g[col]);
      }
    }
    for (int c = 0; c < p->num_cameras; ++c) {
      if (L.cam_off[c] < 0) continue;
      for (size_t m = 0; m < s.cam_tangent[c].size(); ++m)
        euclid(p->camera_params[s.cam_poff[c] + s.cam_tangent[c][m]], g[L.cam_off[c] + m]);
    }
    for (int64_t pt = 0; pt < p->num_points; ++pt) {
      if (L.pt_off[pt] < 0) continue;
      for (int m = 0; m < 3; ++m) euclid(p->xyz[pt * 3 + m], g[nf + L.pt_off[pt] + m]);
    }
    for (size_t c = 0; c < L.cyl_off.size(); ++c) {
      if (L.cyl_off[c] < 0) continue;
      const double* gc = &g[L.cyl_off[c]];
      if (gs.by2) {
        const double* y = &gs.by2p[7 * c];
        for (int m = 0; m < 6; ++m) euclid(y[m], gc[m]);
        mx = std::max(mx, std::fabs(y[6] - std::max(y[6] + -gc[6], 0.0)));
      } else {
        const mi_ba_cylinder& y = gs.g->cylinders[c];
        quat(y.qvec, gc);
        for (int m = 0; m < 3; ++m) euclid(y.tvec[m], gc[3 + m]);
        mx = std::max(mx, std::fabs(y.radius - std::max(y.radius + -gc[6], 0.0)));
        euclid(y.height, gc[7]);
      }
    }
    return mx;
  }
};

}  // namespace

// ===========================================================================
// C ABI for ctypes
// ===========================================================================
extern "C" {

int oracle_num_params(int model) { return NumParams(model); }

// camera_models.h WorldToImage / ImageToWorld for one point.
void oracle_world_to_image(int model, const double* params, double u, double v, double* x, double* y) {
  WorldToImage(model, params, u, v, x, y);
}
void oracle_image_to_world(int model, const double* params, double x, double y, double* u, double* v) {
  ImageToWorld(model, params, x, y, u, v);
}

// BundleAdjustmentCostFunction<M>::Evaluate residuals only (cost_functions.h:57-81).
void oracle_reproj_residual(int model, const double* q, const double* t, const double* X,
                            const double* cam, double ox, double oy, double* r) {
  ReprojResidual<double>(model, q, t, X, cam, ox, oy, r);
}

// projection.cc:111-131 CalculateSquaredReprojectionError(point2D, point3D, qvec, tvec, camera)
double oracle_squared_reprojection_error(int model, const double* params, const double* xy,
                                         const double* X, const double* q, const double* t) {
  double pc[3];
  QuaternionRotatePoint(q, X, pc);
  pc[0] += t[0]; pc[1] += t[1]; pc[2] += t[2];
  if (pc[2] < std::numeric_limits<double>::epsilon()) return std::numeric_limits<double>::max();
  double x, y;
  WorldToImage(model, params, pc[0] / pc[2], pc[1] / pc[2], &x, &y);
  return (x - xy[0]) * (x - xy[0]) + (y - xy[1]) * (y - xy[1]);
}

int oracle_setup_stats(const mi_ba_options* o, mi_ba_problem* p, mi_ba_setup_info* info) {
  Setup s;
  const int st = BuildSetup(o, p, &s);
  if (st) return st;
  info->num_residual_blocks = (int64_t)s.block_obs.size();
  info->num_residuals_reduced = s.num_residuals_reduced;
  info->num_effective_parameters_reduced = s.num_effective_parameters_reduced;
  int64_t vi = 0, vc = 0, vp = 0;
  for (auto v : s.img_var) vi += v;
  for (auto v : s.cam_var) vc += v;
  for (auto v : s.pt_var) vp += v;
  info->num_variable_images = vi;
  info->num_variable_cameras = vc;
  info->num_variable_points = vp;
  info->camera_tangent_size = s.ct;
  return MI_BA_OK;
}

// Residual + tangent Jacobian of every block of the program (program order;
// block_obs[k] = observation index).  Note: normalises config qvecs in place
// exactly as SetUp does.  Returns number of blocks or negative status.
int64_t oracle_reproj_eval(const mi_ba_options* o, mi_ba_problem* p, int64_t* block_obs,
                           double* residuals, double* jacobian, int64_t capacity) {
  Setup s;
  const int st = BuildSetup(o, p, &s);
  if (st) return -st;
  const int64_t nb = (int64_t)s.block_obs.size();
  if (nb > capacity) return nb;
  const int w = 9 + s.ct;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nb; ++b) {
    block_obs[b] = s.block_obs[b];
    double* r = &residuals[2 * b];
    double* J = jacobian ? &jacobian[b * 2 * w] : nullptr;
    EvalBlock(s, p, b, r, J);
    // Ceres' evaluator applies the loss Corrector before the linear solver
    // sees r and J; export them in that (corrected) form.
    double rho[3];
    const double sq = r[0] * r[0] + r[1] * r[1];
    LossEvaluate(o->loss_function_type, o->loss_function_scale, sq, rho);
    ApplyCorrector(rho, sq, 2, r, w, J);
  }
  return nb;
}

// Throughput baseline: residual+Jacobian of all blocks, `repeats` times,
// with the given number of OpenMP threads.  Returns wall seconds of the
// evaluation loop only (setup excluded).
double oracle_reproj_throughput(const mi_ba_options* o, mi_ba_problem* p, int64_t max_blocks,
                                int repeats, int threads, int64_t* blocks_done) {
  Setup s;
  if (BuildSetup(o, p, &s)) return -1.0;
  const int64_t nb = std::min<int64_t>((int64_t)s.block_obs.size(), max_blocks);
  const int w = 9 + s.ct;
  std::vector<double> r(2 * nb), J(2 * w * nb);
  double t0 = 0, t1 = 0;
  {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts); t0 = ts.tv_sec + 1e-9 * ts.tv_nsec;
  }
  for (int rep = 0; rep < repeats; ++rep) {
#pragma omp parallel for schedule(static) num_threads(threads)
    for (int64_t b = 0; b < nb; ++b) EvalBlock(s, p, b, &r[2 * b], &J[b * 2 * w]);
  }
  {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts); t1 = ts.tv_sec + 1e-9 * ts.tv_nsec;
  }
  *blocks_done = nb * repeats;
  return t1 - t0;
}

// Semantic samples: returns count (or negative status).  Arrays sized by
// capacity; layout as mi_ba_download_semantic.
int64_t oracle_semantic_eval(const mi_ba_options* o, mi_ba_problem* p, const mi_ba_semantic* sem,
                             int32_t* sample_pixel, int32_t* status, double* residuals,
                             double* jacobian, int64_t capacity) {
  Setup s;
  const int st = BuildSetup(o, p, &s);
  if (st) return -st;
  SemSetup ss;
  BuildSemSetup(o, p, s, sem, &ss);
  // poses of semantic pairs carry their manifolds even without reprojection
  // blocks (SetUpManifolds, semantic_bundle_adjustment.cc:670-693)
  AddSemanticPoses(p, sem, ss, &s);
  const int64_t n = (int64_t)ss.samples.size();
  if (n > capacity) return n;
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t k = 0; k < n; ++k) {
    sample_pixel[3 * k] = ss.samples[k].pair;
    sample_pixel[3 * k + 1] = ss.samples[k].x;
    sample_pixel[3 * k + 2] = ss.samples[k].y;
    int stt;
    EvalSemantic(p, s, sem, ss, k, &stt, &residuals[k], &jacobian[12 * k]);
    status[k] = stt;
  }
  return n;
}

// SemanticBundleAdjuster::ExportSemanticErrorToCSV (semantic_bundle_adjustment.cc:
// 908-1019): every pixel of image1's grid (y outer, x inner, zero-depth pixels
// included) against image2 at the problem's parameters.  Returns the row
// count (rows written when it fits capacity), or -status.
int64_t oracle_semantic_export(const mi_ba_options* o, mi_ba_problem* p, const mi_ba_semantic* sem, int32_t image1,
                               int32_t image2, int32_t* pixels, int32_t* status, double* error, double* world,
                               int64_t capacity) {
  Setup s;
  const int st = BuildSetup(o, p, &s);
  if (st) return -st;
  SemPlanes planes;
  planes.build(sem, p->num_images);
  const SemRaster& r1 = planes.img[image1];
  const int H = r1.H, W = r1.W, step = sem->pixel_step;
  const int nx = (W + step - 1) / step, ny = (H + step - 1) / step;
  const int64_t n = (int64_t)nx * ny;
  if (n > capacity) return n;
  const int cam1 = p->image_camera[image1];
  const double* K1 = &p->camera_params[s.cam_poff[cam1]];
  const double* q1 = p->qvec + 4 * image1;
  const double* t1 = p->tvec + 3 * image1;
  const double* q2 = p->qvec + 4 * image2;
  const double* t2 = p->tvec + 3 * image2;
  int64_t k = 0;
  for (int y = 0; y < H; y += step) {       // :953-956
    for (int x = 0; x < W; x += step, ++k) {
      const int64_t off = (int64_t)y * W + x;
      SemSample smp;
      smp.pair = 0; smp.x = x; smp.y = y;
      double u1, v1;
      ImageToWorld(s.cam_model[cam1], K1, (double)x, (double)y, &u1, &v1);
      const double depth = (double)r1.depth[off];
      smp.pc1[0] = u1 * depth;
      smp.pc1[1] = v1 * depth;
      smp.pc1[2] = depth;
      smp.label1 = r1.label[off];
      int stt = 0, pxy[2] = {0, 0};
      error[k] = SemanticErrorTo(p, s, sem, image2, planes.img[image2], smp, q1, t1, q2, t2, &stt, &world[3 * k], pxy);
      status[k] = stt;
      pixels[4 * k] = x;
      pixels[4 * k + 1] = y;
      pixels[4 * k + 2] = pxy[0];
      pixels[4 * k + 3] = pxy[1];
    }
  }
  return n;
}

double oracle_semantic_throughput(const mi_ba_options* o, mi_ba_problem* p, const mi_ba_semantic* sem,
                                  int64_t max_samples, int threads, int64_t* done) {
  Setup s;
  if (BuildSetup(o, p, &s)) return -1.0;
  SemSetup ss;
  BuildSemSetup(o, p, s, sem, &ss);
  AddSemanticPoses(p, sem, ss, &s);
  const int64_t n = std::min<int64_t>((int64_t)ss.samples.size(), max_samples);
  std::vector<double> r(n), J(12 * n);
  struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
  const double t0 = ts.tv_sec + 1e-9 * ts.tv_nsec;
#pragma omp parallel for schedule(dynamic, 256) num_threads(threads)
  for (int64_t k = 0; k < n; ++k) {
    int stt;
    EvalSemantic(p, s, sem, ss, k, &stt, &r[k], &J[12 * k]);
  }
  clock_gettime(CLOCK_MONOTONIC, &ts);
  *done = n;
  return ts.tv_sec + 1e-9 * ts.tv_nsec - t0;
}

// The oracle's dense Cholesky (the factorisation its LM applies to the
// reduced camera system, DENSE_SCHUR restated): A row-major n x n, lower
// triangle overwritten with L.  Returns 0, or the 1-based column of the first
// pivot that is not positive.  Rows of L are independent given the columns
// to their left, so the i-loop runs in parallel with unchanged arithmetic.
int oracle_cholesky(double* A, int n) { return CholeskyBlocked(A, n); }

// Property test of the flat test (restated above) against the full CENTRAL
// stencil over every sample of the problem: counts[0] samples, [1] cleared
// by the flat test, [2] cleared samples with a stencil value different from
// the centre residual (the test is sound iff 0), [3] samples with a nonzero
// Jacobian, [4] samples not cleared whose stencil was flat anyway.
int oracle_semantic_flat_property(const mi_ba_options* o, mi_ba_problem* p, const mi_ba_semantic* sem,
                                  int64_t* counts) {
  Setup s;
  const int st = BuildSetup(o, p, &s);
  if (st) return st;
  SemSetup ss;
  BuildSemSetup(o, p, s, sem, &ss);
  std::vector<FlatBounds> pb(sem->num_pairs);
  for (int k = 0; k < sem->num_pairs; ++k) {
    const int i = sem->pairs[2 * k], j = sem->pairs[2 * k + 1];
    FlatStencilBounds(&p->qvec[i * 4], &p->tvec[i * 3], sem->numeric_relative_step_size, &pb[k].rho1, pb[k].dt1);
    FlatStencilBounds(&p->qvec[j * 4], &p->tvec[j * 3], sem->numeric_relative_step_size, &pb[k].rho2, pb[k].dt2);
    double qi[4], ti[3], Ri[9], R2[9];
    PoseInverse(&p->qvec[i * 4], &p->tvec[i * 3], qi, ti);
    QuaternionToRotation(qi, Ri);
    QuaternionToRotation(&p->qvec[j * 4], R2);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        pb[k].C[3 * r + c] = R2[3 * r] * Ri[c] + R2[3 * r + 1] * Ri[3 + c] + R2[3 * r + 2] * Ri[6 + c];
  }
  const int64_t n = (int64_t)ss.samples.size();
  int64_t cleared = 0, bad = 0, nonzero = 0, flat_deferred = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : cleared, bad, nonzero, flat_deferred)
  for (int64_t k = 0; k < n; ++k) {
    const SemSample& smp = ss.samples[k];
    const int i = sem->pairs[2 * smp.pair], j = sem->pairs[2 * smp.pair + 1];
    double x[14];
    for (int m = 0; m < 4; ++m) x[m] = p->qvec[i * 4 + m];
    for (int m = 0; m < 3; ++m) x[4 + m] = p->tvec[i * 3 + m];
    for (int m = 0; m < 4; ++m) x[7 + m] = p->qvec[j * 4 + m];
    for (int m = 0; m < 3; ++m) x[11 + m] = p->tvec[j * 3 + m];
    int stt;
    const double r = SemanticError(p, s, sem, ss, smp, &x[0], &x[4], &x[7], &x[11], &stt);
    const bool var[2] = {ss.pair_var1[smp.pair] != 0, ss.pair_var2[smp.pair] != 0};
    const double min_step = std::sqrt(std::numeric_limits<double>::epsilon());
    bool flat = true, jz = true;
    for (int blk = 0; blk < 2; ++blk) {
      if (!var[blk]) continue;
      for (int m = 0; m < 7; ++m) {
        const int idx = blk * 7 + m;
        const double orig = x[idx];
        const double delta = std::max(min_step, std::fabs(orig) * sem->numeric_relative_step_size);
        x[idx] = orig + delta;
        const double fp = SemanticError(p, s, sem, ss, smp, &x[0], &x[4], &x[7], &x[11], &stt);
        x[idx] = orig - delta;
        const double fm = SemanticError(p, s, sem, ss, smp, &x[0], &x[4], &x[7], &x[11], &stt);
        x[idx] = orig;
        if (fp != r || fm != r) flat = false;
        if (fp != fm) jz = false;
      }
    }
    const bool clears = FlatClears(p, s, sem, ss, smp, pb[smp.pair], var[0], var[1], r);
    cleared += clears;
    bad += clears && !flat;
    nonzero += !jz;
    flat_deferred += !clears && flat;
  }
  counts[0] = n;
  counts[1] = cleared;
  counts[2] = bad;
  counts[3] = nonzero;
  counts[4] = flat_deferred;
  return 0;
}

void oracle_set_flat_bound_scale(double scale) { g_flat_bound_scale = scale; }
void oracle_set_flat_coarse(int coarse) { g_flat_coarse = coarse; }

// Registers (or clears, NULL) the dense factor the LM uses for its reduced
// camera system.
void oracle_set_dense_factor(DenseFactorFn fn) { g_dense_factor = fn; }

// Record the per-iteration LM trace of the next solves into buf (4 int32 per
// iteration, at most cap iterations); null turns it off.
void oracle_set_trace(int32_t* buf, int cap) {
  g_trace = buf;
  g_trace_cap = buf ? cap : 0;
}
// With a trace set: also record the step values into vbuf (4 doubles per
// iteration, the same cap); null turns it off.
void oracle_set_trace_values(double* vbuf) { g_trace_v = vbuf; }

}  // extern "C"

namespace {

// ---------------------------------------------------------------------------
// ITERATIVE_SCHUR + SCHUR_JACOBI, the solver BundleAdjuster::Solve selects
// above 1000 images (bundle_adjustment.cc:276-286; SBA the same,
// semantic_bundle_adjustment.cc:494-499).  Ceres 2.1 is third party and not
// vendored; restated from its published sources:
//   * ImplicitSchurComplement (implicit_schur_complement.cc) with A = J
//     diag(scale) = [E | F] (points are the e blocks):
//       S x  = D_f^2 x + F'(F x - E (E'E + D_e^2)^-1 E'F x)
//       rhs  = F'(b - E (E'E + D_e^2)^-1 E'b)
//       back substitution x_e = (E'E + D_e^2)^-1 E'(b - F x_f)
//     every product through the rows (RightMultiplyF, LeftMultiplyE,
//     RightMultiplyE, LeftMultiplyF), never forming S;
//   * SchurJacobiPreconditioner (schur_jacobi_preconditioner.cc): the
//     diagonal blocks of S, one per f parameter block — qvec (3 tangent),
//     tvec (3, or fewer under a SubsetManifold), the camera's refined
//     intrinsics, and for GSBA the cylinder's qvec / tvec / radius / height
//     (by two points: tvec_1 / tvec_2 / radius) — each inverted through an LLT
//     (BlockRandomAccessDiagonalMatrix::Invert);
//   * ConjugateGradientsSolver (conjugate_gradients_solver.cc): x = 0, r = b;
//     r_tolerance off (LevenbergMarquardtStrategy passes -1); per iteration
//     z = M r, rho = r'z (FAILURE when 0 / inf), p = z or z + (rho / rho_prev)
//     p (FAILURE when beta is 0 / inf), q = S p, pq = p'q (NO_CONVERGENCE when
//     <= 0 / inf, before x moves), alpha = rho / pq (FAILURE when inf),
//     x += alpha p, r = b - S x every residual_reset_period = 10 iterations
//     else r -= alpha q, Q1 = -x'(b + r), stop when i (Q1 - Q0) / Q1 < eta,
//     NO_CONVERGENCE at max_linear_solver_iterations.  A FAILURE is an invalid
//     LM step (TrustRegionMinimizer::ComputeTrustRegionStep); NO_CONVERGENCE
//     and SUCCESS steps are used.
// ---------------------------------------------------------------------------
enum CgTermination { kCgSuccess = 0, kCgNoConvergence = 1, kCgFailure = 2 };

struct ImplicitSchur {
  const Linearization* lin = nullptr;
  const double* scale = nullptr;  // Jacobi scaling, f then e coordinates
  const double* D2 = nullptr;     // LM diagonal D^2 (diag / radius), f then e
  const double* Vinv = nullptr;   // [np3][9] (E'E + D_e^2)^-1
  int nf = 0;
  int64_t np3 = 0;
  std::vector<int64_t> prow_off, prow;  // each point's rows, in row order
  std::vector<int64_t> ft_off, ft_row;  // F transposed: each column's rows, in row order
  std::vector<int> ft_slot;             // the row's f slot of that column
  std::vector<double> rows, te, te2;

  // structure (the rows of each point, the rows of each f column): once per
  // linearization layout (constant over the solve)
  void Structure(const Linearization& L, int nf_, int64_t np3_) {
    lin = &L;
    nf = nf_;
    np3 = np3_;
    constexpr int kF = Linearization::kF;
    const size_t nr = L.rows();
    prow_off.assign(np3 + 1, 0);
    for (size_t R = 0; R < nr; ++R)
      if (L.en[R]) ++prow_off[L.ecol[R * 3] / 3 + 1];
    for (int64_t p = 0; p < np3; ++p) prow_off[p + 1] += prow_off[p];
    prow.assign(prow_off[np3], 0);
    {
      std::vector<int64_t> pos(prow_off.begin(), prow_off.end() - 1);
      for (size_t R = 0; R < nr; ++R)
        if (L.en[R]) prow[pos[L.ecol[R * 3] / 3]++] = (int64_t)R;
    }
    ft_off.assign(nf + 1, 0);
    for (size_t R = 0; R < nr; ++R)
      for (int m = 0; m < L.fn[R]; ++m) ++ft_off[L.fcol[R * kF + m] + 1];
    for (int c = 0; c < nf; ++c) ft_off[c + 1] += ft_off[c];
    ft_row.assign(ft_off[nf], 0);
    ft_slot.assign(ft_off[nf], 0);
    std::vector<int64_t> pos(ft_off.begin(), ft_off.end() - 1);
    for (size_t R = 0; R < nr; ++R)
      for (int m = 0; m < L.fn[R]; ++m) {
        const int64_t k = pos[L.fcol[R * kF + m]]++;
        ft_row[k] = (int64_t)R;
        ft_slot[k] = m;
      }
    rows.assign(nr, 0.0);
    te.assign(3 * np3, 0.0);
    te2.assign(3 * np3, 0.0);
  }
  // out[R] = (F x)[R]
  void RightMultiplyF(const double* x, double* out) const {
    constexpr int kF = Linearization::kF;
    const int64_t nr = (int64_t)lin->rows();
#pragma omp parallel for schedule(static)
    for (int64_t R = 0; R < nr; ++R) {
      double acc = 0.0;
      for (int m = 0; m < lin->fn[R]; ++m) {
        const int32_t c = lin->fcol[R * kF + m];
        acc += (lin->fval[R * kF + m] * scale[c]) * x[c];
      }
      out[R] = acc;
    }
  }
  // e = E' in (per point, its rows in order)
  void LeftMultiplyE(const double* in, double* e) const {
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < np3; ++p) {
      double a[3] = {0.0, 0.0, 0.0};
      for (int64_t k = prow_off[p]; k < prow_off[p + 1]; ++k) {
        const int64_t R = prow[k];
        for (int m = 0; m < 3; ++m) {
          const int64_t c = lin->ecol[R * 3 + m];
          a[c % 3] += (lin->eval[R * 3 + m] * scale[nf + c]) * in[R];
        }
      }
      for (int m = 0; m < 3; ++m) e[3 * p + m] = a[m];
    }
  }
  // out[R] += (E e)[R]
  void RightMultiplyE(const double* e, double* out) const {
    const int64_t nr = (int64_t)lin->rows();
#pragma omp parallel for schedule(static)
    for (int64_t R = 0; R < nr; ++R) {
      if (!lin->en[R]) continue;
      double acc = 0.0;
      for (int m = 0; m < 3; ++m) {
        const int64_t c = lin->ecol[R * 3 + m];
        acc += (lin->eval[R * 3 + m] * scale[nf + c]) * e[c];
      }
      out[R] += acc;
    }
  }
  // y += F' in (per column, its rows in order)
  void LeftMultiplyF(const double* in, double* y) const {
    constexpr int kF = Linearization::kF;
#pragma omp parallel for schedule(static)
    for (int c = 0; c < nf; ++c) {
      double acc = 0.0;
      for (int64_t k = ft_off[c]; k < ft_off[c + 1]; ++k) {
        const int64_t R = ft_row[k];
        acc += (lin->fval[R * kF + ft_slot[k]] * scale[c]) * in[R];
      }
      y[c] += acc;
    }
  }
  void EtEInverse(const double* in, double* out) const {
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < np3; ++p)
      for (int a = 0; a < 3; ++a) {
        double acc = 0.0;
        for (int k = 0; k < 3; ++k) acc += Vinv[p * 9 + a * 3 + k] * in[3 * p + k];
        out[3 * p + a] = acc;
      }
  }
  // ImplicitSchurComplement::RightMultiply
  void RightMultiply(const double* x, double* y) {
    RightMultiplyF(x, rows.data());
    LeftMultiplyE(rows.data(), te.data());
    EtEInverse(te.data(), te2.data());
    for (auto& v : te2) v = -v;
    RightMultiplyE(te2.data(), rows.data());
    for (int c = 0; c < nf; ++c) y[c] = D2[c] * x[c];
    LeftMultiplyF(rows.data(), y);
  }
  // ImplicitSchurComplement::UpdateRhs (b = the residuals)
  void Rhs(const double* b, double* rhs) {
    LeftMultiplyE(b, te.data());
    EtEInverse(te.data(), te2.data());
    const int64_t nr = (int64_t)lin->rows();
    std::fill(rows.begin(), rows.end(), 0.0);
    RightMultiplyE(te2.data(), rows.data());
    for (int64_t R = 0; R < nr; ++R) rows[R] = b[R] - rows[R];
    std::fill(rhs, rhs + nf, 0.0);
    LeftMultiplyF(rows.data(), rhs);
  }
  // ImplicitSchurComplement::BackSubstitute: x_e from x_f
  void BackSubstitute(const double* b, const double* xf, double* xe) {
    RightMultiplyF(xf, rows.data());
    const int64_t nr = (int64_t)lin->rows();
    for (int64_t R = 0; R < nr; ++R) rows[R] = b[R] - rows[R];
    LeftMultiplyE(rows.data(), te.data());
    EtEInverse(te.data(), xe);
  }
};

// The f parameter blocks of the reduced camera system (Ceres column blocks
// after the e blocks): (first column, size).
std::vector<std::pair<int, int>> FBlocks(const Setup& s, const mi_ba_problem* p, const Layout& L,
                                         const GsbaSetup& gs) {
  std::vector<std::pair<int, int>> b;
  for (int i = 0; i < p->num_images; ++i) {
    if (L.img_off[i] < 0) continue;
    b.push_back({L.img_cols[(size_t)i * 6], 3});
    int nt = 0, t0 = -1;
    for (int m = 3; m < 6; ++m)
      if (L.img_cols[(size_t)i * 6 + m] >= 0) { if (t0 < 0) t0 = L.img_cols[(size_t)i * 6 + m]; ++nt; }
    if (nt) b.push_back({t0, nt});
  }
  for (int c = 0; c < p->num_cameras; ++c)
    if (L.cam_off[c] >= 0 && !s.cam_tangent[c].empty()) b.push_back({L.cam_off[c], (int)s.cam_tangent[c].size()});
  for (size_t c = 0; c < L.cyl_off.size(); ++c) {
    if (L.cyl_off[c] < 0) continue;
    const int o = L.cyl_off[c];
    b.push_back({o, 3});
    b.push_back({o + 3, 3});
    b.push_back({o + 6, 1});
    if (!gs.by2) b.push_back({o + 7, 1});
  }
  return b;
}

// Inverse of a small SPD block through its LLT (Eigen llt().solve(I)); the
// upper triangle is read, as selfadjointView<Upper>.
void LltInverse(const std::vector<double>& M, int k, std::vector<double>* inv) {
  std::vector<double> L((size_t)k * k, 0.0);
  for (int j = 0; j < k; ++j) {
    double d = M[(size_t)j * k + j];
    for (int m = 0; m < j; ++m) d -= L[(size_t)j * k + m] * L[(size_t)j * k + m];
    d = std::sqrt(d);
    L[(size_t)j * k + j] = d;
    for (int i = j + 1; i < k; ++i) {
      double v = M[(size_t)j * k + i];  // upper: (j, i)
      for (int m = 0; m < j; ++m) v -= L[(size_t)i * k + m] * L[(size_t)j * k + m];
      L[(size_t)i * k + j] = v / d;
    }
  }
  inv->assign((size_t)k * k, 0.0);
  std::vector<double> y(k);
  for (int c = 0; c < k; ++c) {
    for (int i = 0; i < k; ++i) {
      double v = i == c ? 1.0 : 0.0;
      for (int m = 0; m < i; ++m) v -= L[(size_t)i * k + m] * y[m];
      y[i] = v / L[(size_t)i * k + i];
    }
    for (int i = k - 1; i >= 0; --i) {
      double v = y[i];
      for (int m = i + 1; m < k; ++m) v -= L[(size_t)m * k + i] * y[m];
      y[i] = v / L[(size_t)i * k + i];
    }
    for (int i = 0; i < k; ++i) (*inv)[(size_t)i * k + c] = y[i];
  }
}

// ConjugateGradientsSolver::Solve on the implicit Schur complement with the
// SCHUR_JACOBI blocks.  x (nf) out; returns the CgTermination.
int SchurPcg(ImplicitSchur& A, const std::vector<std::pair<int, int>>& blocks,
             const std::vector<std::vector<double>>& Minv, const double* b, int nf, double eta, int max_it,
             double* x, int* iterations) {
  std::fill(x, x + nf, 0.0);
  *iterations = 0;
  double norm_b = 0.0;
  for (int i = 0; i < nf; ++i) norm_b += b[i] * b[i];
  if (std::sqrt(norm_b) == 0.0) return kCgSuccess;  // "Convergence. |b| = 0."
  std::vector<double> r(b, b + nf), p(nf, 0.0), z(nf), tmp(nf);
  auto zero_or_inf = [](double v) { return v == 0.0 || std::isinf(v); };
  double rho = 1.0;
  double Q0 = 0.0;  // -x'(b + r) at x = 0
  for (int it = 1;; ++it) {
    *iterations = it;
    for (size_t k = 0; k < blocks.size(); ++k) {  // z = M r
      const int o = blocks[k].first, w = blocks[k].second;
      for (int a = 0; a < w; ++a) {
        double acc = 0.0;
        for (int c = 0; c < w; ++c) acc += Minv[k][(size_t)a * w + c] * r[o + c];
        z[o + a] = acc;
      }
    }
    const double last_rho = rho;
    rho = 0.0;
    for (int i = 0; i < nf; ++i) rho += r[i] * z[i];
    if (zero_or_inf(rho)) return kCgFailure;
    if (it == 1) {
      p = z;
    } else {
      const double beta = rho / last_rho;
      if (zero_or_inf(beta)) return kCgFailure;
      for (int i = 0; i < nf; ++i) p[i] = z[i] + beta * p[i];
    }
    std::vector<double>& q = z;
    A.RightMultiply(p.data(), q.data());
    double pq = 0.0;
    for (int i = 0; i < nf; ++i) pq += p[i] * q[i];
    if (pq <= 0.0 || std::isinf(pq)) return kCgNoConvergence;
    const double alpha = rho / pq;
    if (std::isinf(alpha)) return kCgFailure;
    for (int i = 0; i < nf; ++i) x[i] = x[i] + alpha * p[i];
    if (it % 10 == 0) {
      A.RightMultiply(x, tmp.data());
      for (int i = 0; i < nf; ++i) r[i] = b[i] - tmp[i];
    } else {
      for (int i = 0; i < nf; ++i) r[i] = r[i] - alpha * q[i];
    }
    double Q1 = 0.0;
    for (int i = 0; i < nf; ++i) Q1 += x[i] * (b[i] + r[i]);
    Q1 = -1.0 * Q1;
    const double zeta = it * (Q1 - Q0) / Q1;
    if (zeta < eta) return kCgSuccess;
    Q0 = Q1;
    if (it >= max_it) return kCgNoConvergence;
  }
}

// Images in the configuration (bundle_adjustment.cc:276-286 counts
// config.NumImages()).
int64_t ConfigImages(const mi_ba_problem* p) {
  int64_t n = 0;
  for (int i = 0; i < p->num_images; ++i) n += p->image_in_config ? (p->image_in_config[i] != 0) : 1;
  return n;
}

// Full LM solve (Ceres 2.1 LM semantics, restated) with the exact dense
// Schur solve or ITERATIVE_SCHUR, and the optional semantic (SBA) and GSBA
// terms.
int SolveImpl(const mi_ba_options* o, mi_ba_problem* p, const mi_ba_semantic* sem, const mi_ba_gsba* gsba,
              mi_ba_summary* sum) {
  Solver S;
  S.o = o; S.p = p; S.sem = sem;
  std::memset(sum, 0, sizeof(*sum));
  int st = BuildSetup(o, p, &S.s);
  if (st) return st;
  if (sem) {
    BuildSemSetup(o, p, S.s, sem, &S.ss);
    AddSemanticPoses(p, sem, S.ss, &S.s);
  }
  if (gsba) {
    st = BuildGsbaSetup(o, p, S.s, gsba, &S.gs);
    if (st) return st;
    AddGsbaPoses(p, S.gs, &S.s);
  }
  BuildLayout(S.s, p, &S.L, sem, sem ? &S.ss : nullptr, gsba ? &S.gs : nullptr);
  for (size_t b = 0; b < S.s.block_obs.size(); ++b)
    if (S.s.block_reduced[b]) S.reduced.push_back((int64_t)b);
  int64_t ncyl_var = 0;
  for (int c : S.L.cyl_off) ncyl_var += c >= 0 ? 1 : 0;
  sum->num_residuals_reduced =
      S.s.num_residuals_reduced + (int64_t)S.ss.samples.size() + (int64_t)S.gs.blocks.size();
  sum->num_effective_parameters_reduced = S.s.num_effective_parameters_reduced + S.gs.cw() * ncyl_var;
  sum->num_semantic_residuals = (int64_t)S.ss.samples.size();
  if (sum->num_residuals_reduced == 0) return MI_BA_ERR_NO_RESIDUALS;
  // fixed cost of the dropped all-constant blocks
  double fixed = 0.0;
  for (size_t b = 0; b < S.s.block_obs.size(); ++b)
    if (!S.s.block_reduced[b]) fixed += S.BlockCost(b);
  sum->fixed_cost = fixed;
  const int nf = S.L.nf;
  const int64_t ne = S.L.ne;
  const int64_t n = nf + ne;
  Linearization lin;
  S.Linearize(&lin);
  double x_cost = lin.cost;
  sum->initial_cost = x_cost + fixed;
  sum->num_jacobian_evaluations = 1;
  // Jacobi scaling, computed once at iteration 0.
  std::vector<double> colnorm(n, 0.0);
  constexpr int kF = Linearization::kF;
  const size_t nrows = lin.rows();
  for (size_t R = 0; R < nrows; ++R) {
    for (int m = 0; m < lin.fn[R]; ++m) colnorm[lin.fcol[R * kF + m]] += lin.fval[R * kF + m] * lin.fval[R * kF + m];
    for (int m = 0; m < lin.en[R]; ++m) colnorm[nf + lin.ecol[R * 3 + m]] += lin.eval[R * 3 + m] * lin.eval[R * 3 + m];
  }
  std::vector<double> scale(n);
  for (int64_t i = 0; i < n; ++i) scale[i] = 1.0 / (1.0 + std::sqrt(colnorm[i]));
  double radius = o->initial_trust_region_radius;
  double decrease_factor = 2.0;
  bool reuse_diagonal = false;
  std::vector<double> diag(n, 0.0);
  int consecutive_invalid = 0;
  int iteration = 0;
  sum->termination_type = MI_BA_NO_CONVERGENCE;
  const int64_t np3 = ne / 3;
  std::vector<std::vector<double>> W(np3);
  std::vector<std::vector<int>> Wcols(np3);
  std::vector<int> wslot;  // [row][kF] slot of f entry in its point's W
  // linear solver (bundle_adjustment.cc:276-286): the exact Schur solve up
  // to 1000 configured images, ITERATIVE_SCHUR + SCHUR_JACOBI above
  const bool use_pcg = o->linear_solver_type == MI_BA_SOLVER_ITERATIVE_SCHUR ||
                       (o->linear_solver_type == MI_BA_SOLVER_AUTO && ConfigImages(p) > 1000);
  ImplicitSchur isc;
  std::vector<std::pair<int, int>> fblocks;
  if (use_pcg) {
    isc.Structure(lin, nf, np3);
    isc.scale = scale.data();
    fblocks = FBlocks(S.s, p, S.L, S.gs);
  }
  // gradient max norm at the current point (Ceres evaluates it with every
  // Jacobian: IterationZero and each successful step)
  double gmax = S.GradientMaxNorm(lin);
  bool last_successful = true;  // iteration 0 counts as successful
  auto trace = [&](int it, int valid, int success, int cg, int end) {
    if (!g_trace || it < 1 || it > g_trace_cap) return;
    int32_t* t = g_trace + 4 * (size_t)(it - 1);
    t[0] = valid; t[1] = success; t[2] = cg; t[3] = end;
  };
  if (g_trace) std::fill(g_trace, g_trace + 4 * (size_t)g_trace_cap, -1);
  std::vector<double> x_state, c_state;
  while (true) {
    // FinalizeIterationAndCheckIfMinimizerCanContinue: the iteration cap, the
    // gradient tolerance (after a successful step or at iteration 0), the
    // minimum trust-region radius
    if (iteration >= o->max_num_iterations) { sum->termination_type = MI_BA_NO_CONVERGENCE; break; }
    if (last_successful && gmax <= o->gradient_tolerance) { sum->termination_type = MI_BA_CONVERGENCE; break; }
    if (radius <= 1e-32) { sum->termination_type = MI_BA_CONVERGENCE; break; }
    ++iteration;
    // scaled Jacobian column norms -> LM diagonal
    if (!reuse_diagonal) {
      std::fill(diag.begin(), diag.end(), 0.0);
      for (size_t R = 0; R < nrows; ++R) {
        for (int m = 0; m < lin.fn[R]; ++m) {
          const int64_t col = lin.fcol[R * kF + m];
          const double v = lin.fval[R * kF + m] * scale[col];
          diag[col] += v * v;
        }
        for (int m = 0; m < lin.en[R]; ++m) {
          const int64_t col = nf + lin.ecol[R * 3 + m];
          const double v = lin.eval[R * 3 + m] * scale[col];
          diag[col] += v * v;
        }
      }
      for (auto& d : diag) d = std::min(std::max(d, 1e-6), 1e32);
    }
    std::vector<double> D2(n);
    for (int64_t i = 0; i < n; ++i) D2[i] = diag[i] / radius;
    // Normal equations in scaled coordinates, Schur on points.
    std::vector<double> U((size_t)nf * nf, 0.0), g(n, 0.0);
    std::vector<double> V(np3 * 9, 0.0);
    // U and g_f: threads own contiguous row ranges of U (row order of the
    // serial loop per element)
#pragma omp parallel
    {
      const int nt = omp_get_num_threads(), tid = omp_get_thread_num();
      const int r0 = (int)((int64_t)nf * tid / nt), r1 = (int)((int64_t)nf * (tid + 1) / nt);
      for (size_t R = 0; R < nrows; ++R) {
        const double rr = lin.r[R];
        const int32_t* fc = &lin.fcol[R * kF];
        const double* fv = &lin.fval[R * kF];
        const int nfr = lin.fn[R];
        for (int x = 0; x < nfr; ++x) {
          if (fc[x] < r0 || fc[x] >= r1) continue;
          const double va = fv[x] * scale[fc[x]];
          g[fc[x]] += va * rr;
          for (int y = 0; y < nfr; ++y) U[(size_t)fc[x] * nf + fc[y]] += va * fv[y] * scale[fc[y]];
        }
      }
    }
    // e side (V, g_e, W): the row -> W-slot map depends on the structure
    // only, built once; threads own contiguous point ranges (serial row
    // order per element)
    if (wslot.empty()) {
      wslot.assign(nrows * kF, -1);
      for (size_t R = 0; R < nrows; ++R) {
        if (lin.en[R] == 0) continue;
        const int64_t pt = lin.ecol[R * 3] / 3;
        for (int x = 0; x < lin.fn[R]; ++x) {
          const int32_t c = lin.fcol[R * kF + x];
          int slot = -1;
          for (size_t m = 0; m < Wcols[pt].size(); ++m) if (Wcols[pt][m] == c) { slot = (int)m; break; }
          if (slot < 0) { slot = (int)Wcols[pt].size(); Wcols[pt].push_back((int)c); }
          wslot[R * kF + x] = slot;
        }
      }
    }
    for (int64_t pt = 0; pt < np3; ++pt) W[pt].assign(3 * Wcols[pt].size(), 0.0);
#pragma omp parallel
    {
      const int nt = omp_get_num_threads(), tid = omp_get_thread_num();
      const int64_t p0 = np3 * tid / nt, p1 = np3 * (tid + 1) / nt;
      for (size_t R = 0; R < nrows; ++R) {
        if (lin.en[R] == 0) continue;
        const int64_t* ec = &lin.ecol[R * 3];
        const int64_t pt = ec[0] / 3;
        if (pt < p0 || pt >= p1) continue;
        const double rr = lin.r[R];
        const int32_t* fc = &lin.fcol[R * kF];
        const double* fv = &lin.fval[R * kF];
        const int nfr = lin.fn[R];
        const double* ev = &lin.eval[R * 3];
        for (int x = 0; x < 3; ++x) {
          const double va = ev[x] * scale[nf + ec[x]];
          g[nf + ec[x]] += va * rr;
          for (int y = 0; y < 3; ++y) V[pt * 9 + (ec[x] % 3) * 3 + (ec[y] % 3)] += va * ev[y] * scale[nf + ec[y]];
        }
        for (int x = 0; x < nfr; ++x) {
          const int slot = wslot[R * kF + x];
          const double va = fv[x] * scale[fc[x]];
          for (int y = 0; y < 3; ++y) W[pt][slot * 3 + (ec[y] % 3)] += va * ev[y] * scale[nf + ec[y]];
        }
      }
    }
    for (int i = 0; i < nf; ++i) U[(size_t)i * nf + i] += D2[i];
    std::vector<double> Vinv(np3 * 9);
    bool ok = true;
    for (int64_t pt = 0; pt < np3; ++pt) {
      for (int m = 0; m < 3; ++m) V[pt * 9 + m * 4] += D2[nf + pt * 3 + m];
      if (!Inv3(&V[pt * 9], &Vinv[pt * 9])) ok = false;
    }
    std::vector<std::vector<double>> WV(np3);
    if (ok) {
#pragma omp parallel for schedule(static)
      for (int64_t pt = 0; pt < np3; ++pt) {
        const size_t m = Wcols[pt].size();
        WV[pt].assign(m * 3, 0.0);
        for (size_t a = 0; a < m; ++a)
          for (int c2 = 0; c2 < 3; ++c2) {
            double acc = 0.0;
            for (int k = 0; k < 3; ++k) acc += W[pt][a * 3 + k] * Vinv[pt * 9 + k * 3 + c2];
            WV[pt][a * 3 + c2] = acc;
          }
      }
    }
    std::vector<double> step(n, 0.0);
    int cg_its = 0;
    if (use_pcg) {
      if (ok) {
        // SCHUR_JACOBI: the diagonal blocks of S = U - sum_p W_p V_p^-1 W_p'
        // (U carries D_f^2), one per f parameter block, each inverted
        std::vector<int> blk_of(nf, -1), blk_pos(nf, 0);
        for (size_t k = 0; k < fblocks.size(); ++k)
          for (int a = 0; a < fblocks[k].second; ++a) {
            blk_of[fblocks[k].first + a] = (int)k;
            blk_pos[fblocks[k].first + a] = a;
          }
        std::vector<std::vector<double>> M(fblocks.size()), Minv(fblocks.size());
        for (size_t k = 0; k < fblocks.size(); ++k) {
          const int o0 = fblocks[k].first, w = fblocks[k].second;
          M[k].assign((size_t)w * w, 0.0);
          for (int a = 0; a < w; ++a)
            for (int c = 0; c < w; ++c) M[k][(size_t)a * w + c] = U[(size_t)(o0 + a) * nf + o0 + c];
        }
        for (int64_t pt = 0; pt < np3; ++pt) {
          const auto& cols = Wcols[pt];
          for (size_t a = 0; a < cols.size(); ++a)
            for (size_t b2 = 0; b2 < cols.size(); ++b2) {
              const int ka = blk_of[cols[a]];
              if (ka < 0 || ka != blk_of[cols[b2]]) continue;
              double acc = 0.0;
              for (int k = 0; k < 3; ++k) acc += WV[pt][a * 3 + k] * W[pt][b2 * 3 + k];
              M[ka][(size_t)blk_pos[cols[a]] * fblocks[ka].second + blk_pos[cols[b2]]] -= acc;
            }
        }
        for (size_t k = 0; k < fblocks.size(); ++k) LltInverse(M[k], fblocks[k].second, &Minv[k]);
        isc.D2 = D2.data();
        isc.Vinv = Vinv.data();
        std::vector<double> rhs(nf), xf(nf);
        isc.Rhs(lin.r.data(), rhs.data());
        const int term = SchurPcg(isc, fblocks, Minv, rhs.data(), nf, o->eta,
                                  std::max(1, o->max_linear_solver_iterations), xf.data(), &cg_its);
        if (term == kCgFailure) {
          ok = false;
        } else {
          for (int i = 0; i < nf; ++i) step[i] = xf[i];
          isc.BackSubstitute(lin.r.data(), xf.data(), step.data() + nf);
          for (auto& v : step) v = -v;
        }
      }
    } else {
    // S = U - sum W Vinv W^T ; rhs = g_f - sum W Vinv g_e.  Every element
    // of S is updated in point order; threads own contiguous row ranges of S,
    // so the arithmetic is that of the serial loop.
    std::vector<double> Sm = U, rhs(g.begin(), g.begin() + nf);
    cg_its = 1;
    if (ok) {
#pragma omp parallel
      {
        const int nt = omp_get_num_threads(), tid = omp_get_thread_num();
        const int r0 = (int)((int64_t)nf * tid / nt), r1 = (int)((int64_t)nf * (tid + 1) / nt);
        for (int64_t pt = 0; pt < np3; ++pt) {
          const auto& cols = Wcols[pt];
          const size_t m = cols.size();
          for (size_t a = 0; a < m; ++a) {
            if (cols[a] < r0 || cols[a] >= r1) continue;
            for (size_t b2 = 0; b2 < m; ++b2) {
              double acc = 0.0;
              for (int k = 0; k < 3; ++k) acc += WV[pt][a * 3 + k] * W[pt][b2 * 3 + k];
              Sm[(size_t)cols[a] * nf + cols[b2]] -= acc;
            }
          }
        }
      }
      for (int64_t pt = 0; pt < np3; ++pt) {
        const auto& cols = Wcols[pt];
        for (size_t a = 0; a < cols.size(); ++a) {
          double acc = 0.0;
          for (int k = 0; k < 3; ++k) acc += WV[pt][a * 3 + k] * g[nf + pt * 3 + k];
          rhs[cols[a]] -= acc;
        }
      }
    }
    if (ok && nf > 0) ok = Cholesky(Sm, nf);
    if (ok) {
      if (nf > 0) CholSolve(Sm, nf, rhs);
      for (int i = 0; i < nf; ++i) step[i] = rhs[i];
#pragma omp parallel for schedule(static)
      for (int64_t pt = 0; pt < np3; ++pt) {
        double t3[3];
        for (int k = 0; k < 3; ++k) t3[k] = g[nf + pt * 3 + k];
        const auto& cols = Wcols[pt];
        for (size_t a = 0; a < cols.size(); ++a)
          for (int k = 0; k < 3; ++k) t3[k] -= W[pt][a * 3 + k] * step[cols[a]];
        for (int k = 0; k < 3; ++k) {
          double acc = 0.0;
          for (int m2 = 0; m2 < 3; ++m2) acc += Vinv[pt * 9 + k * 3 + m2] * t3[m2];
          step[nf + pt * 3 + k] = acc;
        }
      }
      for (auto& v : step) v = -v;  // Ceres solves (J'J+D'D)x = J'f, step = -x
    }
    }  // exact Schur solve
    reuse_diagonal = true;
    double model_cost_change = 0.0;
    if (ok) {
      std::vector<double> mc(nrows);
#pragma omp parallel for schedule(static)
      for (size_t R = 0; R < nrows; ++R) {
        double mr = 0.0;
        for (int m = 0; m < lin.fn[R]; ++m) mr += lin.fval[R * kF + m] * scale[lin.fcol[R * kF + m]] * step[lin.fcol[R * kF + m]];
        for (int m = 0; m < lin.en[R]; ++m)
          mr += lin.eval[R * 3 + m] * scale[nf + lin.ecol[R * 3 + m]] * step[nf + lin.ecol[R * 3 + m]];
        mc[R] = -(mr * (lin.r[R] + mr / 2.0));
      }
      for (double v : mc) model_cost_change += v;
      ok = model_cost_change > 0.0;
    }
    sum->num_linear_solver_iterations += cg_its;
    if (!ok) {
      ++consecutive_invalid;
      ++sum->num_unsuccessful_steps;
      last_successful = false;
      if (consecutive_invalid > o->max_num_consecutive_invalid_steps) {
        trace(iteration, 0, 0, cg_its, 1);
        sum->termination_type = MI_BA_FAILURE;
        break;
      }
      trace(iteration, 0, 0, cg_its, 0);
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      continue;
    }
    consecutive_invalid = 0;
    std::vector<double> delta(n);
    for (int64_t i = 0; i < n; ++i) delta[i] = step[i] * scale[i];
    // candidate
    std::vector<double> q0(p->qvec, p->qvec + 4 * p->num_images), t0(p->tvec, p->tvec + 3 * p->num_images);
    std::vector<double> c0(p->camera_params, p->camera_params + S.s.cam_poff[p->num_cameras]);
    std::vector<double> x0(p->xyz, p->xyz + 3 * p->num_points);
    std::vector<mi_ba_cylinder> y0;
    if (gsba) y0.assign(gsba->cylinders, gsba->cylinders + gsba->num_cylinders);
    const std::vector<double> by2_0 = S.gs.by2p;
    auto restore = [&]() {
      std::copy(q0.begin(), q0.end(), p->qvec); std::copy(t0.begin(), t0.end(), p->tvec);
      std::copy(c0.begin(), c0.end(), p->camera_params); std::copy(x0.begin(), x0.end(), p->xyz);
      if (gsba) std::copy(y0.begin(), y0.end(), gsba->cylinders);
      S.gs.by2p = by2_0;
    };
    S.State(&x_state);
    S.Plus(delta);
    S.State(&c_state);
    const double candidate_cost = S.Cost();
    // ParameterToleranceReached: step_norm = |x - candidate_x| <=
    // parameter_tolerance (|x| + parameter_tolerance), x the ambient state;
    // FunctionToleranceReached: |cost change| <= function_tolerance * cost.
    // Both return before the candidate is accepted (x_ stays).
    double x_norm2 = 0.0, step_norm2 = 0.0;
    for (size_t i = 0; i < x_state.size(); ++i) {
      x_norm2 += x_state[i] * x_state[i];
      const double d = x_state[i] - c_state[i];
      step_norm2 += d * d;
    }
    const double cost_change = x_cost - candidate_cost;
    const double relative_decrease = cost_change / model_cost_change;
    const bool success = relative_decrease > o->min_relative_decrease;
    if (g_trace_v && iteration >= 1 && iteration <= g_trace_cap) {
      double* v = g_trace_v + 4 * (size_t)(iteration - 1);
      v[0] = std::sqrt(step_norm2);
      v[1] = o->parameter_tolerance * (std::sqrt(x_norm2) + o->parameter_tolerance);
      v[2] = cost_change;
      v[3] = model_cost_change;
    }
    if (std::sqrt(step_norm2) <= o->parameter_tolerance * (std::sqrt(x_norm2) + o->parameter_tolerance) ||
        std::fabs(cost_change) <= o->function_tolerance * x_cost) {
      restore();
      sum->termination_type = MI_BA_CONVERGENCE;
      ++sum->num_unsuccessful_steps;
      trace(iteration, 1, 0, cg_its, 1);
      break;
    }
    trace(iteration, 1, success ? 1 : 0, cg_its, 0);
    if (success) {
      ++sum->num_successful_steps;
      last_successful = true;
      x_cost = candidate_cost;
      radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * relative_decrease - 1.0, 3));
      radius = std::min(1e16, radius);
      decrease_factor = 2.0;
      reuse_diagonal = false;
      // the Jacobian at the new point only feeds the next iteration: skipped
      // after the last allowed one (counted as the solver does, which
      // evaluates it there too); saves a full C4 linearization in the
      // one-iteration parity test
      if (iteration < o->max_num_iterations) {
        S.Linearize(&lin);
        gmax = S.GradientMaxNorm(lin);
      }
      ++sum->num_jacobian_evaluations;
    } else {
      ++sum->num_unsuccessful_steps;
      last_successful = false;
      restore();
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
    }
  }
  sum->final_cost = x_cost + fixed;
  // by 2 points: the cylinders leave as ToCylinder() (exportCylindersToText)
  if (gsba && S.gs.by2 && gsba->refine_geometry)
    for (int c = 0; c < gsba->num_cylinders; ++c) {
      if (S.L.cyl_off[c] < 0) continue;
      mi_ba_cylinder& y = gsba->cylinders[c];
      GsbaBy2ToCylinder(&S.gs.by2p[7 * (size_t)c], y.qvec, y.tvec, &y.radius, &y.height);
    }
  return MI_BA_OK;
}

// The GSBA problem: the reprojection blocks only with include_landmark_error,
// then with ScaledLoss(landmark_error_weight / #2D features of the config
// images) (:729-762); GeometricSemanticBundleAdjuster::Assert (:664-712).
int GsbaProblem(const mi_ba_options* o, const mi_ba_problem* p, const mi_ba_gsba* g, mi_ba_options* oo,
                mi_ba_problem* pp) {
  if (!o || !p || !g) return MI_BA_ERR_INVALID_ARGUMENT;
  if (o->loss_function_type != MI_BA_LOSS_TRIVIAL) return MI_BA_ERR_UNSUPPORTED;
  *oo = *o;
  *pp = *p;
  if (!g->include_landmark_error) {
    pp->num_obs = 0;
  } else {
    int64_t total = 0;
    for (int64_t k = 0; k < p->num_obs; ++k) {
      const int i = p->obs_image[k];
      total += p->image_in_config ? (p->image_in_config[i] != 0) : 1;
    }
    oo->loss_function_type = kLossScaled;
    oo->loss_function_scale = g->landmark_error_weight / (double)std::max<int64_t>(1, total);
  }
  return MI_BA_OK;
}
}  // namespace

extern "C" {

int oracle_solve(const mi_ba_options* o, mi_ba_problem* p, const mi_ba_semantic* sem, mi_ba_summary* sum) {
  return SolveImpl(o, p, sem, nullptr, sum);
}

int oracle_gsba_solve(const mi_ba_options* o, mi_ba_problem* p, mi_ba_gsba* g, mi_ba_summary* sum) {
  mi_ba_options oo;
  mi_ba_problem pp;
  int st = GsbaProblem(o, p, g, &oo, &pp);
  if (st) return st;
  return SolveImpl(&oo, &pp, nullptr, g, sum);
}

// Every GSBA block's residual (1 - IoU) and ambient Jacobian [16]; returns
// the block count (nothing written beyond capacity), or -status.
int64_t oracle_gsba_evaluate(const mi_ba_options* o, mi_ba_problem* p, const mi_ba_gsba* g, int64_t capacity,
                             int32_t* ids, double* residuals, double* jacobians) {
  mi_ba_options oo;
  mi_ba_problem pp;
  int st = GsbaProblem(o, p, g, &oo, &pp);
  if (st) return -st;
  Setup s;
  if ((st = BuildSetup(&oo, &pp, &s))) return -st;
  GsbaSetup gs;
  if ((st = BuildGsbaSetup(&oo, &pp, s, g, &gs))) return -st;
  const int64_t n = (int64_t)gs.blocks.size();
  if (n > capacity) return n;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t k = 0; k < n; ++k) {
    ids[2 * k] = gs.blocks[k].img;
    ids[2 * k + 1] = gs.blocks[k].cyl;
    residuals[k] = GsbaResidual(&pp, s, gs, gs.blocks[k], &jacobians[16 * k]);
  }
  return n;
}

// Trunk masks for tests: the union over `cylinders` of their projected
// quadrilaterals (drawQuadrilateral), per image of the problem.
int oracle_gsba_render(const mi_ba_problem* p, const mi_ba_cylinder* cyl, int ncyl, int H, int W, uint8_t* out) {
  Setup s;
  s.cam_poff.assign(p->num_cameras + 1, 0);
  for (int c = 0; c < p->num_cameras; ++c) s.cam_poff[c + 1] = s.cam_poff[c] + 3;  // SIMPLE_PINHOLE
  for (int i = 0; i < p->num_images; ++i) {
    uint8_t* m = out + (int64_t)i * H * W;
    std::fill(m, m + (int64_t)H * W, 0);
    const double* K = &p->camera_params[s.cam_poff[p->image_camera[i]]];
    for (int c = 0; c < ncyl; ++c) {
      double q[4][2];
      if (!GsbaQuad(&p->qvec[i * 4], &p->tvec[i * 3], K, cyl[c].qvec, cyl[c].tvec, cyl[c].radius, cyl[c].height, q))
        continue;
      GsbaBox box;
      std::vector<uint8_t> mask;
      GsbaDraw(q, W, H, &box, &mask);
      for (int y = 0; y < box.h; ++y)
        for (int x = 0; x < box.w; ++x)
          if (mask[(size_t)y * box.w + x]) m[(int64_t)(box.y + y) * W + box.x + x] = 1;
    }
  }
  return 0;
}

// Cylinder::ComputeSemanticIoU for one configuration (tests).
double oracle_gsba_iou(const double* cq, const double* ct, const double* K, const mi_ba_cylinder* y,
                       const uint8_t* mask, int H, int W) {
  int64_t total = 0;
  for (int64_t k = 0; k < (int64_t)H * W; ++k) total += mask[k] != 0;
  return GsbaIoU(cq, ct, K, y->qvec, y->tvec, y->radius, y->height, mask, H, W, total);
}

}  // extern "C"
