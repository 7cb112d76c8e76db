// setup.cpp — host-side problem assembly (product code); see setup.h.
#include "setup.h"

#include <algorithm>
#include <cmath>

#include "ba_math.h"

namespace miba {

namespace {

void param_groups(int model, std::vector<int>* f, std::vector<int>* pp, std::vector<int>* ex) {
  // camera_models.h *::Initialize{FocalLength,PrincipalPoint,ExtraParams}Idxs
  switch (model) {
    case kSimplePinhole: *f = {0}; *pp = {1, 2}; *ex = {}; break;
    case kPinhole: *f = {0, 1}; *pp = {2, 3}; *ex = {}; break;
    case kSimpleRadial: *f = {0}; *pp = {1, 2}; *ex = {3}; break;
    case kRadial: *f = {0}; *pp = {1, 2}; *ex = {3, 4}; break;
    case kOpenCV: *f = {0, 1}; *pp = {2, 3}; *ex = {4, 5, 6, 7}; break;
    default: break;
  }
}

// CSR adjacency: items grouped by key, preserving original order.
void csr(const int32_t* key, int64_t n, int64_t nkeys, std::vector<int64_t>* off, std::vector<int64_t>* items) {
  off->assign(nkeys + 1, 0);
  for (int64_t k = 0; k < n; ++k) (*off)[key[k] + 1]++;
  for (int64_t k = 0; k < nkeys; ++k) (*off)[k + 1] += (*off)[k];
  items->resize(n);
  std::vector<int64_t> pos(off->begin(), off->end() - 1);
  for (int64_t k = 0; k < n; ++k) (*items)[pos[key[k]]++] = k;
}

}  // namespace

mi_ba_status build_setup(const mi_ba_options& o, mi_ba_problem* p, HostSetup* s) {
  if (!p) return MI_BA_ERR_INVALID_ARGUMENT;
  if (p->num_images < 0 || p->num_cameras < 0 || p->num_points < 0 || p->num_obs < 0)
    return MI_BA_ERR_INVALID_ARGUMENT;
  if (p->num_obs > 0 && (!p->obs_xy || !p->obs_image || !p->obs_point)) return MI_BA_ERR_INVALID_ARGUMENT;
  if (p->num_images > 0 && (!p->qvec || !p->tvec || !p->image_camera)) return MI_BA_ERR_INVALID_ARGUMENT;
  if (p->num_cameras > 0 && !p->camera_params) return MI_BA_ERR_INVALID_ARGUMENT;
  if (p->num_points > 0 && !p->xyz) return MI_BA_ERR_INVALID_ARGUMENT;
  if (o.loss_function_scale < 0) return MI_BA_ERR_INVALID_ARGUMENT;  // BundleAdjustmentOptions::Check
  if (p->num_obs >= (int64_t)0xffffffffLL || p->num_points >= (int64_t)0xffffffffLL)
    return MI_BA_ERR_UNSUPPORTED;
  const int I = p->num_images, C = p->num_cameras;
  const int64_t P = p->num_points, N = p->num_obs;
  for (int i = 0; i < I; ++i)
    if (p->image_camera[i] < 0 || p->image_camera[i] >= C) return MI_BA_ERR_INVALID_ARGUMENT;
  for (int64_t k = 0; k < N; ++k)
    if (p->obs_image[k] < 0 || p->obs_image[k] >= I || p->obs_point[k] < 0 || p->obs_point[k] >= P)
      return MI_BA_ERR_INVALID_ARGUMENT;
  for (int i = 0; i < I; ++i) {
    // BundleAdjustmentConfig::SetConstantPose / SetConstantTvec CHECKs
    // (bundle_adjustment.cc:165-186): tvec subset and constant pose exclusive.
    const bool cp = p->image_constant_pose && p->image_constant_pose[i];
    const uint8_t tm = p->image_constant_tvec ? p->image_constant_tvec[i] : 0;
    if ((tm & ~7u) != 0) return MI_BA_ERR_INVALID_ARGUMENT;
    if (cp && tm) return MI_BA_ERR_INVALID_ARGUMENT;
  }
  // per-camera models (camera_models.h:117-141: unknown ids throw
  // std::domain_error, :140-141)
  if (!p->camera_model_ids && num_params(p->camera_model) < 0) return MI_BA_ERR_UNSUPPORTED;
  s->cam_model.assign(C, 0);
  s->cam_off.assign(C + 1, 0);
  bool mixed = false;
  int np = num_params(p->camera_model);
  for (int c = 0; c < C; ++c) {
    const int m = problem_camera_model(p, c);
    if (num_params(m) < 0) return MI_BA_ERR_UNSUPPORTED;
    s->cam_model[c] = m;
    s->cam_off[c + 1] = s->cam_off[c] + num_params(m);
    if (c == 0) np = num_params(m);
    if (m != s->cam_model[0]) mixed = true;
    np = std::max(np, num_params(m));
  }
  s->model = mixed ? kMixedModels : (C > 0 ? s->cam_model[0] : p->camera_model);
  s->np = np;

  std::vector<int64_t> img_off, img_items, pt_off, pt_items;
  csr(p->obs_image, N, I, &img_off, &img_items);
  csr(p->obs_point, N, P, &pt_off, &pt_items);

  auto in_cfg = [&](int i) { return p->image_in_config ? p->image_in_config[i] != 0 : true; };
  std::vector<uint8_t> cam_in(C, 0), cam_const(C, 0);
  for (int c = 0; c < C; ++c) cam_const[c] = p->camera_constant ? (p->camera_constant[c] != 0) : 0;
  std::vector<int64_t> pt_nobs(P, 0);
  std::vector<int64_t> blocks;
  blocks.reserve(N);
  s->img_var.assign(I, 0);
  s->img_tvec_mask.assign(I, 0);

  // AddImageToProblem (bundle_adjustment.cc:348-427)
  for (int i = 0; i < I; ++i) {
    if (!in_cfg(i)) continue;
    double* q = p->qvec + 4 * (size_t)i;  // NormalizeQuaternion (pose.cc:82-91)
    const double norm = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (norm == 0) {
      q[0] = 1.0;
    } else {
      for (int m = 0; m < 4; ++m) q[m] = q[m] / norm;
    }
    const bool cpose = !o.refine_extrinsics || (p->image_constant_pose && p->image_constant_pose[i]);
    const int64_t nobs = img_off[i + 1] - img_off[i];
    for (int64_t m = img_off[i]; m < img_off[i + 1]; ++m) {
      const int64_t k = img_items[m];
      pt_nobs[p->obs_point[k]] += 1;
      blocks.push_back(k);
    }
    if (nobs > 0) {
      cam_in[p->image_camera[i]] = 1;
      if (!cpose) {
        s->img_var[i] = 1;
        s->img_tvec_mask[i] = p->image_constant_tvec ? p->image_constant_tvec[i] : 0;
      }
    }
  }
  // AddPointToProblem (:429-478): variable points, then constant points.
  if (p->point_config) {
    for (int pass = 1; pass <= 2; ++pass) {
      for (int64_t pt = 0; pt < P; ++pt) {
        if (p->point_config[pt] != pass) continue;
        if (pt_nobs[pt] == pt_off[pt + 1] - pt_off[pt]) continue;
        for (int64_t m = pt_off[pt]; m < pt_off[pt + 1]; ++m) {
          const int64_t k = pt_items[m];
          const int img = p->obs_image[k];
          if (in_cfg(img)) continue;
          pt_nobs[pt] += 1;
          const int cam = p->image_camera[img];
          if (!cam_in[cam]) {
            cam_in[cam] = 1;
            cam_const[cam] = 1;  // config_.SetConstantCamera
          }
          blocks.push_back(k);
        }
      }
    }
  }
  // ParameterizeCameras (:480-516): SubsetManifold over the params the
  // refine flags hold constant, per camera model.
  auto tangent = [&](int model, int* idx) {
    std::vector<int> f, pp, ex;
    param_groups(model, &f, &pp, &ex);
    const int n = num_params(model);
    std::vector<uint8_t> is_const(n, 0);
    if (!o.refine_focal_length) for (int k : f) is_const[k] = 1;
    if (!o.refine_principal_point) for (int k : pp) is_const[k] = 1;
    if (!o.refine_extra_params) for (int k : ex) is_const[k] = 1;
    int ct = 0;
    for (int k = 0; k < n; ++k)
      if (!is_const[k]) {
        if (idx) idx[ct] = k;
        ++ct;
      }
    return ct;
  };
  s->ct = tangent(s->model == kMixedModels ? kOpenCV : s->model, s->cam_tan_idx);
  s->cam_ct.assign(C, 0);
  if (s->model == kMixedModels) {
    s->ct = 0;
    for (int c = 0; c < C; ++c) {
      s->cam_ct[c] = (uint8_t)tangent(s->cam_model[c], nullptr);
      s->ct = std::max<int>(s->ct, s->cam_ct[c]);
    }
  } else {
    for (int c = 0; c < C; ++c) s->cam_ct[c] = (uint8_t)s->ct;
  }
  const bool constant_camera = !o.refine_focal_length && !o.refine_principal_point && !o.refine_extra_params;
  s->cam_var.assign(C, 0);
  for (int c = 0; c < C; ++c)
    s->cam_var[c] = cam_in[c] && !constant_camera && !cam_const[c] && s->cam_ct[c] > 0;
  // ParameterizePoints (:518-530)
  s->pt_var.assign(P, 0);
  for (int64_t pt = 0; pt < P; ++pt) {
    if (pt_nobs[pt] == 0) continue;
    bool constant = (pt_off[pt + 1] - pt_off[pt]) > pt_nobs[pt];
    if (p->point_config && p->point_config[pt] == 2) constant = true;
    s->pt_var[pt] = !constant;
  }
  // Reduced program.
  s->num_residual_blocks = (int64_t)blocks.size();
  s->reduced_obs.clear();
  s->fixed_obs.clear();
  std::vector<uint8_t> used_img(I, 0), used_cam(C, 0);
  int64_t used_pts = 0;
  std::vector<uint8_t> used_pt(P, 0);
  for (int64_t k : blocks) {
    const int img = p->obs_image[k];
    const int cam = p->image_camera[img];
    const int64_t pt = p->obs_point[k];
    const bool vpose = s->img_var[img];
    if (!(vpose || s->cam_var[cam] || s->pt_var[pt])) {
      s->fixed_obs.push_back(k);
      continue;
    }
    s->reduced_obs.push_back(k);
    if (vpose) used_img[img] = 1;
    if (s->cam_var[cam]) used_cam[cam] = 1;
    if (s->pt_var[pt] && !used_pt[pt]) { used_pt[pt] = 1; ++used_pts; }
  }
  s->num_residuals_reduced = 2 * (int64_t)s->reduced_obs.size();
  int64_t ne = 3 * used_pts;
  for (int i = 0; i < I; ++i)
    if (used_img[i]) {
      int masked = 0;
      for (int k = 0; k < 3; ++k) masked += (s->img_tvec_mask[i] >> k) & 1;
      ne += 6 - masked;
    }
  for (int c = 0; c < C; ++c)
    if (used_cam[c]) ne += s->cam_ct[c];
  s->num_effective_parameters_reduced = ne;
  return MI_BA_OK;
}

}  // namespace miba
