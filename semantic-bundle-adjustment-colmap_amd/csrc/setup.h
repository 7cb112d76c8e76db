// setup.h — host-side problem assembly (product code).
//
// Array-based restatement of BundleAdjuster::SetUp / AddImageToProblem /
// AddPointToProblem / ParameterizeCameras / ParameterizePoints
// (src/optim/bundle_adjustment.cc:326-530) plus Ceres' reduced-program rule
// (residual blocks whose parameter blocks are all constant are dropped and
// their cost is reported as fixed_cost).  Linear in the number of
// observations (CSR by image and by point) so it scales to 10M observations.
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/mi_ba.h"

namespace miba {

struct HostSetup {
  int model = 0;       // the problem's camera model, or kMixedModels
  int np = 0;          // params per camera (the largest, mixed models)
  int ct = 0;          // refined intrinsics slots per camera (the largest, mixed models)
  int cam_tan_idx[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // single-model problems
  // per camera: model id, offset of its params in mi_ba_problem::camera_params,
  // refined intrinsics (its slots ct_c..ct-1 are padding: zero Jacobian columns)
  std::vector<int32_t> cam_model;
  std::vector<int64_t> cam_off;
  std::vector<uint8_t> cam_ct;
  std::vector<int64_t> reduced_obs;   // observation index of each reduced block (program order)
  std::vector<int64_t> fixed_obs;     // blocks dropped from the reduced program
  std::vector<uint8_t> img_var;       // pose is a variable parameter block
  std::vector<uint8_t> img_tvec_mask; // SubsetManifold(3, idxs) on tvec
  std::vector<uint8_t> cam_var;
  std::vector<uint8_t> pt_var;
  int64_t num_residual_blocks = 0;
  int64_t num_residuals_reduced = 0;
  int64_t num_effective_parameters_reduced = 0;
};

// Model id of camera c (camera_model_ids, else camera_model).
inline int problem_camera_model(const mi_ba_problem* p, int c) {
  return p->camera_model_ids ? p->camera_model_ids[c] : p->camera_model;
}

// Validates the problem, normalises config qvecs in place (Image::NormalizeQvec
// at bundle_adjustment.cc:355) and fills `s`.
mi_ba_status build_setup(const mi_ba_options& o, mi_ba_problem* p, HostSetup* s);

}  // namespace miba
