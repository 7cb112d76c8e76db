// colmap_amd/bundle_adjustment.h — C++ facade with the reference's API.
//
// Keeps the signatures and semantics COLMAP callers use
// (src/optim/bundle_adjustment.h:49-203, src/optim/semantic_bundle_adjustment.h:
// 53-272 of AlainSchoebi/semantic-bundle-adjustment-colmap) and routes Solve
// to the MI355X library through the C-ABI in mi_ba.h.  Header-only; link
// against libmi_ba.so.
//
//   colmap::BundleAdjustmentOptions          -> colmap_amd::BundleAdjustmentOptions
//   colmap::BundleAdjustmentConfig           -> colmap_amd::BundleAdjustmentConfig
//   colmap::BundleAdjuster                   -> colmap_amd::BundleAdjuster
//   colmap::SemanticBundleAdjustmentOptions  -> colmap_amd::SemanticBundleAdjustmentOptions
//   colmap::SemanticBundleAdjuster           -> colmap_amd::SemanticBundleAdjuster
//   ceres::Solver::Summary (fields read)     -> colmap_amd::SolverSummary
//   colmap::Reconstruction (BA subset)       -> colmap_amd::Reconstruction
//
// Error convention: the reference aborts through glog CHECK or throws; here
// invalid configurations throw std::invalid_argument, unknown camera models
// std::domain_error, reuse of an adjuster std::logic_error, device/runtime
// failures std::runtime_error; Solve returns false when there are no
// residuals (bundle_adjustment.cc:267-269).
#pragma once

#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <fstream>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <exception>
#include <functional>
#include <limits>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../mi_ba.h"
#include "model_io.h"
#include "reconstruction.h"

namespace colmap_amd {

// ---------------------------------------------------------------------------
// Options / config (bundle_adjustment.h:49-167)
// ---------------------------------------------------------------------------
// ceres::CallbackReturnType / IterationSummary / IterationCallback
// (the solver_options.callbacks interface COLMAP's controllers use,
// controllers/bundle_adjustment.cc:43-61,87-88).
enum CallbackReturnType {
  SOLVER_CONTINUE = MI_BA_SOLVER_CONTINUE,
  SOLVER_ABORT = MI_BA_SOLVER_ABORT,
  SOLVER_TERMINATE_SUCCESSFULLY = MI_BA_SOLVER_TERMINATE_SUCCESSFULLY
};
typedef mi_ba_iteration_summary IterationSummary;
class IterationCallback {
 public:
  virtual ~IterationCallback() {}
  virtual CallbackReturnType operator()(const IterationSummary& summary) = 0;
};

struct SolverOptions {  // ceres::Solver::Options subset set by COLMAP
  double function_tolerance = 0.0;
  double gradient_tolerance = 0.0;
  double parameter_tolerance = 0.0;
  bool minimizer_progress_to_stdout = false;
  int max_num_iterations = 100;
  int max_linear_solver_iterations = 200;
  int max_num_consecutive_invalid_steps = 10;
  int max_consecutive_nonmonotonic_steps = 10;
  int num_threads = -1;
  // run in order after every iteration; the first one that does not return
  // SOLVER_CONTINUE decides (Ceres RunCallbacks).  Not owned.
  std::vector<IterationCallback*> callbacks;
  // the Reconstruction holds the current point whenever a callback runs
  bool update_state_every_iteration = false;
};

struct BundleAdjustmentOptions {
  enum class LossFunctionType { TRIVIAL, SOFT_L1, CAUCHY };
  LossFunctionType loss_function_type = LossFunctionType::TRIVIAL;
  double loss_function_scale = 1.0;
  bool refine_focal_length = true;
  bool refine_principal_point = false;
  bool refine_extra_params = true;
  bool refine_extrinsics = true;
  bool print_summary = true;
  int min_num_residuals_for_multi_threading = 50000;  // kept for API parity
  SolverOptions solver_options;
  int device = 0;  // build addition: HIP device ordinal
  // build addition: a flag another thread may set to MI_BA_SOLVER_TERMINATE_
  // SUCCESSFULLY / MI_BA_SOLVER_ABORT to stop the solve at the next
  // iteration boundary (Thread::Stop without a callback); not owned
  const std::atomic<int32_t>* stop_flag = nullptr;

  bool Check() const {
    if (loss_function_scale < 0) throw std::invalid_argument("loss_function_scale must be >= 0");
    return true;
  }
};

class BundleAdjustmentConfig {
 public:
  size_t NumImages() const { return image_ids_.size(); }
  size_t NumPoints() const { return variable_point3D_ids_.size() + constant_point3D_ids_.size(); }
  size_t NumConstantCameras() const { return constant_camera_ids_.size(); }
  size_t NumConstantPoses() const { return constant_poses_.size(); }
  size_t NumConstantTvecs() const { return constant_tvecs_.size(); }
  size_t NumVariablePoints() const { return variable_point3D_ids_.size(); }
  size_t NumConstantPoints() const { return constant_point3D_ids_.size(); }

  // bundle_adjustment.cc:107-138
  size_t NumResiduals(const Reconstruction& reconstruction) const {
    size_t n = 0;
    for (const image_t id : image_ids_) n += reconstruction.GetImage(id).NumPoints3D();
    auto per_point = [&](point3D_t id) {
      size_t m = 0;
      for (const auto& te : reconstruction.GetPoint3D(id).track)
        if (image_ids_.count(te.image_id) == 0) m += 1;
      return m;
    };
    for (const auto id : variable_point3D_ids_) n += per_point(id);
    for (const auto id : constant_point3D_ids_) n += per_point(id);
    return 2 * n;
  }

  void AddImage(image_t id) { image_ids_.insert(id); }
  bool HasImage(image_t id) const { return image_ids_.count(id) != 0; }
  void RemoveImage(image_t id) { image_ids_.erase(id); }

  void SetConstantCamera(camera_t id) { constant_camera_ids_.insert(id); }
  void SetVariableCamera(camera_t id) { constant_camera_ids_.erase(id); }
  bool IsConstantCamera(camera_t id) const { return constant_camera_ids_.count(id) != 0; }

  void SetConstantPose(image_t id) {
    if (!HasImage(id) || HasConstantTvec(id)) throw std::invalid_argument("SetConstantPose");
    constant_poses_.insert(id);
  }
  void SetVariablePose(image_t id) { constant_poses_.erase(id); }
  bool HasConstantPose(image_t id) const { return constant_poses_.count(id) != 0; }

  void SetConstantTvec(image_t id, const std::vector<int>& idxs) {
    std::vector<int> s = idxs;
    std::sort(s.begin(), s.end());
    if (idxs.empty() || idxs.size() > 3 || !HasImage(id) || HasConstantPose(id) ||
        std::adjacent_find(s.begin(), s.end()) != s.end() || s.front() < 0 || s.back() > 2)
      throw std::invalid_argument("SetConstantTvec");
    constant_tvecs_.emplace(id, idxs);
  }
  void RemoveConstantTvec(image_t id) { constant_tvecs_.erase(id); }
  bool HasConstantTvec(image_t id) const { return constant_tvecs_.count(id) != 0; }

  void AddVariablePoint(point3D_t id) {
    if (HasConstantPoint(id)) throw std::invalid_argument("AddVariablePoint");
    variable_point3D_ids_.insert(id);
  }
  void AddConstantPoint(point3D_t id) {
    if (HasVariablePoint(id)) throw std::invalid_argument("AddConstantPoint");
    constant_point3D_ids_.insert(id);
  }
  bool HasPoint(point3D_t id) const { return HasVariablePoint(id) || HasConstantPoint(id); }
  bool HasVariablePoint(point3D_t id) const { return variable_point3D_ids_.count(id) != 0; }
  bool HasConstantPoint(point3D_t id) const { return constant_point3D_ids_.count(id) != 0; }
  void RemoveVariablePoint(point3D_t id) { variable_point3D_ids_.erase(id); }
  void RemoveConstantPoint(point3D_t id) { constant_point3D_ids_.erase(id); }

  const std::unordered_set<image_t>& Images() const { return image_ids_; }
  const std::unordered_set<point3D_t>& VariablePoints() const { return variable_point3D_ids_; }
  const std::unordered_set<point3D_t>& ConstantPoints() const { return constant_point3D_ids_; }
  const std::vector<int>& ConstantTvec(image_t id) const { return constant_tvecs_.at(id); }

 private:
  std::unordered_set<camera_t> constant_camera_ids_;
  std::unordered_set<image_t> image_ids_;
  std::unordered_set<point3D_t> variable_point3D_ids_;
  std::unordered_set<point3D_t> constant_point3D_ids_;
  std::unordered_set<image_t> constant_poses_;
  std::unordered_map<image_t, std::vector<int>> constant_tvecs_;
};

// The ceres::Solver::Summary fields COLMAP reads (PrintSolverSummary).
struct SolverSummary {
  enum TerminationType { CONVERGENCE = 0, NO_CONVERGENCE = 1, FAILURE = 2, USER_SUCCESS = 3, USER_FAILURE = 4 };
  int64_t num_residuals_reduced = 0;
  int64_t num_effective_parameters_reduced = 0;
  int num_successful_steps = 0;
  int num_unsuccessful_steps = 0;
  TerminationType termination_type = FAILURE;
  double initial_cost = 0, final_cost = 0, fixed_cost = 0;
  double total_time_in_seconds = 0;
  double jacobian_evaluation_time_in_seconds = 0;
  int num_jacobian_evaluations = 0;
  int num_linear_solver_iterations = 0;
};

namespace internal {

// mkdir -p (createFolder, util/utils.h:92-105, without emptying the folder)
inline void MakeDirs(const std::string& path) {
  std::string cur;
  for (size_t k = 0; k <= path.size(); ++k) {
    if (k == path.size() || path[k] == '/') {
      if (!cur.empty() && ::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST)
        throw std::runtime_error("cannot create folder " + cur);
    }
    if (k < path.size()) cur += path[k];
  }
}

// Flattened Reconstruction + config (the layout ParallelBundleAdjuster::SetUp
// builds, bundle_adjustment.cc:665-783) with id <-> index maps for write-back.
struct Flat {
  int model = -1;
  std::vector<camera_t> cam_ids;
  std::vector<image_t> img_ids;
  std::vector<point3D_t> pt_ids;
  std::vector<double> cam_params, qvec, tvec, xyz, obs_xy;
  std::vector<int32_t> image_camera, obs_image, obs_point, cam_models;
  std::vector<size_t> cam_offsets;  // params of camera c at [cam_offsets[c], cam_offsets[c + 1])
  std::vector<uint8_t> cam_const, img_cfg, img_cpose, img_ctvec, pt_cfg;
  mi_ba_problem problem{};

  void Build(const Reconstruction& rec, const BundleAdjustmentConfig& cfg) {
    std::unordered_map<camera_t, int32_t> cidx;
    std::unordered_map<image_t, int32_t> iidx;
    std::unordered_map<point3D_t, int32_t> pidx;
    // per-camera models (camera_models.h:117-141), params back to back
    cam_offsets.push_back(0);
    for (const auto& c : rec.cameras) {
      if (model < 0) model = c.second.model_id;
      cidx[c.first] = (int32_t)cam_ids.size();
      cam_ids.push_back(c.first);
      const int np = mi_ba_num_params(c.second.model_id);
      if (np < 0) throw std::domain_error("Camera model does not exist");
      if ((int)c.second.params.size() != np) throw std::invalid_argument("camera params size");
      cam_params.insert(cam_params.end(), c.second.params.begin(), c.second.params.end());
      cam_offsets.push_back(cam_params.size());
      cam_models.push_back(c.second.model_id);
      cam_const.push_back(cfg.IsConstantCamera(c.first) ? 1 : 0);
    }
    for (const auto& p : rec.points3D) {
      pidx[p.first] = (int32_t)pt_ids.size();
      pt_ids.push_back(p.first);
      xyz.insert(xyz.end(), p.second.xyz, p.second.xyz + 3);
      pt_cfg.push_back(cfg.HasVariablePoint(p.first) ? 1 : cfg.HasConstantPoint(p.first) ? 2 : 0);
    }
    for (const auto& im : rec.images) {
      const int32_t i = (int32_t)img_ids.size();
      iidx[im.first] = i;
      img_ids.push_back(im.first);
      qvec.insert(qvec.end(), im.second.qvec, im.second.qvec + 4);
      tvec.insert(tvec.end(), im.second.tvec, im.second.tvec + 3);
      image_camera.push_back(cidx.at(im.second.camera_id));
      img_cfg.push_back(cfg.HasImage(im.first) ? 1 : 0);
      img_cpose.push_back(cfg.HasConstantPose(im.first) ? 1 : 0);
      uint8_t mask = 0;
      if (cfg.HasConstantTvec(im.first))
        for (int k : cfg.ConstantTvec(im.first)) mask |= (uint8_t)(1u << k);
      img_ctvec.push_back(mask);
    }
    // observations: every Point2D with a Point3D (the tracks)
    for (const auto& im : rec.images) {
      for (const auto& p2 : im.second.points2D) {
        if (!p2.HasPoint3D()) continue;
        obs_xy.push_back(p2.xy[0]);
        obs_xy.push_back(p2.xy[1]);
        obs_image.push_back(iidx.at(im.first));
        obs_point.push_back(pidx.at(p2.point3D_id));
      }
    }
    problem.camera_model = model < 0 ? MI_BA_SIMPLE_RADIAL : model;
    problem.num_cameras = (int32_t)cam_ids.size();
    problem.camera_params = cam_params.data();
    problem.camera_constant = cam_const.data();
    problem.num_images = (int32_t)img_ids.size();
    problem.qvec = qvec.data();
    problem.tvec = tvec.data();
    problem.image_camera = image_camera.data();
    problem.image_in_config = img_cfg.data();
    problem.image_constant_pose = img_cpose.data();
    problem.image_constant_tvec = img_ctvec.data();
    problem.num_points = (int64_t)pt_ids.size();
    problem.xyz = xyz.data();
    problem.point_config = pt_cfg.data();
    problem.num_obs = (int64_t)obs_image.size();
    problem.obs_xy = obs_xy.data();
    problem.obs_image = obs_image.data();
    problem.obs_point = obs_point.data();
    problem.camera_model_ids = cam_models.data();
  }

  void WriteBack(Reconstruction* rec) const {
    for (size_t c = 0; c < cam_ids.size(); ++c)
      std::copy(cam_params.begin() + cam_offsets[c], cam_params.begin() + cam_offsets[c + 1],
                rec->cameras.at(cam_ids[c]).params.begin());
    for (size_t i = 0; i < img_ids.size(); ++i) {
      Image& im = rec->images.at(img_ids[i]);
      std::copy(qvec.begin() + 4 * i, qvec.begin() + 4 * i + 4, im.qvec);
      std::copy(tvec.begin() + 3 * i, tvec.begin() + 3 * i + 3, im.tvec);
    }
    for (size_t k = 0; k < pt_ids.size(); ++k)
      std::copy(xyz.begin() + 3 * k, xyz.begin() + 3 * k + 3, rec->points3D.at(pt_ids[k]).xyz);
  }
};

inline mi_ba_options ToOptions(const BundleAdjustmentOptions& o) {
  mi_ba_options m;
  mi_ba_default_options(&m);
  m.loss_function_type = (int32_t)o.loss_function_type;
  m.loss_function_scale = o.loss_function_scale;
  m.refine_focal_length = o.refine_focal_length;
  m.refine_principal_point = o.refine_principal_point;
  m.refine_extra_params = o.refine_extra_params;
  m.refine_extrinsics = o.refine_extrinsics;
  m.print_summary = o.print_summary;
  m.max_num_iterations = o.solver_options.max_num_iterations;
  m.function_tolerance = o.solver_options.function_tolerance;
  m.gradient_tolerance = o.solver_options.gradient_tolerance;
  m.parameter_tolerance = o.solver_options.parameter_tolerance;
  m.max_linear_solver_iterations = o.solver_options.max_linear_solver_iterations;
  m.max_num_consecutive_invalid_steps = o.solver_options.max_num_consecutive_invalid_steps;
  m.device = o.device;
  return m;
}

static_assert(sizeof(std::atomic<int32_t>) == sizeof(int32_t) && alignof(std::atomic<int32_t>) == alignof(int32_t),
              "the stop flag is read as an int32_t");

// solver_options.callbacks through the C-ABI's single callback: the bridge
// runs the caller's callbacks in order; `sync` (set when
// update_state_every_iteration) copies the point the library has just
// written into the flattened arrays back into the caller's objects first.
// No exception crosses the C-ABI callback: one thrown by a callback (or by
// the state copy) is kept, the solve is aborted (SOLVER_ABORT) and Solve
// rethrows it once the library has returned (Rethrow), so it leaves Solve as
// it would leave ceres::Solve.
struct CallbackBridge {
  const std::vector<IterationCallback*>* callbacks = nullptr;
  std::function<void()> sync;
  std::exception_ptr error;
  static int32_t Call(void* user, const mi_ba_iteration_summary* summary) {
    CallbackBridge* b = static_cast<CallbackBridge*>(user);
    try {
      if (b->sync) b->sync();
      for (IterationCallback* cb : *b->callbacks) {
        const CallbackReturnType r = (*cb)(*summary);
        if (r != SOLVER_CONTINUE) return r;
      }
    } catch (...) {
      b->error = std::current_exception();
      return SOLVER_ABORT;
    }
    return SOLVER_CONTINUE;
  }
  void Rethrow() {
    if (error) std::rethrow_exception(error);
  }
};

// Installs the options' callbacks / stop flag into o (bridge must outlive the solve).
inline void InstallCallbacks(const BundleAdjustmentOptions& options, CallbackBridge* bridge,
                             std::function<void()> sync, mi_ba_options* o) {
  o->stop_flag = reinterpret_cast<const int32_t*>(options.stop_flag);
  o->update_state_every_iteration = options.solver_options.update_state_every_iteration ? 1 : 0;
  if (options.solver_options.callbacks.empty()) return;
  bridge->callbacks = &options.solver_options.callbacks;
  if (o->update_state_every_iteration) bridge->sync = std::move(sync);
  o->iteration_callback = &CallbackBridge::Call;
  o->callback_user = bridge;
}

inline SolverSummary ToSummary(const mi_ba_summary& s) {
  SolverSummary o;
  o.num_residuals_reduced = s.num_residuals_reduced;
  o.num_effective_parameters_reduced = s.num_effective_parameters_reduced;
  o.num_successful_steps = s.num_successful_steps;
  o.num_unsuccessful_steps = s.num_unsuccessful_steps;
  o.termination_type = (SolverSummary::TerminationType)s.termination_type;
  o.initial_cost = s.initial_cost;
  o.final_cost = s.final_cost;
  o.fixed_cost = s.fixed_cost;
  o.total_time_in_seconds = s.total_time_in_seconds;
  o.jacobian_evaluation_time_in_seconds = s.jacobian_evaluation_time_in_seconds;
  o.num_jacobian_evaluations = s.num_jacobian_evaluations;
  o.num_linear_solver_iterations = s.num_linear_solver_iterations;
  return o;
}

}  // namespace internal

// Device resources reused by consecutive solves of one host thread (the
// mapper's repeated local BAs): pass the same arena to every Solve.
class SolverArena {
 public:
  SolverArena() = default;
  SolverArena(const SolverArena&) = delete;
  SolverArena& operator=(const SolverArena&) = delete;
  ~SolverArena() { mi_ba_context_destroy(ctx_); }
  mi_ba_context** get() { return &ctx_; }

 private:
  mi_ba_context* ctx_ = nullptr;
};

// ---------------------------------------------------------------------------
// BundleAdjuster (bundle_adjustment.h:171-203)
// ---------------------------------------------------------------------------
class BundleAdjuster {
 public:
  BundleAdjuster(const BundleAdjustmentOptions& options, const BundleAdjustmentConfig& config)
      : options_(options), config_(config) {
    options_.Check();
  }

  // arena (optional): device resources kept across solves (SolverArena)
  bool Solve(Reconstruction* reconstruction, SolverArena* arena = nullptr) {
    if (!reconstruction) throw std::invalid_argument("reconstruction is null");
    if (used_) throw std::logic_error("Cannot use the same BundleAdjuster multiple times");
    used_ = true;
    internal::Flat flat;
    flat.Build(*reconstruction, config_);
    mi_ba_options o = internal::ToOptions(options_);
    internal::CallbackBridge bridge;
    internal::InstallCallbacks(options_, &bridge, [&] { flat.WriteBack(reconstruction); }, &o);
    mi_ba_summary s;
    const mi_ba_status st = arena ? mi_ba_solve_in(arena->get(), &o, &flat.problem, nullptr, &s)
                                  : mi_ba_solve(&o, &flat.problem, nullptr, &s);
    bridge.Rethrow();
    if (st == MI_BA_ERR_NO_RESIDUALS) return false;
    internal::ThrowStatus(st, "BundleAdjuster::Solve");
    summary_ = internal::ToSummary(s);
    flat.WriteBack(reconstruction);
    return true;
  }

  // Problem-assembly counts without solving (host only).
  mi_ba_setup_info SetUpInfo(const Reconstruction& reconstruction) const {
    internal::Flat flat;
    flat.Build(reconstruction, config_);
    const mi_ba_options o = internal::ToOptions(options_);
    mi_ba_setup_info info;
    internal::ThrowStatus(mi_ba_setup_stats(&o, &flat.problem, &info), "SetUpInfo");
    return info;
  }

  const SolverSummary& Summary() const { return summary_; }

 private:
  BundleAdjustmentOptions options_;
  BundleAdjustmentConfig config_;
  SolverSummary summary_;
  bool used_ = false;
};

// ---------------------------------------------------------------------------
// ParallelBundleAdjuster (bundle_adjustment.h:208-268, bundle_adjustment.cc:
// 536-783): the PBA entry point COLMAP's mapper takes for global BA when
// ba_global_use_pba is set (controllers/incremental_mapper.cc:66-71,
// sfm/incremental_mapper.cc:716-747).  Same Options, construction CHECKs,
// IsSupported rule and problem: every config image (SIMPLE_RADIAL, no shared
// intrinsics), the measurements of config images only, every point they see
// variable, per-image camera state (constant pose + intrinsics / fixed
// intrinsics / variable).  PBA's own float LM is replaced by the MI355X
// solver in f64 with Ceres' LM semantics (max_num_iterations from Options);
// Summary() reports that solve's counts and costs.
// ---------------------------------------------------------------------------
class ParallelBundleAdjuster {
 public:
  struct Options {
    bool print_summary = true;
    int max_num_iterations = 50;
    int gpu_index = -1;  // -1: device 0
    int num_threads = -1;
    int min_num_residuals_for_multi_threading = 50000;
    bool Check() const {
      if (max_num_iterations < 0) throw std::invalid_argument("max_num_iterations must be >= 0");
      return true;
    }
  };

  ParallelBundleAdjuster(const Options& options, const BundleAdjustmentOptions& ba_options,
                         const BundleAdjustmentConfig& config)
      : options_(options), ba_options_(ba_options), config_(config) {
    options_.Check();
    ba_options_.Check();
    if (config_.NumConstantCameras() != 0)
      throw std::invalid_argument("PBA does not allow to set individual cameras constant");
    if (config_.NumConstantPoses() != 0)
      throw std::invalid_argument("PBA does not allow to set individual translational elements constant");
    if (config_.NumConstantTvecs() != 0)
      throw std::invalid_argument("PBA does not allow to set individual translational elements constant");
    if (config_.NumVariablePoints() != 0 || config_.NumConstantPoints() != 0)
      throw std::invalid_argument("PBA does not allow to parameterize individual 3D points");
  }

  static bool IsSupported(const BundleAdjustmentOptions& options, const Reconstruction& reconstruction) {
    if (options.refine_principal_point || options.refine_focal_length != options.refine_extra_params) return false;
    std::unordered_set<camera_t> camera_ids;
    for (const auto& im : reconstruction.images) {
      if (!im.second.IsRegistered()) continue;
      const auto cam = reconstruction.cameras.find(im.second.camera_id);
      if (camera_ids.count(im.second.camera_id) != 0 || cam == reconstruction.cameras.end() ||
          cam->second.model_id != MI_BA_SIMPLE_RADIAL)
        return false;
      camera_ids.insert(im.second.camera_id);
    }
    return true;
  }

  bool Solve(Reconstruction* reconstruction) {
    if (!reconstruction) throw std::invalid_argument("reconstruction is null");
    if (used_) throw std::logic_error("Cannot use the same ParallelBundleAdjuster multiple times");
    used_ = true;
    if (ba_options_.refine_principal_point) throw std::invalid_argument("PBA: refine_principal_point");
    if (ba_options_.refine_focal_length != ba_options_.refine_extra_params)
      throw std::invalid_argument("PBA: refine_focal_length != refine_extra_params");
    // AddImagesToProblem (bundle_adjustment.cc:680-728)
    std::unordered_set<camera_t> cams;
    for (const image_t id : config_.Images()) {
      const Image& im = reconstruction->GetImage(id);
      if (!cams.insert(im.camera_id).second) throw std::invalid_argument("PBA does not support shared intrinsics");
      if (reconstruction->GetCamera(im.camera_id).model_id != MI_BA_SIMPLE_RADIAL)
        throw std::domain_error("PBA only supports the SIMPLE_RADIAL camera model");
    }
    // The PBA problem: config images only (their measurements); every point
    // they observe is variable because no other image's observation enters.
    Reconstruction sub;
    for (const image_t id : config_.Images()) {
      const Image& im = reconstruction->GetImage(id);
      sub.AddCamera(reconstruction->GetCamera(im.camera_id));
      Image copy = im;
      for (Point2D& p2 : copy.points2D) p2.point3D_id = kInvalidPoint3DId;
      sub.AddImage(copy);
    }
    std::unordered_map<point3D_t, point3D_t> sub_id;
    for (const image_t id : config_.Images()) {
      const Image& im = reconstruction->GetImage(id);
      for (point2D_t k = 0; k < (point2D_t)im.points2D.size(); ++k) {
        const point3D_t pid = im.points2D[k].point3D_id;
        if (pid == kInvalidPoint3DId) continue;
        auto it = sub_id.find(pid);
        if (it == sub_id.end()) it = sub_id.emplace(pid, sub.AddPoint3D(reconstruction->GetPoint3D(pid).xyz)).first;
        sub.AddObservation(it->second, TrackElement{id, k});
      }
    }
    BundleAdjustmentConfig cfg;
    for (const image_t id : config_.Images()) cfg.AddImage(id);
    BundleAdjustmentOptions o = ba_options_;
    o.solver_options.max_num_iterations = options_.max_num_iterations;
    o.print_summary = options_.print_summary;
    o.device = options_.gpu_index < 0 ? 0 : options_.gpu_index;
    BundleAdjuster ba(o, cfg);
    if (!ba.Solve(&sub)) return false;
    summary_ = ba.Summary();
    // TearDown (:742-766): poses, focal length + distortion, points
    for (const image_t id : config_.Images()) {
      Image& im = reconstruction->GetImage(id);
      const Image& s = sub.GetImage(id);
      std::copy(s.qvec, s.qvec + 4, im.qvec);
      std::copy(s.tvec, s.tvec + 3, im.tvec);
      reconstruction->GetCamera(im.camera_id).params = sub.GetCamera(im.camera_id).params;
    }
    for (const auto& e : sub_id) {
      const double* x = sub.GetPoint3D(e.second).xyz;
      std::copy(x, x + 3, reconstruction->GetPoint3D(e.first).xyz);
    }
    return true;
  }

  const SolverSummary& Summary() const { return summary_; }

 private:
  Options options_;
  BundleAdjustmentOptions ba_options_;
  BundleAdjustmentConfig config_;
  SolverSummary summary_;
  bool used_ = false;
};

// PrintSolverSummary (bundle_adjustment.cc:1142-1196)
inline void PrintSolverSummary(const SolverSummary& s) {
  const char* term = s.termination_type == SolverSummary::CONVERGENCE      ? "Convergence"
                     : s.termination_type == SolverSummary::NO_CONVERGENCE ? "No convergence"
                     : s.termination_type == SolverSummary::FAILURE        ? "Failure"
                     : s.termination_type == SolverSummary::USER_SUCCESS   ? "User success"
                     : s.termination_type == SolverSummary::USER_FAILURE   ? "User failure"
                                                                           : "Unknown";
  std::printf("    Residuals : %lld\n   Parameters : %lld\n   Iterations : %d\n         Time : %g [s]\n"
              " Initial cost : %g [px]\n   Final cost : %g [px]\n  Termination : %s\n\n",
              (long long)s.num_residuals_reduced, (long long)s.num_effective_parameters_reduced,
              s.num_successful_steps + s.num_unsuccessful_steps, s.total_time_in_seconds,
              std::sqrt(s.initial_cost / s.num_residuals_reduced), std::sqrt(s.final_cost / s.num_residuals_reduced),
              term);
}

}  // namespace colmap_amd

// SemanticBundleAdjuster and its options live in semantic_bundle_adjustment.h
// (the reference's file split); included here so existing callers keep working.
#include "semantic_bundle_adjustment.h"
