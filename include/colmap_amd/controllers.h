// colmap_amd/controllers.h — the reference's bundle-adjustment controllers
// (the L3 callers of the boundary) as thin drivers over the facades.
//
//   colmap::BundleAdjustmentController                 src/controllers/bundle_adjustment.cc:65-103
//   colmap::SemanticBundleAdjustmentController         src/controllers/semantic_bundle_adjustment.cc:65-122
//   colmap::GeometricSemanticBundleAdjustmentController src/controllers/geometric_semantic_bundle_adjustment.cc:68-150
//
// Each Run() does what the reference's does: at least two registered images
// (else "ERROR: Need at least two views." and return),
// Reconstruction::FilterObservationsWithNegativeDepth, the gauge (first
// registered pose constant, x of the second registered tvec constant; SBA /
// GSBA: every registered image's camera constant), an iteration callback
// that blocks while the controller is paused and ends the solve with
// SOLVER_TERMINATE_SUCCESSFULLY once it is stopped
// (BundleAdjustmentIterationCallback, controllers/bundle_adjustment.cc:
// 43-61), then Solve.  The reference's controllers are util::Thread
// subclasses; here Run() is synchronous and Stop / Pause / Resume may be
// called from any other thread while it runs (the util::Thread subset the
// callbacks use: threading.h:99-145).  Registered images are taken in
// registration order (Reconstruction::RegImageIds: file order for a model
// read from disk, as reconstruction_->RegImageIds() in the reference), so the
// gauge fixes the same first pose and second tvec as the reference's.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <string>
#include <vector>

#include "bundle_adjustment.h"
#include "geometric_semantic_bundle_adjustment.h"
#include "tiff.h"

namespace colmap_amd {

// Thread::Stop / Pause / Resume / BlockIfPaused / IsStopped.
class ControllerThread {
 public:
  void Stop() {
    stopped_ = true;
    Resume();
  }
  void Pause() {
    std::lock_guard<std::mutex> l(m_);
    paused_ = true;
  }
  void Resume() {
    {
      std::lock_guard<std::mutex> l(m_);
      paused_ = false;
    }
    cv_.notify_all();
  }
  bool IsStopped() const { return stopped_; }
  bool IsPaused() const {
    std::lock_guard<std::mutex> l(m_);
    return paused_;
  }
  void BlockIfPaused() {
    std::unique_lock<std::mutex> l(m_);
    cv_.wait(l, [&] { return !paused_; });
  }

 protected:
  mutable std::mutex m_;
  std::condition_variable cv_;
  bool paused_ = false;
  std::atomic<bool> stopped_{false};
};

namespace internal {
// BundleAdjustmentIterationCallback (controllers/bundle_adjustment.cc:43-61)
class ControllerIterationCallback : public IterationCallback {
 public:
  explicit ControllerIterationCallback(ControllerThread* thread) : thread_(thread) {}
  CallbackReturnType operator()(const IterationSummary&) override {
    thread_->BlockIfPaused();
    return thread_->IsStopped() ? SOLVER_TERMINATE_SUCCESSFULLY : SOLVER_CONTINUE;
  }

 private:
  ControllerThread* thread_;
};

inline std::vector<image_t> RegImageIds(const Reconstruction& r) { return r.RegImageIds(); }
}  // namespace internal

class BundleAdjustmentController : public ControllerThread {
 public:
  BundleAdjustmentController(const BundleAdjustmentOptions& options, Reconstruction* reconstruction)
      : options_(options), reconstruction_(reconstruction) {}

  // controllers/bundle_adjustment.cc:69-103
  void Run() {
    if (!reconstruction_) throw std::invalid_argument("reconstruction is null");
    const std::vector<image_t> reg = internal::RegImageIds(*reconstruction_);
    if (reg.size() < 2) {
      std::printf("ERROR: Need at least two views.\n");
      return;
    }
    num_filtered_ = reconstruction_->FilterObservationsWithNegativeDepth(options_.device);
    BundleAdjustmentOptions ba_options = options_;
    internal::ControllerIterationCallback callback(this);
    ba_options.solver_options.callbacks.push_back(&callback);
    BundleAdjustmentConfig config;
    for (const image_t id : reg) config.AddImage(id);
    config.SetConstantPose(reg[0]);
    config.SetConstantTvec(reg[1], {0});
    BundleAdjuster adjuster(ba_options, config);
    solved_ = adjuster.Solve(reconstruction_);
    summary_ = adjuster.Summary();
  }

  bool Solved() const { return solved_; }
  size_t NumFilteredObservations() const { return num_filtered_; }
  const SolverSummary& Summary() const { return summary_; }

 private:
  BundleAdjustmentOptions options_;
  Reconstruction* reconstruction_;
  SolverSummary summary_;
  size_t num_filtered_ = 0;
  bool solved_ = false;
};

class SemanticBundleAdjustmentController : public ControllerThread {
 public:
  // data_path (nonempty): the folder with depth_tiff/ and semantic_tiff/,
  // overriding options.data_path (SemanticBundleAdjustmentOptions::data_path)
  SemanticBundleAdjustmentController(const SemanticBundleAdjustmentOptions& options, const std::string& data_path,
                                     Reconstruction* reconstruction)
      : options_(options), data_path_(data_path), reconstruction_(reconstruction) {}

  // controllers/semantic_bundle_adjustment.cc:73-122
  void Run() {
    if (!reconstruction_) throw std::invalid_argument("reconstruction is null");
    const std::vector<image_t> reg = internal::RegImageIds(*reconstruction_);
    if (reg.size() < 2) {
      std::printf("ERROR: Need at least two views.\n");
      return;
    }
    num_filtered_ = reconstruction_->FilterObservationsWithNegativeDepth(options_.device);
    SemanticBundleAdjustmentOptions ba_options = options_;
    internal::ControllerIterationCallback callback(this);
    ba_options.solver_options.callbacks.push_back(&callback);
    SemanticBundleAdjustmentConfig config;
    for (const image_t id : reg) config.AddImage(id);
    config.SetConstantPose(reg[0]);
    config.SetConstantTvec(reg[1], {0});
    for (const image_t id : reg) config.SetConstantCamera(reconstruction_->GetImage(id).camera_id);
    if (!data_path_.empty()) ba_options.data_path = data_path_;
    SemanticBundleAdjuster adjuster(ba_options, config);  // the maps from ba_options.data_path
    solved_ = adjuster.Solve(reconstruction_);
    summary_ = adjuster.Summary();
  }

  bool Solved() const { return solved_; }
  size_t NumFilteredObservations() const { return num_filtered_; }
  const SolverSummary& Summary() const { return summary_; }

 private:
  SemanticBundleAdjustmentOptions options_;
  std::string data_path_;
  Reconstruction* reconstruction_;
  SolverSummary summary_;
  size_t num_filtered_ = 0;
  bool solved_ = false;
};

class GeometricSemanticBundleAdjustmentController : public ControllerThread {
 public:
  GeometricSemanticBundleAdjustmentController(const GeometricSemanticBundleAdjustmentOptions& options,
                                              Reconstruction* reconstruction)
      : options_(options), reconstruction_(reconstruction) {}

  // controllers/geometric_semantic_bundle_adjustment.cc:76-150; the
  // cylinders are read from options.input_geometry (Cylinders() afterwards)
  void Run() {
    if (!reconstruction_) throw std::invalid_argument("reconstruction is null");
    const std::vector<image_t> reg = internal::RegImageIds(*reconstruction_);
    if (reg.size() < 2) {
      std::printf("ERROR: Need at least two views.\n");
      return;
    }
    num_filtered_ = reconstruction_->FilterObservationsWithNegativeDepth(options_.device);
    GeometricSemanticBundleAdjustmentOptions ba_options = options_;
    internal::ControllerIterationCallback callback(this);
    ba_options.solver_options.callbacks.push_back(&callback);
    BundleAdjustmentConfig config;
    for (const image_t id : reg) config.AddImage(id);
    config.SetConstantPose(reg[0]);
    config.SetConstantTvec(reg[1], {0});
    for (const image_t id : reg) config.SetConstantCamera(reconstruction_->GetImage(id).camera_id);
    GeometricSemanticBundleAdjuster adjuster(ba_options, config);
    solved_ = adjuster.Solve(reconstruction_);
    summary_ = adjuster.Summary();
    cylinders_ = adjuster.Cylinders();
  }

  bool Solved() const { return solved_; }
  size_t NumFilteredObservations() const { return num_filtered_; }
  const SolverSummary& Summary() const { return summary_; }
  const std::vector<Cylinder>& Cylinders() const { return cylinders_; }

 private:
  GeometricSemanticBundleAdjustmentOptions options_;
  Reconstruction* reconstruction_;
  SolverSummary summary_;
  std::vector<Cylinder> cylinders_;
  size_t num_filtered_ = 0;
  bool solved_ = false;
};

}  // namespace colmap_amd
