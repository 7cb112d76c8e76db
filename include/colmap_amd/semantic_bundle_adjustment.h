// colmap_amd/semantic_bundle_adjustment.h — the semantic BA facade with the
// reference's API (src/optim/semantic_bundle_adjustment.h:53-272 of
// AlainSchoebi/semantic-bundle-adjustment-colmap), on the MI355X library.
// Header-only; link against libmi_ba.so.
//
//   colmap::SemanticBundleAdjustmentOptions  -> colmap_amd::SemanticBundleAdjustmentOptions
//   colmap::SemanticBundleAdjustmentConfig   -> colmap_amd::SemanticBundleAdjustmentConfig
//   colmap::SemanticBundleAdjuster           -> colmap_amd::SemanticBundleAdjuster
//   SemanticBundleAdjuster::ReadDepthAndSemanticMaps -> colmap_amd::LoadSemanticMaps
//
// The reference's construction is SemanticBundleAdjuster(options, config)
// with the maps read inside Solve from options.data_path (SetUp ->
// ReadDepthAndSemanticMaps, semantic_bundle_adjustment.cc:1021-1068); that
// form is kept, next to an overload taking the maps in memory.
#pragma once

#include <algorithm>
#include <cstdio>
#include <exception>
#include <iomanip>
#include <iostream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "bundle_adjustment.h"
#include "tiff.h"

namespace colmap_amd {

// ---------------------------------------------------------------------------
// Semantic BA (semantic_bundle_adjustment.h:53-272)
// ---------------------------------------------------------------------------
struct SemanticBundleAdjustmentOptions : BundleAdjustmentOptions {
  // Data path (semantic_bundle_adjustment.h:58-60): the folder holding
  // depth_tiff/<stem>_depth.tiff and semantic_tiff/<stem>_semantic.tiff of
  // every config image, read by Solve when the adjuster was constructed
  // without maps.
  std::string data_path;
  // Outputs (semantic_bundle_adjustment.h:62-73).  output_path: the refined
  // reconstruction is written there (binary) and to output_path/text after
  // the solve.  visualization_path ("{output_path}/run" resolves to
  // output_path + "/run", as the controller does, controllers/
  // semantic_bundle_adjustment.cc:92-94): every LM iteration k writes the
  // current reconstruction to visualization_path/optim_steps/step_k (binary)
  // and step_k/text (SBACallbackFunctor, semantic_bundle_adjustment.cc:
  // 1086-1123), and with export_csv the semantic error of every grid pixel of
  // every ordered pair of config images to step_k/vis_<image1>_to_<image2>.csv
  // (ExportSemanticErrorToCSV, :908-1019; the rows come from the GPU,
  // mi_ba_semantic_export).  Off by default (output_path empty).  Unlike the
  // reference's createFolders (util/utils.h:101-104), existing folders are
  // never emptied: files of the same names are overwritten, others are kept.
  std::string output_path;
  std::string visualization_path = "{output_path}/run";
  bool export_csv = false;
  double depth_error_threshold = 2;
  int error_computation_pixel_step = 10;
  double numeric_relative_step_size = 1e-3;
  double semantic_weight = 1.0;  // build addition (ScaledLoss weight)
  // Build extension, off by default: the reference accepts SIMPLE_PINHOLE
  // cameras only and throws std::runtime_error for any other model
  // (SemanticBundleAdjuster::Assert, semantic_bundle_adjustment.cc:619-631),
  // as Solve does here unless this is set; with it, PINHOLE, SIMPLE_RADIAL,
  // RADIAL and OPENCV cameras take the same residual through their own
  // ImageToWorld / WorldToImage.
  bool allow_any_camera_model = false;
  SemanticBundleAdjustmentOptions() {
    solver_options.function_tolerance = 1e-8;
    solver_options.gradient_tolerance = 1e-8;
    solver_options.parameter_tolerance = 1e-8;
    // the reference's SBA callbacks read the current point (semantic_bundle_adjustment.h:127-129)
    solver_options.update_state_every_iteration = true;
  }
  std::string ResolvedVisualizationPath() const {
    if (visualization_path == "{output_path}/run") return output_path.empty() ? std::string() : output_path + "/run";
    return visualization_path;
  }
};
typedef BundleAdjustmentConfig SemanticBundleAdjustmentConfig;

// Depth / semantic maps per image name: row-major float32 (the
// matrixFromTiff matrices after their vertical flip, matrix_vis.h:130-176).
// Each image's two maps share one size: sizes[name] = (rows, cols), or, for
// an image without an entry, height x width.  Images may differ in size, as
// in the reference (image 1 sampled on its own grid, the reprojected pixel
// bounds-checked against image 2's own size: semantic_bundle_adjustment.cc:
// 792-799, semantic_cost_functions.h:163).
struct SemanticMaps {
  int height = 0, width = 0;
  std::unordered_map<std::string, std::pair<int, int>> sizes;
  std::unordered_map<std::string, std::vector<float>> depth, semantic;
  std::pair<int, int> Size(const std::string& name) const {
    auto it = sizes.find(name);
    return it == sizes.end() ? std::make_pair(height, width) : it->second;
  }
};

// PrintSemanticSolverSummary (semantic_bundle_adjustment.cc:546-598): the raw
// costs (not RMS pixels as PrintSolverSummary), labels right-aligned in 16
// columns, costs with precision 6.
inline void PrintSemanticSolverSummary(const SolverSummary& s, std::ostream& out = std::cout) {
  const char* term = s.termination_type == SolverSummary::CONVERGENCE      ? "Convergence"
                     : s.termination_type == SolverSummary::NO_CONVERGENCE ? "No convergence"
                     : s.termination_type == SolverSummary::FAILURE        ? "Failure"
                     : s.termination_type == SolverSummary::USER_SUCCESS   ? "User success"
                     : s.termination_type == SolverSummary::USER_FAILURE   ? "User failure"
                                                                           : "Unknown";
  out << std::right << std::setw(16) << "Residuals : " << std::left << s.num_residuals_reduced << std::endl;
  out << std::right << std::setw(16) << "Parameters : " << std::left << s.num_effective_parameters_reduced
      << std::endl;
  out << std::right << std::setw(16) << "Iterations : " << std::left
      << s.num_successful_steps + s.num_unsuccessful_steps << std::endl;
  out << std::right << std::setw(16) << "Time : " << std::left << s.total_time_in_seconds << " [s]" << std::endl;
  out << std::right << std::setw(16) << "Initial cost : " << std::right << std::setprecision(6) << s.initial_cost
      << " " << std::endl;
  out << std::right << std::setw(16) << "Final cost : " << std::right << std::setprecision(6) << s.final_cost << " "
      << std::endl;
  out << std::right << std::setw(16) << "Termination : " << std::right << term << std::endl;
  out << std::endl;
}

// PrintHeading2 (util/misc.cc:197-200)
inline void PrintHeading2(const std::string& heading, std::ostream& out = std::cout) {
  out << std::endl << heading << std::endl;
  out << std::string(std::min<size_t>(heading.size(), 78), '-') << std::endl;
}

// SemanticBundleAdjuster::ReadDepthAndSemanticMaps (semantic_bundle_adjustment.cc:
// 1021-1068): <data_path>/depth_tiff/<stem>_depth.tiff and
// <data_path>/semantic_tiff/<stem>_semantic.tiff of every config image, stem
// = the image name up to its last '.'.  Each image keeps its maps' own size;
// an image's depth and semantic maps must agree (std::invalid_argument).
inline SemanticMaps LoadSemanticMaps(const std::string& data_path, const Reconstruction& reconstruction,
                                     const BundleAdjustmentConfig& config) {
  SemanticMaps maps;
  auto exists = [](const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    return f.good();
  };
  for (const image_t id : config.Images()) {
    const std::string& name = reconstruction.GetImage(id).name;
    const std::string stem = name.substr(0, name.find_last_of('.'));
    const std::string depth_path = data_path + "/depth_tiff/" + stem + "_depth.tiff";
    const std::string semantic_path = data_path + "/semantic_tiff/" + stem + "_semantic.tiff";
    if (!exists(depth_path)) throw std::runtime_error("ERROR: the depth file '" + depth_path + "' does not exist.");
    if (!exists(semantic_path))
      throw std::runtime_error("ERROR: the semantic file '" + semantic_path + "' does not exist.");
    int h0, w0, h1, w1;
    std::vector<float> d = MatrixFromTiff(depth_path, &h0, &w0);
    std::vector<float> l = MatrixFromTiff(semantic_path, &h1, &w1);
    if (h0 != h1 || w0 != w1)
      throw std::invalid_argument("the depth and semantic maps of '" + name + "' differ in size");
    maps.sizes[name] = std::make_pair(h0, w0);
    maps.depth[name] = std::move(d);
    maps.semantic[name] = std::move(l);
  }
  return maps;
}

namespace internal {
// The semantic term of a flattened reconstruction (SemanticBundleAdjuster::
// SetUp, semantic_bundle_adjustment.cc:646-668): every image's maps on their
// own size, planes back to back in flat image order (ABI 4; an image without
// maps, outside the config, gets an empty plane), and every ordered pair of
// config images (:656-661).  `sem` points into the owned vectors.
struct SemanticInputs {
  std::vector<int32_t> img_h, img_w, pairs;
  std::vector<float> depth, label;
  mi_ba_semantic sem{};

  void Build(const Flat& flat, const Reconstruction& rec, const BundleAdjustmentConfig& config,
             const SemanticMaps& maps, const SemanticBundleAdjustmentOptions& options) {
    img_h.assign(flat.img_ids.size(), 0);
    img_w.assign(flat.img_ids.size(), 0);
    for (size_t i = 0; i < flat.img_ids.size(); ++i) {
      const Image& im = rec.GetImage(flat.img_ids[i]);
      auto d = maps.depth.find(im.name), l = maps.semantic.find(im.name);
      if (d == maps.depth.end() || l == maps.semantic.end()) {
        if (config.HasImage(im.image_id)) throw std::runtime_error("missing depth/semantic map for " + im.name);
        continue;
      }
      const std::pair<int, int> hw = maps.Size(im.name);
      if (hw.first <= 0 || hw.second <= 0 || d->second.size() != (size_t)hw.first * hw.second ||
          l->second.size() != d->second.size())
        throw std::invalid_argument("the depth / semantic maps of '" + im.name + "' do not match their size");
      img_h[i] = hw.first;
      img_w[i] = hw.second;
      depth.insert(depth.end(), d->second.begin(), d->second.end());
      label.insert(label.end(), l->second.begin(), l->second.end());
    }
    for (size_t i = 0; i < flat.img_ids.size(); ++i)
      for (size_t j = 0; j < flat.img_ids.size(); ++j)
        if (flat.img_cfg[i] && flat.img_cfg[j]) {
          pairs.push_back((int32_t)i);
          pairs.push_back((int32_t)j);
        }
    static const float kNoMaps = 0.f;  // no image with maps: the library still takes a non-null plane pointer
    sem = mi_ba_semantic{};
    sem.image_height = img_h.data();
    sem.image_width = img_w.data();
    sem.depth = depth.empty() ? &kNoMaps : depth.data();
    sem.label = label.empty() ? &kNoMaps : label.data();
    sem.num_pairs = (int32_t)(pairs.size() / 2);
    sem.pairs = pairs.data();
    sem.pixel_step = options.error_computation_pixel_step;
    sem.depth_error_threshold = options.depth_error_threshold;
    sem.numeric_relative_step_size = options.numeric_relative_step_size;
  }
};
}  // namespace internal

class SemanticBundleAdjuster {
 public:
  // The reference's construction (semantic_bundle_adjustment.h:219-220): the
  // depth / semantic maps are read from options.data_path by Solve.
  SemanticBundleAdjuster(const SemanticBundleAdjustmentOptions& options, const SemanticBundleAdjustmentConfig& config)
      : options_(options), config_(config) {
    options_.Check();
  }
  // Build addition: the maps given in memory (options.data_path unused).
  SemanticBundleAdjuster(const SemanticBundleAdjustmentOptions& options, const SemanticBundleAdjustmentConfig& config,
                         const SemanticMaps& maps)
      : options_(options), config_(config), maps_(maps), have_maps_(true) {
    options_.Check();
  }

  bool Solve(Reconstruction* reconstruction) {
    if (!reconstruction) throw std::invalid_argument("reconstruction is null");
    if (used_) throw std::logic_error("Cannot use the same BundleAdjuster multiple times");
    used_ = true;
    // SemanticBundleAdjuster::Assert (semantic_bundle_adjustment.cc:604-644),
    // in its order and with its messages
    for (const image_t id : config_.Images()) {
      const Image& im = reconstruction->GetImage(id);
      if (!config_.IsConstantCamera(im.camera_id))
        throw std::runtime_error("ERROR: camera intrinsics of image '" + im.name +
                                 "' are not set to constant. This is not supported.");
    }
    if (!options_.allow_any_camera_model)
      for (const image_t id : config_.Images()) {
        const Image& im = reconstruction->GetImage(id);
        if (reconstruction->GetCamera(im.camera_id).model_id != MI_BA_SIMPLE_PINHOLE)
          throw std::runtime_error("ERROR: the only supported camera model is SimplePinholeCameraModel.");
      }
    if (!options_.refine_extrinsics)
      throw std::runtime_error("ERROR: the argument 'refine_extrinsics' must be set to true.");
    // SetUp -> ReadDepthAndSemanticMaps (:1021-1068)
    if (!have_maps_) {
      maps_ = LoadSemanticMaps(options_.data_path, *reconstruction, config_);
      have_maps_ = true;
    }
    internal::Flat flat;
    flat.Build(*reconstruction, config_);
    // The pose-only semantic problem: no reprojection blocks.
    flat.problem.num_obs = 0;
    internal::SemanticInputs in;
    in.Build(flat, *reconstruction, config_, maps_, options_);
    const mi_ba_semantic& sem = in.sem;
    mi_ba_options o = internal::ToOptions(options_);
    o.semantic_weight = options_.semantic_weight;
    o.print_summary = 0;  // the SBA prints its own report (PrintSemanticSolverSummary, below)
    // the per-iteration snapshot writer runs after the caller's callbacks
    // (Solve pushes the SBACallbackFunctor last, semantic_bundle_adjustment.cc:519-520)
    const std::string steps = options_.ResolvedVisualizationPath();
    SolverArena arena;  // the live context, for the CSV rows inside the callback
    SemanticBundleAdjustmentOptions cb_options = options_;
    struct StepWriter : IterationCallback {
      SemanticBundleAdjuster* sba;
      Reconstruction* rec;
      const internal::Flat* flat;
      SolverArena* arena;
      std::string steps;
      // A snapshot that cannot be written is reported and the optimisation
      // goes on, as the reference's writers do ("Unable to open the file",
      // ExportSemanticErrorToCSV :934-937); nothing is thrown into the solver.
      CallbackReturnType operator()(const IterationSummary& it) override {
        std::printf("\nOptimization Iteration %d Update\n%-16s%.6g\n%-16s%.6g\n", it.iteration, "Cost: ", it.cost,
                    "Cost change: ", it.cost_change);
        try {
          sba->WriteStep(*rec, *flat, *arena->get(), steps + "/optim_steps/step_" + std::to_string(it.iteration));
        } catch (const std::exception& e) {
          std::printf("Unable to write the optimization step %d: %s\n", it.iteration, e.what());
        }
        return SOLVER_CONTINUE;
      }
    } writer;
    writer.sba = this;
    writer.rec = reconstruction;
    writer.flat = &flat;
    writer.arena = &arena;
    writer.steps = steps;
    if (!steps.empty()) {
      cb_options.solver_options.callbacks.push_back(&writer);
      cb_options.solver_options.update_state_every_iteration = true;
    }
    internal::CallbackBridge bridge;
    internal::InstallCallbacks(cb_options, &bridge, [&] { flat.WriteBack(reconstruction); }, &o);
    mi_ba_summary s;
    const mi_ba_status st = mi_ba_solve_in(arena.get(), &o, &flat.problem, &sem, &s);
    bridge.Rethrow();
    if (st == MI_BA_ERR_NO_RESIDUALS) return false;
    internal::ThrowStatus(st, "SemanticBundleAdjuster::Solve");
    summary_ = internal::ToSummary(s);
    if (options_.print_summary) {  // :526-529
      PrintHeading2("Semantic Bundle Adjustment Report");
      PrintSemanticSolverSummary(summary_);
    }
    flat.WriteBack(reconstruction);
    if (!options_.output_path.empty()) {  // :531-538
      internal::MakeDirs(options_.output_path + "/text");
      WriteModelBinary(options_.output_path, *reconstruction);
      WriteModelText(options_.output_path + "/text", *reconstruction);
    }
    return true;
  }

  const SolverSummary& Summary() const { return summary_; }

  // One snapshot (SBACallbackFunctor::operator(), semantic_bundle_adjustment.cc:
  // 1090-1123): the reconstruction's current state to dir (binary) and
  // dir/text, and with export_csv every ordered pair of config images'
  // ExportSemanticErrorToCSV file dir/vis_<name1>_to_<name2>.csv.
  void WriteStep(const Reconstruction& rec, const internal::Flat& flat, mi_ba_context* ctx, const std::string& dir) {
    internal::MakeDirs(dir + "/text");
    if (options_.export_csv) {
      std::vector<int32_t> pix, status;
      std::vector<double> err, world;
      for (size_t a = 0; a < flat.img_ids.size(); ++a) {
        if (!flat.img_cfg[a]) continue;
        for (size_t b = 0; b < flat.img_ids.size(); ++b) {
          if (a == b || !flat.img_cfg[b]) continue;
          int64_t n = 0;
          internal::ThrowStatus(mi_ba_semantic_export(ctx, (int32_t)a, (int32_t)b, &n, nullptr, nullptr, nullptr, nullptr),
                                "ExportSemanticErrorToCSV");
          pix.resize(4 * n);
          status.resize(n);
          err.resize(n);
          world.resize(3 * n);
          internal::ThrowStatus(mi_ba_semantic_export(ctx, (int32_t)a, (int32_t)b, &n, pix.data(), status.data(),
                                                      err.data(), world.data()),
                                "ExportSemanticErrorToCSV");
          const std::string path = dir + "/vis_" + rec.GetImage(flat.img_ids[a]).name + "_to_" +
                                   rec.GetImage(flat.img_ids[b]).name + ".csv";
          std::ofstream f(path);
          if (!f.is_open()) {  // :934-937: reported, the other files are still written
            std::printf("Unable to open the file '%s'\n", path.c_str());
            continue;
          }
          // :994-1007: default stream formatting, the error as float
          f << "Type,SemanticError,X1,Y1,X2,Y2,X3D,Y3D,Z3D\n";
          for (int64_t k = 0; k < n; ++k)
            f << status[k] << "," << (float)err[k] << "," << pix[4 * k] << "," << pix[4 * k + 1] << ","
              << pix[4 * k + 2] << "," << pix[4 * k + 3] << "," << world[3 * k] << "," << world[3 * k + 1] << ","
              << world[3 * k + 2] << "\n";
        }
      }
    }
    WriteModelBinary(dir, rec);
    WriteModelText(dir + "/text", rec);
  }

 private:
  SemanticBundleAdjustmentOptions options_;
  SemanticBundleAdjustmentConfig config_;
  SemanticMaps maps_;
  bool have_maps_ = false;
  SolverSummary summary_;
  bool used_ = false;
};

}  // namespace colmap_amd
