// colmap_amd/geometric_semantic_bundle_adjustment.h — C++ facade of the
// reference's GSBA (header-only; links libmi_ba.so).
//
//   colmap::Cylinder (q, t, radius, height; text I/O)      src/util/cylinder.h:153-631
//   colmap::GeometricSemanticBundleAdjustmentOptions        src/optim/geometric_semantic_bundle_adjustment.h:51-150
//   colmap::GeometricSemanticBundleAdjuster<Cylinder>        ...bundle_adjustment.cc:481-1338
//   colmap::GeometricSemanticBundleAdjuster<CylinderBy2Points> (cylinder_parametrization
//     "by_2_points"; src/util/cylinder_by_2_points.h, ...bundle_adjustment.cc:917-1010,1185-1213)
//
// Solve(reconstruction, cylinders): reads <data_path>/depth_tiff and
// semantic_tiff maps of the config images (ReadDepthAndSemanticMaps,
// :1298-1336), builds the trunk masks (semantic == trunk_semantic_class) and
// runs mi_ba_gsba_solve; poses (and cylinders when refine_geometry) are
// written back.  The reference's per-iteration visualisation / CSV exports
// (:1482-1558) are not part of the solve and are not reproduced.
#pragma once

#include <cstdio>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "bundle_adjustment.h"
#include "tiff.h"

namespace colmap_amd {

struct Cylinder {
  double qvec[4] = {1, 0, 0, 0};
  double tvec[3] = {0, 0, 0};
  double radius = 1.0;
  double height = 1.0;

  // Cylinder::to_string / Cylinder(const std::string&) (cylinder.h:216-256):
  // "q w x y z t x y z r R h H"
  std::string ToString() const {
    std::ostringstream o;
    o.precision(17);
    o << "q " << qvec[0] << " " << qvec[1] << " " << qvec[2] << " " << qvec[3] << " t " << tvec[0] << " " << tvec[1]
      << " " << tvec[2] << " r " << radius << " h " << height;
    return o.str();
  }
  static Cylinder FromString(const std::string& line) {
    std::istringstream is(line);
    Cylinder c;
    std::string tag;
    auto expect = [&](const char* t) {
      if (!(is >> tag) || tag != t) throw std::runtime_error("ERROR: creating Cylinder from string failed.");
    };
    expect("q");
    for (double& v : c.qvec) is >> v;
    expect("t");
    for (double& v : c.tvec) is >> v;
    expect("r");
    is >> c.radius;
    expect("h");
    is >> c.height;
    if (!is) throw std::runtime_error("ERROR: creating Cylinder from string failed.");
    if (c.radius <= 0) c.radius = 1e-4;  // Cylinder::Check
    if (c.height <= 0) c.height = 1e-4;
    return c;
  }
};

// pushBackCylindersReadFromText / exportCylindersToText (cylinder.h:606-628)
inline std::vector<Cylinder> ReadCylindersText(const std::string& path) {
  std::ifstream f(path);
  if (!f.is_open()) throw std::runtime_error("cannot open " + path);
  std::vector<Cylinder> out;
  std::string line;
  while (std::getline(f, line))
    if (line.find_first_not_of(" \t\r\n") != std::string::npos) out.push_back(Cylinder::FromString(line));
  return out;
}
inline void WriteCylindersText(const std::string& path, const std::vector<Cylinder>& cylinders) {
  std::ofstream f(path, std::ios::trunc);
  if (!f.is_open()) throw std::runtime_error("cannot open " + path);
  for (const Cylinder& c : cylinders) f << c.ToString() << "\n";
}

enum class CylinderParametrization { DEFAULT, BY2POINTS };

struct GeometricSemanticBundleAdjustmentOptions : BundleAdjustmentOptions {
  std::string data_path;               // folder with depth_tiff/ and semantic_tiff/
  std::string input_geometry;          // cylinder text file (Solve(reconstruction) reads it)
  double trunk_semantic_class = 250.;
  bool refine_geometry = true;
  bool include_landmark_error = false;
  double landmark_error_weight = 1;
  double numeric_relative_step_size = 1e-3;
  // "default" (GeometricSemanticBundleAdjuster<Cylinder>) or "by_2_points"
  // (<CylinderBy2Points>): geometric_semantic_bundle_adjustment.h:49-95
  std::string cylinder_parametrization = "default";

  CylinderParametrization GetCylinderParametrization() const {
    if (cylinder_parametrization == "default") return CylinderParametrization::DEFAULT;
    if (cylinder_parametrization == "by_2_points") return CylinderParametrization::BY2POINTS;
    throw std::runtime_error("ERROR: '" + cylinder_parametrization + "' is not a valid cylinder parametrization.");
  }
};

class GeometricSemanticBundleAdjuster {
 public:
  GeometricSemanticBundleAdjuster(const GeometricSemanticBundleAdjustmentOptions& options,
                                  const BundleAdjustmentConfig& config)
      : options_(options), config_(config) {
    options_.Check();
  }

  // Reads the cylinders from options.input_geometry (SetUp, :800-806).
  bool Solve(Reconstruction* reconstruction) {
    std::vector<Cylinder> cylinders = ReadCylindersText(options_.input_geometry);
    const bool ok = Solve(reconstruction, &cylinders);
    cylinders_ = cylinders;
    return ok;
  }

  bool Solve(Reconstruction* reconstruction, std::vector<Cylinder>* cylinders) {
    if (!reconstruction || !cylinders) throw std::invalid_argument("null argument");
    if (used_) throw std::logic_error("Cannot use the same BundleAdjuster multiple times");
    used_ = true;
    // Assert (:664-712)
    for (const image_t id : config_.Images()) {
      const Image& im = reconstruction->GetImage(id);
      if (!config_.IsConstantCamera(im.camera_id))
        throw std::runtime_error("ERROR: camera intrinsics of image '" + im.name +
                                 "' are not set to constant. This is not supported.");
      if (reconstruction->GetCamera(im.camera_id).model_id != MI_BA_SIMPLE_PINHOLE)
        throw std::runtime_error("ERROR: the only supported camera model is SimplePinholeCameraModel.");
    }
    if (options_.loss_function_type != BundleAdjustmentOptions::LossFunctionType::TRIVIAL)
      throw std::runtime_error("ERROR: the only supported loss function is 'LossFunctionType::TRIVIAL'.");
    internal::Flat flat;
    flat.Build(*reconstruction, config_);
    // trunk masks of the config images (ReadDepthAndSemanticMaps, :1298-1336)
    // each on its own map's size (the IoU is rasterised on that size,
    // :1530-1531), planes back to back (ABI 4)
    const SemanticMaps maps = LoadSemanticMaps(options_.data_path, *reconstruction, config_);
    std::vector<int32_t> mask_h(flat.img_ids.size(), 0), mask_w(flat.img_ids.size(), 0);
    std::vector<uint8_t> masks;
    for (size_t i = 0; i < flat.img_ids.size(); ++i) {
      const Image& im = reconstruction->GetImage(flat.img_ids[i]);
      auto it = maps.semantic.find(im.name);
      if (it == maps.semantic.end()) continue;  // not a config image
      const std::pair<int, int> hw = maps.Size(im.name);
      mask_h[i] = hw.first;
      mask_w[i] = hw.second;
      for (const float v : it->second) masks.push_back((double)v == options_.trunk_semantic_class ? 1 : 0);
    }
    if (masks.empty()) masks.push_back(0);  // a non-null plane pointer
    std::vector<mi_ba_cylinder> cyl(cylinders->size());
    for (size_t c = 0; c < cyl.size(); ++c) {
      const Cylinder& y = (*cylinders)[c];
      std::copy(y.qvec, y.qvec + 4, cyl[c].qvec);
      std::copy(y.tvec, y.tvec + 3, cyl[c].tvec);
      cyl[c].radius = y.radius;
      cyl[c].height = y.height;
    }
    mi_ba_gsba g;
    mi_ba_default_gsba(&g);
    g.image_height = mask_h.data();
    g.image_width = mask_w.data();
    g.trunk_mask = masks.data();
    g.num_cylinders = (int32_t)cyl.size();
    g.cylinders = cyl.data();
    g.refine_geometry = options_.refine_geometry;
    g.numeric_relative_step_size = options_.numeric_relative_step_size;
    g.include_landmark_error = options_.include_landmark_error;
    g.landmark_error_weight = options_.landmark_error_weight;
    g.cylinder_parametrization = options_.GetCylinderParametrization() == CylinderParametrization::BY2POINTS
                                     ? MI_BA_CYLINDER_BY_2_POINTS
                                     : MI_BA_CYLINDER_DEFAULT;
    mi_ba_options o = internal::ToOptions(options_);
    internal::CallbackBridge bridge;
    internal::InstallCallbacks(options_, &bridge, [&] {
      flat.WriteBack(reconstruction);
      CopyCylinders(cyl, cylinders);
    }, &o);
    mi_ba_summary s;
    const mi_ba_status st = mi_ba_gsba_solve(&o, &flat.problem, &g, &s);
    bridge.Rethrow();
    if (st == MI_BA_ERR_NO_RESIDUALS) return false;
    internal::ThrowStatus(st, "GeometricSemanticBundleAdjuster::Solve");
    summary_ = internal::ToSummary(s);
    flat.WriteBack(reconstruction);
    CopyCylinders(cyl, cylinders);
    return true;
  }

  const SolverSummary& Summary() const { return summary_; }
  const std::vector<Cylinder>& Cylinders() const { return cylinders_; }

 private:
  static void CopyCylinders(const std::vector<mi_ba_cylinder>& cyl, std::vector<Cylinder>* cylinders) {
    for (size_t c = 0; c < cyl.size(); ++c) {
      Cylinder& y = (*cylinders)[c];
      std::copy(cyl[c].qvec, cyl[c].qvec + 4, y.qvec);
      std::copy(cyl[c].tvec, cyl[c].tvec + 3, y.tvec);
      y.radius = cyl[c].radius;
      y.height = cyl[c].height;
    }
  }

  GeometricSemanticBundleAdjustmentOptions options_;
  BundleAdjustmentConfig config_;
  SolverSummary summary_;
  std::vector<Cylinder> cylinders_;
  bool used_ = false;
};

}  // namespace colmap_amd
