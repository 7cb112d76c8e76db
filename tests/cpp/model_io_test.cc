// model_io_test.cc — drives include/colmap_amd/model_io.h and tiff.h for
// tests/test_model_io.py (host only).
//
//   model_io_test dump <model dir>                 canonical JSON of the model
//   model_io_test write <model dir> <bin> <txt>    read, write both formats
//   model_io_test tiff <file> <out.f32>            H W on stdout, raster bytes to out
//   model_io_test maps <data dir> <model dir>      LoadSemanticMaps over every image
//   model_io_test ba <model dir> <out dir> [iters]  the bundle_adjuster workflow
//       (exe/sfm.cc RunBundleAdjuster + BundleAdjustmentController::Run,
//       controllers/bundle_adjustment.cc:69-101): read, every registered image
//       in the config, pose of the first constant, tvec x of the second
//       constant, Solve on the GPU, write binary
//   model_io_test gsba <model dir> <data dir> <cylinders in> <cylinders out> [iters] [parametrization]
//       GeometricSemanticBundleAdjuster: every registered image, first pose
//       constant, cameras constant, maps from <data dir>, cylinders file I/O
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>

#include "colmap_amd/geometric_semantic_bundle_adjustment.h"
#include "colmap_amd/model_io.h"
#include "colmap_amd/tiff.h"

using namespace colmap_amd;

static void Num(double v) { std::printf("%.17g", v); }

static void Dump(const Reconstruction& r) {
  std::printf("{\"cameras\": {");
  bool first = true;
  for (const auto& e : r.cameras) {
    std::printf("%s\"%u\": [%d, %llu, %llu, [", first ? "" : ", ", e.first, e.second.model_id,
                (unsigned long long)e.second.width, (unsigned long long)e.second.height);
    for (size_t k = 0; k < e.second.params.size(); ++k) {
      if (k) std::printf(", ");
      Num(e.second.params[k]);
    }
    std::printf("]]");
    first = false;
  }
  std::printf("}, \"images\": {");
  first = true;
  for (const auto& e : r.images) {
    const Image& im = e.second;
    std::printf("%s\"%u\": [[", first ? "" : ", ", e.first);
    for (int k = 0; k < 4; ++k) { if (k) std::printf(", "); Num(im.qvec[k]); }
    std::printf("], [");
    for (int k = 0; k < 3; ++k) { if (k) std::printf(", "); Num(im.tvec[k]); }
    std::printf("], %u, \"%s\", [", im.camera_id, im.name.c_str());
    for (size_t k = 0; k < im.points2D.size(); ++k) {
      const Point2D& p = im.points2D[k];
      std::printf("%s[", k ? ", " : "");
      Num(p.xy[0]);
      std::printf(", ");
      Num(p.xy[1]);
      std::printf(", %lld]", p.HasPoint3D() ? (long long)p.point3D_id : -1LL);
    }
    std::printf("]]");
    first = false;
  }
  std::printf("}, \"points3D\": {");
  first = true;
  for (const auto& e : r.points3D) {
    const Point3D& p = e.second;
    std::printf("%s\"%llu\": [[", first ? "" : ", ", (unsigned long long)e.first);
    for (int k = 0; k < 3; ++k) { if (k) std::printf(", "); Num(p.xyz[k]); }
    std::printf("], [%d, %d, %d], ", p.color[0], p.color[1], p.color[2]);
    Num(p.error);
    std::printf(", [");
    for (size_t k = 0; k < p.track.size(); ++k)
      std::printf("%s[%u, %u]", k ? ", " : "", p.track[k].image_id, p.track[k].point2D_idx);
    std::printf("]]");
    first = false;
  }
  std::printf("}}\n");
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const std::string mode = argv[1];
  try {
    if (mode == "dump") {
      Reconstruction r;
      ReadModel(argv[2], &r);
      Dump(r);
    } else if (mode == "write" && argc == 5) {
      Reconstruction r;
      ReadModel(argv[2], &r);
      WriteModelBinary(argv[3], r);
      WriteModelText(argv[4], r);
    } else if (mode == "tiff" && argc == 4) {
      int h, w;
      const std::vector<float> m = MatrixFromTiff(argv[2], &h, &w);
      std::printf("%d %d\n", h, w);
      std::ofstream f(argv[3], std::ios::binary);
      f.write(reinterpret_cast<const char*>(m.data()), (std::streamsize)(m.size() * sizeof(float)));
    } else if (mode == "maps" && argc == 4) {
      Reconstruction r;
      ReadModel(argv[3], &r);
      BundleAdjustmentConfig cfg;
      for (const auto& e : r.images) cfg.AddImage(e.first);
      const SemanticMaps maps = LoadSemanticMaps(argv[2], r, cfg);
      // the maps' size when every image shares it, else -1 -1 (each image keeps its own)
      int h = -2, w = -2;
      for (const auto& e : maps.sizes) {
        if (h == -2) {
          h = e.second.first;
          w = e.second.second;
        } else if (h != e.second.first || w != e.second.second) {
          h = w = -1;
        }
      }
      std::printf("%d %d %zu %zu\n", h, w, maps.depth.size(), maps.semantic.size());
    } else if (mode == "ba" && argc >= 4) {
      Reconstruction r;
      ReadModel(argv[2], &r);
      std::vector<image_t> reg;
      for (const auto& e : r.images)
        if (e.second.IsRegistered()) reg.push_back(e.first);
      if (reg.size() < 2) {
        std::printf("ERROR: Need at least two views.\n");
        return 3;
      }
      BundleAdjustmentConfig cfg;
      for (image_t id : reg) cfg.AddImage(id);
      cfg.SetConstantPose(reg[0]);
      cfg.SetConstantTvec(reg[1], {0});
      BundleAdjustmentOptions o;
      o.print_summary = false;
      if (argc >= 5) o.solver_options.max_num_iterations = std::atoi(argv[4]);
      BundleAdjuster ba(o, cfg);
      if (!ba.Solve(&r)) return 4;
      WriteModelBinary(argv[3], r);
      std::printf("%.17g %.17g %d %d\n", ba.Summary().initial_cost, ba.Summary().final_cost,
                  ba.Summary().num_successful_steps, ba.Summary().num_unsuccessful_steps);
    } else if (mode == "gsba" && argc >= 6) {
      Reconstruction r;
      ReadModel(argv[2], &r);
      BundleAdjustmentConfig cfg;
      bool first = true;
      for (const auto& e : r.images) {
        cfg.AddImage(e.first);
        if (first) cfg.SetConstantPose(e.first);
        first = false;
      }
      for (const auto& c : r.cameras) cfg.SetConstantCamera(c.first);
      GeometricSemanticBundleAdjustmentOptions o;
      o.print_summary = false;
      o.data_path = argv[3];
      o.input_geometry = argv[4];
      if (argc >= 7) o.solver_options.max_num_iterations = std::atoi(argv[6]);
      if (argc >= 8) o.cylinder_parametrization = argv[7];
      GeometricSemanticBundleAdjuster gsba(o, cfg);
      if (!gsba.Solve(&r)) return 4;
      WriteCylindersText(argv[5], gsba.Cylinders());
      std::printf("%.17g %.17g %d %d\n", gsba.Summary().initial_cost, gsba.Summary().final_cost,
                  gsba.Summary().num_successful_steps, gsba.Summary().num_unsuccessful_steps);
    } else {
      return 2;
    }
  } catch (const std::exception& e) {
    std::printf("EXCEPTION %s\n", e.what());
    return 3;
  }
  return 0;
}
