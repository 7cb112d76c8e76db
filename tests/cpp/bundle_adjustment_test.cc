// bundle_adjustment_test.cc — the reference's BundleAdjuster tests
// (src/optim/bundle_adjustment_test.cc:111-642), rerun through the
// colmap_amd facade (include/colmap_amd/bundle_adjustment.h) on libmi_ba.so.
//
//   ./bundle_adjustment_test counts   structural counts only (host, no GPU)
//   ./bundle_adjustment_test solve    full Solve on the MI355X + the
//                                     CheckVariable*/CheckConstant* assertions
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "colmap_amd/bundle_adjustment.h"

using namespace colmap_amd;

static int g_failures = 0;
#define CHECK_T(cond)                                                        \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::printf("  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);        \
      ++g_failures;                                                          \
    }                                                                        \
  } while (0)

static std::mt19937* g_prng = nullptr;
static double RandomReal(double a, double b) { return std::uniform_real_distribution<double>(a, b)(*g_prng); }

// GenerateReconstruction (bundle_adjustment_test.cc:123-184), SIMPLE_RADIAL,
// f = 1.2 * 1000, identity rotations, tvec = (U, U, 10), U(-2, 2) noise.
static Reconstruction GenerateReconstruction(int num_images, int num_points) {
  std::mt19937 prng(0);
  g_prng = &prng;
  Reconstruction rec;
  std::vector<point3D_t> ids;
  for (int i = 0; i < num_points; ++i) {
    double xyz[3];
    xyz[0] = RandomReal(-1, 1);
    xyz[1] = RandomReal(-1, 1);
    xyz[2] = RandomReal(-1, 1);
    ids.push_back(rec.AddPoint3D(xyz));
  }
  for (int i = 0; i < num_images; ++i) {
    Camera cam;
    cam.camera_id = (camera_t)i;
    cam.model_id = MI_BA_SIMPLE_RADIAL;
    cam.params = {1.2 * 1000, 500, 500, 0};
    rec.AddCamera(cam);
    Image im;
    im.image_id = (image_t)i;
    im.camera_id = (camera_t)i;
    im.name = std::to_string(i);
    im.tvec[0] = RandomReal(-1.0, 1.0);
    im.tvec[1] = RandomReal(-1.0, 1.0);
    im.tvec[2] = 10;
    for (point3D_t id : ids) {
      const double* X = rec.GetPoint3D(id).xyz;
      const double px = X[0] + im.tvec[0], py = X[1] + im.tvec[1], pz = X[2] + im.tvec[2];
      const double u = px / pz, v = py / pz;  // SIMPLE_RADIAL with k = 0
      Point2D p2;
      p2.xy[0] = 1200 * u + 500 + RandomReal(-2.0, 2.0);
      p2.xy[1] = 1200 * v + 500 + RandomReal(-2.0, 2.0);
      im.points2D.push_back(p2);
    }
    rec.AddImage(im);
  }
  for (int i = 0; i < num_images; ++i) {
    point2D_t idx = 0;
    for (point3D_t id : ids) rec.AddObservation(id, TrackElement{(image_t)i, idx++});
  }
  return rec;
}

static bool Same(const double* a, const double* b, int n) { return std::memcmp(a, b, sizeof(double) * n) == 0; }
static void CheckVariableCamera(Reconstruction& r, const Reconstruction& o, camera_t c) {
  const auto& a = r.GetCamera(c).params;
  const auto& b = o.cameras.at(c).params;
  CHECK_T(a[0] != b[0]);  // focal
  CHECK_T(a[3] != b[3]);  // radial
}
static void CheckConstantCamera(Reconstruction& r, const Reconstruction& o, camera_t c) {
  CHECK_T(r.GetCamera(c).params == o.cameras.at(c).params);
}
static void CheckConstantImage(Reconstruction& r, const Reconstruction& o, image_t i) {
  CHECK_T(Same(r.GetImage(i).qvec, o.GetImage(i).qvec, 4));
  CHECK_T(Same(r.GetImage(i).tvec, o.GetImage(i).tvec, 3));
}
static void CheckVariableImage(Reconstruction& r, const Reconstruction& o, image_t i) {
  CHECK_T(!Same(r.GetImage(i).qvec, o.GetImage(i).qvec, 4));
  CHECK_T(!Same(r.GetImage(i).tvec, o.GetImage(i).tvec, 3));
}
static void CheckConstantXImage(Reconstruction& r, const Reconstruction& o, image_t i) {
  CHECK_T(!Same(r.GetImage(i).qvec, o.GetImage(i).qvec, 4));
  CHECK_T(r.GetImage(i).tvec[0] == o.GetImage(i).tvec[0]);
}
static void CheckVariablePoint(Reconstruction& r, const Reconstruction& o, point3D_t p) {
  CHECK_T(!Same(r.GetPoint3D(p).xyz, o.GetPoint3D(p).xyz, 3));
}
static void CheckConstantPoint(Reconstruction& r, const Reconstruction& o, point3D_t p) {
  CHECK_T(Same(r.GetPoint3D(p).xyz, o.GetPoint3D(p).xyz, 3));
}

struct Case {
  std::string name;
  std::function<void(bool solve)> run;
};

// Runs counts (always) and, in solve mode, Solve + checks.
static void Expect(bool solve, BundleAdjuster& ba, Reconstruction& rec, int64_t residuals, int64_t params,
                   const std::function<void(Reconstruction&, const Reconstruction&)>& checks) {
  const mi_ba_setup_info info = ba.SetUpInfo(rec);
  CHECK_T(info.num_residuals_reduced == residuals);
  CHECK_T(info.num_effective_parameters_reduced == params);
  if (!solve) return;
  const Reconstruction orig = rec;
  CHECK_T(ba.Solve(&rec));
  CHECK_T(ba.Summary().num_residuals_reduced == residuals);
  CHECK_T(ba.Summary().num_effective_parameters_reduced == params);
  CHECK_T(ba.Summary().final_cost <= ba.Summary().initial_cost);
  checks(rec, orig);
  bool threw = false;
  try {
    ba.Solve(&rec);
  } catch (const std::logic_error&) {
    threw = true;
  }
  CHECK_T(threw);  // "Cannot use the same BundleAdjuster multiple times"
}

int main(int argc, char** argv) {
  const bool solve = argc > 1 && std::string(argv[1]) == "solve";
  std::vector<Case> cases;

  cases.push_back({"TestConfigNumObservations", [](bool) {
    Reconstruction rec = GenerateReconstruction(4, 100);
    BundleAdjustmentConfig config;
    config.AddImage(0);
    config.AddImage(1);
    CHECK_T(config.NumResiduals(rec) == 400);
    config.AddVariablePoint(1);
    CHECK_T(config.NumResiduals(rec) == 404);
    config.AddConstantPoint(2);
    CHECK_T(config.NumResiduals(rec) == 408);
    config.AddImage(2);
    CHECK_T(config.NumResiduals(rec) == 604);
    config.AddImage(3);
    CHECK_T(config.NumResiduals(rec) == 800);
  }});

  cases.push_back({"TestTwoView", [](bool s) {
    Reconstruction rec = GenerateReconstruction(2, 100);
    BundleAdjustmentConfig config;
    config.AddImage(0);
    config.AddImage(1);
    config.SetConstantPose(0);
    config.SetConstantTvec(1, {0});
    BundleAdjustmentOptions options;
    options.print_summary = false;
    BundleAdjuster ba(options, config);
    Expect(s, ba, rec, 400, 309, [](Reconstruction& r, const Reconstruction& o) {
      CheckVariableCamera(r, o, 0);
      CheckConstantImage(r, o, 0);
      CheckVariableCamera(r, o, 1);
      CheckConstantXImage(r, o, 1);
      for (auto& p : r.points3D) CheckVariablePoint(r, o, p.first);
    });
  }});

  cases.push_back({"TestTwoViewConstantCamera", [](bool s) {
    Reconstruction rec = GenerateReconstruction(2, 100);
    BundleAdjustmentConfig config;
    config.AddImage(0);
    config.AddImage(1);
    config.SetConstantPose(0);
    config.SetConstantPose(1);
    config.SetConstantCamera(0);
    BundleAdjustmentOptions options;
    options.print_summary = false;
    BundleAdjuster ba(options, config);
    Expect(s, ba, rec, 400, 302, [](Reconstruction& r, const Reconstruction& o) {
      CheckConstantCamera(r, o, 0);
      CheckConstantImage(r, o, 0);
      CheckVariableCamera(r, o, 1);
      CheckConstantImage(r, o, 1);
      for (auto& p : r.points3D) CheckVariablePoint(r, o, p.first);
    });
  }});

  cases.push_back({"TestPartiallyContainedTracks", [](bool s) {
    Reconstruction rec = GenerateReconstruction(3, 100);
    const point3D_t variable_id = rec.GetImage(2).points2D[0].point3D_id;
    rec.DeleteObservation(2, 0);
    BundleAdjustmentConfig config;
    config.AddImage(0);
    config.AddImage(1);
    config.SetConstantPose(0);
    config.SetConstantPose(1);
    BundleAdjustmentOptions options;
    options.print_summary = false;
    BundleAdjuster ba(options, config);
    Expect(s, ba, rec, 400, 7, [variable_id](Reconstruction& r, const Reconstruction& o) {
      CheckVariableCamera(r, o, 0);
      CheckConstantImage(r, o, 0);
      CheckVariableCamera(r, o, 1);
      CheckConstantImage(r, o, 1);
      CheckConstantCamera(r, o, 2);
      CheckConstantImage(r, o, 2);
      for (auto& p : r.points3D) {
        if (p.first == variable_id) CheckVariablePoint(r, o, p.first);
        else CheckConstantPoint(r, o, p.first);
      }
    });
  }});

  cases.push_back({"TestPartiallyContainedTracksForceToOptimizePoint", [](bool s) {
    Reconstruction rec = GenerateReconstruction(3, 100);
    const point3D_t variable_id = rec.GetImage(2).points2D[0].point3D_id;
    const point3D_t add_variable_id = rec.GetImage(2).points2D[1].point3D_id;
    const point3D_t add_constant_id = rec.GetImage(2).points2D[2].point3D_id;
    rec.DeleteObservation(2, 0);
    BundleAdjustmentConfig config;
    config.AddImage(0);
    config.AddImage(1);
    config.SetConstantPose(0);
    config.SetConstantPose(1);
    config.AddVariablePoint(add_variable_id);
    config.AddConstantPoint(add_constant_id);
    BundleAdjustmentOptions options;
    options.print_summary = false;
    BundleAdjuster ba(options, config);
    Expect(s, ba, rec, 402, 10, [=](Reconstruction& r, const Reconstruction& o) {
      CheckVariableCamera(r, o, 0);
      CheckConstantImage(r, o, 0);
      CheckVariableCamera(r, o, 1);
      CheckConstantImage(r, o, 1);
      CheckConstantCamera(r, o, 2);
      CheckConstantImage(r, o, 2);
      for (auto& p : r.points3D) {
        if (p.first == variable_id || p.first == add_variable_id) CheckVariablePoint(r, o, p.first);
        else CheckConstantPoint(r, o, p.first);
      }
    });
  }});

  cases.push_back({"TestConstantPoints", [](bool s) {
    Reconstruction rec = GenerateReconstruction(2, 100);
    BundleAdjustmentConfig config;
    config.AddImage(0);
    config.AddImage(1);
    config.SetConstantPose(0);
    config.SetConstantPose(1);
    config.AddConstantPoint(1);
    config.AddConstantPoint(2);
    BundleAdjustmentOptions options;
    options.print_summary = false;
    BundleAdjuster ba(options, config);
    Expect(s, ba, rec, 400, 298, [](Reconstruction& r, const Reconstruction& o) {
      CheckVariableCamera(r, o, 0);
      CheckConstantImage(r, o, 0);
      CheckVariableCamera(r, o, 1);
      CheckConstantImage(r, o, 1);
      for (auto& p : r.points3D) {
        if (p.first == 1 || p.first == 2) CheckConstantPoint(r, o, p.first);
        else CheckVariablePoint(r, o, p.first);
      }
    });
  }});

  cases.push_back({"TestVariableImage", [](bool s) {
    Reconstruction rec = GenerateReconstruction(3, 100);
    BundleAdjustmentConfig config;
    config.AddImage(0);
    config.AddImage(1);
    config.AddImage(2);
    config.SetConstantPose(0);
    config.SetConstantTvec(1, {0});
    BundleAdjustmentOptions options;
    options.print_summary = false;
    BundleAdjuster ba(options, config);
    Expect(s, ba, rec, 600, 317, [](Reconstruction& r, const Reconstruction& o) {
      CheckVariableCamera(r, o, 0);
      CheckConstantImage(r, o, 0);
      CheckVariableCamera(r, o, 1);
      CheckConstantXImage(r, o, 1);
      CheckVariableCamera(r, o, 2);
      CheckVariableImage(r, o, 2);
      for (auto& p : r.points3D) CheckVariablePoint(r, o, p.first);
    });
  }});

  auto focal_case = [](const char* flag, int64_t params) {
    return [flag, params](bool s) {
      Reconstruction rec = GenerateReconstruction(2, 100);
      BundleAdjustmentConfig config;
      config.AddImage(0);
      config.AddImage(1);
      config.SetConstantPose(0);
      config.SetConstantTvec(1, {0});
      BundleAdjustmentOptions options;
      options.print_summary = false;
      const std::string f(flag);
      if (f == "focal") options.refine_focal_length = false;
      if (f == "pp") options.refine_principal_point = true;
      if (f == "extra") options.refine_extra_params = false;
      BundleAdjuster ba(options, config);
      Expect(s, ba, rec, 400, params, [f](Reconstruction& r, const Reconstruction& o) {
        CheckConstantImage(r, o, 0);
        CheckConstantXImage(r, o, 1);
        for (camera_t c = 0; c < 2; ++c) {
          const auto& a = r.GetCamera(c).params;
          const auto& b = o.cameras.at(c).params;
          if (f == "focal") { CHECK_T(a[0] == b[0]); CHECK_T(a[3] != b[3]); }
          if (f == "pp") { CHECK_T(a[0] != b[0]); CHECK_T(a[1] != b[1]); CHECK_T(a[2] != b[2]); CHECK_T(a[3] != b[3]); }
          if (f == "extra") { CHECK_T(a[0] != b[0]); CHECK_T(a[3] == b[3]); }
        }
        for (auto& p : r.points3D) CheckVariablePoint(r, o, p.first);
      });
    };
  };
  cases.push_back({"TestConstantFocalLength", focal_case("focal", 307)});
  cases.push_back({"TestVariablePrincipalPoint", focal_case("pp", 313)});
  cases.push_back({"TestConstantExtraParam", focal_case("extra", 307)});

  // Build addition: cameras of different models in one problem (the
  // reference dispatches the model per camera, camera_models.h:117-141,
  // bundle_adjustment.cc:396-406).  Counts: SIMPLE_RADIAL f,k + PINHOLE
  // fx,fy + OPENCV fx,fy,k1,k2,p1,p2 = 10; poses 0 + 5 + 6; points 300.
  cases.push_back({"TestMixedCameraModels", [](bool s) {
    Reconstruction rec = GenerateReconstruction(3, 100);
    rec.GetCamera(1).model_id = MI_BA_PINHOLE;
    rec.GetCamera(1).params = {1200, 1200, 500, 500};
    rec.GetCamera(2).model_id = MI_BA_OPENCV;
    rec.GetCamera(2).params = {1200, 1200, 500, 500, 0, 0, 0, 0};
    BundleAdjustmentConfig config;
    config.AddImage(0);
    config.AddImage(1);
    config.AddImage(2);
    config.SetConstantPose(0);
    config.SetConstantTvec(1, {0});
    BundleAdjustmentOptions options;
    options.print_summary = false;
    BundleAdjuster ba(options, config);
    Expect(s, ba, rec, 600, 321, [](Reconstruction& r, const Reconstruction& o) {
      CheckVariableCamera(r, o, 0);
      const auto& p1 = r.GetCamera(1).params;
      const auto& q1 = o.cameras.at(1).params;
      CHECK_T(p1[0] != q1[0] && p1[1] != q1[1] && p1[2] == q1[2] && p1[3] == q1[3]);
      const auto& p2 = r.GetCamera(2).params;
      const auto& q2 = o.cameras.at(2).params;
      CHECK_T(p2[0] != q2[0] && p2[1] != q2[1] && p2[2] == q2[2] && p2[3] == q2[3]);
      for (int k = 4; k < 8; ++k) CHECK_T(p2[k] != q2[k]);
      CheckConstantImage(r, o, 0);
      CheckConstantXImage(r, o, 1);
      CheckVariableImage(r, o, 2);
      for (auto& p : r.points3D) CheckVariablePoint(r, o, p.first);
    });
  }});

  // SemanticBundleAdjuster through the facade (semantic_bundle_adjustment.h:
  // 217-225): Assert (cc:604-644) on the host, then a pose-only semantic
  // solve over every ordered pair of three images looking at a labelled plane.
  cases.push_back({"TestSemanticBundleAdjuster", [](bool s) {
    Reconstruction rec = GenerateReconstruction(3, 10);
    const int H = 60, W = 60;
    SemanticMaps maps;
    maps.height = H;
    maps.width = W;
    for (auto& e : rec.images) {
      Image& im = e.second;
      std::vector<float> depth((size_t)H * W), label((size_t)H * W);
      // the plane z = 0 at camera depth tvec[2] = 10; labels: 0.5-wide checkerboard
      for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
          const double d = im.tvec[2];
          const double X = (x - 500.0 + 470.0) / 1200.0 * d - im.tvec[0];
          const double Y = (y - 500.0 + 470.0) / 1200.0 * d - im.tvec[1];
          depth[(size_t)y * W + x] = (float)d;
          label[(size_t)y * W + x] = (float)((((int)std::floor(X / 0.05) + (int)std::floor(Y / 0.05)) % 2 + 2) % 2);
        }
      maps.depth[im.name] = depth;
      maps.semantic[im.name] = label;
      // a principal point near the raster so the pairs overlap inside it; the
      // SIMPLE_RADIAL model first (the reference's Assert rejects it)
      rec.GetCamera(im.camera_id).params = {1200, 30, 30, 0};
      im.tvec[0] += 0.002 * (double)im.image_id;  // pose error for the semantic term to pull on
    }
    SemanticBundleAdjustmentOptions options;
    options.print_summary = false;
    options.error_computation_pixel_step = 3;
    SemanticBundleAdjustmentConfig config;
    for (image_t i = 0; i < 3; ++i) config.AddImage(i);
    config.SetConstantPose(0);
    {
      SemanticBundleAdjuster bad(options, config, maps);  // cameras not constant: Assert throws
      bool threw = false;
      try { bad.Solve(&rec); } catch (const std::runtime_error&) { threw = true; }
      CHECK_T(threw);
    }
    for (camera_t c = 0; c < 3; ++c) config.SetConstantCamera(c);
    {
      // not SIMPLE_PINHOLE: Assert throws (cc:619-631) unless the extension is asked for
      SemanticBundleAdjuster bad(options, config, maps);
      std::string what;
      try { bad.Solve(&rec); } catch (const std::runtime_error& e) { what = e.what(); }
      CHECK_T(what == "ERROR: the only supported camera model is SimplePinholeCameraModel.");
    }
    {
      SemanticBundleAdjustmentOptions o2 = options;
      o2.refine_extrinsics = false;  // (with SIMPLE_PINHOLE cameras) the third check
      Reconstruction pin = rec;
      for (auto& c : pin.cameras) {
        c.second.model_id = MI_BA_SIMPLE_PINHOLE;
        c.second.params = {1200, 30, 30};
      }
      SemanticBundleAdjuster bad(o2, config, maps);
      std::string what;
      try { bad.Solve(&pin); } catch (const std::runtime_error& e) { what = e.what(); }
      CHECK_T(what == "ERROR: the argument 'refine_extrinsics' must be set to true.");
    }
    if (s) {
      // the extension: a SIMPLE_RADIAL (k = 0) solve equals the SIMPLE_PINHOLE one
      SemanticBundleAdjustmentOptions o2 = options;
      o2.allow_any_camera_model = true;
      Reconstruction rad = rec, pin = rec;
      for (auto& c : pin.cameras) {
        c.second.model_id = MI_BA_SIMPLE_PINHOLE;
        c.second.params = {1200, 30, 30};
      }
      SemanticBundleAdjuster a(o2, config, maps), b(options, config, maps);
      CHECK_T(a.Solve(&rad));
      CHECK_T(b.Solve(&pin));
      CHECK_T(a.Summary().final_cost == b.Summary().final_cost);
    }
    for (auto& c : rec.cameras) {
      c.second.model_id = MI_BA_SIMPLE_PINHOLE;
      c.second.params = {1200, 30, 30};
    }
    if (!s) return;
    const Reconstruction orig = rec;
    SemanticBundleAdjuster sba(options, config, maps);
    CHECK_T(sba.Solve(&rec));
    CHECK_T(sba.Summary().num_residuals_reduced > 0);
    CHECK_T(sba.Summary().final_cost <= sba.Summary().initial_cost);
    CheckConstantImage(rec, orig, 0);
    for (camera_t c = 0; c < 3; ++c) CheckConstantCamera(rec, orig, c);
    for (auto& p : rec.points3D) CheckConstantPoint(rec, orig, p.first);
  }});

  // SBA outputs (SBACallbackFunctor, semantic_bundle_adjustment.cc:1086-1123;
  // ExportSemanticErrorToCSV :908-1019; the final write :531-538): every
  // iteration's step_k model equals the state the caller's callback saw at
  // that iteration, the CSV files hold every grid pixel of every ordered pair
  // and their errors sum to twice the iteration's cost (TRIVIAL loss, weight
  // 1, no zero-depth pixel, every pair in the problem), the final model is
  // written to output_path.
  cases.push_back({"TestSemanticBundleAdjusterSnapshots", [](bool s) {
    if (!s) return;
    Reconstruction rec = GenerateReconstruction(3, 10);
    const int H = 60, W = 60, step = 3;
    SemanticMaps maps;
    maps.height = H;
    maps.width = W;
    for (auto& e : rec.images) {
      Image& im = e.second;
      // overlapping views (GenerateReconstruction's tvec spread is 8x the
      // 0.5-wide footprint): the maps are rendered at these poses, then the
      // poses move by 0.02 per image so the semantic cost is not zero.  The
      // numeric-diff step is 1e-3 of each coordinate (sqrt(eps) at 0): with
      // identity rotations only translations of ~5 step across pixels
      // (0.6 px here), so the gradient is not zero either
      im.tvec[0] = 5.0 + 0.05 * (double)im.image_id;
      im.tvec[1] = 5.0 + 0.03 * (double)im.image_id;
      std::vector<float> depth((size_t)H * W), label((size_t)H * W);
      for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
          const double d = im.tvec[2];
          const double X = (x - 500.0 + 470.0) / 1200.0 * d - im.tvec[0];
          const double Y = (y - 500.0 + 470.0) / 1200.0 * d - im.tvec[1];
          depth[(size_t)y * W + x] = (float)d;
          label[(size_t)y * W + x] = (float)((((int)std::floor(X / 0.05) + (int)std::floor(Y / 0.05)) % 2 + 2) % 2);
        }
      maps.depth[im.name] = depth;
      maps.semantic[im.name] = label;
      Camera& cam = rec.GetCamera(im.camera_id);
      cam.model_id = MI_BA_SIMPLE_PINHOLE;
      cam.params = {1200, 30, 30};
      im.tvec[0] += 0.02 * (double)im.image_id;
    }
    char tmpl[] = "/tmp/sba_out_XXXXXX";
    const char* dir = mkdtemp(tmpl);
    CHECK_T(dir != nullptr);
    if (!dir) return;
    const std::string out(dir);
    SemanticBundleAdjustmentOptions options;
    options.print_summary = false;
    options.error_computation_pixel_step = step;
    options.output_path = out;
    options.export_csv = true;
    options.solver_options.max_num_iterations = 4;
    SemanticBundleAdjustmentConfig config;
    for (image_t i = 0; i < 3; ++i) config.AddImage(i);
    config.SetConstantPose(0);
    for (camera_t c = 0; c < 3; ++c) config.SetConstantCamera(c);
    std::vector<Reconstruction> seen;
    std::vector<double> costs;
    struct Saver : IterationCallback {
      std::function<void(const IterationSummary&)> fn;
      CallbackReturnType operator()(const IterationSummary& it) override { fn(it); return SOLVER_CONTINUE; }
    } saver;
    saver.fn = [&](const IterationSummary& it) {
      seen.push_back(rec);
      costs.push_back(it.cost);
    };
    options.solver_options.callbacks.push_back(&saver);
    SemanticBundleAdjuster sba(options, config, maps);
    CHECK_T(sba.Solve(&rec));
    CHECK_T(seen.size() >= 2);
    const int grid = ((W + step - 1) / step) * ((H + step - 1) / step);
    for (size_t k = 0; k < seen.size(); ++k) {
      const std::string sd = out + "/run/optim_steps/step_" + std::to_string(k);
      Reconstruction bin, txt;
      ReadModelBinary(sd, &bin);
      ReadModelText(sd + "/text", &txt);
      for (const auto& e : seen[k].images) {
        const Image& a = e.second;
        const Image& b = bin.GetImage(e.first);
        const Image& t = txt.GetImage(e.first);
        for (int m = 0; m < 3; ++m) CHECK_T(b.tvec[m] == a.tvec[m] && t.tvec[m] == a.tvec[m]);
        for (int m = 0; m < 4; ++m)
          CHECK_T(std::fabs(b.qvec[m] - a.qvec[m]) <= 1e-15 && std::fabs(t.qvec[m] - a.qvec[m]) <= 1e-15);
      }
      long errors = 0;
      for (image_t i = 0; i < 3; ++i)
        for (image_t j = 0; j < 3; ++j) {
          if (i == j) continue;
          std::ifstream f(sd + "/vis_" + std::to_string(i) + "_to_" + std::to_string(j) + ".csv");
          CHECK_T(f.is_open());
          std::string line;
          std::getline(f, line);
          CHECK_T(line == "Type,SemanticError,X1,Y1,X2,Y2,X3D,Y3D,Z3D");
          int rows = 0;
          while (std::getline(f, line)) {
            std::stringstream ls(line);
            std::string type, err;
            std::getline(ls, type, ',');
            std::getline(ls, err, ',');
            CHECK_T(type == "10" || type == "-1" || type == "-2");
            CHECK_T(err == "0" || err == "1");
            errors += err == "1";
            ++rows;
          }
          CHECK_T(rows == grid);
        }
      CHECK_T(0.5 * (double)errors == costs[k]);
    }
    Reconstruction fin;
    ReadModelBinary(out, &fin);
    for (const auto& e : rec.images)
      for (int m = 0; m < 3; ++m) CHECK_T(fin.GetImage(e.first).tvec[m] == e.second.tvec[m]);
    if (std::system(("rm -rf '" + out + "'").c_str()) != 0) std::printf("  (could not remove %s)\n", out.c_str());
  }});

  // Reconstruction::FilterPoints3DWithLargeReprojectionError
  // (reconstruction.cc:1472-1525) on the GPU against its rule restated here.
  cases.push_back({"TestFilterPoints3D", [](bool s) {
    if (!s) return;
    Reconstruction rec = GenerateReconstruction(3, 100);
    // outliers: point p gets p % 4 of its observations moved by 30 px
    for (auto& e : rec.points3D) {
      int n = 0;
      for (const TrackElement& te : e.second.track)
        if (n++ < (int)(e.first % 4)) rec.GetImage(te.image_id).points2D[te.point2D_idx].xy[0] += 30.0;
    }
    const Reconstruction orig = rec;
    std::unordered_set<point3D_t> ids;
    for (auto& e : rec.points3D) ids.insert(e.first);
    const double max_err = 5.0;
    // expected: squared error of each element (SIMPLE_RADIAL, k = 0, identity rotations)
    size_t expect = 0;
    std::vector<point3D_t> expect_deleted;
    for (auto& e : orig.points3D) {
      size_t bad = 0;
      for (const TrackElement& te : e.second.track) {
        const Image& im = orig.GetImage(te.image_id);
        const double* X = e.second.xyz;
        const double pz = X[2] + im.tvec[2];
        const double x = 1200 * (X[0] + im.tvec[0]) / pz + 500, y = 1200 * (X[1] + im.tvec[1]) / pz + 500;
        const double* o = im.points2D[te.point2D_idx].xy;
        if ((x - o[0]) * (x - o[0]) + (y - o[1]) * (y - o[1]) > max_err * max_err) ++bad;
      }
      if (bad >= e.second.track.size() - 1) {
        expect += e.second.track.size();
        expect_deleted.push_back(e.first);
      } else {
        expect += bad;
      }
    }
    const size_t n = rec.FilterPoints3DWithLargeReprojectionError(max_err, ids);
    CHECK_T(n == expect);
    CHECK_T(rec.points3D.size() == orig.points3D.size() - expect_deleted.size());
    for (point3D_t id : expect_deleted) CHECK_T(rec.points3D.count(id) == 0);
    for (auto& e : rec.points3D) {
      CHECK_T(e.second.track.size() == 3 - e.first % 4);
      CHECK_T(e.second.error >= 0.0 && e.second.error < max_err);
    }
  }});

  // ParallelBundleAdjuster (bundle_adjustment.cc:536-783) routed to the GPU
  // solver: the PBA problem has the config images' measurements only, so
  // every point they see is variable (here: images 0 and 1 of 3, 400
  // residuals, 2 * (6 + 2) + 300 parameters).
  cases.push_back({"TestParallelBundleAdjuster", [](bool s) {
    Reconstruction rec = GenerateReconstruction(3, 100);
    BundleAdjustmentOptions options;
    options.print_summary = false;
    CHECK_T(ParallelBundleAdjuster::IsSupported(options, rec));
    BundleAdjustmentOptions pp = options;
    pp.refine_principal_point = true;
    CHECK_T(!ParallelBundleAdjuster::IsSupported(pp, rec));
    BundleAdjustmentOptions ex = options;
    ex.refine_extra_params = false;
    CHECK_T(!ParallelBundleAdjuster::IsSupported(ex, rec));
    Reconstruction shared = rec;
    shared.GetImage(1).camera_id = 0;
    CHECK_T(!ParallelBundleAdjuster::IsSupported(options, shared));
    Reconstruction pinhole = rec;
    pinhole.GetCamera(2).model_id = MI_BA_PINHOLE;
    pinhole.GetCamera(2).params = {1200, 1200, 500, 500};
    CHECK_T(!ParallelBundleAdjuster::IsSupported(options, pinhole));
    ParallelBundleAdjuster::Options po;
    po.print_summary = false;
    {
      BundleAdjustmentConfig bad;
      bad.AddImage(0);
      bad.SetConstantCamera(0);
      bool threw = false;
      try { ParallelBundleAdjuster pba(po, options, bad); } catch (const std::invalid_argument&) { threw = true; }
      CHECK_T(threw);
      bad = BundleAdjustmentConfig();
      bad.AddImage(0);
      bad.AddVariablePoint(1);
      threw = false;
      try { ParallelBundleAdjuster pba(po, options, bad); } catch (const std::invalid_argument&) { threw = true; }
      CHECK_T(threw);
    }
    if (!s) return;
    BundleAdjustmentConfig config;
    config.AddImage(0);
    config.AddImage(1);
    const Reconstruction orig = rec;
    ParallelBundleAdjuster pba(po, options, config);
    CHECK_T(pba.Solve(&rec));
    CHECK_T(pba.Summary().num_residuals_reduced == 400);
    CHECK_T(pba.Summary().num_effective_parameters_reduced == 2 * (6 + 2) + 300);
    CHECK_T(pba.Summary().final_cost <= pba.Summary().initial_cost);
    CheckVariableImage(rec, orig, 0);
    CheckVariableImage(rec, orig, 1);
    CheckVariableCamera(rec, orig, 0);
    CheckVariableCamera(rec, orig, 1);
    CheckConstantImage(rec, orig, 2);
    CheckConstantCamera(rec, orig, 2);
    for (auto& p : rec.points3D) CheckVariablePoint(rec, orig, p.first);
    bool threw = false;
    try { pba.Solve(&rec); } catch (const std::logic_error&) { threw = true; }
    CHECK_T(threw);
  }});

  cases.push_back({"TestInvalidConfig", [](bool) {
    BundleAdjustmentConfig config;
    bool threw = false;
    try { config.SetConstantPose(7); } catch (const std::invalid_argument&) { threw = true; }
    CHECK_T(threw);
    config.AddImage(1);
    config.SetConstantTvec(1, {0});
    threw = false;
    try { config.SetConstantPose(1); } catch (const std::invalid_argument&) { threw = true; }
    CHECK_T(threw);
  }});

  for (auto& c : cases) {
    const int before = g_failures;
    try {
      c.run(solve);
    } catch (const std::exception& e) {
      std::printf("  EXCEPTION %s\n", e.what());
      ++g_failures;
    }
    std::printf("%s %s\n", g_failures == before ? "PASS" : "FAIL", c.name.c_str());
  }
  std::printf("%d failure(s)\n", g_failures);
  return g_failures == 0 ? 0 : 1;
}
