// controllers_test.cc — the facade's controllers, iteration callbacks and
// Reconstruction filters (include/colmap_amd/controllers.h,
// bundle_adjustment.h) on libmi_ba.so.
//
//   ./controllers_test host   host-only cases (no GPU)
//   ./controllers_test gpu    every case (the filters and solves need the MI355X)
//
// Known answers transcribed from the reference's tests:
//   TestFilterObservationsWithNegativeDepth  src/base/reconstruction_test.cc:510-531
//   TestFilterPoints3D (reprojection half)   src/base/reconstruction_test.cc:415-434
// Registration order: ReadImagesText / ReadImagesBinary register images in
// file order (reconstruction.cc:1599-1600,1826-1827); the controllers' gauge
// takes RegImageIds()[0] / [1] (controllers/bundle_adjustment.cc:91-94).
// Callback semantics: ceres::IterationCallback as the reference's controllers
// use it (controllers/bundle_adjustment.cc:43-61,87-88) and the SBA snapshot
// callback's update_state_every_iteration (semantic_bundle_adjustment.h:129,
// semantic_bundle_adjustment.cc:1086-1123).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "colmap_amd/controllers.h"
#include "colmap_amd/model_io.h"

#include <cstdlib>
#include <fstream>

using namespace colmap_amd;

static int g_failures = 0;
#define CHECK_T(cond)                                                        \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::printf("  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);        \
      ++g_failures;                                                          \
    }                                                                        \
  } while (0)

// GenerateReconstruction of reconstruction_test.cc:43-66: one PINHOLE camera
// (InitializeWithName("PINHOLE", 1, 1, 1): f = 1, principal point (0.5, 0.5)),
// num_images registered images at the identity pose with 10 points2D at (0, 0).
static Reconstruction TinyReconstruction(int num_images) {
  Reconstruction rec;
  Camera cam;
  cam.camera_id = 1;
  cam.model_id = MI_BA_PINHOLE;
  cam.width = cam.height = 1;
  cam.params = {1, 1, 0.5, 0.5};
  rec.AddCamera(cam);
  for (int i = 1; i <= num_images; ++i) {
    Image im;
    im.image_id = (image_t)i;
    im.camera_id = 1;
    im.name = "image" + std::to_string(i);
    im.points2D.assign(10, Point2D());
    rec.AddImage(im);
  }
  return rec;
}

// bundle_adjustment_test.cc:123-184 with a small rotation and OPENCV-free
// SIMPLE_RADIAL cameras (f = 1200, identity rotation, tvec (U, U, 10)).
static Reconstruction SolveScene(int num_images, int num_points) {
  std::mt19937 prng(0);
  auto U = [&](double a, double b) { return std::uniform_real_distribution<double>(a, b)(prng); };
  Reconstruction rec;
  std::vector<point3D_t> ids;
  for (int i = 0; i < num_points; ++i) {
    double xyz[3] = {U(-1, 1), U(-1, 1), U(-1, 1)};
    ids.push_back(rec.AddPoint3D(xyz));
  }
  for (int i = 0; i < num_images; ++i) {
    Camera cam;
    cam.camera_id = (camera_t)i;
    cam.model_id = MI_BA_SIMPLE_RADIAL;
    cam.params = {1200, 500, 500, 0};
    rec.AddCamera(cam);
    Image im;
    im.image_id = (image_t)i;
    im.camera_id = (camera_t)i;
    im.name = std::to_string(i);
    im.tvec[0] = U(-1, 1);
    im.tvec[1] = U(-1, 1);
    im.tvec[2] = 10;
    for (point3D_t id : ids) {
      const double* X = rec.GetPoint3D(id).xyz;
      const double px = X[0] + im.tvec[0], py = X[1] + im.tvec[1], pz = X[2] + im.tvec[2];
      Point2D p2;
      p2.xy[0] = 1200 * px / pz + 500 + U(-2, 2);
      p2.xy[1] = 1200 * py / pz + 500 + U(-2, 2);
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

// Parameters equal within rel (0: bitwise).  Solves that should agree are
// compared within 1e-9 relative: the normal-equation reductions use float
// atomics, so two runs of one problem may differ in the last bits.
static bool SameParams(const Reconstruction& a, const Reconstruction& b, double rel = 1e-9) {
  auto close = [&](double x, double y) { return std::fabs(x - y) <= rel * std::max(1.0, std::fabs(y)); };
  for (const auto& e : a.images) {
    const Image& o = b.images.at(e.first);
    for (int m = 0; m < 4; ++m) if (!close(e.second.qvec[m], o.qvec[m])) return false;
    for (int m = 0; m < 3; ++m) if (!close(e.second.tvec[m], o.tvec[m])) return false;
  }
  for (const auto& e : a.points3D)
    for (int m = 0; m < 3; ++m) if (!close(e.second.xyz[m], b.points3D.at(e.first).xyz[m])) return false;
  for (const auto& e : a.cameras) {
    const auto& q = b.cameras.at(e.first).params;
    for (size_t m = 0; m < q.size(); ++m) if (!close(e.second.params[m], q[m])) return false;
  }
  return true;
}

static BundleAdjustmentConfig GaugeConfig(const Reconstruction& rec) {
  BundleAdjustmentConfig c;
  for (const auto& e : rec.images) c.AddImage(e.first);
  c.SetConstantPose(0);
  c.SetConstantTvec(1, {0});
  return c;
}

struct LambdaCallback : IterationCallback {
  std::function<CallbackReturnType(const IterationSummary&)> fn;
  explicit LambdaCallback(std::function<CallbackReturnType(const IterationSummary&)> f) : fn(std::move(f)) {}
  CallbackReturnType operator()(const IterationSummary& s) override { return fn(s); }
};

struct Case {
  std::string name;
  bool gpu;
  std::function<void()> run;
};

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::string(argv[1]) == "gpu";
  std::vector<Case> cases;

  // Reconstruction::DeleteObservation: a track of length <= 2 takes its point
  // with it (reconstruction.cc:257-277).
  cases.push_back({"TestDeleteObservationShortTrack", false, [] {
    Reconstruction rec = TinyReconstruction(3);
    const double x[3] = {0, 0, 1};
    const point3D_t a = rec.AddPoint3D(x);
    rec.AddObservation(a, TrackElement{1, 0});
    rec.AddObservation(a, TrackElement{2, 0});
    rec.AddObservation(a, TrackElement{3, 0});
    rec.DeleteObservation(3, 0);
    CHECK_T(rec.points3D.count(a) == 1 && rec.points3D.at(a).track.size() == 2);
    CHECK_T(!rec.GetImage(3).points2D[0].HasPoint3D());
    rec.DeleteObservation(2, 0);
    CHECK_T(rec.points3D.count(a) == 0);
    CHECK_T(!rec.GetImage(1).points2D[0].HasPoint3D() && !rec.GetImage(2).points2D[0].HasPoint3D());
  }});

  // reconstruction_test.cc:510-531
  cases.push_back({"TestFilterObservationsWithNegativeDepth", true, [] {
    Reconstruction rec = TinyReconstruction(2);
    const double x[3] = {0, 0, 1};
    const point3D_t id = rec.AddPoint3D(x);
    CHECK_T(rec.points3D.size() == 1);
    rec.FilterObservationsWithNegativeDepth();
    CHECK_T(rec.points3D.size() == 1);
    rec.GetPoint3D(id).xyz[2] = 0.001;
    rec.FilterObservationsWithNegativeDepth();
    CHECK_T(rec.points3D.size() == 1);
    rec.GetPoint3D(id).xyz[2] = 0.0;
    rec.FilterObservationsWithNegativeDepth();
    CHECK_T(rec.points3D.size() == 1);
    rec.AddObservation(id, TrackElement{1, 0});
    rec.GetPoint3D(id).xyz[2] = 0.001;
    CHECK_T(rec.FilterObservationsWithNegativeDepth() == 0);
    CHECK_T(rec.points3D.size() == 1);
    rec.GetPoint3D(id).xyz[2] = 0.0;
    CHECK_T(rec.FilterObservationsWithNegativeDepth() == 1);
    CHECK_T(rec.points3D.size() == 0);
  }});

  // Only registered images are visited; a deleted point's later observations
  // are not counted again.
  cases.push_back({"TestFilterNegativeDepthOrderAndRegistration", true, [] {
    Reconstruction rec = TinyReconstruction(4);
    const double behind[3] = {0, 0, -1};
    const point3D_t a = rec.AddPoint3D(behind);  // track 2: the first deletion removes it
    rec.AddObservation(a, TrackElement{1, 0});
    rec.AddObservation(a, TrackElement{2, 0});
    const point3D_t b = rec.AddPoint3D(behind);  // track 3 with one unregistered image
    rec.AddObservation(b, TrackElement{1, 1});
    rec.AddObservation(b, TrackElement{2, 1});
    rec.AddObservation(b, TrackElement{3, 1});
    rec.GetImage(3).registered = false;
    const double front[3] = {0.1, 0.2, 3};
    const point3D_t c = rec.AddPoint3D(front);
    rec.AddObservation(c, TrackElement{1, 2});
    rec.AddObservation(c, TrackElement{4, 2});
    // image 1: a (deletes a: length 2), b (3 -> 2); image 2: b (length 2 -> deleted)
    CHECK_T(rec.FilterObservationsWithNegativeDepth() == 3);
    CHECK_T(rec.points3D.count(a) == 0 && rec.points3D.count(b) == 0 && rec.points3D.count(c) == 1);
    CHECK_T(rec.points3D.at(c).track.size() == 2);
  }});

  // reconstruction_test.cc:425-434, the reprojection-error half of
  // TestFilterPoints3D: (-0.6, -0.5, 1) seen at (0, 0) by both images
  // projects 0.1 px away: kept at 0.1, deleted at 0.09.
  cases.push_back({"TestFilterPoints3DReprojectionKnownAnswers", true, [] {
    Reconstruction rec = TinyReconstruction(2);
    const double x3[3] = {-0.5, -0.5, 1};
    const point3D_t id3 = rec.AddPoint3D(x3);
    rec.AddObservation(id3, TrackElement{1, 0});
    rec.AddObservation(id3, TrackElement{2, 0});
    CHECK_T(rec.FilterPoints3DWithLargeReprojectionError(0.0, {id3}) == 0);
    CHECK_T(rec.points3D.size() == 1);
    rec.DeletePoint3D(id3);
    const double x4[3] = {-0.6, -0.5, 1};
    const point3D_t id4 = rec.AddPoint3D(x4);
    rec.AddObservation(id4, TrackElement{1, 0});
    rec.AddObservation(id4, TrackElement{2, 0});
    CHECK_T(rec.FilterPoints3DWithLargeReprojectionError(0.1, {id4}) == 0);
    CHECK_T(rec.points3D.size() == 1);
    CHECK_T(rec.FilterPoints3DWithLargeReprojectionError(0.09, {id4}) == 2);
    CHECK_T(rec.points3D.size() == 0);
  }});

  // A callback ending the solve with SOLVER_TERMINATE_SUCCESSFULLY at
  // iteration k leaves the parameters of a max_num_iterations = k solve.
  cases.push_back({"TestCallbackTerminateEqualsMaxIterations", true, [] {
    for (int k : {0, 1, 3}) {
      Reconstruction ref = SolveScene(3, 60), rec = ref;
      BundleAdjustmentOptions o;
      o.print_summary = false;
      o.solver_options.max_num_iterations = k;
      BundleAdjuster a(o, GaugeConfig(ref));
      CHECK_T(a.Solve(&ref));
      CHECK_T(a.Summary().termination_type == SolverSummary::NO_CONVERGENCE);
      BundleAdjustmentOptions o2;
      o2.print_summary = false;
      std::vector<int> seen;
      LambdaCallback cb([&](const IterationSummary& s) {
        seen.push_back(s.iteration);
        return s.iteration == k ? SOLVER_TERMINATE_SUCCESSFULLY : SOLVER_CONTINUE;
      });
      o2.solver_options.callbacks.push_back(&cb);
      BundleAdjuster b(o2, GaugeConfig(rec));
      CHECK_T(b.Solve(&rec));
      CHECK_T(b.Summary().termination_type == SolverSummary::USER_SUCCESS);
      CHECK_T((int)seen.size() == k + 1);
      for (int i = 0; i <= k && i < (int)seen.size(); ++i) CHECK_T(seen[i] == i);
      CHECK_T(SameParams(ref, rec));
      CHECK_T(std::fabs(b.Summary().final_cost - a.Summary().final_cost) <= 1e-12 * a.Summary().final_cost);
    }
  }});

  // SOLVER_ABORT: USER_FAILURE, the caller's parameters untouched (Ceres
  // copies no state back after USER_FAILURE); with
  // update_state_every_iteration they hold the point of the last callback.
  cases.push_back({"TestCallbackAbortAndUpdateState", true, [] {
    Reconstruction orig = SolveScene(3, 60), rec = orig;
    for (auto& e : orig.images) {  // SetUp normalises the config qvecs
      double* q = e.second.qvec;
      const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
      for (int m = 0; m < 4; ++m) q[m] /= n;
    }
    BundleAdjustmentOptions o;
    o.print_summary = false;
    LambdaCallback abort_at2([](const IterationSummary& s) { return s.iteration == 2 ? SOLVER_ABORT : SOLVER_CONTINUE; });
    o.solver_options.callbacks.push_back(&abort_at2);
    BundleAdjuster a(o, GaugeConfig(rec));
    CHECK_T(a.Solve(&rec));
    CHECK_T(a.Summary().termination_type == SolverSummary::USER_FAILURE);
    CHECK_T(SameParams(orig, rec, 0.0));
    // update_state_every_iteration: snapshots per iteration, abort at 2
    auto run_k = [](int k) {
      Reconstruction r = SolveScene(3, 60);
      BundleAdjustmentOptions o2;
      o2.print_summary = false;
      o2.solver_options.max_num_iterations = k;
      BundleAdjuster b(o2, GaugeConfig(r));
      CHECK_T(b.Solve(&r));
      return r;
    };
    const Reconstruction one = run_k(1), two = run_k(2);
    Reconstruction upd = SolveScene(3, 60);
    std::vector<Reconstruction> snaps;
    BundleAdjustmentOptions o3;
    o3.print_summary = false;
    o3.solver_options.update_state_every_iteration = true;
    LambdaCallback snap([&](const IterationSummary& s) {
      snaps.push_back(upd);
      return s.iteration == 2 ? SOLVER_ABORT : SOLVER_CONTINUE;
    });
    o3.solver_options.callbacks.push_back(&snap);
    BundleAdjuster c(o3, GaugeConfig(upd));
    CHECK_T(c.Solve(&upd));
    CHECK_T(c.Summary().termination_type == SolverSummary::USER_FAILURE);
    CHECK_T(snaps.size() == 3);
    if (snaps.size() == 3) {
      CHECK_T(SameParams(snaps[0], orig));
      CHECK_T(SameParams(snaps[1], one));
      CHECK_T(SameParams(snaps[2], two));
    }
    CHECK_T(SameParams(upd, two));
  }});

  // The stop flag (Thread::Stop without a callback): set before the solve,
  // the LM stops after iteration 0.
  cases.push_back({"TestStopFlag", true, [] {
    Reconstruction rec = SolveScene(3, 60);
    std::atomic<int32_t> stop{MI_BA_SOLVER_TERMINATE_SUCCESSFULLY};
    BundleAdjustmentOptions o;
    o.print_summary = false;
    o.stop_flag = &stop;
    BundleAdjuster a(o, GaugeConfig(rec));
    CHECK_T(a.Solve(&rec));
    CHECK_T(a.Summary().termination_type == SolverSummary::USER_SUCCESS);
    CHECK_T(a.Summary().num_successful_steps + a.Summary().num_unsuccessful_steps == 0);
    CHECK_T(a.Summary().final_cost == a.Summary().initial_cost);
  }});

  // BundleAdjustmentController: negative-depth observations filtered before
  // the solve, Pause blocks the LM in the callback until Resume, Stop ends
  // it with USER_SUCCESS (controllers/bundle_adjustment.cc:43-103).
  cases.push_back({"TestBundleAdjustmentController", true, [] {
    Reconstruction rec = SolveScene(4, 80);
    // one point moved behind every camera: depth -0.5, three of its four
    // observations deleted, the third deletion taking the point
    const point3D_t moved = rec.points3D.begin()->first;
    rec.GetPoint3D(moved).xyz[2] = -10.5;
    BundleAdjustmentOptions o;
    o.print_summary = false;
    std::thread resumer;
    BundleAdjustmentController* final_ctl = nullptr;
    LambdaCallback self([&](const IterationSummary& s) {
      if (s.iteration == 1) {
        final_ctl->Pause();
        resumer = std::thread([&] {
          std::this_thread::sleep_for(std::chrono::milliseconds(60));
          final_ctl->Resume();
        });
      }
      if (s.iteration == 3) final_ctl->Stop();
      return SOLVER_CONTINUE;
    });
    BundleAdjustmentOptions of = o;
    of.solver_options.callbacks.assign(1, &self);
    BundleAdjustmentController fc(of, &rec);
    final_ctl = &fc;
    const auto t0 = std::chrono::steady_clock::now();
    fc.Run();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (resumer.joinable()) resumer.join();
    CHECK_T(fc.Solved());
    CHECK_T(fc.NumFilteredObservations() == 3);
    CHECK_T(rec.points3D.count(moved) == 0);
    CHECK_T(fc.Summary().termination_type == SolverSummary::USER_SUCCESS);
    CHECK_T(fc.Summary().num_successful_steps + fc.Summary().num_unsuccessful_steps == 3);
    CHECK_T(ms >= 60.0);
    CHECK_T(fc.IsStopped());
  }});

  // A model whose images.txt is not in image-id order: RegImageIds follows
  // the file, RegisterImage / DeRegisterImage append / remove.
  cases.push_back({"TestRegImageIdsFileOrder", false, [] {
    char tmpl[] = "/tmp/reg_order_XXXXXX";
    const char* dir = mkdtemp(tmpl);
    CHECK_T(dir != nullptr);
    if (!dir) return;
    const std::string d(dir);
    std::ofstream(d + "/cameras.txt") << "1 SIMPLE_RADIAL 100 100 100 50 50 0\n";
    std::ofstream(d + "/images.txt") << "5 1 0 0 0 0 0 10 1 a.png\n10 20 1\n"
                                        "2 1 0 0 0 0.5 0 10 1 b.png\n11 21 1\n"
                                        "9 1 0 0 0 -0.5 0 10 1 c.png\n12 22 1\n";
    std::ofstream(d + "/points3D.txt") << "1 0 0 0 0 0 0 -1 5 0 2 0 9 0\n";
    Reconstruction rec;
    ReadModelText(d, &rec);
    CHECK_T((rec.RegImageIds() == std::vector<image_t>{5, 2, 9}));
    rec.DeRegisterImage(2);
    CHECK_T((rec.RegImageIds() == std::vector<image_t>{5, 9}));
    CHECK_T(!rec.GetImage(2).IsRegistered() && rec.points3D.at(1).track.size() == 2);
    rec.RegisterImage(2);
    CHECK_T((rec.RegImageIds() == std::vector<image_t>{5, 9, 2}));
    // the binary round trip keeps a registration order of the same images
    WriteModelBinary(d, rec);
    Reconstruction back;
    ReadModelBinary(d, &back);
    std::vector<image_t> ids = back.RegImageIds();
    std::sort(ids.begin(), ids.end());
    CHECK_T((ids == std::vector<image_t>{2, 5, 9}));
    for (const char* f : {"cameras", "images", "points3D"}) {
      std::remove((d + "/" + f + ".txt").c_str());
      std::remove((d + "/" + f + ".bin").c_str());
    }
    rmdir(dir);
  }});

  // The controller's gauge follows the registration order: images registered
  // as 2, 0, 3, 1 fix image 2's pose and image 0's tvec x.
  cases.push_back({"TestControllerGaugeFollowsRegistrationOrder", true, [] {
    const Reconstruction base = SolveScene(4, 80);
    Reconstruction rec;
    rec.cameras = base.cameras;
    rec.points3D = base.points3D;
    for (image_t id : {2u, 0u, 3u, 1u}) rec.AddImage(base.images.at(id));
    CHECK_T((rec.RegImageIds() == std::vector<image_t>{2, 0, 3, 1}));
    Image before2 = rec.GetImage(2), before0 = rec.GetImage(0), before1 = rec.GetImage(1);
    BundleAdjustmentOptions o;
    o.print_summary = false;
    BundleAdjustmentController ctl(o, &rec);
    ctl.Run();
    CHECK_T(ctl.Solved());
    const Image& a2 = rec.GetImage(2);
    const Image& a0 = rec.GetImage(0);
    const Image& a1 = rec.GetImage(1);
    for (int m = 0; m < 3; ++m) CHECK_T(a2.tvec[m] == before2.tvec[m]);
    CHECK_T(a0.tvec[0] == before0.tvec[0]);
    CHECK_T(a0.tvec[1] != before0.tvec[1]);
    CHECK_T(a1.tvec[0] != before1.tvec[0]);
  }});

  // Fewer than two registered images: the reference prints an error and returns.
  cases.push_back({"TestControllerNeedsTwoViews", false, [] {
    Reconstruction rec = TinyReconstruction(2);
    rec.GetImage(2).registered = false;
    BundleAdjustmentOptions o;
    BundleAdjustmentController ctl(o, &rec);
    ctl.Run();
    CHECK_T(!ctl.Solved());
  }});

  for (auto& c : cases) {
    if (c.gpu && !gpu) continue;
    const int before = g_failures;
    try {
      c.run();
    } catch (const std::exception& e) {
      std::printf("  EXCEPTION %s\n", e.what());
      ++g_failures;
    }
    std::printf("%s %s\n", g_failures == before ? "PASS" : "FAIL", c.name.c_str());
  }
  std::printf("%d failure(s)\n", g_failures);
  return g_failures == 0 ? 0 : 1;
}
