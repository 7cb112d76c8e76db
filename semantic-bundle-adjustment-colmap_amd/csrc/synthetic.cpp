// synthetic.cpp — synthetic BA scenes (fixture/benchmark tool, host only).
// See include/mi_ba_synthetic.h for the restated reference generator.
#include "../../include/mi_ba_synthetic.h"

#include <algorithm>
#include <cmath>
#include <random>
#include <vector>

#include "ba_math.h"

using namespace miba;

namespace {

void init_params(int model, double f, double c, const double* extra, double* out) {
  // *CameraModel::InitializeParams (camera_models.h) + extra params
  switch (model) {
    case kSimplePinhole: out[0] = f; out[1] = c; out[2] = c; break;
    case kPinhole: out[0] = f; out[1] = f; out[2] = c; out[3] = c; break;
    case kSimpleRadial: out[0] = f; out[1] = c; out[2] = c; out[3] = extra[0]; break;
    case kRadial: out[0] = f; out[1] = c; out[2] = c; out[3] = extra[0]; out[4] = extra[1]; break;
    case kOpenCV:
      out[0] = f; out[1] = f; out[2] = c; out[3] = c;
      for (int k = 0; k < 4; ++k) out[4 + k] = extra[k];
      break;
    default: break;
  }
}

void project(int model, const double* prm, const double* q, const double* t, const double* X, double* xy) {
  const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const double qn[4] = {q[0] / n, q[1] / n, q[2] / n, q[3] / n};
  double P[3];
  unit_quat_rotate(qn, X, P);
  P[0] += t[0]; P[1] += t[1]; P[2] += t[2];
  const double u = P[0] / P[2], v = P[1] / P[2];
  dispatch_model(model, [&](auto m) {
    constexpr int M = decltype(m)::value;
    world_to_image<M>(prm, u, v, &xy[0], &xy[1]);
  });
}

}  // namespace

extern "C" {

int64_t mi_ba_synth_num_obs(const mi_ba_synth_config* cfg) {
  if (!cfg) return -1;
  if (cfg->track_length <= 0) return (int64_t)cfg->num_images * cfg->num_points;
  return (int64_t)std::min(cfg->track_length, cfg->num_images) * cfg->num_points;
}

int32_t mi_ba_synth_generate(const mi_ba_synth_config* cfg, double* camera_params, double* qvec, double* tvec,
                             int32_t* image_camera, double* xyz, double* obs_xy, int32_t* obs_image,
                             int32_t* obs_point) {
  const int np = num_params(cfg->camera_model);
  if (np < 0 || cfg->num_images <= 0 || cfg->num_points < 0) return 1;
  std::mt19937 prng(cfg->seed);  // SetPRNGSeed (random.cc:42-44)
  auto random_real = [&](double a, double b) { return std::uniform_real_distribution<double>(a, b)(prng); };
  const int I = cfg->num_images;
  const int64_t P = cfg->num_points;
  // GeneratePointCloud (bundle_adjustment_test.cc:111-121)
  for (int64_t k = 0; k < P; ++k) {
    xyz[3 * k + 0] = random_real(-1, 1);
    xyz[3 * k + 1] = random_real(-1, 1);
    xyz[3 * k + 2] = random_real(-1, 1);
  }
  const double f = cfg->focal_factor * cfg->image_size;
  const double c = cfg->image_size / 2.0;
  const double noise = cfg->noise;
  if (cfg->track_length <= 0) {
    // reference generator: per image, camera + pose, then all points
    int64_t o = 0;
    for (int i = 0; i < I; ++i) {
      init_params(cfg->camera_model, f, c, cfg->extra, camera_params + (size_t)np * i);
      image_camera[i] = i;
      qvec[4 * i] = 1; qvec[4 * i + 1] = 0; qvec[4 * i + 2] = 0; qvec[4 * i + 3] = 0;
      tvec[3 * i] = random_real(-1.0, 1.0);
      tvec[3 * i + 1] = random_real(-1.0, 1.0);
      tvec[3 * i + 2] = 10;
      for (int64_t k = 0; k < P; ++k, ++o) {
        double xy[2];
        project(cfg->camera_model, camera_params + (size_t)np * i, qvec + 4 * i, tvec + 3 * i, xyz + 3 * k, xy);
        const double nx = random_real(-noise, noise);
        const double ny = random_real(-noise, noise);
        obs_xy[2 * o] = xy[0] + nx;
        obs_xy[2 * o + 1] = xy[1] + ny;
        obs_image[o] = i;
        obs_point[o] = (int32_t)k;
      }
    }
    return 0;
  }
  // scaled variant: small random rotations, L distinct images per point
  for (int i = 0; i < I; ++i) {
    init_params(cfg->camera_model, f, c, cfg->extra, camera_params + (size_t)np * i);
    image_camera[i] = i;
    const double r = cfg->rotation_range;
    double a[3] = {0, 0, 0};
    if (r > 0) {
      a[0] = random_real(-r, r);
      a[1] = random_real(-r, r);
      a[2] = random_real(-r, r);
    }
    const double th = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    if (th > 0) {
      const double s = std::sin(th / 2) / th;
      qvec[4 * i] = std::cos(th / 2);
      qvec[4 * i + 1] = s * a[0];
      qvec[4 * i + 2] = s * a[1];
      qvec[4 * i + 3] = s * a[2];
    } else {
      qvec[4 * i] = 1; qvec[4 * i + 1] = 0; qvec[4 * i + 2] = 0; qvec[4 * i + 3] = 0;
    }
    tvec[3 * i] = random_real(-1.0, 1.0);
    tvec[3 * i + 1] = random_real(-1.0, 1.0);
    tvec[3 * i + 2] = 10;
  }
  const int L = std::min(cfg->track_length, I);
  std::uniform_int_distribution<int> pick(0, I - 1);
  std::vector<int> imgs(L);
  int64_t o = 0;
  for (int64_t k = 0; k < P; ++k) {
    for (int m = 0; m < L; ++m) {
      int cand;
      do {
        cand = pick(prng);
      } while (std::find(imgs.begin(), imgs.begin() + m, cand) != imgs.begin() + m);
      imgs[m] = cand;
    }
    std::sort(imgs.begin(), imgs.end());
    for (int m = 0; m < L; ++m, ++o) {
      const int i = imgs[m];
      double xy[2];
      project(cfg->camera_model, camera_params + (size_t)np * i, qvec + 4 * i, tvec + 3 * i, xyz + 3 * k, xy);
      const double nx = random_real(-noise, noise);
      const double ny = random_real(-noise, noise);
      obs_xy[2 * o] = xy[0] + nx;
      obs_xy[2 * o + 1] = xy[1] + ny;
      obs_image[o] = i;
      obs_point[o] = (int32_t)k;
    }
  }
  return 0;
}

int32_t mi_ba_synth_render(int32_t model, int32_t num_images, const double* camera_params, const double* qvec,
                           const double* tvec, const int32_t* image_camera, int32_t H, int32_t W, double plane_z,
                           double cell, float* depth, float* label) {
  const int np = num_params(model);
  if (np < 0 || H <= 0 || W <= 0) return 1;
  // normalized coordinates of every pixel, per distinct camera parameter set
  std::vector<std::vector<double>> tables;
  std::vector<const double*> table_params;
  std::vector<int> table_of(num_images, -1);
  for (int i = 0; i < num_images; ++i) {
    const double* prm = camera_params + (size_t)np * image_camera[i];
    int found = -1;
    for (size_t t = 0; t < table_params.size(); ++t)
      if (std::equal(prm, prm + np, table_params[t])) { found = (int)t; break; }
    if (found < 0) {
      found = (int)tables.size();
      table_params.push_back(prm);
      tables.emplace_back((size_t)2 * H * W);
      std::vector<double>& tab = tables.back();
#pragma omp parallel for schedule(static)
      for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
          double u = 0, v = 0;
          dispatch_model(model, [&](auto m) {
            constexpr int M = decltype(m)::value;
            image_to_world<M>(prm, (double)x, (double)y, &u, &v);
          });
          tab[2 * ((size_t)y * W + x)] = u;
          tab[2 * ((size_t)y * W + x) + 1] = v;
        }
    }
    table_of[i] = found;
  }
#pragma omp parallel for schedule(dynamic, 1)
  for (int i = 0; i < num_images; ++i) {
    const double* q = qvec + 4 * (size_t)i;
    const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const double qn[4] = {q[0] / n, q[1] / n, q[2] / n, q[3] / n};
    double R[9];
    unit_quat_matrix(qn, R);
    const double* t = tvec + 3 * (size_t)i;
    // camera centre C = -R^T t
    const double Cw[3] = {-(R[0] * t[0] + R[3] * t[1] + R[6] * t[2]), -(R[1] * t[0] + R[4] * t[1] + R[7] * t[2]),
                          -(R[2] * t[0] + R[5] * t[1] + R[8] * t[2])};
    const std::vector<double>& tab = tables[table_of[i]];
    float* dd = depth + (size_t)i * H * W;
    float* ll = label + (size_t)i * H * W;
    for (size_t pix = 0; pix < (size_t)H * W; ++pix) {
      const double u = tab[2 * pix], v = tab[2 * pix + 1];
      // ray direction in world: R^T (u, v, 1)
      const double dw[3] = {R[0] * u + R[3] * v + R[6], R[1] * u + R[4] * v + R[7], R[2] * u + R[5] * v + R[8]};
      double s = dw[2] != 0.0 ? (plane_z - Cw[2]) / dw[2] : -1.0;
      if (!(s > 0.0)) {
        dd[pix] = 0.0f;
        ll[pix] = 0.0f;
        continue;
      }
      const double X = Cw[0] + s * dw[0], Y = Cw[1] + s * dw[1];
      const long a = (long)std::floor(X / cell) + (long)std::floor(Y / cell);
      dd[pix] = (float)s;
      ll[pix] = (float)(((a % 8) + 8) % 8);
    }
  }
  return 0;
}

}  // extern "C"
