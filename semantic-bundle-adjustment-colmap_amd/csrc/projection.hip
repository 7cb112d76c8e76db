// projection.hip — reprojection errors of every observation and the
// post-BA track filter (product code).
//
//   mi_ba_squared_reprojection_errors  <- CalculateSquaredReprojectionError
//                                         (src/base/projection.cc:111-128)
//   mi_ba_filter_points3d              <- Reconstruction::
//                                         FilterPoints3DWithLargeReprojectionError
//                                         (src/base/reconstruction.cc:1470-1525)
//   mi_ba_positive_depth               <- the HasPointPositiveDepth test of
//                                         Reconstruction::FilterObservationsWithNegativeDepth
//                                         (src/base/reconstruction.cc:647-665)
//
// One lane per observation (error) and one lane per point (filter decision
// over its track, CSR by point built on the host in track order).  Both are
// HBM-bound byte streams: per observation 16 B xy + 8 B indices in, 8 B out,
// plus the point / pose / camera gathers (L2-resident per image).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstring>
#include <vector>

#include "../../include/mi_ba.h"
#include "ba_math.h"
#include "setup.h"

namespace miba {
namespace {

constexpr int kTB = 256;

struct ProjArgs {
  const double2* xy;
  const int32_t* obs_image;
  const int32_t* obs_point;
  const double* qt;       // [I][8] q(4) t(3) pad
  const double* cam;      // [C][8]
  const uint8_t* cam_model;
  const int32_t* img_cam;
  const double* X;        // [P][3]
  int64_t n;
};

// QuaternionRotatePoint (pose.cc): normalise, then rotate.
__device__ inline void rotate_normalized(const double q[4], const double p[3], double r[3]) {
  const double s = 1.0 / sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const double u[4] = {s * q[0], s * q[1], s * q[2], s * q[3]};
  unit_quat_rotate(u, p, r);
}

__global__ __launch_bounds__(kTB) void sq_reproj_error_kernel(ProjArgs a, double* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * kTB + threadIdx.x;
  if (k >= a.n) return;
  const int img = a.obs_image[k];
  const int64_t pt = a.obs_point[k];
  const double* qt = a.qt + 8 * (size_t)img;
  const double q[4] = {qt[0], qt[1], qt[2], qt[3]};
  const double X[3] = {a.X[3 * pt], a.X[3 * pt + 1], a.X[3 * pt + 2]};
  double P[3];
  rotate_normalized(q, X, P);
  P[0] += qt[4];
  P[1] += qt[5];
  P[2] += qt[6];
  // point behind the camera (projection.cc:118-121)
  if (P[2] < DBL_EPSILON) {
    out[k] = DBL_MAX;
    return;
  }
  const int cam = a.img_cam[img];
  double prm[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) prm[m] = a.cam[8 * (size_t)cam + m];
  double x, y;
  world_to_image_any(a.cam_model[cam], prm, P[0] / P[2], P[1] / P[2], &x, &y);
  const double2 o = a.xy[k];
  out[k] = (x - o.x) * (x - o.x) + (y - o.y) * (y - o.y);
}

// HasPointPositiveDepth(image.ProjectionMatrix(), X) (projection.cc:191-195)
// for every observation: the third row of [R | t] with R =
// Eigen::Quaterniond(qvec).normalized().toRotationMatrix() (pose.cc
// QuaternionToRotationMatrix), dotted with (X, 1), >= DBL_EPSILON.  The
// products are kept unfused and in Eigen's order (SSE2 squaredNorm pairs
// (x, z) and (y, w); the strided row dot sums left to right), as the
// reference's x86-64 build evaluates them.  Observations of images outside
// image_mask are kept.
__global__ __launch_bounds__(kTB) void positive_depth_kernel(ProjArgs a, const uint8_t* __restrict__ image_mask,
                                                              uint8_t* __restrict__ keep) {
#pragma clang fp contract(off)
  const int64_t k = (int64_t)blockIdx.x * kTB + threadIdx.x;
  if (k >= a.n) return;
  const int img = a.obs_image[k];
  if (image_mask && !image_mask[img]) {
    keep[k] = 1;
    return;
  }
  const int64_t pt = a.obs_point[k];
  const double* qt = a.qt + 8 * (size_t)img;
  const double w = qt[0], x = qt[1], y = qt[2], z = qt[3];
  const double sq = (x * x + z * z) + (y * y + w * w);
  double nw = w, nx = x, ny = y, nz = z;
  if (sq > 0.0) {
    const double n = sqrt(sq);
    nw = w / n;
    nx = x / n;
    ny = y / n;
    nz = z / n;
  }
  const double tx = 2.0 * nx, ty = 2.0 * ny, tz = 2.0 * nz;
  const double twx = tx * nw, twy = ty * nw;
  const double txx = tx * nx, txz = tz * nx, tyy = ty * ny, tyz = tz * ny;
  const double r20 = txz - twy, r21 = tyz + twx, r22 = 1.0 - (txx + tyy);
  const double depth = ((r20 * a.X[3 * pt] + r21 * a.X[3 * pt + 1]) + r22 * a.X[3 * pt + 2]) + qt[6] * 1.0;
  keep[k] = depth >= DBL_EPSILON ? 1 : 0;
}

// reconstruction.cc:1480-1521 for one point: track elements with squared
// error above max_sq are deleted; if that leaves fewer than two, the whole
// point is; otherwise its error is the mean reprojection error of what stays.
__global__ __launch_bounds__(kTB) void filter_points_kernel(const int64_t* __restrict__ off,
                                                           const int64_t* __restrict__ items,
                                                           const double* __restrict__ sq, int64_t P,
                                                           const uint8_t* __restrict__ point_mask, double max_sq,
                                                           uint8_t* __restrict__ obs_keep,
                                                           uint8_t* __restrict__ point_keep,
                                                           double* __restrict__ point_error,
                                                           int64_t* __restrict__ filtered) {
  const int64_t p = (int64_t)blockIdx.x * kTB + threadIdx.x;
  if (p >= P) return;
  const int64_t b = off[p], e = off[p + 1], len = e - b;
  int64_t nf = 0;
  if (point_mask && !point_mask[p]) {
    point_keep[p] = 1;
    for (int64_t m = b; m < e; ++m) obs_keep[items[m]] = 1;
  } else if (len < 2) {
    point_keep[p] = 0;
    nf = len;
    for (int64_t m = b; m < e; ++m) obs_keep[items[m]] = 0;
  } else {
    double sum = 0.0;
    int64_t bad = 0;
    for (int64_t m = b; m < e; ++m) {
      const double s = sq[items[m]];
      if (s > max_sq) {
        ++bad;
      } else {
        sum += sqrt(s);
      }
    }
    if (bad >= len - 1) {
      point_keep[p] = 0;
      nf = len;
      for (int64_t m = b; m < e; ++m) obs_keep[items[m]] = 0;
    } else {
      point_keep[p] = 1;
      nf = bad;
      for (int64_t m = b; m < e; ++m) obs_keep[items[m]] = sq[items[m]] > max_sq ? 0 : 1;
      point_error[p] = sum / (double)(len - bad);
    }
  }
  filtered[p] = nf;
}

struct Buf {
  void* p = nullptr;
  ~Buf() {
    if (p) (void)hipFree(p);
  }
  template <typename T>
  T* alloc(size_t n) {
    if (hipMalloc(&p, n == 0 ? 8 : n * sizeof(T)) != hipSuccess) p = nullptr;
    return static_cast<T*>(p);
  }
};

// Uploads the problem's observations and parameters for the projection
// kernels; fills `a`.
mi_ba_status upload(const mi_ba_problem* p, const HostSetup& s, Buf* b, ProjArgs* a) {
  const int I = p->num_images, C = p->num_cameras;
  const int64_t P = p->num_points, N = p->num_obs;
  std::vector<double> qt(8 * (size_t)I, 0.0), cm(8 * (size_t)C, 0.0);
  std::vector<uint8_t> cmod(C);
  for (int i = 0; i < I; ++i) {
    for (int m = 0; m < 4; ++m) qt[8 * (size_t)i + m] = p->qvec[4 * (size_t)i + m];
    for (int m = 0; m < 3; ++m) qt[8 * (size_t)i + 4 + m] = p->tvec[3 * (size_t)i + m];
  }
  for (int c = 0; c < C; ++c) {
    cmod[c] = (uint8_t)s.cam_model[c];
    for (int64_t m = s.cam_off[c]; m < s.cam_off[c + 1]; ++m) cm[8 * (size_t)c + (m - s.cam_off[c])] = p->camera_params[m];
  }
  double2* xy = b[0].alloc<double2>(N);
  int32_t* oi = b[1].alloc<int32_t>(N);
  int32_t* op = b[2].alloc<int32_t>(N);
  double* dqt = b[3].alloc<double>(qt.size());
  double* dcm = b[4].alloc<double>(cm.size());
  uint8_t* dmod = b[5].alloc<uint8_t>(C);
  int32_t* dic = b[6].alloc<int32_t>(I);
  double* dX = b[7].alloc<double>(3 * (size_t)P);
  if (!xy || !oi || !op || !dqt || !dcm || !dmod || !dic || !dX) return MI_BA_ERR_OUT_OF_MEMORY;
  if ((N && (hipMemcpy(xy, p->obs_xy, N * 16, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(oi, p->obs_image, N * 4, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(op, p->obs_point, N * 4, hipMemcpyHostToDevice) != hipSuccess)) ||
      (I && (hipMemcpy(dqt, qt.data(), qt.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(dic, p->image_camera, I * 4, hipMemcpyHostToDevice) != hipSuccess)) ||
      (C && (hipMemcpy(dcm, cm.data(), cm.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(dmod, cmod.data(), C, hipMemcpyHostToDevice) != hipSuccess)) ||
      (P && hipMemcpy(dX, p->xyz, 3 * P * 8, hipMemcpyHostToDevice) != hipSuccess))
    return MI_BA_ERR_HIP;
  *a = ProjArgs{xy, oi, op, dqt, dcm, dmod, dic, dX, N};
  return MI_BA_OK;
}

// Validation shared with problem assembly (indices in range, known models);
// no qvec normalisation here (QuaternionRotatePoint normalises itself).
mi_ba_status check(const mi_ba_problem* p, HostSetup* s) {
  if (!p || p->num_obs < 0 || p->num_images < 0 || p->num_cameras < 0 || p->num_points < 0)
    return MI_BA_ERR_INVALID_ARGUMENT;
  if (p->num_obs > 0 && (!p->obs_xy || !p->obs_image || !p->obs_point)) return MI_BA_ERR_INVALID_ARGUMENT;
  if (p->num_images > 0 && (!p->qvec || !p->tvec || !p->image_camera)) return MI_BA_ERR_INVALID_ARGUMENT;
  if (p->num_cameras > 0 && !p->camera_params) return MI_BA_ERR_INVALID_ARGUMENT;
  if (p->num_points > 0 && !p->xyz) return MI_BA_ERR_INVALID_ARGUMENT;
  const int C = p->num_cameras;
  s->cam_model.assign(C, 0);
  s->cam_off.assign(C + 1, 0);
  for (int c = 0; c < C; ++c) {
    const int m = problem_camera_model(p, c);
    if (num_params(m) < 0) return MI_BA_ERR_UNSUPPORTED;
    s->cam_model[c] = m;
    s->cam_off[c + 1] = s->cam_off[c] + num_params(m);
  }
  for (int i = 0; i < p->num_images; ++i)
    if (p->image_camera[i] < 0 || p->image_camera[i] >= C) return MI_BA_ERR_INVALID_ARGUMENT;
  for (int64_t k = 0; k < p->num_obs; ++k)
    if (p->obs_image[k] < 0 || p->obs_image[k] >= p->num_images || p->obs_point[k] < 0 ||
        p->obs_point[k] >= p->num_points)
      return MI_BA_ERR_INVALID_ARGUMENT;
  return MI_BA_OK;
}

mi_ba_status set_device(int32_t device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return MI_BA_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return MI_BA_ERR_INVALID_ARGUMENT;
  if (hipSetDevice(device) != hipSuccess) return MI_BA_ERR_HIP;
  return MI_BA_OK;
}

}  // namespace
}  // namespace miba

using namespace miba;

extern "C" mi_ba_status mi_ba_squared_reprojection_errors(const mi_ba_problem* problem, int32_t device,
                                                         double* sq_errors) {
  HostSetup s;
  mi_ba_status st = check(problem, &s);
  if (st != MI_BA_OK) return st;
  if (problem->num_obs > 0 && !sq_errors) return MI_BA_ERR_INVALID_ARGUMENT;
  if ((st = set_device(device)) != MI_BA_OK) return st;
  const int64_t N = problem->num_obs;
  if (N == 0) return MI_BA_OK;
  Buf b[9];
  ProjArgs a;
  if ((st = upload(problem, s, b, &a)) != MI_BA_OK) return st;
  double* d_sq = b[8].alloc<double>(N);
  if (!d_sq) return MI_BA_ERR_OUT_OF_MEMORY;
  hipLaunchKernelGGL(sq_reproj_error_kernel, dim3((unsigned)((N + kTB - 1) / kTB)), dim3(kTB), 0, 0, a, d_sq);
  if (hipGetLastError() != hipSuccess) return MI_BA_ERR_HIP;
  if (hipMemcpy(sq_errors, d_sq, N * 8, hipMemcpyDeviceToHost) != hipSuccess) return MI_BA_ERR_HIP;
  return MI_BA_OK;
}

extern "C" mi_ba_status mi_ba_filter_points3d(const mi_ba_problem* problem, double max_reproj_error,
                                             const uint8_t* point_mask, int32_t device, uint8_t* obs_keep,
                                             uint8_t* point_keep, double* point_error, int64_t* num_filtered) {
  HostSetup s;
  mi_ba_status st = check(problem, &s);
  if (st != MI_BA_OK) return st;
  const int64_t N = problem->num_obs, P = problem->num_points;
  if ((N > 0 && !obs_keep) || (P > 0 && (!point_keep || !point_error)) || !num_filtered)
    return MI_BA_ERR_INVALID_ARGUMENT;
  if ((st = set_device(device)) != MI_BA_OK) return st;
  *num_filtered = 0;
  if (P == 0) return MI_BA_OK;
  // CSR by point, observations of a point in their order in the problem
  // (the flattener emits them in Track order)
  std::vector<int64_t> off(P + 1, 0), items(N);
  for (int64_t k = 0; k < N; ++k) off[problem->obs_point[k] + 1]++;
  for (int64_t p = 0; p < P; ++p) off[p + 1] += off[p];
  {
    std::vector<int64_t> pos(off.begin(), off.end() - 1);
    for (int64_t k = 0; k < N; ++k) items[pos[problem->obs_point[k]]++] = k;
  }
  Buf b[16];
  ProjArgs a;
  if ((st = upload(problem, s, b, &a)) != MI_BA_OK) return st;
  double* d_sq = b[8].alloc<double>(N);
  int64_t* d_off = b[9].alloc<int64_t>(P + 1);
  int64_t* d_items = b[10].alloc<int64_t>(N);
  uint8_t* d_mask = point_mask ? b[11].alloc<uint8_t>(P) : nullptr;
  uint8_t* d_okeep = b[12].alloc<uint8_t>(N);
  uint8_t* d_pkeep = b[13].alloc<uint8_t>(P);
  double* d_perr = b[14].alloc<double>(P);
  int64_t* d_nf = b[15].alloc<int64_t>(P);
  if (!d_sq || !d_off || !d_items || (point_mask && !d_mask) || !d_okeep || !d_pkeep || !d_perr || !d_nf)
    return MI_BA_ERR_OUT_OF_MEMORY;
  // point_error of points that keep no error value stays what the caller had
  if (hipMemcpy(d_off, off.data(), (P + 1) * 8, hipMemcpyHostToDevice) != hipSuccess ||
      (N && hipMemcpy(d_items, items.data(), N * 8, hipMemcpyHostToDevice) != hipSuccess) ||
      (point_mask && hipMemcpy(d_mask, point_mask, P, hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(d_perr, point_error, P * 8, hipMemcpyHostToDevice) != hipSuccess)
    return MI_BA_ERR_HIP;
  if (N) hipLaunchKernelGGL(sq_reproj_error_kernel, dim3((unsigned)((N + kTB - 1) / kTB)), dim3(kTB), 0, 0, a, d_sq);
  hipLaunchKernelGGL(filter_points_kernel, dim3((unsigned)((P + kTB - 1) / kTB)), dim3(kTB), 0, 0, d_off, d_items,
                     d_sq, P, d_mask, max_reproj_error * max_reproj_error, d_okeep, d_pkeep, d_perr, d_nf);
  if (hipGetLastError() != hipSuccess) return MI_BA_ERR_HIP;
  std::vector<int64_t> nf(P);
  if ((N && hipMemcpy(obs_keep, d_okeep, N, hipMemcpyDeviceToHost) != hipSuccess) ||
      hipMemcpy(point_keep, d_pkeep, P, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(point_error, d_perr, P * 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(nf.data(), d_nf, P * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return MI_BA_ERR_HIP;
  int64_t total = 0;
  for (int64_t v : nf) total += v;
  *num_filtered = total;
  return MI_BA_OK;
}

extern "C" mi_ba_status mi_ba_positive_depth(const mi_ba_problem* problem, const uint8_t* image_mask, int32_t device,
                                            uint8_t* obs_keep, int64_t* num_negative) {
  HostSetup s;
  mi_ba_status st = check(problem, &s);
  if (st != MI_BA_OK) return st;
  const int64_t N = problem->num_obs;
  if ((N > 0 && !obs_keep) || !num_negative) return MI_BA_ERR_INVALID_ARGUMENT;
  if ((st = set_device(device)) != MI_BA_OK) return st;
  *num_negative = 0;
  if (N == 0) return MI_BA_OK;
  Buf b[11];
  ProjArgs a;
  if ((st = upload(problem, s, b, &a)) != MI_BA_OK) return st;
  const int I = problem->num_images;
  uint8_t* d_mask = image_mask ? b[8].alloc<uint8_t>(I) : nullptr;
  uint8_t* d_keep = b[9].alloc<uint8_t>(N);
  if ((image_mask && !d_mask) || !d_keep) return MI_BA_ERR_OUT_OF_MEMORY;
  if (image_mask && I && hipMemcpy(d_mask, image_mask, I, hipMemcpyHostToDevice) != hipSuccess) return MI_BA_ERR_HIP;
  hipLaunchKernelGGL(positive_depth_kernel, dim3((unsigned)((N + kTB - 1) / kTB)), dim3(kTB), 0, 0, a, d_mask, d_keep);
  if (hipGetLastError() != hipSuccess) return MI_BA_ERR_HIP;
  if (hipMemcpy(obs_keep, d_keep, N, hipMemcpyDeviceToHost) != hipSuccess) return MI_BA_ERR_HIP;
  int64_t neg = 0;
  for (int64_t k = 0; k < N; ++k) neg += obs_keep[k] == 0;
  *num_negative = neg;
  return MI_BA_OK;
}
