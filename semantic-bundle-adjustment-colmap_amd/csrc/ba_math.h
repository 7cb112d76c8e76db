// ba_math.h — host/device math of the semantic-BA hot path (product code).
//
// Restates, for gfx950 kernels and the host setup, the per-observation math
// of the reference (AlainSchoebi/semantic-bundle-adjustment-colmap):
//   camera models   src/base/camera_models.h:545-588, 614-637, 640-690,
//                   714-757, 760-810, 853-902
//   reprojection    src/base/cost_functions.h:57-81, 116-142
//   rotations       Ceres 2.1 rotation.h (3rd party, restated) and
//                   src/util/rotation_extension.h:43-98
// Jacobians are analytic (hand-derived), not dual numbers: the oracle uses
// dual numbers, so parity tests compare two independent derivations.
#pragma once

#include <cmath>
#include <cstdint>
#include <type_traits>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MI_HD __host__ __device__ inline
#else
#define MI_HD inline
#endif

namespace miba {

enum CameraModelId { kSimplePinhole = 0, kPinhole = 1, kSimpleRadial = 2, kRadial = 3, kOpenCV = 4 };
constexpr int kNumModels = 5;

MI_HD int num_params(int model) {
  return model == kSimplePinhole ? 3 : model == kPinhole ? 4 : model == kSimpleRadial ? 4
       : model == kRadial ? 5 : model == kOpenCV ? 8 : -1;
}

template <int M> struct Model;
template <> struct Model<kSimplePinhole> { static constexpr int kNumParams = 3; };
template <> struct Model<kPinhole> { static constexpr int kNumParams = 4; };
template <> struct Model<kSimpleRadial> { static constexpr int kNumParams = 4; };
template <> struct Model<kRadial> { static constexpr int kNumParams = 5; };
template <> struct Model<kOpenCV> { static constexpr int kNumParams = 8; };
// Kernel instantiation for problems whose cameras use different models
// (camera_models.h:117-141 dispatches per camera): the model is read per
// camera at run time, parameters are held in 8-wide slots.
constexpr int kMixedModels = 15;
template <> struct Model<kMixedModels> { static constexpr int kNumParams = 8; };

// ---------------------------------------------------------------------------
// Rotations (Ceres 2.1 rotation.h, restated)
// ---------------------------------------------------------------------------
MI_HD void unit_quat_rotate(const double q[4], const double p[3], double r[3]) {
  const double t2 = q[0] * q[1];
  const double t3 = q[0] * q[2];
  const double t4 = q[0] * q[3];
  const double t5 = -(q[1] * q[1]);
  const double t6 = q[1] * q[2];
  const double t7 = q[1] * q[3];
  const double t8 = -(q[2] * q[2]);
  const double t9 = q[2] * q[3];
  const double t1 = -(q[3] * q[3]);
  r[0] = 2.0 * ((t8 + t1) * p[0] + (t6 - t4) * p[1] + (t3 + t7) * p[2]) + p[0];
  r[1] = 2.0 * ((t4 + t6) * p[0] + (t5 + t1) * p[1] + (t9 - t2) * p[2]) + p[1];
  r[2] = 2.0 * ((t7 - t3) * p[0] + (t2 + t9) * p[1] + (t5 + t8) * p[2]) + p[2];
}

// d(unit_quat_rotate(q, p))/dq, 3x4 row-major, exact for non-unit q.
MI_HD void unit_quat_rotate_dq(const double q[4], const double p[3], double D[12]) {
  const double q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  const double p0 = p[0], p1 = p[1], p2 = p[2];
  D[0] = 2.0 * (q2 * p2 - q3 * p1);
  D[1] = 2.0 * (q2 * p1 + q3 * p2);
  D[2] = 2.0 * (q1 * p1 + q0 * p2 - 2.0 * q2 * p0);
  D[3] = 2.0 * (q1 * p2 - q0 * p1 - 2.0 * q3 * p0);
  D[4] = 2.0 * (q3 * p0 - q1 * p2);
  D[5] = 2.0 * (q2 * p0 - q0 * p2 - 2.0 * q1 * p1);
  D[6] = 2.0 * (q1 * p0 + q3 * p2);
  D[7] = 2.0 * (q0 * p0 + q2 * p2 - 2.0 * q3 * p1);
  D[8] = 2.0 * (q1 * p1 - q2 * p0);
  D[9] = 2.0 * (q3 * p0 + q0 * p1 - 2.0 * q1 * p2);
  D[10] = 2.0 * (q3 * p1 - q0 * p0 - 2.0 * q2 * p2);
  D[11] = 2.0 * (q1 * p0 + q2 * p1);
}

// Rotation matrix of unit_quat_rotate (linear in p), row-major.
MI_HD void unit_quat_matrix(const double q[4], double R[9]) {
  const double t2 = q[0] * q[1], t3 = q[0] * q[2], t4 = q[0] * q[3];
  const double t5 = -(q[1] * q[1]), t6 = q[1] * q[2], t7 = q[1] * q[3];
  const double t8 = -(q[2] * q[2]), t9 = q[2] * q[3], t1 = -(q[3] * q[3]);
  R[0] = 2.0 * (t8 + t1) + 1.0; R[1] = 2.0 * (t6 - t4);       R[2] = 2.0 * (t3 + t7);
  R[3] = 2.0 * (t4 + t6);       R[4] = 2.0 * (t5 + t1) + 1.0; R[5] = 2.0 * (t9 - t2);
  R[6] = 2.0 * (t7 - t3);       R[7] = 2.0 * (t2 + t9);       R[8] = 2.0 * (t5 + t8) + 1.0;
}

// Ceres 2.1 QuaternionManifold::PlusJacobian (4x3 row-major).
MI_HD void quat_plus_jacobian(const double x[4], double J[12]) {
  J[0] = -x[1]; J[1] = -x[2];  J[2] = -x[3];
  J[3] = x[0];  J[4] = x[3];   J[5] = -x[2];
  J[6] = -x[3]; J[7] = x[0];   J[8] = x[1];
  J[9] = x[2];  J[10] = -x[1]; J[11] = x[0];
}

// Ceres 2.1 QuaternionManifold::Plus.
MI_HD void quat_plus(const double x[4], const double d[3], double out[4]) {
  const double nd = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd == 0.0) {
    out[0] = x[0]; out[1] = x[1]; out[2] = x[2]; out[3] = x[3];
    return;
  }
  const double s = sin(nd) / nd;
  const double a0 = cos(nd), a1 = s * d[0], a2 = s * d[1], a3 = s * d[2];
  out[0] = a0 * x[0] - a1 * x[1] - a2 * x[2] - a3 * x[3];
  out[1] = a0 * x[1] + a1 * x[0] + a2 * x[3] - a3 * x[2];
  out[2] = a0 * x[2] - a1 * x[3] + a2 * x[0] + a3 * x[1];
  out[3] = a0 * x[3] + a1 * x[2] - a2 * x[1] + a3 * x[0];
}

// ---------------------------------------------------------------------------
// Camera models: distortion, projection, and their analytic derivatives.
// ---------------------------------------------------------------------------
template <int M>
MI_HD void distortion(const double* ex, double u, double v, double* du, double* dv) {
  if constexpr (M == kSimpleRadial) {
    const double k = ex[0];
    const double u2 = u * u, v2 = v * v, r2 = u2 + v2;
    const double radial = k * r2;
    *du = u * radial;
    *dv = v * radial;
  } else if constexpr (M == kRadial) {
    const double k1 = ex[0], k2 = ex[1];
    const double u2 = u * u, v2 = v * v, r2 = u2 + v2;
    const double radial = k1 * r2 + k2 * r2 * r2;
    *du = u * radial;
    *dv = v * radial;
  } else if constexpr (M == kOpenCV) {
    const double k1 = ex[0], k2 = ex[1], p1 = ex[2], p2 = ex[3];
    const double u2 = u * u, uv = u * v, v2 = v * v, r2 = u2 + v2;
    const double radial = k1 * r2 + k2 * r2 * r2;
    *du = u * radial + 2.0 * p1 * uv + p2 * (r2 + 2.0 * u2);
    *dv = v * radial + 2.0 * p2 * uv + p1 * (r2 + 2.0 * v2);
  } else {
    *du = 0.0;
    *dv = 0.0;
  }
}

template <int M>
MI_HD void world_to_image(const double* prm, double u, double v, double* x, double* y) {
  if constexpr (M == kSimplePinhole) {
    *x = prm[0] * u + prm[1];
    *y = prm[0] * v + prm[2];
  } else if constexpr (M == kPinhole) {
    *x = prm[0] * u + prm[2];
    *y = prm[1] * v + prm[3];
  } else if constexpr (M == kSimpleRadial || M == kRadial) {
    double du, dv;
    distortion<M>(prm + 3, u, v, &du, &dv);
    const double xd = u + du, yd = v + dv;
    *x = prm[0] * xd + prm[1];
    *y = prm[0] * yd + prm[2];
  } else {
    double du, dv;
    distortion<M>(prm + 4, u, v, &du, &dv);
    const double xd = u + du, yd = v + dv;
    *x = prm[0] * xd + prm[2];
    *y = prm[1] * yd + prm[3];
  }
}

// Projection plus derivatives: A = d(x,y)/d(u,v) (2x2 row-major) and
// Jp = d(x,y)/dparams (2 x kNumParams row-major).
template <int M>
MI_HD void world_to_image_jac(const double* prm, double u, double v, double* x, double* y,
                              double A[4], double* Jp) {
  constexpr int np = Model<M>::kNumParams;
  for (int i = 0; i < 2 * np; ++i) Jp[i] = 0.0;
  if constexpr (M == kSimplePinhole) {
    const double f = prm[0];
    *x = f * u + prm[1];
    *y = f * v + prm[2];
    A[0] = f; A[1] = 0.0; A[2] = 0.0; A[3] = f;
    Jp[0] = u; Jp[1] = 1.0;
    Jp[np + 0] = v; Jp[np + 2] = 1.0;
  } else if constexpr (M == kPinhole) {
    *x = prm[0] * u + prm[2];
    *y = prm[1] * v + prm[3];
    A[0] = prm[0]; A[1] = 0.0; A[2] = 0.0; A[3] = prm[1];
    Jp[0] = u; Jp[2] = 1.0;
    Jp[np + 1] = v; Jp[np + 3] = 1.0;
  } else if constexpr (M == kSimpleRadial) {
    const double f = prm[0], k = prm[3];
    const double u2 = u * u, v2 = v * v, r2 = u2 + v2;
    const double radial = k * r2;
    const double xd = u + u * radial, yd = v + v * radial;
    *x = f * xd + prm[1];
    *y = f * yd + prm[2];
    const double two_k_uv = 2.0 * k * u * v;
    A[0] = f * (1.0 + radial + 2.0 * k * u2);
    A[1] = f * two_k_uv;
    A[2] = f * two_k_uv;
    A[3] = f * (1.0 + radial + 2.0 * k * v2);
    Jp[0] = xd; Jp[1] = 1.0; Jp[3] = f * u * r2;
    Jp[np + 0] = yd; Jp[np + 2] = 1.0; Jp[np + 3] = f * v * r2;
  } else if constexpr (M == kRadial) {
    const double f = prm[0], k1 = prm[3], k2 = prm[4];
    const double u2 = u * u, v2 = v * v, r2 = u2 + v2;
    const double radial = k1 * r2 + k2 * r2 * r2;
    const double g = 2.0 * (k1 + 2.0 * k2 * r2);  // d radial / d(u) = g*u
    const double xd = u + u * radial, yd = v + v * radial;
    *x = f * xd + prm[1];
    *y = f * yd + prm[2];
    A[0] = f * (1.0 + radial + g * u2);
    A[1] = f * (g * u * v);
    A[2] = f * (g * u * v);
    A[3] = f * (1.0 + radial + g * v2);
    Jp[0] = xd; Jp[1] = 1.0; Jp[3] = f * u * r2; Jp[4] = f * u * r2 * r2;
    Jp[np + 0] = yd; Jp[np + 2] = 1.0; Jp[np + 3] = f * v * r2; Jp[np + 4] = f * v * r2 * r2;
  } else {  // OPENCV
    const double fx = prm[0], fy = prm[1], k1 = prm[4], k2 = prm[5], p1 = prm[6], p2 = prm[7];
    const double u2 = u * u, uv = u * v, v2 = v * v, r2 = u2 + v2;
    const double radial = k1 * r2 + k2 * r2 * r2;
    const double g = 2.0 * (k1 + 2.0 * k2 * r2);
    const double xd = u + u * radial + 2.0 * p1 * uv + p2 * (r2 + 2.0 * u2);
    const double yd = v + v * radial + 2.0 * p2 * uv + p1 * (r2 + 2.0 * v2);
    *x = fx * xd + prm[2];
    *y = fy * yd + prm[3];
    A[0] = fx * (1.0 + radial + g * u2 + 2.0 * p1 * v + 6.0 * p2 * u);
    A[1] = fx * (g * uv + 2.0 * p1 * u + 2.0 * p2 * v);
    A[2] = fy * (g * uv + 2.0 * p2 * v + 2.0 * p1 * u);
    A[3] = fy * (1.0 + radial + g * v2 + 2.0 * p2 * u + 6.0 * p1 * v);
    Jp[0] = xd; Jp[2] = 1.0;
    Jp[4] = fx * u * r2; Jp[5] = fx * u * r2 * r2; Jp[6] = fx * 2.0 * uv; Jp[7] = fx * (r2 + 2.0 * u2);
    Jp[np + 1] = yd; Jp[np + 3] = 1.0;
    Jp[np + 4] = fy * v * r2; Jp[np + 5] = fy * v * r2 * r2; Jp[np + 6] = fy * (r2 + 2.0 * v2);
    Jp[np + 7] = fy * 2.0 * uv;
  }
}

// camera_models.h:545-588 IterativeUndistortion (Eigen 2x2 inverse form).
template <int M>
MI_HD void iterative_undistortion(const double* ex, double* u, double* v) {
  const double eps = 2.220446049250313e-16;
  const double x00 = *u, x01 = *v;
  double x0 = *u, x1 = *v;
  for (int i = 0; i < 100; ++i) {
    const double s0 = fmax(eps, fabs(1e-6 * x0));
    const double s1 = fmax(eps, fabs(1e-6 * x1));
    double d0, d1, b00, b01, f00, f01, b10, b11, f10, f11;
    distortion<M>(ex, x0, x1, &d0, &d1);
    distortion<M>(ex, x0 - s0, x1, &b00, &b01);
    distortion<M>(ex, x0 + s0, x1, &f00, &f01);
    distortion<M>(ex, x0, x1 - s1, &b10, &b11);
    distortion<M>(ex, x0, x1 + s1, &f10, &f11);
    const double J00 = 1 + (f00 - b00) / (2 * s0);
    const double J01 = (f10 - b10) / (2 * s1);
    const double J10 = (f01 - b01) / (2 * s0);
    const double J11 = 1 + (f11 - b11) / (2 * s1);
    const double invdet = 1.0 / (J00 * J11 - J10 * J01);
    const double e0 = x0 + d0 - x00, e1 = x1 + d1 - x01;
    const double st0 = (J11 * invdet) * e0 + (-J01 * invdet) * e1;
    const double st1 = (-J10 * invdet) * e0 + (J00 * invdet) * e1;
    x0 -= st0;
    x1 -= st1;
    if (st0 * st0 + st1 * st1 < 1e-10) break;
  }
  *u = x0;
  *v = x1;
}

template <int M>
MI_HD void image_to_world(const double* prm, double x, double y, double* u, double* v) {
  if constexpr (M == kSimplePinhole) {
    *u = (x - prm[1]) / prm[0];
    *v = (y - prm[2]) / prm[0];
  } else if constexpr (M == kPinhole) {
    *u = (x - prm[2]) / prm[0];
    *v = (y - prm[3]) / prm[1];
  } else if constexpr (M == kSimpleRadial || M == kRadial) {
    *u = (x - prm[1]) / prm[0];
    *v = (y - prm[2]) / prm[0];
    iterative_undistortion<M>(prm + 3, u, v);
  } else {
    *u = (x - prm[2]) / prm[0];
    *v = (y - prm[3]) / prm[1];
    iterative_undistortion<M>(prm + 4, u, v);
  }
}

// Run-time dispatch on a per-camera model id (host and device).
template <typename F>
MI_HD void switch_model(int model, F&& f) {
  switch (model) {
    case kSimplePinhole: f(std::integral_constant<int, kSimplePinhole>{}); break;
    case kPinhole: f(std::integral_constant<int, kPinhole>{}); break;
    case kSimpleRadial: f(std::integral_constant<int, kSimpleRadial>{}); break;
    case kRadial: f(std::integral_constant<int, kRadial>{}); break;
    default: f(std::integral_constant<int, kOpenCV>{}); break;
  }
}

// Projection of a camera whose model is known only at run time; Jp8 is
// d(x,y)/dparams in 8-wide rows (2 x 8, unused columns zero).
MI_HD void world_to_image_any(int model, const double* prm, double u, double v, double* x, double* y) {
  switch_model(model, [&](auto m) { world_to_image<decltype(m)::value>(prm, u, v, x, y); });
}
MI_HD void world_to_image_jac_any(int model, const double* prm, double u, double v, double* x, double* y,
                                  double A[4], double Jp8[16]) {
  switch_model(model, [&](auto m) {
    constexpr int M = decltype(m)::value;
    constexpr int np = Model<M>::kNumParams;
    double Jp[2 * np];
    world_to_image_jac<M>(prm, u, v, x, y, A, Jp);
    for (int rw = 0; rw < 2; ++rw)
      for (int k = 0; k < 8; ++k) Jp8[rw * 8 + k] = k < np ? Jp[rw * np + k] : 0.0;
  });
}
MI_HD void image_to_world_any(int model, const double* prm, double x, double y, double* u, double* v) {
  switch_model(model, [&](auto m) { image_to_world<decltype(m)::value>(prm, x, y, u, v); });
}

// Runtime dispatch helpers for host code.
template <typename F>
inline void dispatch_model(int model, F&& f) {
  switch (model) {
    case kSimplePinhole: f(std::integral_constant<int, kSimplePinhole>{}); break;
    case kPinhole: f(std::integral_constant<int, kPinhole>{}); break;
    case kSimpleRadial: f(std::integral_constant<int, kSimpleRadial>{}); break;
    case kRadial: f(std::integral_constant<int, kRadial>{}); break;
    case kOpenCV: f(std::integral_constant<int, kOpenCV>{}); break;
    default: break;
  }
}

// ---------------------------------------------------------------------------
// Loss functions (Ceres 2.1 TrivialLoss / SoftLOneLoss / CauchyLoss, restated)
// and the Corrector's residual/Jacobian scale for the rho'' <= 0 branch
// (every loss used here: Trivial rho''=0, SoftL1/Cauchy rho''<0).
// ---------------------------------------------------------------------------
// kLossScaled: ceres::ScaledLoss(nullptr, scale), internal (the GSBA
// landmark term, geometric_semantic_bundle_adjustment.cc:758-762).
enum LossType { kLossTrivial = 0, kLossSoftL1 = 1, kLossCauchy = 2, kLossScaled = 3 };

MI_HD void loss_eval(int type, double scale, double s, double rho[3]) {
  if (type == kLossScaled) {
    rho[0] = scale * s;
    rho[1] = scale;
    rho[2] = 0.0;
  } else if (type == kLossSoftL1) {
    const double b = scale * scale, c = 1.0 / b;
    const double sum = 1.0 + s * c;
    const double tmp = sqrt(sum);
    rho[0] = 2.0 * b * (tmp - 1.0);
    rho[1] = fmax(2.2250738585072014e-308, 1.0 / tmp);
    rho[2] = -(c * rho[1]) / (2.0 * sum);
  } else if (type == kLossCauchy) {
    const double b = scale * scale, c = 1.0 / b;
    const double sum = 1.0 + s * c;
    const double inv = 1.0 / sum;
    rho[0] = b * log(sum);
    rho[1] = fmax(2.2250738585072014e-308, inv);
    rho[2] = -c * (inv * inv);
  } else {
    rho[0] = s;
    rho[1] = 1.0;
    rho[2] = 0.0;
  }
}

// static_cast<int>(double) as executed by the reference's x86-64 build
// (cvttsd2si: NaN / out of range -> INT_MIN); gfx950's conversion saturates,
// so the bounds are handled explicitly.
MI_HD int32_t cast_to_int_x86(double x) {
  if (!(x > -2147483649.0 && x < 2147483648.0)) return (int32_t)0x80000000;
  return (int32_t)x;
}

}  // namespace miba
