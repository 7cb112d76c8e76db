// oracle_math.h — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's per-observation math, used by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER.
// The product (semantic-bundle-adjustment-colmap_amd/csrc) never includes or
// links this file.
//
// Reference (AlainSchoebi/semantic-bundle-adjustment-colmap, read as text):
//   camera models        src/base/camera_models.h:545-588 (IterativeUndistortion),
//                        :614-637 (SIMPLE_PINHOLE), :640-690 (PINHOLE),
//                        :714-757 (SIMPLE_RADIAL), :760-810 (RADIAL),
//                        :853-902 (OPENCV)
//   rotation helpers     Ceres 2.1 rotation.h (3rd party, not vendored):
//                        UnitQuaternionRotatePoint, QuaternionRotatePoint,
//                        QuaternionToScaledRotation / QuaternionToRotation
//                        (restated);
//                        src/util/rotation_extension.h:43-98 (PoseInverse,
//                        QuaternionInverseRotation, PoseTransformPoint)
//   quaternion manifold  Ceres 2.1 QuaternionManifold::PlusJacobian (restated)
//
// Compiled with -ffp-contract=off: the reference is built for baseline x86-64
// (no FMA contraction), so every product/sum rounds separately, as here.
#pragma once

#include <cmath>
#include <cstdint>
#include <limits>

namespace oracle {

// ---------------------------------------------------------------------------
// Minimal forward-mode dual number (the arithmetic of ceres::Jet), so that the
// oracle's Jacobians come from differentiating the reference formulas exactly
// as AutoDiffCostFunction does — independent of the GPU's hand-derived ones.
// ---------------------------------------------------------------------------
template <int N>
struct Jet {
  double a;
  double v[N];
  Jet() : a(0) { for (int i = 0; i < N; ++i) v[i] = 0; }
  explicit Jet(double x) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; }
  Jet(double x, int k) : a(x) {
    for (int i = 0; i < N; ++i) v[i] = 0;
    v[k] = 1.0;
  }
};
template <int N> inline Jet<N> operator+(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> h(f.a + g.a); for (int i = 0; i < N; ++i) h.v[i] = f.v[i] + g.v[i]; return h;
}
template <int N> inline Jet<N> operator-(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> h(f.a - g.a); for (int i = 0; i < N; ++i) h.v[i] = f.v[i] - g.v[i]; return h;
}
template <int N> inline Jet<N> operator-(const Jet<N>& f) {
  Jet<N> h(-f.a); for (int i = 0; i < N; ++i) h.v[i] = -f.v[i]; return h;
}
template <int N> inline Jet<N> operator*(const Jet<N>& f, const Jet<N>& g) {
  Jet<N> h(f.a * g.a);
  for (int i = 0; i < N; ++i) h.v[i] = f.a * g.v[i] + f.v[i] * g.a;
  return h;
}
template <int N> inline Jet<N> operator*(double s, const Jet<N>& f) {
  Jet<N> h(s * f.a); for (int i = 0; i < N; ++i) h.v[i] = s * f.v[i]; return h;
}
template <int N> inline Jet<N> operator*(const Jet<N>& f, double s) {
  Jet<N> h(f.a * s); for (int i = 0; i < N; ++i) h.v[i] = f.v[i] * s; return h;
}
// ceres jet.h operator/: a_inverse = 1/g.a; abyb = f.a*a_inverse;
// (f.v - abyb*g.v) * a_inverse
template <int N> inline Jet<N> operator/(const Jet<N>& f, const Jet<N>& g) {
  const double a_inverse = 1.0 / g.a;
  const double abyb = f.a * a_inverse;
  Jet<N> h(abyb);
  for (int i = 0; i < N; ++i) h.v[i] = (f.v[i] - abyb * g.v[i]) * a_inverse;
  return h;
}
template <int N> inline Jet<N>& operator+=(Jet<N>& f, const Jet<N>& g) { f = f + g; return f; }
template <int N> inline Jet<N>& operator-=(Jet<N>& f, const Jet<N>& g) { f = f - g; return f; }
template <int N> inline Jet<N>& operator/=(Jet<N>& f, const Jet<N>& g) { f = f / g; return f; }

inline double T2(double) { return 2.0; }
template <typename T> inline T Const(double x) { return T(x); }

// ---------------------------------------------------------------------------
// Ceres rotation.h (restated; Ceres 2.1 is not vendored in the reference).
// ---------------------------------------------------------------------------
template <typename T>
inline void UnitQuaternionRotatePoint(const T q[4], const T pt[3], T result[3]) {
  const T t2 = q[0] * q[1];
  const T t3 = q[0] * q[2];
  const T t4 = q[0] * q[3];
  const T t5 = -(q[1] * q[1]);
  const T t6 = q[1] * q[2];
  const T t7 = q[1] * q[3];
  const T t8 = -(q[2] * q[2]);
  const T t9 = q[2] * q[3];
  const T t1 = -(q[3] * q[3]);
  const T two(2.0);
  result[0] = two * ((t8 + t1) * pt[0] + (t6 - t4) * pt[1] + (t3 + t7) * pt[2]) + pt[0];
  result[1] = two * ((t4 + t6) * pt[0] + (t5 + t1) * pt[1] + (t9 - t2) * pt[2]) + pt[1];
  result[2] = two * ((t7 - t3) * pt[0] + (t2 + t9) * pt[1] + (t5 + t8) * pt[2]) + pt[2];
}

inline void QuaternionRotatePoint(const double q[4], const double pt[3], double result[3]) {
  const double scale = 1.0 / std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const double unit[4] = {scale * q[0], scale * q[1], scale * q[2], scale * q[3]};
  UnitQuaternionRotatePoint(unit, pt, result);
}

// QuaternionToRotation (row-major R) = QuaternionToScaledRotation * 1/|q|^2
inline void QuaternionToRotation(const double q[4], double R[9]) {
  const double a = q[0], b = q[1], c = q[2], d = q[3];
  const double aa = a * a, ab = a * b, ac = a * c, ad = a * d;
  const double bb = b * b, bc = b * c, bd = b * d;
  const double cc = c * c, cd = c * d, dd = d * d;
  R[0] = aa + bb - cc - dd; R[1] = 2.0 * (bc - ad);  R[2] = 2.0 * (ac + bd);
  R[3] = 2.0 * (ad + bc);  R[4] = aa - bb + cc - dd; R[5] = 2.0 * (cd - ab);
  R[6] = 2.0 * (bd - ac);  R[7] = 2.0 * (ab + cd);  R[8] = aa - bb - cc + dd;
  double normalizer = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  normalizer = 1.0 / normalizer;
  for (int i = 0; i < 9; ++i) R[i] *= normalizer;
}

// rotation_extension.h:65-79
inline void QuaternionInverseRotation(const double q[4], double q_inverse[4]) {
  const double scale = 1.0 / std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const double unit[4] = {scale * q[0], scale * q[1], scale * q[2], scale * q[3]};
  q_inverse[0] = unit[0];
  q_inverse[1] = -unit[1];
  q_inverse[2] = -unit[2];
  q_inverse[3] = -unit[3];
}

// rotation_extension.h:43-57
inline void PoseInverse(const double q[4], const double t[3], double q_inv[4], double t_inv[3]) {
  QuaternionInverseRotation(q, q_inv);
  double R[9];
  QuaternionToRotation(q_inv, R);
  t_inv[0] = -(R[0] * t[0] + R[1] * t[1] + R[2] * t[2]);
  t_inv[1] = -(R[3] * t[0] + R[4] * t[1] + R[5] * t[2]);
  t_inv[2] = -(R[6] * t[0] + R[7] * t[1] + R[8] * t[2]);
}

// rotation_extension.h:81-88
inline void PoseTransformPoint(const double q[4], const double t[3], const double pt[3], double r[3]) {
  QuaternionRotatePoint(q, pt, r);
  r[0] += t[0];
  r[1] += t[1];
  r[2] += t[2];
}

// Ceres 2.1 QuaternionManifold::PlusJacobian, 4x3 row-major.
inline void QuaternionPlusJacobian(const double x[4], double J[12]) {
  J[0] = -x[1]; J[1] = -x[2];  J[2] = -x[3];
  J[3] = x[0];  J[4] = x[3];   J[5] = -x[2];
  J[6] = -x[3]; J[7] = x[0];   J[8] = x[1];
  J[9] = x[2];  J[10] = -x[1]; J[11] = x[0];
}

// Ceres 2.1 QuaternionManifold::Plus: [cos|d|, sin|d|/|d| d] (x) x
inline void QuaternionPlus(const double x[4], const double delta[3], double out[4]) {
  const double norm_delta = std::sqrt(delta[0] * delta[0] + delta[1] * delta[1] + delta[2] * delta[2]);
  if (norm_delta == 0.0) {
    for (int i = 0; i < 4; ++i) out[i] = x[i];
    return;
  }
  const double sin_delta_by_delta = std::sin(norm_delta) / norm_delta;
  const double q_delta[4] = {std::cos(norm_delta), sin_delta_by_delta * delta[0],
                             sin_delta_by_delta * delta[1], sin_delta_by_delta * delta[2]};
  // QuaternionProduct(q_delta, x)
  out[0] = q_delta[0] * x[0] - q_delta[1] * x[1] - q_delta[2] * x[2] - q_delta[3] * x[3];
  out[1] = q_delta[0] * x[1] + q_delta[1] * x[0] + q_delta[2] * x[3] - q_delta[3] * x[2];
  out[2] = q_delta[0] * x[2] - q_delta[1] * x[3] + q_delta[2] * x[0] + q_delta[3] * x[1];
  out[3] = q_delta[0] * x[3] + q_delta[1] * x[2] - q_delta[2] * x[1] + q_delta[3] * x[0];
}

// ---------------------------------------------------------------------------
// Camera models (camera_models.h)
// ---------------------------------------------------------------------------
enum { SIMPLE_PINHOLE = 0, PINHOLE = 1, SIMPLE_RADIAL = 2, RADIAL = 3, OPENCV = 4 };

inline int NumParams(int model) {
  switch (model) {
    case SIMPLE_PINHOLE: return 3;
    case PINHOLE: return 4;
    case SIMPLE_RADIAL: return 4;
    case RADIAL: return 5;
    case OPENCV: return 8;
  }
  return -1;
}

// camera_models.h *::InitializeFocalLengthIdxs / PrincipalPointIdxs / ExtraParamsIdxs
inline void ParamGroups(int model, int* f, int* nf, int* pp, int* npp, int* ex, int* nex) {
  *nf = *npp = *nex = 0;
  switch (model) {
    case SIMPLE_PINHOLE: f[(*nf)++] = 0; pp[(*npp)++] = 1; pp[(*npp)++] = 2; break;
    case PINHOLE: f[(*nf)++] = 0; f[(*nf)++] = 1; pp[(*npp)++] = 2; pp[(*npp)++] = 3; break;
    case SIMPLE_RADIAL: f[(*nf)++] = 0; pp[(*npp)++] = 1; pp[(*npp)++] = 2; ex[(*nex)++] = 3; break;
    case RADIAL: f[(*nf)++] = 0; pp[(*npp)++] = 1; pp[(*npp)++] = 2; ex[(*nex)++] = 3; ex[(*nex)++] = 4; break;
    case OPENCV:
      f[(*nf)++] = 0; f[(*nf)++] = 1; pp[(*npp)++] = 2; pp[(*npp)++] = 3;
      for (int k = 4; k < 8; ++k) ex[(*nex)++] = k;
      break;
  }
}

template <typename T>
inline void Distortion(int model, const T* extra, const T u, const T v, T* du, T* dv) {
  switch (model) {
    case SIMPLE_RADIAL: {  // camera_models.h:746-757
      const T k = extra[0];
      const T u2 = u * u;
      const T v2 = v * v;
      const T r2 = u2 + v2;
      const T radial = k * r2;
      *du = u * radial;
      *dv = v * radial;
      return;
    }
    case RADIAL: {  // camera_models.h:799-810
      const T k1 = extra[0];
      const T k2 = extra[1];
      const T u2 = u * u;
      const T v2 = v * v;
      const T r2 = u2 + v2;
      const T radial = k1 * r2 + k2 * r2 * r2;
      *du = u * radial;
      *dv = v * radial;
      return;
    }
    case OPENCV: {  // camera_models.h:887-902
      const T k1 = extra[0];
      const T k2 = extra[1];
      const T p1 = extra[2];
      const T p2 = extra[3];
      const T u2 = u * u;
      const T uv = u * v;
      const T v2 = v * v;
      const T r2 = u2 + v2;
      const T radial = k1 * r2 + k2 * r2 * r2;
      const T two(2.0);
      *du = u * radial + two * p1 * uv + p2 * (r2 + two * u2);
      *dv = v * radial + two * p2 * uv + p1 * (r2 + two * v2);
      return;
    }
    default:
      *du = T(0.0);
      *dv = T(0.0);
  }
}

template <typename T>
inline void WorldToImage(int model, const T* params, const T u, const T v, T* x, T* y) {
  switch (model) {
    case SIMPLE_PINHOLE: {  // :614-626
      const T f = params[0], c1 = params[1], c2 = params[2];
      *x = f * u + c1;
      *y = f * v + c2;
      return;
    }
    case PINHOLE: {
      const T f1 = params[0], f2 = params[1], c1 = params[2], c2 = params[3];
      *x = f1 * u + c1;
      *y = f2 * v + c2;
      return;
    }
    case SIMPLE_RADIAL:
    case RADIAL: {  // :714-730
      const T f = params[0], c1 = params[1], c2 = params[2];
      T du, dv;
      Distortion(model, &params[3], u, v, &du, &dv);
      *x = u + du;
      *y = v + dv;
      *x = f * *x + c1;
      *y = f * *y + c2;
      return;
    }
    case OPENCV: {  // :853-870
      const T f1 = params[0], f2 = params[1], c1 = params[2], c2 = params[3];
      T du, dv;
      Distortion(model, &params[4], u, v, &du, &dv);
      *x = u + du;
      *y = v + dv;
      *x = f1 * *x + c1;
      *y = f2 * *y + c2;
      return;
    }
  }
}

// camera_models.h:545-588 (Eigen 2x2 inverse: invdet = 1/det,
// det = m00*m11 - m10*m01)
inline void IterativeUndistortion(int model, const double* extra, double* u, double* v) {
  const int kNumIterations = 100;
  const double kMaxStepNorm = 1e-10;
  const double kRelStepSize = 1e-6;
  const double x0[2] = {*u, *v};
  double x[2] = {*u, *v};
  for (int i = 0; i < kNumIterations; ++i) {
    const double step0 = std::max(std::numeric_limits<double>::epsilon(), std::abs(kRelStepSize * x[0]));
    const double step1 = std::max(std::numeric_limits<double>::epsilon(), std::abs(kRelStepSize * x[1]));
    double dx[2], dx_0b[2], dx_0f[2], dx_1b[2], dx_1f[2];
    Distortion(model, extra, x[0], x[1], &dx[0], &dx[1]);
    Distortion(model, extra, x[0] - step0, x[1], &dx_0b[0], &dx_0b[1]);
    Distortion(model, extra, x[0] + step0, x[1], &dx_0f[0], &dx_0f[1]);
    Distortion(model, extra, x[0], x[1] - step1, &dx_1b[0], &dx_1b[1]);
    Distortion(model, extra, x[0], x[1] + step1, &dx_1f[0], &dx_1f[1]);
    const double J00 = 1 + (dx_0f[0] - dx_0b[0]) / (2 * step0);
    const double J01 = (dx_1f[0] - dx_1b[0]) / (2 * step1);
    const double J10 = (dx_0f[1] - dx_0b[1]) / (2 * step0);
    const double J11 = 1 + (dx_1f[1] - dx_1b[1]) / (2 * step1);
    const double det = J00 * J11 - J10 * J01;
    const double invdet = 1.0 / det;
    const double i00 = J11 * invdet, i01 = -J01 * invdet, i10 = -J10 * invdet, i11 = J00 * invdet;
    const double e0 = x[0] + dx[0] - x0[0];
    const double e1 = x[1] + dx[1] - x0[1];
    const double s0 = i00 * e0 + i01 * e1;
    const double s1 = i10 * e0 + i11 * e1;
    x[0] -= s0;
    x[1] -= s1;
    if (s0 * s0 + s1 * s1 < kMaxStepNorm) break;
  }
  *u = x[0];
  *v = x[1];
}

inline void ImageToWorld(int model, const double* params, double x, double y, double* u, double* v) {
  *u = x;
  *v = y;
  switch (model) {
    case SIMPLE_PINHOLE:
      *u = (x - params[1]) / params[0];
      *v = (y - params[2]) / params[0];
      return;
    case PINHOLE:
      *u = (x - params[2]) / params[0];
      *v = (y - params[3]) / params[1];
      return;
    case SIMPLE_RADIAL:
    case RADIAL:
      *u = (x - params[1]) / params[0];
      *v = (y - params[2]) / params[0];
      IterativeUndistortion(model, &params[3], u, v);
      return;
    case OPENCV:
      *u = (x - params[2]) / params[0];
      *v = (y - params[3]) / params[1];
      IterativeUndistortion(model, &params[4], u, v);
      return;
  }
}

// static_cast<int>(double) as the reference's x86-64 build executes it
// (cvttsd2si): NaN or out-of-range -> INT_MIN.
inline int32_t CastToIntX86(double x) {
  if (!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
  return static_cast<int32_t>(x);
}

}  // namespace oracle
