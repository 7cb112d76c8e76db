// semantic.hip — semantic-label residuals on gfx950 (product code).
//
// Compiled with -ffp-contract=off: the residual is a 0/1 step of rounded
// reprojected pixels, so the evaluation keeps the reference's operation
// order (semantic_cost_functions.h:103-205, rotation_extension.h:43-88)
// without FMA contraction — bitwise identical to the CPU reference build.
//
// One lane per sampled pixel; each lane evaluates the Ceres CENTRAL
// numeric-diff stencil over the ambient pose parameters (1 + 2*7 per
// variable pose: 29 evaluations for a variable-variable block, 15 with one
// constant pose), then applies QuaternionManifold / SubsetManifold.
// Samples are grouped by image pair; one workgroup per pair-aligned tile, so
// the pair's poses are wave-uniform and J'J, J'r reduce in LDS (one atomic
// flush per tile).
#include <hip/hip_runtime.h>

#include <map>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>

#include "ba_math.h"
#include "kernels.h"
#include "semantic.h"

namespace miba {

namespace {

constexpr double kMinStep = 1.4901161193847656e-08;  // sqrt(DBL_EPSILON) = 2^-26

struct SemArgs {
  const SemSample* samples;
  const SemPair* pairs;
  const double* qt;
  const double* cam;
  const uint32_t* img_cam;
  const uint8_t* cam_model;  // [C] model id per camera (mixed-model cost kernel)
  const uint32_t* img_flags;
  const uint32_t* raster_slot;
  const SlotInfo* slots;  // [slot] plane offsets and size of each raster slot
  const float2* dl;   // interleaved (depth, label) rasters, one plane per slot (SlotInfo::off)
  const float4* wsum; // 3x3 window summaries, the rasters' layout (window_summary_kernel) or null
  const uint8_t* lab8; // label planes, the rasters' layout (label_index_kernel) or null
  const float2* dtile; // tile depth ranges, one plane per slot (SlotInfo::toff; depth_tile_kernel)
  const float* pal;    // [256] label values of the lab8 indices
  // the raster of the current pair's second image (per pair: with_pair); 0 in
  // the kernel arguments
  int TW;
  int H, W;
  double threshold;
  double rel_step;
  int64_t ns;
  int loss_type;
  double loss_scale;
  double weight;
};

__device__ inline void quat_rotate_point(const double q[4], const double pt[3], double r[3]) {
  const double scale = 1.0 / sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const double unit[4] = {scale * q[0], scale * q[1], scale * q[2], scale * q[3]};
  unit_quat_rotate(unit, pt, r);
}

// compute_semantic_error (semantic_cost_functions.h:87-208), the reference's
// operation sequence.
// pw_out / pxy_out (nullable): the world point and the rounded pixel in image
// 2 (compute_semantic_error's return_point3D / return_point2D_2).
template <int M>
__device__ inline double semantic_error(const SemArgs& a, const double pc1[3], float label1, const double* q1,
                                        const double* t1, const double* q2, const double* t2, const double* K2,
                                        const float2* dl2, int* status, double* pw_out = nullptr,
                                        int* pxy_out = nullptr) {
  // PoseInverse (rotation_extension.h:43-57)
  const double sc = 1.0 / sqrt(q1[0] * q1[0] + q1[1] * q1[1] + q1[2] * q1[2] + q1[3] * q1[3]);
  const double qi[4] = {sc * q1[0], -(sc * q1[1]), -(sc * q1[2]), -(sc * q1[3])};
  // QuaternionToRotation(q_inv)
  const double aa = qi[0] * qi[0], ab = qi[0] * qi[1], ac = qi[0] * qi[2], ad = qi[0] * qi[3];
  const double bb = qi[1] * qi[1], bc = qi[1] * qi[2], bd = qi[1] * qi[3];
  const double cc = qi[2] * qi[2], cd = qi[2] * qi[3], dd = qi[3] * qi[3];
  double R[9];
  R[0] = aa + bb - cc - dd; R[1] = 2.0 * (bc - ad);  R[2] = 2.0 * (ac + bd);
  R[3] = 2.0 * (ad + bc);  R[4] = aa - bb + cc - dd; R[5] = 2.0 * (cd - ab);
  R[6] = 2.0 * (bd - ac);  R[7] = 2.0 * (ab + cd);  R[8] = aa - bb - cc + dd;
  double nrm = qi[0] * qi[0] + qi[1] * qi[1] + qi[2] * qi[2] + qi[3] * qi[3];
  nrm = 1.0 / nrm;
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] *= nrm;
  const double ti[3] = {-(R[0] * t1[0] + R[1] * t1[1] + R[2] * t1[2]), -(R[3] * t1[0] + R[4] * t1[1] + R[5] * t1[2]),
                        -(R[6] * t1[0] + R[7] * t1[1] + R[8] * t1[2])};
  // PoseTransformPoint(q_inv, t_inv, P_c1) -> world
  double pw[3];
  quat_rotate_point(qi, pc1, pw);
  pw[0] += ti[0];
  pw[1] += ti[1];
  pw[2] += ti[2];
  if (pw_out) {
    pw_out[0] = pw[0];
    pw_out[1] = pw[1];
    pw_out[2] = pw[2];
  }
  // PoseTransformPoint(q2, t2, P_w) -> camera 2
  double p2[3];
  quat_rotate_point(q2, pw, p2);
  p2[0] += t2[0];
  p2[1] += t2[1];
  p2[2] += t2[2];
  const double u2 = p2[0] / p2[2];
  const double v2 = p2[1] / p2[2];
  const double measured_depth_2 = p2[2];
  double x2, y2;
  world_to_image<M>(K2, u2, v2, &x2, &y2);
  const int px = cast_to_int_x86(round(x2));
  const int py = cast_to_int_x86(round(y2));
  if (pxy_out) {
    pxy_out[0] = px;
    pxy_out[1] = py;
  }
  if (px < 0 || px >= a.W || py < 0 || py >= a.H) {
    *status = MI_BA_OUT_OF_BOUNDS;
    return 0.0;
  }
  const float2 s = dl2[(size_t)py * a.W + px];
  const double depth_2 = (double)s.x;
  if (fabs(depth_2 - measured_depth_2) > a.threshold) {
    *status = MI_BA_INVALID_DEPTH;
    return 0.0;
  }
  *status = MI_BA_VALID;
  return (label1 == s.y) ? 0.0 : 1.0;
}

// ---------------------------------------------------------------------------
// The centre evaluation split into its pose-1 / pose-2 stages (each stage is
// exactly the operation sequence of semantic_error above, so the centre value
// is bitwise the reference's).
// ---------------------------------------------------------------------------
struct Pose1Stage {   // depends on q1 (and P_c1)
  double R[9];        // QuaternionToRotation(q_inv)
  double rot[3];      // QuaternionRotatePoint(q_inv, P_c1)
};

__device__ inline void pose1_stage(const double* q1, const double pc1[3], Pose1Stage& s) {
  const double sc = 1.0 / sqrt(q1[0] * q1[0] + q1[1] * q1[1] + q1[2] * q1[2] + q1[3] * q1[3]);
  const double qi[4] = {sc * q1[0], -(sc * q1[1]), -(sc * q1[2]), -(sc * q1[3])};
  const double aa = qi[0] * qi[0], ab = qi[0] * qi[1], ac = qi[0] * qi[2], ad = qi[0] * qi[3];
  const double bb = qi[1] * qi[1], bc = qi[1] * qi[2], bd = qi[1] * qi[3];
  const double cc = qi[2] * qi[2], cd = qi[2] * qi[3], dd = qi[3] * qi[3];
  s.R[0] = aa + bb - cc - dd; s.R[1] = 2.0 * (bc - ad);  s.R[2] = 2.0 * (ac + bd);
  s.R[3] = 2.0 * (ad + bc);  s.R[4] = aa - bb + cc - dd; s.R[5] = 2.0 * (cd - ab);
  s.R[6] = 2.0 * (bd - ac);  s.R[7] = 2.0 * (ab + cd);  s.R[8] = aa - bb - cc + dd;
  double nrm = qi[0] * qi[0] + qi[1] * qi[1] + qi[2] * qi[2] + qi[3] * qi[3];
  nrm = 1.0 / nrm;
#pragma unroll
  for (int k = 0; k < 9; ++k) s.R[k] *= nrm;
  quat_rotate_point(qi, pc1, s.rot);
}

__device__ inline void unit_quat(const double* q, double u[4]) {
  const double scale = 1.0 / sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  u[0] = scale * q[0];
  u[1] = scale * q[1];
  u[2] = scale * q[2];
  u[3] = scale * q[3];
}

struct PixelCache {   // the centre evaluation's raster read
  int px, py;
  float depth, label;
  bool valid;
};

// Projection into image 2 and the raster tests (semantic_cost_functions.h:141-205),
// reference operation order; records the centre pixel.
template <int M>
__device__ inline double project_centre(const SemArgs& a, const double p2[3], float label1, const double* K2,
                                        const float2* dl2, PixelCache& pc, int* status) {
  const double u2 = p2[0] / p2[2];
  const double v2 = p2[1] / p2[2];
  const double measured_depth_2 = p2[2];
  double x2, y2;
  world_to_image<M>(K2, u2, v2, &x2, &y2);
  const int px = cast_to_int_x86(round(x2));
  const int py = cast_to_int_x86(round(y2));
  if (px < 0 || px >= a.W || py < 0 || py >= a.H) {
    *status = MI_BA_OUT_OF_BOUNDS;
    return 0.0;
  }
  const float2 s = dl2[(size_t)py * a.W + px];
  pc.px = px; pc.py = py; pc.depth = s.x; pc.label = s.y; pc.valid = true;
  if (fabs((double)s.x - measured_depth_2) > a.threshold) {
    *status = MI_BA_INVALID_DEPTH;
    return 0.0;
  }
  *status = MI_BA_VALID;
  return (label1 == s.y) ? 0.0 : 1.0;
}

// ---------------------------------------------------------------------------
// Stencil evaluations.  The residual is a step function: it depends on the
// perturbed evaluation only through round(x2), round(y2) and the sign of
// |depth - z| - threshold.  Each perturbed camera-2 point is therefore formed
// by a cheaper, equally accurate route (unnormalised rotation matrices, one
// reciprocal, the stage quantities of the centre), and its outcome is taken
// when every one of those three decisions clears a margin far above the
// rounding difference between this route and the reference's (both are
// within ~1e-12 px / ~1e-15 |p| of the exact value; the margins are 1e-6 px
// and 1e-9 in depth, scaled by the magnitudes involved).  Otherwise the
// evaluation is redone with the reference operation sequence
// (semantic_error).  The stencil values, hence J, are the reference's
// bit for bit.
// ---------------------------------------------------------------------------
// Unnormalised rotation matrix: Rot(q) v = Q(q) v / |q|^2 (row-major).
__device__ inline void quat_matrix_un(const double q[4], double Q[9]) {
  const double a = q[0], b = q[1], c = q[2], d = q[3];
  const double aa = a * a, bb = b * b, cc = c * c, dd = d * d;
  const double ab = a * b, ac = a * c, ad = a * d, bc = b * c, bd = b * d, cd = c * d;
  Q[0] = aa + bb - cc - dd; Q[1] = 2.0 * (bc - ad);  Q[2] = 2.0 * (ac + bd);
  Q[3] = 2.0 * (bc + ad);  Q[4] = aa - bb + cc - dd; Q[5] = 2.0 * (cd - ab);
  Q[6] = 2.0 * (bd - ac);  Q[7] = 2.0 * (ab + cd);  Q[8] = aa - bb - cc + dd;
}

[[maybe_unused]] __device__ inline double rcp_refined(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  r = fma(r, fma(-x, r, 1.0), r);
  return r;
}

template <int M>
__device__ inline double distortion_gain(const double* K, double r2) {
  constexpr int np = Model<M>::kNumParams;
  double s = 0.0;
  if constexpr (M == kSimpleRadial || M == kRadial) {
#pragma unroll
    for (int k = 3; k < np; ++k) s += fabs(K[k]);
  } else if constexpr (M == kOpenCV) {
#pragma unroll
    for (int k = 4; k < np; ++k) s += fabs(K[k]);
  }
  const double g = 1.0 + r2;
  return 1.0 + s * g * g * g;
}

// The camera models with FMA contraction, for resolve's fast route only (an
// outcome is taken only when it clears resolve's margins, which are orders of
// magnitude above the rounding difference contraction makes; the reference
// operation sequence, semantic_error, stays uncontracted).
template <int M>
__device__ inline void world_to_image_fma(const double* K, double u, double v, double* x, double* y) {
#pragma clang fp contract(fast)
  if constexpr (M == kSimplePinhole) {
    *x = K[0] * u + K[1];
    *y = K[0] * v + K[2];
  } else if constexpr (M == kPinhole) {
    *x = K[0] * u + K[2];
    *y = K[1] * v + K[3];
  } else if constexpr (M == kSimpleRadial || M == kRadial) {
    const double r2 = u * u + v * v;
    double rad = K[3] * r2;
    if constexpr (M == kRadial) rad = rad + K[4] * r2 * r2;
    *x = K[0] * (u + u * rad) + K[1];
    *y = K[0] * (v + v * rad) + K[2];
  } else {
    const double k1 = K[4], k2 = K[5], p1 = K[6], p2 = K[7];
    const double u2 = u * u, uv = u * v, v2 = v * v, r2 = u2 + v2;
    const double rad = k1 * r2 + k2 * r2 * r2;
    const double du = u * rad + 2.0 * p1 * uv + p2 * (r2 + 2.0 * u2);
    const double dv = v * rad + 2.0 * p2 * uv + p1 * (r2 + 2.0 * v2);
    *x = K[0] * (u + du) + K[2];
    *y = K[1] * (v + dv) + K[3];
  }
}

// A p + t, contracted (fast route's perturbed camera-2 point)
__device__ inline void matvec3_t_fma(const double* A, double v0, double v1, double v2, const double* t,
                                     double pp[3]) {
#pragma clang fp contract(fast)
#pragma unroll
  for (int c = 0; c < 3; ++c) pp[c] = A[3 * c] * v0 + A[3 * c + 1] * v1 + A[3 * c + 2] * v2 + t[c];
}

// Outcome of one stencil evaluation from its camera-2 point p; false when a
// decision is inside the margin (caller falls back to semantic_error).
// mag bounds the magnitudes p was formed from (L1 norms).  FAST: the
// projection with FMA contraction (world_to_image_fma).
// FAST also takes the pixel margin's model term from the sample's centre
// (exk = 2e-11 * kscale at the centre, margin_model_term): a stencil point's
// u, v, 1/z differ from the centre's by ~1e-3 relative, so twice the centre's
// bound covers every point of the stencil; and one Newton step of the
// reciprocal (2^-44 relative, ~1e-10 px at 1000 px, far inside the 1e-6 px
// margin).
template <int M>
__device__ inline double margin_model_term(const double* K2, const double p[3], double mag) {
  const double iz = 1.0 / p[2];
  const double u = p[0] * iz, v = p[1] * iz;
  return 2e-11 * (fabs(K2[0]) + fabs(K2[1])) * distortion_gain<M>(K2, u * u + v * v) * (1.0 + fabs(u) + fabs(v)) *
         (1.0 + mag * fabs(iz));
}

template <int M, bool FAST = false>
__device__ inline bool resolve(const SemArgs& a, const double p[3], double mag, float label1, const double* K2,
                               const float2* dl2, const PixelCache& pc, double& f, double exk = 0.0) {
  double iz;
  if constexpr (FAST) {
    const double x0 = p[2];
    double r = __builtin_amdgcn_rcp(x0);
    iz = fma(r, fma(-x0, r, 1.0), r);
  } else {
    iz = rcp_refined(p[2]);
  }
  const double u = p[0] * iz, v = p[1] * iz;
  double x, y;
  if constexpr (FAST)
    world_to_image_fma<M>(K2, u, v, &x, &y);
  else
    world_to_image<M>(K2, u, v, &x, &y);
  if (!(fabs(x) < 1e8 && fabs(y) < 1e8 && fabs(u) < 1e6 && fabs(v) < 1e6)) return false;
  double ex;
  if constexpr (FAST) {
    ex = 1e-6 + exk + 1e-11 * (fabs(x) + fabs(y));
  } else {
    const double kscale = (fabs(K2[0]) + fabs(K2[1])) * distortion_gain<M>(K2, u * u + v * v) *
                          (1.0 + fabs(u) + fabs(v)) * (1.0 + mag * fabs(iz));
    ex = 1e-6 + 1e-11 * (kscale + fabs(x) + fabs(y));
  }
  const double fx = floor(x), fy = floor(y);
  const double rx = x - fx, ry = y - fy;
  if (!(fabs(rx - 0.5) > ex && fabs(ry - 0.5) > ex)) return false;
  const int px = (int)fx + (rx > 0.5 ? 1 : 0);
  const int py = (int)fy + (ry > 0.5 ? 1 : 0);
  if (px < 0 || px >= a.W || py < 0 || py >= a.H) {
    f = 0.0;
    return true;
  }
  float2 s;
  if (pc.valid && px == pc.px && py == pc.py) {
    s = make_float2(pc.depth, pc.label);
  } else {
    s = dl2[(size_t)py * a.W + px];
  }
  const double dd = fabs((double)s.x - p[2]) - a.threshold;
  if (!(fabs(dd) > 1e-9 * (1.0 + fabs((double)s.x) + mag))) return false;
  f = (dd > 0.0) ? 0.0 : ((label1 == s.y) ? 0.0 : 1.0);
  return true;
}

// Per-pair constants of one linearization (pose dependent, sample
// independent), formed with the reference's operation sequence so that the
// per-sample centre evaluation continues it bit for bit.  Every workgroup
// works on one pair, so these are wave-uniform (scalar loads/registers).
struct PairConst {
  double q1[4], t1[3], q2[4], t2[3];  // raw parameters (stencil base)
  double uqi[4];                      // normalised q_inv as QuaternionRotatePoint uses it
  double ti[3];                       // t_inv = -(R t1)
  double u2[4];                       // normalised q2
  double R2[9];                       // rotation of u2 (stencil)
  double C[9];                        // R2 R: d P_2 / d t1 = -C (stencil)
  double K2[8];                       // camera of image j
  uint32_t var1, var2, mask1, mask2;  // variable poses, constant-tvec masks
  uint32_t slot, H2, W2, TW2;        // image j's raster slot, its size, its tiles per row
  uint64_t roff, toff;                // its plane in the rasters / label planes, in the tiles
  // stencil tables, e = 2 m + minus over the 14 ambient parameters
  double pert[28];                    // perturbed parameter value
  double ood[14];                     // (1 / delta) / 2, Ceres CENTRAL
  double A[16][9];                    // q1 points (e 0..7): R2 Q(q1')^T / |q1'|^2; q2 (e 14..21): Q(q2') / |q2'|^2
  double pj[8][3];                    // PlusJacobian rows of q1 (0..3) and q2 (4..7)
  // displacement bounds of the camera-2 point over the stencil (flat test):
  // |P_2' - P_2| <= rho1 |P_c1 - t1| (q1 points), rho2 |P_w| (q2 points);
  // t1 point k moves it by dt1[k] C[:, k], t2 point k by dt2[k] e_k
  double rho1, rho2, dt1[3], dt2[3];
};

// The kernel arguments with the pair's second-image raster size (image j's own
// H x W: the bounds test of semantic_cost_functions.h:163).
__device__ __forceinline__ SemArgs with_pair(const SemArgs& ak, const PairConst* __restrict__ P) {
  SemArgs a = ak;
  a.H = (int)P->H2;
  a.W = (int)P->W2;
  a.TW = (int)P->TW2;
  return a;
}

// Bounds of one pose's stencil (the flat test): a perturbed quaternion q' =
// q + d e_k rotates by ||R(q') - R(q)|| = 2 sin(angle(q, q')) <= 2 d_perp /
// (|q| - d), d_perp = d sqrt(1 - q_k^2 / |q|^2) the step's component normal
// to q; a translation step moves the point by d.  d is the stencil's actual
// |q_k' - q_k| (Ceres' delta, as stencil_prep forms it).
__device__ inline void stencil_bounds(const double* q, const double* t, double rel_step, double* rho, double dt[3]) {
  const double nq2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  const double nq = sqrt(nq2);
  double r = 0.0;
  for (int k = 0; k < 4; ++k) {
    const double delta = fmax(kMinStep, fabs(q[k]) * rel_step);
    const double d = fmax(fabs((q[k] + delta) - q[k]), fabs(q[k] - (q[k] - delta)));
    const double perp = d * sqrt(fmax(0.0, 1.0 - q[k] * q[k] / nq2));
    const double den = nq - d;
    r = fmax(r, den > 0.0 ? 2.0 * perp / den : INFINITY);
  }
  *rho = r * 1.001;
  for (int k = 0; k < 3; ++k) {
    const double delta = fmax(kMinStep, fabs(t[k]) * rel_step);
    dt[k] = fmax(fabs((t[k] + delta) - t[k]), fabs(t[k] - (t[k] - delta))) * 1.001;
  }
}

// Stencil entries of one pair: one lane per stencil point (perturbed value,
// the Ceres step 1/(2 delta) with the lane-side operation sequence of the
// reference, the perturbed rotation map).
__device__ inline void stencil_prep(const double* q1, const double* t1, const double* q2, const double* t2,
                                    double rel_step, int e, PairConst* __restrict__ P) {
  const int m = e >> 1;
  const bool minus = e & 1;
  const int grp = m < 4 ? 0 : (m < 7 ? 1 : (m < 11 ? 2 : 3));
  const int k = m - (grp == 0 ? 0 : (grp == 1 ? 4 : (grp == 2 ? 7 : 11)));
  const double orig = grp == 0 ? q1[k] : (grp == 1 ? t1[k] : (grp == 2 ? q2[k] : t2[k]));
  const double delta = fmax(kMinStep, fabs(orig) * rel_step);
  const double pert = minus ? orig - delta : orig + delta;
  P->pert[e] = pert;
  if (minus) {
    double one_over_delta = 1.0 / delta;
    one_over_delta /= 2;
    P->ood[m] = one_over_delta;
  }
  if (grp == 1 || grp == 3) return;
  const double* q = grp == 0 ? q1 : q2;
  double qq[4] = {q[0], q[1], q[2], q[3]};
  qq[k] = pert;
  double Q[9];
  quat_matrix_un(qq, Q);
  const double in = 1.0 / (qq[0] * qq[0] + qq[1] * qq[1] + qq[2] * qq[2] + qq[3] * qq[3]);
  double* A = P->A[grp == 0 ? e : e - 6];
  if (grp == 0) {
    double u2[4], R2[9];
    unit_quat(q2, u2);
    unit_quat_matrix(u2, R2);
    for (int r = 0; r < 3; ++r)
      for (int j = 0; j < 3; ++j)
        A[3 * r + j] = (R2[3 * r] * Q[3 * j] + R2[3 * r + 1] * Q[3 * j + 1] + R2[3 * r + 2] * Q[3 * j + 2]) * in;
  } else {
    for (int c = 0; c < 9; ++c) A[c] = Q[c] * in;
  }
  if (minus) {
    double PJ[12];
    quat_plus_jacobian(q, PJ);
    for (int c = 0; c < 3; ++c) P->pj[(grp == 0 ? 0 : 4) + k][c] = PJ[3 * k + c];
  }
}

// Two pairs per 64-lane workgroup: lanes 0..27 of each half fill the stencil
// tables, lane 28 the pair's base constants.  The pair's accumulator record
// (blk_stride doubles of pair_blk) and deferred-sample count are cleared here
// too (two launches fewer than separate memsets).
__global__ void semantic_pair_prep_kernel(const SemPair* __restrict__ pairs, int npairs, const double* __restrict__ qt,
                                          const double* __restrict__ cam, const uint32_t* __restrict__ img_cam,
                                          const uint32_t* __restrict__ img_flags,
                                          const uint32_t* __restrict__ raster_slot,
                                          const SlotInfo* __restrict__ slots, double rel_step,
                                          PairConst* __restrict__ out, double* __restrict__ pair_blk, int blk_stride,
                                          uint32_t* __restrict__ pair_cnt, uint32_t* __restrict__ zero_n = nullptr,
                                          int nzero = 0) {
  const int k = blockIdx.x * 2 + (threadIdx.x >> 5);
  const int lane = threadIdx.x & 31;
  if (zero_n && blockIdx.x == 0 && (int)threadIdx.x < nzero) zero_n[threadIdx.x] = 0u;  // the deferred pass's counts
  if (k >= npairs) return;
  for (int e = lane; e < blk_stride; e += 32) pair_blk[(size_t)k * blk_stride + e] = 0.0;
  if (pair_cnt && lane == 31) pair_cnt[k] = 0u;
  if (lane > 28) return;
  const SemPair pr = pairs[k];
  if (lane < 28) {
    const double* a1 = qt + 8 * (size_t)pr.i;
    const double* a2 = qt + 8 * (size_t)pr.j;
    const double q1[4] = {a1[0], a1[1], a1[2], a1[3]}, t1[3] = {a1[4], a1[5], a1[6]};
    const double q2[4] = {a2[0], a2[1], a2[2], a2[3]}, t2[3] = {a2[4], a2[5], a2[6]};
    stencil_prep(q1, t1, q2, t2, rel_step, lane, out + k);
    return;
  }
  PairConst& P = out[k];
  const double* a1 = qt + 8 * (size_t)pr.i;
  const double* a2 = qt + 8 * (size_t)pr.j;
  for (int m = 0; m < 4; ++m) { P.q1[m] = a1[m]; P.q2[m] = a2[m]; }
  for (int m = 0; m < 3; ++m) { P.t1[m] = a1[4 + m]; P.t2[m] = a2[4 + m]; }
  // PoseInverse + QuaternionToRotation (pose1_stage), t_inv (pose1_world)
  Pose1Stage s;
  const double zero[3] = {0.0, 0.0, 0.0};
  pose1_stage(P.q1, zero, s);
  {
    const double* q1 = P.q1;
    const double sc = 1.0 / sqrt(q1[0] * q1[0] + q1[1] * q1[1] + q1[2] * q1[2] + q1[3] * q1[3]);
    const double qi[4] = {sc * q1[0], -(sc * q1[1]), -(sc * q1[2]), -(sc * q1[3])};
    // quat_rotate_point(qi, .) normalisation
    const double scale = 1.0 / sqrt(qi[0] * qi[0] + qi[1] * qi[1] + qi[2] * qi[2] + qi[3] * qi[3]);
    for (int m = 0; m < 4; ++m) P.uqi[m] = scale * qi[m];
  }
  P.ti[0] = -(s.R[0] * P.t1[0] + s.R[1] * P.t1[1] + s.R[2] * P.t1[2]);
  P.ti[1] = -(s.R[3] * P.t1[0] + s.R[4] * P.t1[1] + s.R[5] * P.t1[2]);
  P.ti[2] = -(s.R[6] * P.t1[0] + s.R[7] * P.t1[1] + s.R[8] * P.t1[2]);
  unit_quat(P.q2, P.u2);
  unit_quat_matrix(P.u2, P.R2);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      P.C[3 * r + c] = P.R2[3 * r] * s.R[c] + P.R2[3 * r + 1] * s.R[3 + c] + P.R2[3 * r + 2] * s.R[6 + c];
  const double* K = cam + 8 * (size_t)img_cam[pr.j];
  for (int m = 0; m < 8; ++m) P.K2[m] = K[m];
  P.var1 = pr.var1;
  P.var2 = pr.var2;
  P.mask1 = (img_flags[pr.i] >> 1) & 7u;
  P.mask2 = (img_flags[pr.j] >> 1) & 7u;
  P.slot = raster_slot[pr.j];
  const SlotInfo si = slots[P.slot];
  P.H2 = (uint32_t)si.H;
  P.W2 = (uint32_t)si.W;
  P.TW2 = (uint32_t)si.TW;
  P.roff = si.off;
  P.toff = si.toff;
  stencil_bounds(P.q1, P.t1, rel_step, &P.rho1, P.dt1);
  stencil_bounds(P.q2, P.t2, rel_step, &P.rho2, P.dt2);
}

// Per-pair record: loss-corrected J'J (packed 12x12 upper, 78) and J'r (12).
constexpr int kPairVals = 78 + 12;
constexpr int kPairStride = 96;  // padded record per pair
constexpr int kSemRow = 13;      // LDS row: corrected J (12), corrected r

// One workgroup per pair-aligned tile of <= 256 samples, one lane per sample:
// centre residual (reference sequence), the CENTRAL stencil over the
// variable poses' ambient parameters (rolled loop, outcome resolution above),
// QuaternionManifold / SubsetManifold, the ScaledLoss Corrector, and the
// tile's J'J / J'r / cost reduced in LDS with one atomic flush per value.
// Per-sample r / status / J are stored only when requested (parity and
// download); the solver consumes the pair records.
// Reference-order evaluation of one stencil point (the fallback when
// resolve's margins are not cleared), out of line: four group loops share it.
template <int M>
__device__ __forceinline__ double stencil_reference(const SemArgs& a, const PairConst* __restrict__ P, int grp, int k,
                                                 double pert, const double pc1[3], float label1, const double* K2,
                                                 const float2* dl2) {
  double qq1[4], tt1[3], qq2[4], tt2[3];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    qq1[c] = (grp == 0 && c == k) ? pert : P->q1[c];
    qq2[c] = (grp == 2 && c == k) ? pert : P->q2[c];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    tt1[c] = (grp == 1 && c == k) ? pert : P->t1[c];
    tt2[c] = (grp == 3 && c == k) ? pert : P->t2[c];
  }
  int st2;
  return semantic_error<M>(a, pc1, label1, qq1, tt1, qq2, tt2, K2, dl2, &st2);
}

// One stencil point e (ambient coordinate k of group GRP: 0 q1, 1 t1, 2 q2,
// 3 t2): the perturbed camera-2 point from the pair table, its outcome by
// resolve, or the reference sequence inside the margins.
template <bool FAST, int GRP>
__device__ __forceinline__ void stencil_pp(const PairConst* __restrict__ P, int e, int k, const double w[3],
                                           const double pw[3], const double p2[3], double pp[3]) {
  if constexpr (GRP == 0 || GRP == 2) {
    // q1: P_2' = R2 Q(q1')^T (P_c1 - t1) / |q1'|^2 + t2;  q2: P_2' = Q(q2') P_w / |q2'|^2 + t2
    const double* A = P->A[GRP == 0 ? e : e - 6];
    const double* v = GRP == 0 ? w : pw;
    if constexpr (FAST) {
      matvec3_t_fma(A, v[0], v[1], v[2], P->t2, pp);
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c) pp[c] = A[3 * c] * v[0] + A[3 * c + 1] * v[1] + A[3 * c + 2] * v[2] + P->t2[c];
    }
  } else if constexpr (GRP == 1) {  // t1: P_2' = P_2 - C (t1' - t1)
    const double dt = P->pert[e] - P->t1[k];
#pragma unroll
    for (int c = 0; c < 3; ++c) pp[c] = p2[c] - dt * P->C[3 * c + k];
  } else {  // t2: P_2' = P_2 + (t2' - t2)
    const double dt = P->pert[e] - P->t2[k];
#pragma unroll
    for (int c = 0; c < 3; ++c) pp[c] = p2[c] + (c == k ? dt : 0.0);
  }
}

template <int M, bool FAST, int GRP>
__device__ __forceinline__ double stencil_point(const SemArgs& a, const PairConst* __restrict__ P, int e, int k,
                                                const double w[3], const double pw[3], const double p2[3],
                                                double mag, const double pc1[3], float label1, const double* K2,
                                                const float2* dl2, const PixelCache& pc, double exk) {
  const double pert = P->pert[e];
  double pp[3];
  stencil_pp<FAST, GRP>(P, e, k, w, pw, p2, pp);
  double f;
  if (!resolve<M, FAST>(a, pp, mag, label1, K2, dl2, pc, f, exk))
    f = stencil_reference<M>(a, P, GRP, k, pert, pc1, label1, K2, dl2);
  return f;
}

// The per-point route over every variable pose (one rolled loop per parameter
// group, so the tangent row stays in registers): tangent columns accumulate
// from 0.0 in m order, exactly as J_tangent = J_ambient * PlusJacobian does.
template <int M, bool FAST>
__device__ __forceinline__ void stencil_rolled(const SemArgs& a, const PairConst* __restrict__ P, const double w[3],
                                               const double pw[3], const double p2[3], double mag, const double pc1[3],
                                               float label1, const double* K2, const float2* dl2, const PixelCache& pc,
                                               double exk, double Jt[12]) {
  double jq1[3] = {0.0, 0.0, 0.0}, jt1[3] = {0.0, 0.0, 0.0}, jq2[3] = {0.0, 0.0, 0.0}, jt2[3] = {0.0, 0.0, 0.0};
  if (P->var1) {
#pragma unroll 1
    for (int m = 0; m < 4; ++m) {
      double fp = 0.0, fm = 0.0;
#pragma unroll 1
      for (int sg = 0; sg < 2; ++sg) {
        const double f = stencil_point<M, FAST, 0>(a, P, 2 * m + sg, m, w, pw, p2, mag, pc1, label1, K2, dl2, pc, exk);
        fp = sg == 0 ? f : fp;
        fm = sg == 1 ? f : fm;
      }
      const double jm = (fp - fm) * P->ood[m];
      const double* pj = P->pj[m];
#pragma unroll
      for (int c = 0; c < 3; ++c) jq1[c] = jq1[c] + jm * pj[c];
    }
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
      const int m = 4 + k;
      double fp = 0.0, fm = 0.0;
#pragma unroll 1
      for (int sg = 0; sg < 2; ++sg) {
        const double f = stencil_point<M, FAST, 1>(a, P, 2 * m + sg, k, w, pw, p2, mag, pc1, label1, K2, dl2, pc, exk);
        fp = sg == 0 ? f : fp;
        fm = sg == 1 ? f : fm;
      }
      const double jm = (fp - fm) * P->ood[m];
      const double v = ((P->mask1 >> k) & 1u) ? 0.0 : jm;
#pragma unroll
      for (int c = 0; c < 3; ++c) jt1[c] = c == k ? v : jt1[c];
    }
  }
  if (P->var2) {
#pragma unroll 1
    for (int k = 0; k < 4; ++k) {
      const int m = 7 + k;
      double fp = 0.0, fm = 0.0;
#pragma unroll 1
      for (int sg = 0; sg < 2; ++sg) {
        const double f = stencil_point<M, FAST, 2>(a, P, 2 * m + sg, k, w, pw, p2, mag, pc1, label1, K2, dl2, pc, exk);
        fp = sg == 0 ? f : fp;
        fm = sg == 1 ? f : fm;
      }
      const double jm = (fp - fm) * P->ood[m];
      const double* pj = P->pj[4 + k];
#pragma unroll
      for (int c = 0; c < 3; ++c) jq2[c] = jq2[c] + jm * pj[c];
    }
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
      const int m = 11 + k;
      double fp = 0.0, fm = 0.0;
#pragma unroll 1
      for (int sg = 0; sg < 2; ++sg) {
        const double f = stencil_point<M, FAST, 3>(a, P, 2 * m + sg, k, w, pw, p2, mag, pc1, label1, K2, dl2, pc, exk);
        fp = sg == 0 ? f : fp;
        fm = sg == 1 ? f : fm;
      }
      const double jm = (fp - fm) * P->ood[m];
      const double v = ((P->mask2 >> k) & 1u) ? 0.0 : jm;
#pragma unroll
      for (int c = 0; c < 3; ++c) jt2[c] = c == k ? v : jt2[c];
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    Jt[c] = jq1[c];
    Jt[3 + c] = jt1[c];
    Jt[6 + c] = jq2[c];
    Jt[9 + c] = jt2[c];
  }
}

// ---------------------------------------------------------------------------
// Batched stencil.  The per-point route waits on one raster read per stencil
// point (a dependent gather inside a rolled loop: ~29 serial memory round
// trips per wave).  Here a step of NB parameters (2 NB points) forms every
// perturbed pixel first, issues the step's raster reads together and then
// takes the decisions — the same decisions with the same margins as resolve.
// A point whose decision falls inside a margin does not fall back on its own:
// it marks the sample, and the sample is redone by the per-point route
// (stencil_rolled, which falls back to the reference sequence), so the
// values stay the reference's bit for bit.
// ---------------------------------------------------------------------------
struct FlatBox {
  int x0, y0, ncol, nrow;  // reachable pixels (x0 .. x0 + ncol - 1, y0 .. y0 + nrow - 1)
  double d;                // bound of the depth change
};

// First half of resolve: 0 = inside a pixel margin (redo), 1 = out of bounds
// (f = 0), 2 = raster test at *idx (pixel *pxo, *pyo) needed.
template <int M, bool FAST>
__device__ __forceinline__ int probe_pixel(const SemArgs& a, const double p[3], double mag, const double* K2,
                                           double exk, int* idx, int* pxo = nullptr, int* pyo = nullptr) {
  double iz;
  if constexpr (FAST) {
    const double x0 = p[2];
    double r = __builtin_amdgcn_rcp(x0);
    iz = fma(r, fma(-x0, r, 1.0), r);
  } else {
    iz = rcp_refined(p[2]);
  }
  const double u = p[0] * iz, v = p[1] * iz;
  double x, y;
  if constexpr (FAST)
    world_to_image_fma<M>(K2, u, v, &x, &y);
  else
    world_to_image<M>(K2, u, v, &x, &y);
  if (!(fabs(x) < 1e8 && fabs(y) < 1e8 && fabs(u) < 1e6 && fabs(v) < 1e6)) return 0;
  double ex;
  if constexpr (FAST) {
    ex = 1e-6 + exk + 1e-11 * (fabs(x) + fabs(y));
  } else {
    const double kscale = (fabs(K2[0]) + fabs(K2[1])) * distortion_gain<M>(K2, u * u + v * v) *
                          (1.0 + fabs(u) + fabs(v)) * (1.0 + mag * fabs(iz));
    ex = 1e-6 + 1e-11 * (kscale + fabs(x) + fabs(y));
  }
  const double fx = floor(x), fy = floor(y);
  const double rx = x - fx, ry = y - fy;
  if (!(fabs(rx - 0.5) > ex && fabs(ry - 0.5) > ex)) return 0;
  const int px = (int)fx + (rx > 0.5 ? 1 : 0);
  const int py = (int)fy + (ry > 0.5 ? 1 : 0);
  if (px < 0 || px >= a.W || py < 0 || py >= a.H) return 1;
  *idx = py * a.W + px;
  if (pxo) {
    *pxo = px;
    *pyo = py;
  }
  return 2;
}

// Second half of resolve: the depth decision (false = inside its margin).
__device__ __forceinline__ bool probe_depth(const SemArgs& a, float2 s, double z, double mag, float label1,
                                            double* f) {
  const double dd = fabs((double)s.x - z) - a.threshold;
  if (!(fabs(dd) > 1e-9 * (1.0 + fabs((double)s.x) + mag))) return false;
  *f = (dd > 0.0) ? 0.0 : ((label1 == s.y) ? 0.0 : 1.0);
  return true;
}

// One step: parameters k0 .. k0 + NB - 1 (< n) of group GRP, global index
// m0 + j for parameter k0 + j; fp / fm the + / - values.  cidx: a pixel the
// lane has read already (the centre's), read again by points with no raster
// test so that every read of the step issues unconditionally.
// box (nullable): the sample's reachable 3 x 3 box of raster pixels (fb), read
// once into the lane's LDS slot: every stencil point's pixel lies in it (the
// flat test's bound), so the step takes its pixels from LDS instead of the
// raster (a pixel outside it, which the bound rules out, is read from the
// raster all the same).
template <int M, bool FAST, int GRP, int NB>
__device__ __forceinline__ bool stencil_step(const SemArgs& a, const PairConst* __restrict__ P, int m0, int k0, int n,
                                             const double w[3], const double pw[3], const double p2[3], double mag,
                                             float label1, const double* K2, const float2* __restrict__ dl2, int cidx,
                                             double exk, double fp[NB], double fm[NB], const float2* box = nullptr,
                                             const FlatBox* fb = nullptr) {
  int code[2 * NB], idx[2 * NB], bq[2 * NB];
  double z[2 * NB];
#pragma unroll
  for (int j = 0; j < 2 * NB; ++j) {
    code[j] = 1;
    idx[j] = cidx;
    bq[j] = -1;
    z[j] = 0.0;
    if (k0 + j / 2 < n) {
      double pp[3];
      stencil_pp<FAST, GRP>(P, 2 * (m0 + j / 2) + (j & 1), k0 + j / 2, w, pw, p2, pp);
      z[j] = pp[2];
      int ix = cidx, px = 0, py = 0;
      code[j] = probe_pixel<M, FAST>(a, pp, mag, K2, exk, &ix, &px, &py);
      idx[j] = code[j] == 2 ? ix : cidx;
      if (box && code[j] == 2) {
        const int dx = px - fb->x0, dy = py - fb->y0;
        if (dx >= 0 && dx < fb->ncol && dy >= 0 && dy < fb->nrow) bq[j] = dy * 3 + dx;
      }
    }
  }
  float2 s[2 * NB];
#pragma unroll
  for (int j = 0; j < 2 * NB; ++j) s[j] = bq[j] >= 0 ? box[bq[j]] : dl2[idx[j]];
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 2 * NB; ++j) {
    double f = 0.0;
    if (code[j] == 0 || (code[j] == 2 && !probe_depth(a, s[j], z[j], mag, label1, &f))) ok = false;
    if (j & 1)
      fm[j / 2] = f;
    else
      fp[j / 2] = f;
  }
  return ok;
}

// The stencil in steps of NB parameters; false when some point's decision was
// inside a margin (Jt is then not the reference's: redo with stencil_rolled).
// Accumulation order as stencil_rolled.
template <int M, bool FAST, int NB>
__device__ __forceinline__ bool stencil_batched(const SemArgs& a, const PairConst* __restrict__ P, const double w[3],
                                                const double pw[3], const double p2[3], double mag, float label1,
                                                const double* K2, const float2* dl2, int cidx, double exk,
                                                double Jt[12], const float2* box = nullptr,
                                                const FlatBox* fb = nullptr) {
  double jq1[3] = {0.0, 0.0, 0.0}, jt1[3] = {0.0, 0.0, 0.0}, jq2[3] = {0.0, 0.0, 0.0}, jt2[3] = {0.0, 0.0, 0.0};
  bool ok = true;
  if (P->var1) {
#pragma unroll 1
    for (int k = 0; k < 4; k += NB) {
      double fp[NB], fm[NB];
      ok &= stencil_step<M, FAST, 0, NB>(a, P, k, k, 4, w, pw, p2, mag, label1, K2, dl2, cidx, exk, fp, fm,
                                                box, fb);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (k + j < 4) {
          const double jm = (fp[j] - fm[j]) * P->ood[k + j];
          const double* pj = P->pj[k + j];
#pragma unroll
          for (int c = 0; c < 3; ++c) jq1[c] = jq1[c] + jm * pj[c];
        }
      }
    }
#pragma unroll 1
    for (int k = 0; k < 3; k += NB) {
      double fp[NB], fm[NB];
      ok &= stencil_step<M, FAST, 1, NB>(a, P, 4 + k, k, 3, w, pw, p2, mag, label1, K2, dl2, cidx, exk, fp, fm,
                                                box, fb);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (k + j < 3) {
          const double jm = (fp[j] - fm[j]) * P->ood[4 + k + j];
          const double v = ((P->mask1 >> (k + j)) & 1u) ? 0.0 : jm;
#pragma unroll
          for (int c = 0; c < 3; ++c) jt1[c] = c == k + j ? v : jt1[c];
        }
      }
    }
  }
  if (P->var2) {
#pragma unroll 1
    for (int k = 0; k < 4; k += NB) {
      double fp[NB], fm[NB];
      ok &= stencil_step<M, FAST, 2, NB>(a, P, 7 + k, k, 4, w, pw, p2, mag, label1, K2, dl2, cidx, exk, fp, fm,
                                                box, fb);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (k + j < 4) {
          const double jm = (fp[j] - fm[j]) * P->ood[7 + k + j];
          const double* pj = P->pj[4 + k + j];
#pragma unroll
          for (int c = 0; c < 3; ++c) jq2[c] = jq2[c] + jm * pj[c];
        }
      }
    }
#pragma unroll 1
    for (int k = 0; k < 3; k += NB) {
      double fp[NB], fm[NB];
      ok &= stencil_step<M, FAST, 3, NB>(a, P, 11 + k, k, 3, w, pw, p2, mag, label1, K2, dl2, cidx, exk, fp, fm,
                                                box, fb);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (k + j < 3) {
          const double jm = (fp[j] - fm[j]) * P->ood[11 + k + j];
          const double v = ((P->mask2 >> (k + j)) & 1u) ? 0.0 : jm;
#pragma unroll
          for (int c = 0; c < 3; ++c) jt2[c] = c == k + j ? v : jt2[c];
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    Jt[c] = jq1[c];
    Jt[3 + c] = jt1[c];
    Jt[6 + c] = jq2[c];
    Jt[9 + c] = jt2[c];
  }
  return ok;
}

// One workgroup per pair-aligned tile of <= 256 samples, one lane per sample:
// centre residual (reference sequence), the CENTRAL stencil over the
// variable poses' ambient parameters (one rolled loop per parameter group, so
// the tangent row stays in registers), QuaternionManifold / SubsetManifold,
// the ScaledLoss Corrector, and the tile's J'J / J'r / cost reduced through
// LDS in two 128-row halves (13 KB of LDS per workgroup: occupancy is set by
// registers, not LDS) with one atomic flush per value.  Per-sample r /
// status / J are stored only when requested (parity and download); the
// solver consumes the pair records.
// ---------------------------------------------------------------------------
// Centre evaluation of one sample (reference operation sequence) and the
// quantities its stencil starts from.
// ---------------------------------------------------------------------------
struct Centre {
  double pw[3], p2[3], w[3];
  double r, mag, exk;
  PixelCache pc;
  int st;
};

template <int M, bool FAST>
__device__ __forceinline__ void centre_eval(const SemArgs& a, const PairConst* __restrict__ P, const SemSample& smp,
                                            const double* K2, const float2* dl2, Centre& c) {
  // QuaternionRotatePoint(q_inv, P_c1) + t_inv, then pose 2
  double rot[3];
  unit_quat_rotate(P->uqi, smp.pc1, rot);
  c.pw[0] = rot[0] + P->ti[0];
  c.pw[1] = rot[1] + P->ti[1];
  c.pw[2] = rot[2] + P->ti[2];
  double rot2[3];
  unit_quat_rotate(P->u2, c.pw, rot2);
  c.p2[0] = rot2[0] + P->t2[0];
  c.p2[1] = rot2[1] + P->t2[1];
  c.p2[2] = rot2[2] + P->t2[2];
  c.pc.valid = false;
  c.pc.px = c.pc.py = 0;
  c.pc.depth = c.pc.label = 0.f;
  c.st = 0;
  c.r = project_centre<M>(a, c.p2, smp.label1, K2, dl2, c.pc, &c.st);
  c.mag = fabs(smp.pc1[0]) + fabs(smp.pc1[1]) + fabs(smp.pc1[2]) + fabs(P->t1[0]) + fabs(P->t1[1]) +
          fabs(P->t1[2]) + fabs(c.pw[0]) + fabs(c.pw[1]) + fabs(c.pw[2]) + fabs(P->t2[0]) + fabs(P->t2[1]) +
          fabs(P->t2[2]);
  c.w[0] = smp.pc1[0] - P->t1[0];
  c.w[1] = smp.pc1[1] - P->t1[1];
  c.w[2] = smp.pc1[2] - P->t1[2];
  c.exk = FAST ? margin_model_term<M>(K2, c.p2, c.mag) : 0.0;
}

// Stencil: parameter m = 0..13 over (q1, t1, q2, t2), + then - (Ceres
// CENTRAL order), e = 2 m + minus.  Everything that depends only on the pair
// and the stencil point (perturbed value, 1/(2 delta), the perturbed rotation
// folded into one 3x3 map, PlusJacobian rows) comes from the per-pair table
// as wave-uniform scalar loads; a lane forms one mat-vec per point.
// Returns true when the batched route had to be redone per point (a decision
// inside a margin; semantic_diag 2 counts them).
template <int M, bool FAST, int NB>
__device__ __forceinline__ bool stencil_full(const SemArgs& a, const PairConst* __restrict__ P, const Centre& c,
                                             const SemSample& smp, const double* K2, const float2* dl2,
                                             double Jt[12], const float2* box = nullptr,
                                             const FlatBox* fb = nullptr) {
  if constexpr (NB > 0) {
    const int cidx = c.pc.valid ? c.pc.py * a.W + c.pc.px : 0;
    if (!stencil_batched<M, FAST, NB>(a, P, c.w, c.pw, c.p2, c.mag, smp.label1, K2, dl2, cidx, c.exk, Jt, box, fb)) {
      stencil_rolled<M, FAST>(a, P, c.w, c.pw, c.p2, c.mag, smp.pc1, smp.label1, K2, dl2, c.pc, c.exk, Jt);
      return true;
    }
    return false;
  } else {
    stencil_rolled<M, FAST>(a, P, c.w, c.pw, c.p2, c.mag, smp.pc1, smp.label1, K2, dl2, c.pc, c.exk, Jt);
    return true;
  }
}

// ---------------------------------------------------------------------------
// Flat test.  Most samples have a zero Jacobian: every stencil point lands on
// a pixel with the centre's outcome.  This proves it without evaluating the
// stencil (DESIGN.md §4 has the derivation):
//  (1) every stencil point's camera-2 point P' lies within a componentwise
//      bound (ax, ay, az) of the centre's P (per class of stencil points:
//      PairConst bounds), so with z' >= z - az > 0, u' - u = (dPx - u dPz) /
//      (z + dPz) gives |du| <= (ax + |u| az) / (z - az) exactly (v alike);
//  (2) the pixel x(u, v) = f (u + D(u, v)) + c moves by the mean value
//      theorem by |dx| <= (|A00| + Hx s) du + (|A01| + Hx s) dv, s = du + dv,
//      A = d(x, y) / d(u, v) at the centre and Hx = |fx| H(rho) a bound of
//      every second derivative of x over the box |(u, v)| <= rho
//      (second_derivative_bound: the radial terms u r^2 / u r^4 give 6 rho /
//      20 rho^3, the tangential ones 6 (|p1| + |p2|); 0 for the pinholes);
//  (3) the reference's computed pixel differs from the exact one by rounding
//      far below resolve's margin ex, so round() can only reach the pixels
//      round(x - bx) .. round(x + bx), bx = bound + ex; the depth compared
//      moves by at most az.
// When every pixel of that box gives the centre's outcome for every depth
// within az (outside the margin), every stencil value equals the centre's
// residual: all CENTRAL differences are +0.0 and J = +0.0 exactly as the
// reference's accumulation yields.  Otherwise (or on any doubt: depth near
// zero, huge coordinates, a box wider than 3 x 3) the sample takes the full
// stencil.  tests/test_semantic_flat_property.py checks the oracle's
// restatement of this test against the full stencil on >= 1e7 samples.
// ---------------------------------------------------------------------------

// Bound H(rho) of every second derivative of the distortion map (u, v) ->
// u + Du(u, v) (and v + Dv) over |(u, v)| <= rho, per unit focal length:
//   d2(u r^2) <= 6 rho, d2(u r^4) <= 20 rho^3 (all of d2/du2, d2/dudv,
//   d2/dv2; v alike), d2 of the OPENCV tangential terms <= 6 (|p1| + |p2|).
template <int M>
__device__ __forceinline__ double second_derivative_bound(const double* K, double rho) {
  if constexpr (M == kSimpleRadial) {
    return 6.0 * fabs(K[3]) * rho;
  } else if constexpr (M == kRadial) {
    return 6.0 * fabs(K[3]) * rho + 20.0 * fabs(K[4]) * rho * rho * rho;
  } else if constexpr (M == kOpenCV) {
    return 6.0 * fabs(K[4]) * rho + 20.0 * fabs(K[5]) * rho * rho * rho + 6.0 * (fabs(K[6]) + fabs(K[7]));
  } else {
    return 0.0;
  }
}

// Geometry half of the flat test: false when the sample cannot be cleared
// whatever the raster holds.  c needs p2, pw, w, mag (not the raster).
template <int M>
__device__ __forceinline__ bool flat_box(const PairConst* __restrict__ P, const Centre& c, const double* K2,
                                         FlatBox& fb) {
  const double z = c.p2[2];
  if (!(z > 0.0)) return false;  // NaN-safe
  const double iz = 1.0 / z;
  const double u = c.p2[0] * iz, v = c.p2[1] * iz;
  constexpr int np = Model<M>::kNumParams;
  double x, y, A[4], Jp[2 * np];
  world_to_image_jac<M>(K2, u, v, &x, &y, A, Jp);
  if (!(fabs(x) < 1e8 && fabs(y) < 1e8 && fabs(u) < 1e6 && fabs(v) < 1e6)) return false;
  // per class of stencil points, componentwise bounds (ax, ay, az) of the
  // camera-2 point's displacement: du <= (ax + |u| az) / (z - az), dv alike
  // (one reciprocal for every class: 1 / (z - az_max) bounds each 1 / (z - az))
  const double dq1 = P->var1 ? P->rho1 * sqrt(c.w[0] * c.w[0] + c.w[1] * c.w[1] + c.w[2] * c.w[2]) * (1.0 + 1e-12) : 0.0;
  const double dq2 = P->var2 ? P->rho2 * sqrt(c.pw[0] * c.pw[0] + c.pw[1] * c.pw[1] + c.pw[2] * c.pw[2]) * (1.0 + 1e-12) : 0.0;
  double az_max = fmax(dq1, dq2);
  if (P->var1)
    az_max = fmax(az_max, fmax(P->dt1[0] * fabs(P->C[6]), fmax(P->dt1[1] * fabs(P->C[7]), P->dt1[2] * fabs(P->C[8]))));
  if (P->var2) az_max = fmax(az_max, P->dt2[2]);
  if (!(z - az_max > 0.5 * z)) return false;
  const double iden = 1.0 / (z - az_max) * (1.0 + 1e-12);
  // the classes' (du, dv): q1, t1 x3, q2, t2 x3
  double cu[8], cv[8];
  int nc = 0;
  auto cls = [&](double ax, double ay, double az) {
    cu[nc] = (ax + fabs(u) * az) * iden;
    cv[nc] = (ay + fabs(v) * az) * iden;
    ++nc;
  };
  if (P->var1) {
    cls(dq1, dq1, dq1);
#pragma unroll
    for (int k = 0; k < 3; ++k)
      cls(P->dt1[k] * fabs(P->C[k]), P->dt1[k] * fabs(P->C[3 + k]), P->dt1[k] * fabs(P->C[6 + k]));
  }
  if (P->var2) {
    cls(dq2, dq2, dq2);
    cls(P->dt2[0], 0.0, 0.0);
    cls(0.0, P->dt2[1], 0.0);
    cls(0.0, 0.0, P->dt2[2]);
  }
  double gm = 0.0;
  for (int k = 0; k < nc; ++k) gm = fmax(gm, fmax(cu[k], cv[k]));
  if (!(gm < 0.1)) return false;  // a stencil this wide is never cleared (and keeps rho finite)
  const double ru = fabs(u) + gm, rv = fabs(v) + gm;
  const double H = second_derivative_bound<M>(K2, sqrt(ru * ru + rv * rv) * (1.0 + 1e-12));
  const double fx = fabs(K2[0]);
  const double fy = (M == kPinhole || M == kOpenCV) ? fabs(K2[1]) : fabs(K2[0]);
  double bxm = 0.0, bym = 0.0;
  for (int k = 0; k < nc; ++k) {
    const double sk = cu[k] + cv[k];
    bxm = fmax(bxm, (fabs(A[0]) + fx * H * sk) * cu[k] + (fabs(A[1]) + fx * H * sk) * cv[k]);
    bym = fmax(bym, (fabs(A[2]) + fy * H * sk) * cu[k] + (fabs(A[3]) + fy * H * sk) * cv[k]);
  }
  const double gain = distortion_gain<M>(K2, u * u + v * v);
  const double kscale = (fabs(K2[0]) + fabs(K2[1])) * gain * (1.0 + fabs(u) + fabs(v)) * (1.0 + c.mag * fabs(iz));
  const double ex = 1e-6 + 1e-11 * (kscale + fabs(x) + fabs(y));
  const double bx = bxm * (1.0 + 1e-12) + ex;
  const double by = bym * (1.0 + 1e-12) + ex;
  // round() is monotone: the reachable pixels are round(x - bx) .. round(x + bx)
  fb.x0 = (int)round(x - bx);
  fb.y0 = (int)round(y - by);
  fb.ncol = (int)round(x + bx) - fb.x0 + 1;
  fb.nrow = (int)round(y + by) - fb.y0 + 1;
  fb.d = az_max;
  return fb.ncol <= 3 && fb.nrow <= 3;
}

// Upper bounds of |A| = |d(x, y) / d(u, v)| at (u, v) from the radius alone
// (triangle inequality on the models' derivatives, 2 |u v| <= r^2, |u|, |v|
// <= r <= |u| + |v|): radial u r^2 gives d/du <= 3 r^2, d/dv <= r^2; u r^4
// gives 5 r^4, 2 r^4; the OPENCV tangential terms 2 p1 u v + p2 (r^2 + 2 u^2)
// give (2 |p1| + 6 |p2|) r1 and 2 (|p1| + |p2|) r1 (v alike with p1, p2
// swapped), r1 = |u| + |v|.
template <int M>
__device__ __forceinline__ void image_jac_bound(const double* K, double u, double v, double Ah[4]) {
  const double r2 = u * u + v * v, r1 = fabs(u) + fabs(v);
  if constexpr (M == kSimplePinhole) {
    Ah[0] = Ah[3] = fabs(K[0]);
    Ah[1] = Ah[2] = 0.0;
  } else if constexpr (M == kPinhole) {
    Ah[0] = fabs(K[0]);
    Ah[3] = fabs(K[1]);
    Ah[1] = Ah[2] = 0.0;
  } else if constexpr (M == kSimpleRadial) {
    const double k = fabs(K[3]);
    Ah[0] = Ah[3] = fabs(K[0]) * (1.0 + 3.0 * k * r2);
    Ah[1] = Ah[2] = fabs(K[0]) * (k * r2);
  } else if constexpr (M == kRadial) {
    const double k1 = fabs(K[3]), k2 = fabs(K[4]);
    Ah[0] = Ah[3] = fabs(K[0]) * (1.0 + 3.0 * k1 * r2 + 5.0 * k2 * r2 * r2);
    Ah[1] = Ah[2] = fabs(K[0]) * (k1 * r2 + 2.0 * k2 * r2 * r2);
  } else {
    const double k1 = fabs(K[4]), k2 = fabs(K[5]), p1 = fabs(K[6]), p2 = fabs(K[7]);
    const double rad = 3.0 * k1 * r2 + 5.0 * k2 * r2 * r2, off = k1 * r2 + 2.0 * k2 * r2 * r2 + 2.0 * (p1 + p2) * r1;
    Ah[0] = fabs(K[0]) * (1.0 + rad + (2.0 * p1 + 6.0 * p2) * r1);
    Ah[1] = fabs(K[0]) * off;
    Ah[2] = fabs(K[1]) * off;
    Ah[3] = fabs(K[1]) * (1.0 + rad + (6.0 * p1 + 2.0 * p2) * r1);
  }
}

// flat_box with the per-class displacement bounds replaced by their
// componentwise maxima (ax, ay, az) over the classes: each class's pixel
// bound is monotone in its (ax, ay, az) and in 1 / (z - az), so the one bound
// covers every class — a box at most marginally wider, without the per-class
// loops.  The centre's own (u, v) and pixel (x, y) (the reference sequence)
// serve as the expansion point and |A| is bounded from the radius
// (image_jac_bound), so no camera-model Jacobian is evaluated.  The depth
// bound az is flat_box's.  Restated in the oracle (FlatClears, coarse form)
// for tests/test_semantic_flat_property.py.
template <int M, bool EXACT_A = false, bool GROUPS = false>
__device__ __forceinline__ bool flat_box_coarse(const PairConst* __restrict__ P, const Centre& c, const double* K2,
                                                double u, double v, double x, double y, FlatBox& fb) {
  const double z = c.p2[2];
  if (!(z > 0.0)) return false;  // NaN-safe
  double Ae[4];
  if constexpr (EXACT_A) {  // semantic_flat_coarse 2: A at the centre from the camera model's Jacobian
    constexpr int np = Model<M>::kNumParams;
    double Jp[2 * np];
    world_to_image_jac<M>(K2, u, v, &x, &y, Ae, Jp);
  }
  if (!(fabs(x) < 1e8 && fabs(y) < 1e8 && fabs(u) < 1e6 && fabs(v) < 1e6)) return false;
  // rotation classes (isotropic dq) and translation classes (componentwise
  // maxima of the t1 / t2 steps); GROUPS: bounded separately, else together
  double dq = 0.0, tx = 0.0, ty = 0.0, tz = 0.0;
  if (P->var1) {
    dq = P->rho1 * sqrt(c.w[0] * c.w[0] + c.w[1] * c.w[1] + c.w[2] * c.w[2]) * (1.0 + 1e-12);
    tx = fmax(P->dt1[0] * fabs(P->C[0]), fmax(P->dt1[1] * fabs(P->C[1]), P->dt1[2] * fabs(P->C[2])));
    ty = fmax(P->dt1[0] * fabs(P->C[3]), fmax(P->dt1[1] * fabs(P->C[4]), P->dt1[2] * fabs(P->C[5])));
    tz = fmax(P->dt1[0] * fabs(P->C[6]), fmax(P->dt1[1] * fabs(P->C[7]), P->dt1[2] * fabs(P->C[8])));
  }
  if (P->var2) {
    dq = fmax(dq, P->rho2 * sqrt(c.pw[0] * c.pw[0] + c.pw[1] * c.pw[1] + c.pw[2] * c.pw[2]) * (1.0 + 1e-12));
    tx = fmax(tx, P->dt2[0]);
    ty = fmax(ty, P->dt2[1]);
    tz = fmax(tz, P->dt2[2]);
  }
  const double az = fmax(dq, tz);
  if (!(z - az > 0.5 * z)) return false;
  const double iden = 1.0 / (z - az) * (1.0 + 1e-12);
  // (cu, cv) of the group(s): the rotation group's and the translation group's
  const double cu_r = (dq + fabs(u) * dq) * iden, cv_r = (dq + fabs(v) * dq) * iden;
  const double cu_t = (tx + fabs(u) * tz) * iden, cv_t = (ty + fabs(v) * tz) * iden;
  const double cu = fmax(cu_r, cu_t), cv = fmax(cv_r, cv_t);
  const double gm = fmax(cu, cv);
  if (!(gm < 0.1)) return false;  // a stencil this wide is never cleared (and keeps rho finite)
  const double ru = fabs(u) + gm, rv = fabs(v) + gm;
  const double H = second_derivative_bound<M>(K2, sqrt(ru * ru + rv * rv) * (1.0 + 1e-12));
  const double fx = fabs(K2[0]);
  const double fy = (M == kPinhole || M == kOpenCV) ? fabs(K2[1]) : fabs(K2[0]);
  double Ah[4];
  if constexpr (EXACT_A) {
#pragma unroll
    for (int k = 0; k < 4; ++k) Ah[k] = fabs(Ae[k]);
  } else {
    image_jac_bound<M>(K2, u, v, Ah);
  }
  double bxm, bym;
  if constexpr (GROUPS) {
    const double sr = cu_r + cv_r, st = cu_t + cv_t;
    bxm = fmax((Ah[0] + fx * H * sr) * cu_r + (Ah[1] + fx * H * sr) * cv_r,
               (Ah[0] + fx * H * st) * cu_t + (Ah[1] + fx * H * st) * cv_t);
    bym = fmax((Ah[2] + fy * H * sr) * cu_r + (Ah[3] + fy * H * sr) * cv_r,
               (Ah[2] + fy * H * st) * cu_t + (Ah[3] + fy * H * st) * cv_t);
  } else {
    const double sk = cu + cv;
    bxm = (Ah[0] + fx * H * sk) * cu + (Ah[1] + fx * H * sk) * cv;
    bym = (Ah[2] + fy * H * sk) * cu + (Ah[3] + fy * H * sk) * cv;
  }
  const double gain = distortion_gain<M>(K2, u * u + v * v);
  const double kscale = (fabs(K2[0]) + fabs(K2[1])) * gain * (1.0 + fabs(u) + fabs(v)) * (1.0 + c.mag * fabs(1.0 / z));
  const double ex = 1e-6 + 1e-11 * (kscale + fabs(x) + fabs(y));
  const double bx = bxm * (1.0 + 1e-12) + ex;
  const double by = bym * (1.0 + 1e-12) + ex;
  fb.x0 = (int)round(x - bx);
  fb.y0 = (int)round(y - by);
  fb.ncol = (int)round(x + bx) - fb.x0 + 1;
  fb.nrow = (int)round(y + by) - fb.y0 + 1;
  fb.d = az;
  return fb.ncol <= 3 && fb.nrow <= 3;
}

// Box entry q (of 3 x 3): raster index to read (pixel 0 when q is outside the
// box or the raster — read and ignored, so every read issues unconditionally).
__device__ __forceinline__ int flat_index(const SemArgs& a, const FlatBox& fb, bool cand, int q) {
  const int px = fb.x0 + q % 3, py = fb.y0 + q / 3;
  const bool in = cand && q % 3 < fb.ncol && q / 3 < fb.nrow && px >= 0 && px < a.W && py >= 0 && py < a.H;
  return in ? py * a.W + px : 0;
}

// Raster half: every box pixel gives the centre's outcome r for every depth
// within d of z (outside the margin).
__device__ __forceinline__ bool flat_check(const SemArgs& a, const FlatBox& fb, const float2 s[9], double z,
                                           double mag, float label1, double r) {
  bool flat = true;
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const int px = fb.x0 + q % 3, py = fb.y0 + q / 3;
    if (q % 3 < fb.ncol && q / 3 < fb.nrow) {
      double f = 0.0;
      if (px >= 0 && px < a.W && py >= 0 && py < a.H) {
        const double dz = fabs((double)s[q].x - z) - a.threshold;
        if (!(fabs(dz) > fb.d + 1e-9 * (1.0 + fabs((double)s[q].x) + mag))) flat = false;
        f = dz > 0.0 ? 0.0 : (label1 == s[q].y ? 0.0 : 1.0);
      }
      if (f != r) flat = false;
    }
  }
  return flat;
}

template <int M>
__device__ __forceinline__ bool stencil_flat(const SemArgs& a, const PairConst* __restrict__ P, const Centre& c,
                                             float label1, const double* K2, const float2* __restrict__ dl2) {
  FlatBox fb;
  if (!flat_box<M>(P, c, K2, fb)) return false;
  float2 s[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) s[q] = dl2[flat_index(a, fb, true, q)];
  return flat_check(a, fb, s, c.p2[2], c.mag, label1, c.r);
}

// NB > 0: the batched stencil (NB parameters per step), the per-point route
// only for samples with a decision inside a margin.  FLAT: the flat test
// first; the samples it cannot clear are gathered into the workgroup's first
// lanes (one sample per lane) and only those evaluate the stencil, so a
// workgroup with few of them keeps most of its waves free.
template <int M, bool FAST = false, int NB = 0, bool FLAT = false>
__global__ __launch_bounds__(kBlock) void semantic_linearize_kernel(SemArgs ak, const SemTile* __restrict__ tiles,
                                                                     const PairConst* __restrict__ pcs,
                                                                     double* __restrict__ pair_blk,
                                                                     double* __restrict__ cost_partial,
                                                                     double* __restrict__ r_out,
                                                                     int32_t* __restrict__ status_out,
                                                                     double* __restrict__ J_out, int write_samples) {
  constexpr int kHalf = kBlock / 2;
  // sbuf: the tile's rows for the J'J reduction (kHalf x kSemRow), earlier
  // (FLAT) the stencil results of the gathered samples (kBlock x 12)
  constexpr int kBuf = FLAT ? kBlock * 12 : kHalf * kSemRow;
  __shared__ double sbuf[kBuf];
  __shared__ double spart[2 * kPairVals];
  __shared__ double sred[4];
  __shared__ int slist[FLAT ? kBlock : 1];
  __shared__ int scnt[kBlock / 64];
  double* sJ = sbuf;
  const SemTile t = tiles[blockIdx.x];
  const PairConst* __restrict__ P = pcs + t.pair;
  const SemArgs a = with_pair(ak, P);
  const int tid = threadIdx.x;
  const bool active = tid < (int)t.count;
  const int64_t n = (int64_t)t.start + tid;
  const float2* dl2 = a.dl + P->roff;
  const double* K2 = P->K2;
  double cost = 0.0;
  double rowv[kSemRow];
#pragma unroll
  for (int k = 0; k < kSemRow; ++k) rowv[k] = 0.0;
  double r = 0.0;
  int st = 0;
  double Jt[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) Jt[k] = 0.0;
  bool deferred = false;  // FLAT: stencil evaluated by a gathered lane
  if (active) {
    const SemSample smp = a.samples[n];
    Centre c;
    centre_eval<M, FAST>(a, P, smp, K2, dl2, c);
    r = c.r;
    st = c.st;
    if constexpr (FLAT)
      deferred = !stencil_flat<M>(a, P, c, smp.label1, K2, dl2);  // flat: Jt stays +0.0
    else
      stencil_full<M, FAST, NB>(a, P, c, smp, K2, dl2, Jt);
  }
  if constexpr (FLAT) {
    // gather the deferred samples into lanes 0 .. nd-1 (workgroup order)
    const int lane = tid & 63;
    const unsigned long long bal = __ballot(deferred);
    if (lane == 0) scnt[tid >> 6] = __popcll(bal);
    __syncthreads();
    int base = 0, nd = 0;
#pragma unroll
    for (int wv = 0; wv < kBlock / 64; ++wv) {
      base += wv < (tid >> 6) ? scnt[wv] : 0;
      nd += scnt[wv];
    }
    const int slot = base + __popcll(bal & ((1ull << lane) - 1ull));
    if (deferred) slist[slot] = tid;
    __syncthreads();
    if (tid < nd) {
      const SemSample smp = a.samples[(int64_t)t.start + slist[tid]];
      Centre c;
      centre_eval<M, FAST>(a, P, smp, K2, dl2, c);
      double Jd[12];
      stencil_full<M, FAST, NB>(a, P, c, smp, K2, dl2, Jd);
#pragma unroll
      for (int k = 0; k < 12; ++k) sbuf[tid * 12 + k] = Jd[k];
    }
    __syncthreads();
    if (deferred) {
#pragma unroll
      for (int k = 0; k < 12; ++k) Jt[k] = sbuf[slot * 12 + k];
    }
    __syncthreads();  // sbuf is reused by the reduction below
  }
  if (active) {
    if (write_samples) {
      r_out[n] = r;
      status_out[n] = st + ((write_samples & 2) && deferred ? 0x1000 : 0);  // 2: mark deferred samples (diagnostic)
      double2* jo = reinterpret_cast<double2*>(J_out + 12 * n);
#pragma unroll
      for (int m = 0; m < 6; ++m) jo[m] = make_double2(Jt[2 * m], Jt[2 * m + 1]);
    }
    // ScaledLoss(w) + loss, Corrector rho'' <= 0 branch: sqrt(w * rho')
    double rho[3];
    loss_eval(a.loss_type, a.loss_scale, r * r, rho);
    cost = 0.5 * (a.weight * rho[0]);
    const double sc = sqrt(a.weight * rho[1]);
#pragma unroll
    for (int m = 0; m < 12; ++m) rowv[m] = Jt[m] * sc;
    rowv[12] = r * sc;
  }
  // tile J'J (78) and J'r (12): the rows pass through LDS in two halves
  // (threads 0..127, then 128..255); 2 x 90 threads over interleaved rows
  int ca = 0, cb = 0;
  const int h = tid / kPairVals, e = tid - h * kPairVals;
  if (tid < 2 * kPairVals) {
    if (e < 78) {
      int a_ = 0, rem = e;
      while (rem >= 12 - a_) { rem -= 12 - a_; ++a_; }
      ca = a_;
      cb = a_ + rem;
    } else {
      ca = e - 78;
      cb = 12;
    }
  }
  double acc = 0.0;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (tid / kHalf == half) {
      double* row = sJ + (tid - half * kHalf) * kSemRow;
#pragma unroll
      for (int k = 0; k < kSemRow; ++k) row[k] = rowv[k];
    }
    __syncthreads();
    const int cnt = min(kHalf, (int)t.count - half * kHalf);
    if (tid < 2 * kPairVals)
      for (int q = h; q < cnt; q += 2) acc += sJ[q * kSemRow + ca] * sJ[q * kSemRow + cb];
    __syncthreads();
  }
  if (tid < 2 * kPairVals) spart[tid] = acc;
  double v = cost;
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if ((tid & 63) == 0) sred[tid >> 6] = v;
  __syncthreads();
  if (tid < kPairVals) atomicAdd(pair_blk + (size_t)t.pair * kPairStride + tid, spart[tid] + spart[kPairVals + tid]);
  if (tid == 0) cost_partial[blockIdx.x] = sred[0] + sred[1] + sred[2] + sred[3];
}

// ---------------------------------------------------------------------------
// Two-pass linearization (semantic_variant 6).  A sample the flat test clears
// has J = +0.0: its row adds nothing to J'J or J'r, only its cost.  Pass 1
// (one workgroup per tile) evaluates every sample's centre, cost and flat
// test and appends the samples it cannot clear to their pair's region of a
// deferred list (one atomic per wave).  Pass 2 runs the full stencil on the
// deferred samples only, 64 per workgroup and all of one pair (wave-uniform
// pair table), and reduces their J'J / J'r into the pair block — dense
// waves, unlike in-tile compaction, which leaves most waves of a tile idle.
// ---------------------------------------------------------------------------
// The 3x3 window summary of pixel p (window_summary_kernel): the window with
// top-left corner p = (x, y), inside the raster, every label == the first
// (not NaN): {min depth, max depth, label, 0}; any other window: dmin = NaN.
// It decides a sample of the flat pass alone (no centre or box read) when the
// window holding the sample's box lies on one side of the depth test with
// the flat test's margin for every depth in it: then every box pixel, the
// centre pixel among them, has the outcome the window's label (valid side)
// or INVALID_DEPTH (invalid side) gives, exactly as flat_check and the centre
// evaluation would find pixel by pixel (fabs(s - z) is monotone in s, and the
// margin 1e-9 (1 + |s| + mag) in |s|).  Undecided samples read the raster.
__device__ __forceinline__ bool window_decides(const SemArgs& a, const FlatBox& fb, const float4& w, double z,
                                               double mag, float label1, int* st, double* r) {
  const double dmin = (double)w.x, dmax = (double)w.y;
  if (!(dmin <= dmax)) return false;  // NaN: a mixed-label or edge window
  const double margin = fb.d + 1e-9 * (1.0 + fmax(fabs(dmin), fabs(dmax)) + mag);
  const double far = fmax(fabs(dmax - z), fabs(dmin - z));
  const double dzmax = far - a.threshold;
  if (dzmax < 0.0 && -dzmax > margin) {
    *st = MI_BA_VALID;
    *r = (label1 == w.z) ? 0.0 : 1.0;
    return true;
  }
  const double nearest = (z >= dmin && z <= dmax) ? 0.0 : fmin(fabs(dmin - z), fabs(dmax - z));
  const double dzmin = nearest - a.threshold;
  if (dzmin > 0.0 && dzmin > margin) {
    *st = MI_BA_INVALID_DEPTH;
    *r = 0.0;
    return true;
  }
  return false;
}

// grid (pixel blocks of the largest plane, slots)
__global__ __launch_bounds__(256) void window_summary_kernel(const float2* __restrict__ dl,
                                                             const SlotInfo* __restrict__ slots,
                                                             float4* __restrict__ out) {
  const SlotInfo si = slots[blockIdx.y];
  const int H = si.H, W = si.W;
  const int64_t rem = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (rem >= (int64_t)H * W) return;
  const int64_t k = (int64_t)si.off + rem;
  const int y = (int)(rem / W), x = (int)(rem - (int64_t)y * W);
  float4 o = make_float4(__builtin_nanf(""), 0.f, 0.f, 0.f);
  if (x + 2 < W && y + 2 < H) {
    const float2* base = dl + k;
    const float L = base[0].y;
    float dmin = base[0].x, dmax = base[0].x;
    bool uniform = true;
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const float2 v = base[(q / 3) * W + q % 3];
      uniform = uniform && (v.y == L);
      dmin = fminf(dmin, v.x);
      dmax = fmaxf(dmax, v.x);
      if (v.x != v.x) uniform = false;  // NaN depth: the pixel test is left to the raster
    }
    if (uniform) o = make_float4(dmin, dmax, L, 0.f);
  }
  out[k] = o;
}

// Label planes.  The palette: every distinct label bit pattern of the
// rasters in an open-addressed table of 256 keys (bit pattern | 1 << 32, 0 =
// empty); more than 256 distinct labels sets *overflow and the planes are not
// used.  Comparing the sample's label with pal[index] is the comparison with
// the raster's label itself (the same bits), NaN and signed zeros included.
__device__ __forceinline__ uint32_t pal_hash(uint32_t b) {
  b ^= b >> 16;
  b *= 0x7feb352du;
  b ^= b >> 15;
  return b & 255u;
}

__global__ __launch_bounds__(256) void label_palette_kernel(const float2* __restrict__ dl, int64_t n,
                                                            unsigned long long* keys, unsigned* overflow) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const uint32_t bits = __float_as_uint(dl[k].y);
  const unsigned long long key = (unsigned long long)bits | (1ull << 32);
  uint32_t h = pal_hash(bits);
  for (int probe = 0; probe < 256; ++probe, h = (h + 1u) & 255u) {
    const unsigned long long cur = __hip_atomic_load(keys + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return;
    if (cur == 0ull) {
      const unsigned long long prev = atomicCAS(keys + h, 0ull, key);
      if (prev == 0ull || prev == key) return;
    }
  }
  atomicOr(overflow, 1u);
}

__global__ __launch_bounds__(256) void label_index_kernel(const float2* __restrict__ dl, int64_t n,
                                                          const unsigned long long* __restrict__ keys,
                                                          uint8_t* __restrict__ lab8) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const uint32_t bits = __float_as_uint(dl[k].y);
  const unsigned long long key = (unsigned long long)bits | (1ull << 32);
  uint32_t h = pal_hash(bits);
  for (int probe = 0; probe < 256 && keys[h] != key; ++probe) h = (h + 1u) & 255u;
  lab8[k] = (uint8_t)h;
}

// grid (tile blocks of the largest tile plane, slots)
__global__ __launch_bounds__(256) void depth_tile_kernel(const float2* __restrict__ dl,
                                                         const SlotInfo* __restrict__ slots, float2* __restrict__ out) {
  const SlotInfo si = slots[blockIdx.y];
  const int H = si.H, W = si.W, TW = si.TW, TH = (H + 7) / 8;
  const int rem = (int)(blockIdx.x * 256 + threadIdx.x);
  if (rem >= TH * TW) return;
  const int64_t k = (int64_t)si.toff + rem;
  const int ty = rem / TW, tx = rem - ty * TW;
  const float2* base = dl + si.off;
  float dmin = __builtin_inff(), dmax = -__builtin_inff();
  bool nan = false;
  const int y1 = min(8 * ty + 10, H), x1 = min(8 * tx + 10, W);
  for (int y = 8 * ty; y < y1; ++y)
    for (int x = 8 * tx; x < x1; ++x) {
      const float d = base[(int64_t)y * W + x].x;
      nan = nan || d != d;
      dmin = fminf(dmin, d);
      dmax = fmaxf(dmax, d);
    }
  out[k] = nan ? make_float2(__builtin_nanf(""), __builtin_nanf("")) : make_float2(dmin, dmax);
}

// The depth side of every pixel of a box in one tile: 1 when every depth in
// [dmin, dmax] passes the depth test with the flat test's margin (|d - z| is
// convex in d: its maximum over the range is at an end), 2 when every depth
// fails it with the margin, 0 undecided (a NaN range included).
__device__ __forceinline__ int tile_depth_side(const SemArgs& a, const FlatBox& fb, float2 dr, double z, double mag) {
  const double dmin = (double)dr.x, dmax = (double)dr.y;
  if (!(dmin <= dmax)) return 0;
  const double margin = fb.d + 1e-9 * (1.0 + fmax(fabs(dmin), fabs(dmax)) + mag);
  const double far = fmax(fabs(dmax - z), fabs(dmin - z));
  if (a.threshold - far > margin) return 1;
  const double nearest = (z >= dmin && z <= dmax) ? 0.0 : fmin(fabs(dmin - z), fabs(dmax - z));
  if (nearest - a.threshold > margin) return 2;
  return 0;
}

template <int M, bool FAST, bool WS = false, bool LP = false, int COARSE = 0>
__global__ __launch_bounds__(kBlock) void semantic_flat_kernel(SemArgs ak, const SemTile* __restrict__ tiles,
                                                               const PairConst* __restrict__ pcs,
                                                               unsigned long long* __restrict__ dmask,
                                                               double* __restrict__ cost_partial,
                                                               double* __restrict__ r_out,
                                                               int32_t* __restrict__ status_out,
                                                               double* __restrict__ J_out, int write_samples) {
  __shared__ double sred[kBlock / 64];
  __shared__ float spal[LP ? 256 : 1];
  const SemTile t = tiles[blockIdx.x];
  const PairConst* __restrict__ P = pcs + t.pair;
  const SemArgs a = with_pair(ak, P);
  const int tid = threadIdx.x, lane = tid & 63;
  const bool active = tid < (int)t.count;
  const int64_t n = (int64_t)t.start + tid;
  const float2* dl2 = a.dl + P->roff;
  const double* K2 = P->K2;
  double cost = 0.0;
  bool deferred = false;
  if constexpr (LP) {
    static_assert(kBlock >= 256, "one palette entry per thread");
    spal[tid] = a.pal[tid];
    __syncthreads();
  }
  if (active) {
    const SemSample smp = a.samples[n];
    // centre geometry (reference sequence, as centre_eval / project_centre)
    Centre c;
    double rot[3];
    unit_quat_rotate(P->uqi, smp.pc1, rot);
    c.pw[0] = rot[0] + P->ti[0];
    c.pw[1] = rot[1] + P->ti[1];
    c.pw[2] = rot[2] + P->ti[2];
    double rot2[3];
    unit_quat_rotate(P->u2, c.pw, rot2);
    c.p2[0] = rot2[0] + P->t2[0];
    c.p2[1] = rot2[1] + P->t2[1];
    c.p2[2] = rot2[2] + P->t2[2];
    c.mag = fabs(smp.pc1[0]) + fabs(smp.pc1[1]) + fabs(smp.pc1[2]) + fabs(P->t1[0]) + fabs(P->t1[1]) +
            fabs(P->t1[2]) + fabs(c.pw[0]) + fabs(c.pw[1]) + fabs(c.pw[2]) + fabs(P->t2[0]) + fabs(P->t2[1]) +
            fabs(P->t2[2]);
    c.w[0] = smp.pc1[0] - P->t1[0];
    c.w[1] = smp.pc1[1] - P->t1[1];
    c.w[2] = smp.pc1[2] - P->t1[2];
    const double u2 = c.p2[0] / c.p2[2];
    const double v2 = c.p2[1] / c.p2[2];
    double x2, y2;
    world_to_image<M>(K2, u2, v2, &x2, &y2);
    const int cpx = cast_to_int_x86(round(x2));
    const int cpy = cast_to_int_x86(round(y2));
    const bool cin = !(cpx < 0 || cpx >= a.W || cpy < 0 || cpy >= a.H);
    FlatBox fb;
    const bool cand = COARSE == 3   ? flat_box_coarse<M, false, true>(P, c, K2, u2, v2, x2, y2, fb)
                      : COARSE == 2 ? flat_box_coarse<M, true>(P, c, K2, u2, v2, x2, y2, fb)
                      : COARSE == 1 ? flat_box_coarse<M>(P, c, K2, u2, v2, x2, y2, fb)
                                    : flat_box<M>(P, c, K2, fb);
    bool decided = false;   // the centre outcome and the flat test are settled without the raster
    bool resolved = false;  // the centre outcome is settled (the flat test may have failed)
    if constexpr (LP) {
      // label planes: one 8-B tile depth range (a line shared by the wave's
      // neighbouring samples) settles the depth test of the whole box; on the
      // valid side the box's labels come from the 1-B label plane
      if (cand && fb.x0 >= 0 && fb.y0 >= 0 && fb.x0 + fb.ncol <= a.W && fb.y0 + fb.nrow <= a.H && cpx >= fb.x0 &&
          cpx < fb.x0 + fb.ncol && cpy >= fb.y0 && cpy < fb.y0 + fb.nrow) {
        // the tile range and the box's labels requested together (one round
        // trip; the labels go unused when the depth test settles the box invalid)
        const float2 dr = a.dtile[P->toff + (size_t)(fb.y0 >> 3) * a.TW + (fb.x0 >> 3)];
        const uint8_t* lp = a.lab8 + P->roff + (size_t)fb.y0 * a.W + fb.x0;
        const uint8_t lc = lp[(size_t)(cpy - fb.y0) * a.W + (cpx - fb.x0)];
        uint8_t L[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) L[q] = (q % 3 < fb.ncol && q / 3 < fb.nrow) ? lp[(size_t)(q / 3) * a.W + q % 3] : lc;
        const int side = tile_depth_side(a, fb, dr, c.p2[2], c.mag);
        if (side == 2) {
          c.st = MI_BA_INVALID_DEPTH;
          c.r = 0.0;
          decided = resolved = true;
        } else if (side == 1) {
          c.st = MI_BA_VALID;
          c.r = (smp.label1 == spal[lc]) ? 0.0 : 1.0;
          bool flat = true;
#pragma unroll
          for (int q = 0; q < 9; ++q) flat = flat && ((smp.label1 == spal[L[q]]) ? 0.0 : 1.0) == c.r;
          resolved = true;
          decided = flat;
          deferred = !flat;
        }
      }
    }
    if constexpr (WS) {
      // one 16-B read of the window holding the box (its top-left pixel)
      if (!resolved && cand && fb.x0 >= 0 && fb.y0 >= 0 && fb.x0 + 2 < a.W && fb.y0 + 2 < a.H) {
        const float4 w = a.wsum[P->roff + (size_t)fb.y0 * a.W + fb.x0];
        decided = resolved = window_decides(a, fb, w, c.p2[2], c.mag, smp.label1, &c.st, &c.r);
      }
    }
    if (!resolved && cand &&
        (fb.x0 + fb.ncol <= 0 || fb.x0 >= a.W || fb.y0 + fb.nrow <= 0 || fb.y0 >= a.H)) {
      // every reachable pixel (the centre's among them) lies outside the
      // raster: the centre and every stencil point are OUT_OF_BOUNDS (f = 0),
      // the flat test's outcome without a raster read (14 % of C4's samples)
      c.st = MI_BA_OUT_OF_BOUNDS;
      c.r = 0.0;
      decided = resolved = true;
    }
    if (!resolved) {
      // every raster read of the sample in one round trip: the centre pixel and the box
      const float2 sc = dl2[cin ? cpy * a.W + cpx : 0];
      float2 s[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) s[q] = dl2[flat_index(a, fb, cand, q)];
      // centre outcome (semantic_cost_functions.h:141-205)
      if (!cin) {
        c.st = MI_BA_OUT_OF_BOUNDS;
        c.r = 0.0;
      } else if (fabs((double)sc.x - c.p2[2]) > a.threshold) {
        c.st = MI_BA_INVALID_DEPTH;
        c.r = 0.0;
      } else {
        c.st = MI_BA_VALID;
        c.r = (smp.label1 == sc.y) ? 0.0 : 1.0;
      }
      deferred = !(cand && flat_check(a, fb, s, c.p2[2], c.mag, smp.label1, c.r));
    }
    double rho[3];
    loss_eval(a.loss_type, a.loss_scale, c.r * c.r, rho);
    cost = 0.5 * (a.weight * rho[0]);
    if (write_samples) {
      r_out[n] = c.r;
      status_out[n] = c.st + ((write_samples & 2) && deferred ? 0x1000 : 0) + ((write_samples & 4) && decided ? 0x4000 : 0);
      if (!deferred) {
        double2* jo = reinterpret_cast<double2*>(J_out + 12 * n);
#pragma unroll
        for (int m = 0; m < 6; ++m) jo[m] = make_double2(0.0, 0.0);
      }
    }
  }
  // the wave's deferred samples as one mask word (tile-major, 4 words per
  // tile): deferred_order_kernel lists them per pair in sample order
  const unsigned long long bal = __ballot(deferred);
  if (lane == 0) dmask[(size_t)blockIdx.x * (kBlock / 64) + (tid >> 6)] = bal;
  double v = cost;
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane == 0) sred[tid >> 6] = v;
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) s += sred[w];
    cost_partial[blockIdx.x] = s;
  }
}

// Pass 2: chunk = 64 consecutive entries of one pair's deferred region
// (chunks past the pair's count exit at once).
// WPE: minimum waves per SIMD asked of the register allocator (tools-build
// variants; the default build's 128 VGPRs give 4 waves per SIMD, 16 of these
// 64-thread workgroups per CU)
template <int M, bool FAST, int NB, bool BOX = false, int WPE = 1>
__global__ __launch_bounds__(64, WPE) void semantic_deferred_kernel(SemArgs ak, const uint2* __restrict__ chunks,
                                                              const uint32_t* __restrict__ ccount,
                                                              const PairConst* __restrict__ pcs,
                                                              const uint32_t* __restrict__ pair_cnt,
                                                              const uint32_t* __restrict__ dlist,
                                                              const uint32_t* __restrict__ pair_chunk0,
                                                              double* __restrict__ cpart,
                                                              double* __restrict__ J_out, int write_samples,
                                                              int32_t* __restrict__ status_out = nullptr) {
  __shared__ double sJ[64 * kSemRow];
  __shared__ float2 sbox[BOX ? 64 * 9 : 1];  // BOX: each lane's 3 x 3 box of raster pixels
  // ccount (the compacted list's length, deferred_compact_kernel): a grid of
  // resident workgroups loops over the non-empty chunks; null: one chunk per
  // workgroup over the whole static list (empty chunks exit at once)
  const uint32_t nch = ccount ? *ccount : blockIdx.x + 1;
  const uint32_t stride = ccount ? gridDim.x : 1u;
  for (uint32_t ci = blockIdx.x; ci < nch; ci += stride) {
  const uint2 ch = chunks[ci];  // (pair, first entry)
  const uint32_t cnt = pair_cnt[ch.x];
  if (ch.y >= cnt) continue;  // workgroup-uniform
  const PairConst* __restrict__ P = pcs + ch.x;
  const SemArgs a = with_pair(ak, P);
  const int lane = threadIdx.x;
  const uint32_t k = ch.y + lane;
  const uint32_t pstart = a.pairs[ch.x].start;
  const float2* dl2 = a.dl + P->roff;
  const double* K2 = P->K2;
  double rowv[kSemRow];
#pragma unroll
  for (int q = 0; q < kSemRow; ++q) rowv[q] = 0.0;
  if (k < cnt) {
    const int64_t n = (int64_t)pstart + dlist[pstart + k];
    const SemSample smp = a.samples[n];
    Centre c;
    centre_eval<M, FAST>(a, P, smp, K2, dl2, c);
    double Jt[12];
    bool redone;
    if constexpr (BOX) {
      // the reachable box (the flat test's bound), read in one round trip:
      // the stencil's steps then take their pixels from LDS
      FlatBox fb;
      if (flat_box<M>(P, c, K2, fb)) {
        float2* mine = sbox + 9 * lane;
#pragma unroll
        for (int q = 0; q < 9; ++q) mine[q] = dl2[flat_index(a, fb, true, q)];
        redone = stencil_full<M, FAST, NB>(a, P, c, smp, K2, dl2, Jt, mine, &fb);
      } else {
        redone = stencil_full<M, FAST, NB>(a, P, c, smp, K2, dl2, Jt);
      }
    } else {
      redone = stencil_full<M, FAST, NB>(a, P, c, smp, K2, dl2, Jt);
    }
    if ((write_samples & 4) && status_out && redone) status_out[n] += 0x10000;  // diagnostic
    if (write_samples) {
      double2* jo = reinterpret_cast<double2*>(J_out + 12 * n);
#pragma unroll
      for (int m = 0; m < 6; ++m) jo[m] = make_double2(Jt[2 * m], Jt[2 * m + 1]);
    }
    double rho[3];
    loss_eval(a.loss_type, a.loss_scale, c.r * c.r, rho);
    const double sc = sqrt(a.weight * rho[1]);
#pragma unroll
    for (int m = 0; m < 12; ++m) rowv[m] = Jt[m] * sc;
    rowv[12] = c.r * sc;
  }
#pragma unroll
  for (int q = 0; q < kSemRow; ++q) sJ[lane * kSemRow + q] = rowv[q];
  __syncthreads();
  const int rows = min(64, (int)(cnt - ch.y));
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int e = lane + 64 * h;
    if (e < kPairVals) {
      int ca, cb;
      if (e < 78) {
        int a_ = 0, rem = e;
        while (rem >= 12 - a_) { rem -= 12 - a_; ++a_; }
        ca = a_;
        cb = a_ + rem;
      } else {
        ca = e - 78;
        cb = 12;
      }
      double acc = 0.0;
      for (int q = 0; q < rows; ++q) acc += sJ[q * kSemRow + ca] * sJ[q * kSemRow + cb];
      // the chunk's J'J / J'r, summed per pair in chunk order (pair_reduce_kernel)
      cpart[((size_t)pair_chunk0[ch.x] + ch.y / 64) * kPairVals + e] = acc;
    }
  }
  __syncthreads();  // sJ / sbox are rewritten by the next chunk
  }
}

// The pair's deferred samples in sample order from the flat pass's wave masks
// (one workgroup per pair; a pair's tiles are consecutive, 256 samples each
// from the pair's start, so mask word w covers samples 64 w .. 64 w + 63):
// popcounts, a workgroup scan, each set bit's offset.  pair_cnt = their
// number.  Sample order makes every chunk of the deferred pass, hence every
// pair block sum, the same run to run.
__global__ __launch_bounds__(256) void deferred_order_kernel(const unsigned long long* __restrict__ dmask,
                                                             const uint32_t* __restrict__ pair_tile0,
                                                             const SemPair* __restrict__ pairs,
                                                             uint32_t* __restrict__ pair_cnt,
                                                             uint32_t* __restrict__ dlist) {
  __shared__ uint32_t sc[256];
  const int p = blockIdx.x, tid = threadIdx.x;
  const SemPair pr = pairs[p];
  const uint32_t words = (pr.count + 63) / 64;
  const unsigned long long* mk = dmask + (size_t)pair_tile0[p] * (kBlock / 64);
  uint32_t base = 0;
  for (uint32_t w0 = 0; w0 < words; w0 += 256) {
    const uint32_t w = w0 + tid;
    const unsigned long long m = w < words ? mk[w] : 0ull;
    const uint32_t c = (uint32_t)__popcll(m);
    sc[tid] = c;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {  // inclusive scan (Hillis-Steele)
      const uint32_t v = tid >= off ? sc[tid - off] : 0u;
      __syncthreads();
      sc[tid] += v;
      __syncthreads();
    }
    uint32_t o = base + sc[tid] - c;
    for (unsigned long long r = m; r; r &= r - 1) dlist[pr.start + o++] = 64 * w + (uint32_t)__ffsll((long long)r) - 1;
    base += sc[255];
    __syncthreads();
  }
  if (tid == 0) pair_cnt[p] = base;
}

// Pair blocks from the deferred pass's chunk partials, summed in chunk order
// (one workgroup per pair; a pair without deferred samples gets zeros: its
// cleared samples have J = 0).
__global__ __launch_bounds__(128) void pair_reduce_kernel(const uint32_t* __restrict__ pair_cnt,
                                                          const uint32_t* __restrict__ pair_chunk0,
                                                          const double* __restrict__ cpart,
                                                          double* __restrict__ pair_blk) {
  const int p = blockIdx.x, e = threadIdx.x;
  if (e >= kPairVals) return;
  const uint32_t nch = (pair_cnt[p] + 63) / 64;
  const double* c = cpart + (size_t)pair_chunk0[p] * kPairVals + e;
  double v = 0.0;
  for (uint32_t j = 0; j < nch; ++j) v += c[(size_t)j * kPairVals];
  pair_blk[(size_t)p * kPairStride + e] = v;
}

// The deferred pass's work list: the static list of every pair's possible
// 64-entry chunks (grouped by model, model_chunks) filtered to the chunks the
// flat pass filled (first entry < pair_cnt), per model into the same region
// of `out`, counts in cnt[model] (zeroed before).  Launching one workgroup per
// static chunk instead spent the deferred pass's time dispatching the ~92 %
// that are empty (80k workgroups for 6.4k chunks at C4).  One atomic per
// workgroup and model; the order within a model is the atomics' (the pair sums already
// accumulate by atomics in any order).
struct ModelRanges {
  int b[kNumModels + 1];
};

__global__ __launch_bounds__(256) void deferred_compact_kernel(const uint2* __restrict__ chunks, int nchunks,
                                                               const uint32_t* __restrict__ pair_cnt, ModelRanges mr,
                                                               uint2* __restrict__ out, uint32_t* __restrict__ cnt) {
  // one atomic per workgroup and model: per-wave counts through LDS, the
  // workgroup's base per model, then each wave's offset inside it
  __shared__ uint32_t swc[4][kNumModels];
  __shared__ uint32_t sbase[kNumModels];
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool valid = i < nchunks;
  uint2 ch = make_uint2(0u, 0u);
  int m = 0;
  bool live = false;
  if (valid) {
    ch = chunks[i];
    live = ch.y < pair_cnt[ch.x];
    while (m + 1 < kNumModels && i >= mr.b[m + 1]) ++m;
  }
  uint32_t rank = 0;  // the lane's rank among its wave's live chunks of its model
#pragma unroll
  for (int mm = 0; mm < kNumModels; ++mm) {
    const unsigned long long sel = __ballot(live && m == mm);
    if (lane == 0) swc[wv][mm] = (uint32_t)__popcll(sel);
    if (live && m == mm) rank = (uint32_t)__popcll(sel & ((1ull << lane) - 1ull));
  }
  __syncthreads();
  if (threadIdx.x < kNumModels) {
    const uint32_t tot = swc[0][threadIdx.x] + swc[1][threadIdx.x] + swc[2][threadIdx.x] + swc[3][threadIdx.x];
    sbase[threadIdx.x] = tot ? atomicAdd(cnt + threadIdx.x, tot) : 0u;
  }
  __syncthreads();
  if (live) {
    uint32_t off = sbase[m];
    for (int w = 0; w < wv; ++w) off += swc[w][m];
    out[mr.b[m] + off + rank] = ch;
  }
}

template <int M>
__global__ __launch_bounds__(kBlock) void semantic_cost_kernel(SemArgs a, double* __restrict__ partial) {
  __shared__ double sred[4];
  const int64_t n = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double c = 0.0;
  if (n < a.ns) {
    const SemSample smp = a.samples[n];
    const SemPair pr = a.pairs[smp.pair];
    const double* qt1 = a.qt + 8 * (size_t)pr.i;
    const double* qt2 = a.qt + 8 * (size_t)pr.j;
    const double q1[4] = {qt1[0], qt1[1], qt1[2], qt1[3]}, t1[3] = {qt1[4], qt1[5], qt1[6]};
    const double q2[4] = {qt2[0], qt2[1], qt2[2], qt2[3]}, t2[3] = {qt2[4], qt2[5], qt2[6]};
    constexpr int np = Model<M>::kNumParams;
    double K2[np];
    const uint32_t cam2 = a.img_cam[pr.j];
    const double* kc = a.cam + 8 * (size_t)cam2;
#pragma unroll
    for (int m = 0; m < np; ++m) K2[m] = kc[m];
    const SlotInfo si = a.slots[a.raster_slot[pr.j]];
    SemArgs aj = a;  // image j's raster size
    aj.H = si.H;
    aj.W = si.W;
    int st;
    double r;
    if constexpr (M == kMixedModels) {
      switch_model(a.cam_model[cam2], [&](auto m) {
        r = semantic_error<decltype(m)::value>(aj, smp.pc1, smp.label1, q1, t1, q2, t2, K2, a.dl + si.off, &st);
      });
    } else {
      r = semantic_error<M>(aj, smp.pc1, smp.label1, q1, t1, q2, t2, K2, a.dl + si.off, &st);
    }
    double rho[3];
    loss_eval(a.loss_type, a.loss_scale, r * r, rho);
    c = 0.5 * (a.weight * rho[0]);
  }
  // block sum
  double v = c;
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = sred[0] + sred[1] + sred[2] + sred[3];
}

__device__ inline int sym12(int a, int b) {  // a <= b
  return a * 12 - (a * (a - 1)) / 2 + (b - a);
}

// Fold pair blocks into the per-image Schur-Jacobi blocks, b, diag(U).
// The pair blocks folded into their images' slots deterministically: each
// image (or S block) sums its pairs in pair order (img_pairs / sblk_ent,
// built once), no float atomics.  Entry (pair << 1) | side: the image is the
// pair's first (side 0) or second (1) pose; a pose that is not variable takes
// nothing.

// Schur-Jacobi pose block (21), b (6) and diag(U) (6) of every image: one
// 64-thread workgroup per image, thread e one of the 33 values.
__global__ void semantic_fblock_kernel(const SemPair* __restrict__ pairs, const uint32_t* __restrict__ img_pairs_off,
                                       const uint32_t* __restrict__ img_pairs, const double* __restrict__ pair_blk,
                                       double* __restrict__ pose_blk, double* __restrict__ bvec,
                                       double* __restrict__ udiag) {
  const uint32_t img = blockIdx.x;
  const int e = threadIdx.x;
  if (e >= 33) return;
  int a = 0, b = 0;
  if (e < 21) {
    int rem = e;
    while (rem >= 6 - a) { rem -= 6 - a; ++a; }
    b = a + rem;
  } else {
    a = b = (e - 21) % 6;
  }
  double v = 0.0;
  bool any = false;
  for (uint32_t q = img_pairs_off[img]; q < img_pairs_off[img + 1]; ++q) {
    const uint32_t k = img_pairs[q] >> 1, side = img_pairs[q] & 1u;
    const SemPair pr = pairs[k];
    if (!(side ? pr.var2 : pr.var1)) continue;
    const double* B = pair_blk + (size_t)k * kPairStride;
    const int base = 6 * (int)side;
    v += e < 21 || e >= 27 ? B[sym12(base + a, base + b)] : B[78 + base + a];
    any = true;
  }
  if (!any) return;
  if (e < 21)
    pose_blk[21 * (size_t)img + e] += v;
  else if (e < 27)
    bvec[6 * (size_t)img + a] += v;
  else
    udiag[6 * (size_t)img + a] += v;
}

// g += J'r of the pair blocks on the image's pose (the raw gradient of the
// gradient tolerance test).
__global__ void semantic_gradient_kernel(const SemPair* __restrict__ pairs, const uint32_t* __restrict__ img_pairs_off,
                                         const uint32_t* __restrict__ img_pairs, const double* __restrict__ pair_blk,
                                         double* __restrict__ g) {
  const uint32_t img = blockIdx.x;
  const int a = threadIdx.x;
  if (a >= 6) return;
  double v = 0.0;
  for (uint32_t q = img_pairs_off[img]; q < img_pairs_off[img + 1]; ++q) {
    const uint32_t k = img_pairs[q] >> 1, side = img_pairs[q] & 1u;
    const SemPair pr = pairs[k];
    if (!(side ? pr.var2 : pr.var1)) continue;
    v += pair_blk[(size_t)k * kPairStride + 78 + 6 * side + a];
  }
  g[6 * (size_t)img + a] += v;
}

// y += M x on the image's pose rows: row (6 side + a) of each pair's M times
// the pair's two poses of x.
__global__ void semantic_product_kernel(const SemPair* __restrict__ pairs, const uint32_t* __restrict__ img_pairs_off,
                                        const uint32_t* __restrict__ img_pairs, const double* __restrict__ pair_blk,
                                        const double* __restrict__ x, double* __restrict__ y) {
  const uint32_t img = blockIdx.x;
  const int a = threadIdx.x;
  if (a >= 6) return;
  double v = 0.0;
  bool any = false;
  for (uint32_t q = img_pairs_off[img]; q < img_pairs_off[img + 1]; ++q) {
    const uint32_t k = img_pairs[q] >> 1, side = img_pairs[q] & 1u;
    const SemPair pr = pairs[k];
    if (!(side ? pr.var2 : pr.var1)) continue;
    const double* B = pair_blk + (size_t)k * kPairStride;
    const int r = 6 * (int)side + a;
    double s = 0.0;
    for (int c = 0; c < 12; ++c) {
      const bool vc = c < 6 ? pr.var1 : pr.var2;
      const double xc = vc ? x[6 * (size_t)(c < 6 ? pr.i : pr.j) + c % 6] : 0.0;
      s += B[r <= c ? sym12(r, c) : sym12(c, r)] * xc;
    }
    v += s;
    any = true;
  }
  if (any) y[6 * (size_t)img + a] += v;
}

// Pair blocks into the explicit reduced camera system (upper triangle,
// row-major with leading dimension lds): one workgroup per 6 x 6 S block (i,
// j), i <= j, thread (a, b); the block's contributions in pair order.  Entry
// flag: diagonal block — image i is the pair's first (M11) or second (M22)
// pose; off-diagonal — rows i are the pair's first pose (M[a][6 + b]) or its
// second (M[6 + a][b]).
__global__ void semantic_dense_kernel(const SemPair* __restrict__ pairs, const uint2* __restrict__ sblk,
                                      const uint32_t* __restrict__ sblk_off, const uint32_t* __restrict__ sblk_ent,
                                      const double* __restrict__ pair_blk, int64_t lds, double* __restrict__ S) {
  const uint2 bl = sblk[blockIdx.x];
  const int a = threadIdx.x / 6, b = threadIdx.x % 6;
  if (threadIdx.x >= 36 || (bl.x == bl.y && a > b)) return;
  double v = 0.0;
  bool any = false;
  for (uint32_t q = sblk_off[blockIdx.x]; q < sblk_off[blockIdx.x + 1]; ++q) {
    const uint32_t k = sblk_ent[q] >> 1, f = sblk_ent[q] & 1u;
    const SemPair pr = pairs[k];
    int A, B;
    bool va, vb;
    if (bl.x == bl.y) {
      A = 6 * (int)f + a;
      B = 6 * (int)f + b;
      va = vb = f ? pr.var2 : pr.var1;
    } else if (!f) {
      A = a;
      B = 6 + b;
      va = pr.var1;
      vb = pr.var2;
    } else {
      A = 6 + a;
      B = b;
      va = pr.var2;
      vb = pr.var1;
    }
    if (!va || !vb) continue;
    v += pair_blk[(size_t)k * kPairStride + (A <= B ? sym12(A, B) : sym12(B, A))];
    any = true;
  }
  if (any) S[(6 * (int64_t)bl.x + a) * lds + 6 * (int64_t)bl.y + b] += v;
}

// model cost change -(g'd + d'Md/2) per pair, one partial per wave (summed
// by launch_sum in a fixed order)
__global__ void semantic_model_kernel(const SemPair* __restrict__ pairs, int npairs,
                                      const double* __restrict__ pair_blk, const double* __restrict__ df,
                                      double* __restrict__ partial) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  double v = 0.0;
  if (k < npairs) {
    const SemPair pr = pairs[k];
    const double* B = pair_blk + (size_t)k * kPairStride;
    double d[12];
    for (int m = 0; m < 6; ++m) {
      d[m] = pr.var1 ? df[6 * (size_t)pr.i + m] : 0.0;
      d[6 + m] = pr.var2 ? df[6 * (size_t)pr.j + m] : 0.0;
    }
    double gd = 0.0, dMd = 0.0;
    for (int a = 0; a < 12; ++a) {
      gd += B[78 + a] * d[a];
      double s = 0.0;
      for (int b = 0; b < 12; ++b) s += B[a <= b ? sym12(a, b) : sym12(b, a)] * d[b];
      dMd += d[a] * s;
    }
    v = -(gd + 0.5 * dMd);
  }
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if (threadIdx.x == 0) partial[blockIdx.x] = v;
}

// ExportSemanticErrorToCSV (semantic_bundle_adjustment.cc:908-1019): every
// pixel of image i's grid (y outer, x inner, step `step`; zero-depth pixels
// included, unlike the problem's samples) evaluated against image j at the
// current parameters by compute_semantic_error — status, error, the rounded
// pixel in image j and the world point.  One lane per grid pixel.
__global__ __launch_bounds__(kBlock) void semantic_export_kernel(SemArgs a, uint32_t i, uint32_t j, int step, int nx,
                                                                  int64_t n, int32_t* __restrict__ pix,
                                                                  int32_t* __restrict__ status,
                                                                  double* __restrict__ err,
                                                                  double* __restrict__ world) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const int x = (int)(k % nx) * step, y = (int)(k / nx) * step;
  const uint32_t cam1 = a.img_cam[i], cam2 = a.img_cam[j];
  const double* K1 = a.cam + 8 * (size_t)cam1;
  const double* kc = a.cam + 8 * (size_t)cam2;
  double K2[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) K2[m] = kc[m];
  const SlotInfo s1 = a.slots[a.raster_slot[i]], s2 = a.slots[a.raster_slot[j]];
  const float2 c1 = a.dl[s1.off + (size_t)y * s1.W + x];
  double u1 = 0.0, v1 = 0.0;
  image_to_world_any(a.cam_model[cam1], K1, (double)x, (double)y, &u1, &v1);
  const double depth = (double)c1.x;
  const double pc1[3] = {u1 * depth, v1 * depth, depth};
  const double* qt1 = a.qt + 8 * (size_t)i;
  const double* qt2 = a.qt + 8 * (size_t)j;
  const double q1[4] = {qt1[0], qt1[1], qt1[2], qt1[3]}, t1[3] = {qt1[4], qt1[5], qt1[6]};
  const double q2[4] = {qt2[0], qt2[1], qt2[2], qt2[3]}, t2[3] = {qt2[4], qt2[5], qt2[6]};
  const float2* dl2 = a.dl + s2.off;
  SemArgs aj = a;  // image j's raster size
  aj.H = s2.H;
  aj.W = s2.W;
  int st = 0;
  double r = 0.0, pw[3] = {0.0, 0.0, 0.0};
  int pxy[2] = {0, 0};
  switch_model(a.cam_model[cam2], [&](auto m) {
    r = semantic_error<decltype(m)::value>(aj, pc1, c1.y, q1, t1, q2, t2, K2, dl2, &st, pw, pxy);
  });
  pix[4 * k] = x;
  pix[4 * k + 1] = y;
  pix[4 * k + 2] = pxy[0];
  pix[4 * k + 3] = pxy[1];
  status[k] = st;
  err[k] = r;
  world[3 * k] = pw[0];
  world[3 * k + 1] = pw[1];
  world[3 * k + 2] = pw[2];
}

SemArgs make_args(mi_ba_context* ctx, const double* qt, const double* cam) {
  SemanticState* S = ctx->sem;
  SemArgs a;
  a.samples = S->samples.ptr;
  a.pairs = S->pairs.ptr;
  a.qt = qt;
  a.cam = cam;
  a.img_cam = ctx->dev.img_cam;
  a.cam_model = ctx->dev.cam_model;
  a.img_flags = ctx->dev.img_flags;
  a.raster_slot = S->raster_slot.ptr;
  a.slots = S->slots.ptr;
  a.dl = S->dl.ptr;
  a.wsum = S->use_wsum ? S->wsum.ptr : nullptr;
  a.lab8 = S->use_lp ? S->lab8.ptr : nullptr;
  a.dtile = S->use_lp ? S->dtile.ptr : nullptr;
  a.pal = S->use_lp ? S->pal.ptr : nullptr;
  a.TW = 0;  // per pair (with_pair)
  a.H = 0;
  a.W = 0;
  a.threshold = S->depth_threshold;
  a.rel_step = S->rel_step;
  a.ns = S->ns;
  a.loss_type = ctx->options.loss_function_type;
  a.loss_scale = ctx->options.loss_function_scale;
  a.weight = ctx->options.semantic_weight;
  return a;
}

}  // namespace

mi_ba_status semantic_create(mi_ba_context* ctx, const mi_ba_semantic* sem) {
  const mi_ba_problem* p = &ctx->problem;
  const mi_ba_options& o = ctx->options;
  const bool per_image = sem->image_height || sem->image_width;
  if ((per_image && !(sem->image_height && sem->image_width)) ||
      (!per_image && (sem->height <= 0 || sem->width <= 0)) || !sem->depth || !sem->label || sem->num_pairs < 0 ||
      (sem->num_pairs > 0 && !sem->pairs) || sem->pixel_step <= 0)
    return MI_BA_ERR_INVALID_ARGUMENT;
  const int I = p->num_images;
  // each image's raster size and plane (ABI 4: per-image sizes, planes back to
  // back in image order)
  std::vector<int32_t> img_h(I), img_w(I);
  std::vector<size_t> img_off(I);
  {
    size_t off = 0;
    for (int i = 0; i < I; ++i) {
      img_h[i] = per_image ? sem->image_height[i] : sem->height;
      img_w[i] = per_image ? sem->image_width[i] : sem->width;
      if (img_h[i] < 0 || img_w[i] < 0) return MI_BA_ERR_INVALID_ARGUMENT;
      img_off[i] = off;
      off += (size_t)img_h[i] * img_w[i];
    }
  }
  for (int k = 0; k < sem->num_pairs; ++k) {
    const int i = sem->pairs[2 * k], j = sem->pairs[2 * k + 1];
    if (i < 0 || i >= I || j < 0 || j >= I) return MI_BA_ERR_INVALID_ARGUMENT;
    if (i != j && (img_h[i] <= 0 || img_w[i] <= 0 || img_h[j] <= 0 || img_w[j] <= 0))
      return MI_BA_ERR_INVALID_ARGUMENT;
  }
  auto* S = new SemanticState();
  ctx->sem = S;
  S->img_h = img_h;
  S->img_w = img_w;
  S->depth_threshold = sem->depth_error_threshold;
  S->rel_step = sem->numeric_relative_step_size;
  S->step = sem->pixel_step;
  const HostSetup& hs = ctx->setup;
  auto const_pose = [&](int i) {
    return !o.refine_extrinsics || (p->image_constant_pose && p->image_constant_pose[i]);
  };
  std::vector<SemSample> samples;
  std::vector<SemTile> tiles;
  std::vector<int32_t> slot(I, -1);
  std::vector<int> slot_images;
  for (int k = 0; k < sem->num_pairs; ++k) {
    const int i = sem->pairs[2 * k], j = sem->pairs[2 * k + 1];
    if (i < 0 || i >= I || j < 0 || j >= I) { semantic_destroy(ctx); return MI_BA_ERR_INVALID_ARGUMENT; }
    // AddImagePairToProblem: skip i == j (:703) and both-constant pairs (:784-789)
    if (i == j) continue;
    const bool c1 = const_pose(i), c2 = const_pose(j);
    if (c1 && c2) continue;
    SemPair pr;
    pr.i = (uint32_t)i;
    pr.j = (uint32_t)j;
    pr.var1 = !c1;
    pr.var2 = !c2;
    pr.start = (uint32_t)samples.size();
    const double* K1 = p->camera_params + hs.cam_off[p->image_camera[i]];
    const int model1 = hs.cam_model[p->image_camera[i]];
    const float* d1 = sem->depth + img_off[i];
    const float* l1 = sem->label + img_off[i];
    const int H = img_h[i], W = img_w[i];  // image 1's own size (:792-793)
    const uint32_t pair_idx = (uint32_t)S->pairs_host.size();
    // pixel grid: y outer, x inner (:796-799); skip depth < 1e-4 (:806-814)
    for (int y = 0; y < H; y += sem->pixel_step) {
      for (int x = 0; x < W; x += sem->pixel_step) {
        const float depth = d1[(size_t)y * W + x];
        if (depth < 1e-4) continue;
        double u1 = 0, v1 = 0;
        image_to_world_any(model1, K1, (double)x, (double)y, &u1, &v1);
        SemSample smp;
        smp.pc1[0] = u1 * (double)depth;
        smp.pc1[1] = v1 * (double)depth;
        smp.pc1[2] = (double)depth;
        smp.label1 = l1[(size_t)y * W + x];
        smp.pair = pair_idx;
        samples.push_back(smp);
        S->sample_pixel_host.push_back((int32_t)k);
        S->sample_pixel_host.push_back(x);
        S->sample_pixel_host.push_back(y);
      }
    }
    pr.count = (uint32_t)(samples.size() - pr.start);
    for (uint32_t t0 = 0; t0 < pr.count; t0 += kBlock) {  // one workgroup per tile
      SemTile t;
      t.pair = pair_idx;
      t.start = pr.start + t0;
      t.count = std::min<uint32_t>(kBlock, pr.count - t0);
      t.pad = 0;
      tiles.push_back(t);
    }
    S->pairs_host.push_back(pr);
    if (slot[j] < 0) {
      slot[j] = (int32_t)slot_images.size();
      slot_images.push_back(j);
    }
    // poses touched by semantic blocks are variable parameter blocks
    // (SetUpManifolds, semantic_bundle_adjustment.cc:670-693)
    if (!c1 && !ctx->setup.img_var[i]) {
      ctx->setup.img_var[i] = 1;
      ctx->setup.img_tvec_mask[i] = p->image_constant_tvec ? p->image_constant_tvec[i] : 0;
      int masked = 0;
      for (int b = 0; b < 3; ++b) masked += (ctx->setup.img_tvec_mask[i] >> b) & 1;
      ctx->setup.num_effective_parameters_reduced += 6 - masked;
    }
    if (!c2 && !ctx->setup.img_var[j]) {
      ctx->setup.img_var[j] = 1;
      ctx->setup.img_tvec_mask[j] = p->image_constant_tvec ? p->image_constant_tvec[j] : 0;
      int masked = 0;
      for (int b = 0; b < 3; ++b) masked += (ctx->setup.img_tvec_mask[j] >> b) & 1;
      ctx->setup.num_effective_parameters_reduced += 6 - masked;
    }
  }
  S->ns = (int64_t)samples.size();
  S->npairs = (int)S->pairs_host.size();
  // refresh image flags on the device (poses made variable by the semantic term)
  {
    std::vector<uint32_t> fl(I);
    for (int i = 0; i < I; ++i)
      fl[i] = (ctx->setup.img_var[i] ? 1u : 0u) | ((uint32_t)ctx->setup.img_tvec_mask[i] << 1);
    if (I && hipMemcpy(ctx->img_flags.ptr, fl.data(), I * 4, hipMemcpyHostToDevice) != hipSuccess) {
      return MI_BA_ERR_HIP;
    }
  }
  // the slots' planes (rasters / label planes / window summaries) and tile planes
  S->slots_host.resize(slot_images.size());
  {
    uint64_t off = 0, toff = 0;
    for (size_t k = 0; k < slot_images.size(); ++k) {
      const int j = slot_images[k];
      SlotInfo& si = S->slots_host[k];
      si.H = img_h[j];
      si.W = img_w[j];
      si.TW = (si.W + 7) / 8;
      si.pad = 0;
      si.off = off;
      si.toff = toff;
      const int64_t plane = (int64_t)si.H * si.W, tiles = (int64_t)((si.H + 7) / 8) * si.TW;
      if (plane > INT32_MAX - 256) return MI_BA_ERR_INVALID_ARGUMENT;  // per-slot kernels index a plane in int
      off += (uint64_t)plane;
      toff += (uint64_t)tiles;
      S->max_plane = std::max<int>(S->max_plane, (int)plane);
      S->max_tiles = std::max<int>(S->max_tiles, (int)tiles);
    }
    S->npix = (int64_t)off;
    S->ntile = (int64_t)toff;
  }
  std::vector<uint32_t> slot_u(I, 0);
  for (int i = 0; i < I; ++i) slot_u[i] = slot[i] < 0 ? 0u : (uint32_t)slot[i];
  S->nslots = (int)slot_images.size();
  S->has_raster.assign(I, 0);
  for (int i = 0; i < I; ++i) S->has_raster[i] = slot[i] >= 0;
  // tiles grouped by the model of the pair's second camera (one launch per
  // model present; order within a model unchanged)
  {
    auto tile_model = [&](const SemTile& t) { return hs.cam_model[p->image_camera[S->pairs_host[t.pair].j]]; };
    std::stable_sort(tiles.begin(), tiles.end(),
                     [&](const SemTile& x, const SemTile& y) { return tile_model(x) < tile_model(y); });
    for (int m = 0; m <= kNumModels; ++m) S->model_tiles[m] = 0;
    for (const SemTile& t : tiles) S->model_tiles[tile_model(t) + 1]++;
    for (int m = 0; m < kNumModels; ++m) S->model_tiles[m + 1] += S->model_tiles[m];
  }
  S->ntiles = (int)tiles.size();
  // 64-entry chunks of every pair's deferred region, grouped by model like the tiles
  std::vector<uint2> chunks;
  {
    std::vector<std::vector<uint2>> per(kNumModels);
    for (int k = 0; k < S->npairs; ++k) {
      const SemPair& pr = S->pairs_host[k];
      const int m = hs.cam_model[p->image_camera[pr.j]];
      for (uint32_t off = 0; off < pr.count; off += 64) per[m].push_back(make_uint2((uint32_t)k, off));
    }
    S->model_chunks[0] = 0;
    for (int m = 0; m < kNumModels; ++m) {
      chunks.insert(chunks.end(), per[m].begin(), per[m].end());
      S->model_chunks[m + 1] = (int)chunks.size();
    }
  }
  if (S->pair_cnt.alloc(std::max(1, S->npairs)) || S->dlist.alloc(std::max<int64_t>(1, S->ns)) ||
      S->chunks.alloc(std::max<size_t>(1, chunks.size())) || S->dchunks.alloc(std::max<size_t>(1, chunks.size())) ||
      S->dcount.alloc(kNumModels))
    return MI_BA_ERR_OUT_OF_MEMORY;
  // deterministic sums (see SemanticState)
  {
    const int np = S->npairs;
    std::vector<uint32_t> tile0(std::max(1, np), 0), chunk0(std::max(1, np), 0);
    for (size_t k = tiles.size(); k-- > 0;) tile0[tiles[k].pair] = (uint32_t)k;  // first tile of each pair
    std::vector<uint32_t> nchk(std::max(1, np), 0);
    for (const uint2& c : chunks) ++nchk[c.x];
    for (size_t k = chunks.size(); k-- > 0;) chunk0[chunks[k].x] = (uint32_t)k;
    // a pair's tiles and chunks are consecutive (grouped by model, pair order inside)
    for (int k = 0; k < np; ++k) {
      const SemPair& pr = S->pairs_host[k];
      const uint32_t nt = (pr.count + kBlock - 1) / kBlock;
      for (uint32_t j = 0; j < nt; ++j)
        if (tiles[tile0[k] + j].pair != (uint32_t)k || tiles[tile0[k] + j].start != pr.start + j * kBlock)
          return MI_BA_ERR_HIP;
      for (uint32_t j = 0; j < nchk[k]; ++j)
        if (chunks[chunk0[k] + j].x != (uint32_t)k || chunks[chunk0[k] + j].y != 64 * j) return MI_BA_ERR_HIP;
    }
    // the pairs of each image, and the S blocks' contributions
    std::vector<uint32_t> ipo(I + 1, 0), ip;
    for (int k = 0; k < np; ++k) {
      ++ipo[S->pairs_host[k].i + 1];
      ++ipo[S->pairs_host[k].j + 1];
    }
    for (int i = 0; i < I; ++i) ipo[i + 1] += ipo[i];
    ip.resize(ipo[I]);
    {
      std::vector<uint32_t> pos(ipo.begin(), ipo.end() - 1);
      for (int k = 0; k < np; ++k) {
        ip[pos[S->pairs_host[k].i]++] = (uint32_t)k << 1;
        ip[pos[S->pairs_host[k].j]++] = (uint32_t)k << 1 | 1u;
      }
    }
    std::map<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>> blocks;
    for (int k = 0; k < np; ++k) {
      const SemPair& pr = S->pairs_host[k];
      blocks[{pr.i, pr.i}].push_back((uint32_t)k << 1);       // M11 on image i's diagonal block
      blocks[{pr.j, pr.j}].push_back((uint32_t)k << 1 | 1u);  // M22 on image j's
      if (pr.i < pr.j)
        blocks[{pr.i, pr.j}].push_back((uint32_t)k << 1);      // rows i (first), columns j
      else
        blocks[{pr.j, pr.i}].push_back((uint32_t)k << 1 | 1u); // rows j (second), columns i
    }
    std::vector<uint2> sb;
    std::vector<uint32_t> so(1, 0), se;
    for (auto& b : blocks) {
      sb.push_back(make_uint2(b.first.first, b.first.second));
      se.insert(se.end(), b.second.begin(), b.second.end());
      so.push_back((uint32_t)se.size());
    }
    S->nsblk = (int)sb.size();
    if (S->dmask.alloc(std::max<size_t>(1, tiles.size()) * (kBlock / 64)) || S->pair_tile0.alloc(tile0.size()) ||
        S->pair_chunk0.alloc(chunk0.size()) || S->cpart.alloc(std::max<size_t>(1, chunks.size()) * kPairVals) ||
        S->img_pairs_off.alloc(ipo.size()) || S->img_pairs.alloc(std::max<size_t>(1, ip.size())) ||
        S->sblk.alloc(std::max<size_t>(1, sb.size())) || S->sblk_off.alloc(so.size()) ||
        S->sblk_ent.alloc(std::max<size_t>(1, se.size())) || S->mpart.alloc((std::max(1, np) + 63) / 64))
      return MI_BA_ERR_OUT_OF_MEMORY;
    if (hipMemcpy(S->pair_tile0.ptr, tile0.data(), tile0.size() * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(S->pair_chunk0.ptr, chunk0.data(), chunk0.size() * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(S->img_pairs_off.ptr, ipo.data(), ipo.size() * 4, hipMemcpyHostToDevice) ||
        (!ip.empty() && hipMemcpy(S->img_pairs.ptr, ip.data(), ip.size() * 4, hipMemcpyHostToDevice)) ||
        (!sb.empty() && hipMemcpy(S->sblk.ptr, sb.data(), sb.size() * sizeof(uint2), hipMemcpyHostToDevice)) ||
        hipMemcpy(S->sblk_off.ptr, so.data(), so.size() * 4, hipMemcpyHostToDevice) ||
        (!se.empty() && hipMemcpy(S->sblk_ent.ptr, se.data(), se.size() * 4, hipMemcpyHostToDevice)))
      return MI_BA_ERR_HIP;
  }
  {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) ||
        ncu <= 0)
      ncu = 256;
    S->n_cu = ncu;
  }
  if (!chunks.empty() && hipMemcpy(S->chunks.ptr, chunks.data(), chunks.size() * sizeof(uint2), hipMemcpyHostToDevice))
    return MI_BA_ERR_HIP;
  if (S->samples.alloc(S->ns) || S->pairs.alloc(S->npairs) || S->raster_slot.alloc(I) ||
      S->slots.alloc(std::max<size_t>(1, S->slots_host.size())) ||
      S->dl.alloc(std::max<size_t>(1, (size_t)S->npix)) || S->r.alloc(S->ns) ||
      S->status.alloc(S->ns) || S->J.alloc(12 * S->ns) ||
      S->pair_blk.alloc((size_t)kPairStride * std::max(1, S->npairs)) || S->tiles.alloc(tiles.size()) ||
      S->pconst.alloc(sizeof(PairConst) / sizeof(double) * std::max(1, S->npairs)))
    return MI_BA_ERR_OUT_OF_MEMORY;
  S->npartial = std::max<int64_t>({(int64_t)tiles.size(), (S->ns + kBlock - 1) / kBlock, (int64_t)1});
  if (S->partial.alloc(S->npartial)) return MI_BA_ERR_OUT_OF_MEMORY;
  if ((S->ns && hipMemcpy(S->samples.ptr, samples.data(), S->ns * sizeof(SemSample), hipMemcpyHostToDevice)) ||
      (S->npairs &&
       hipMemcpy(S->pairs.ptr, S->pairs_host.data(), S->npairs * sizeof(SemPair), hipMemcpyHostToDevice)) ||
      (I && hipMemcpy(S->raster_slot.ptr, slot_u.data(), I * 4, hipMemcpyHostToDevice)) ||
      (!S->slots_host.empty() && hipMemcpy(S->slots.ptr, S->slots_host.data(), S->slots_host.size() * sizeof(SlotInfo),
                                           hipMemcpyHostToDevice)) ||
      (!tiles.empty() &&
       hipMemcpy(S->tiles.ptr, tiles.data(), tiles.size() * sizeof(SemTile), hipMemcpyHostToDevice)))
    return MI_BA_ERR_HIP;
  // rasters interleaved (depth, label): one 8-B gather per pixel test
  std::vector<float2> buf((size_t)S->max_plane);
  for (size_t s = 0; s < slot_images.size(); ++s) {
    const int j = slot_images[s];
    const size_t plane = (size_t)img_h[j] * img_w[j];
    const float* d = sem->depth + img_off[j];
    const float* l = sem->label + img_off[j];
    for (size_t k = 0; k < plane; ++k) buf[k] = make_float2(d[k], l[k]);
    if (hipMemcpy(S->dl.ptr + S->slots_host[s].off, buf.data(), plane * sizeof(float2), hipMemcpyHostToDevice))
      return MI_BA_ERR_HIP;
  }
  // the flat pass's label planes (3.9M of 5.0M C4 samples settled without the
  // float rasters, 1.1 GB), else (more than 256 distinct labels) the 3x3
  // window summaries (2.8M, 16 B per raster pixel): semantic step 0.41 ->
  // 0.39 ms at C4 either way (profiles/r4_ab_semantic_label_planes.jsonl);
  // without the memory for them the flat pass reads the rasters alone
  mi_ba_status st = semantic_set_label_planes(ctx, true);
  if (st == MI_BA_ERR_HIP) return st;
  if (!S->use_lp && semantic_set_window_summary(ctx, true) == MI_BA_ERR_HIP) return MI_BA_ERR_HIP;
  return MI_BA_OK;
}

mi_ba_status semantic_export(mi_ba_context* ctx, int32_t image1, int32_t image2, int64_t* count, int32_t* pixels,
                             int32_t* status, double* error, double* world) {
  SemanticState* S = ctx->sem;
  const int I = ctx->problem.num_images;
  if (!S || !count || image1 < 0 || image1 >= I || image2 < 0 || image2 >= I || image1 == image2)
    return MI_BA_ERR_INVALID_ARGUMENT;
  // image 1's own grid (ExportSemanticErrorToCSV loops over image 1's map, :953-956)
  const int H1 = S->img_h[image1], W1 = S->img_w[image1];
  const int nx = (W1 + S->step - 1) / S->step, ny = (H1 + S->step - 1) / S->step;
  const int64_t n = (int64_t)nx * ny;
  *count = n;
  if (!pixels) return MI_BA_OK;
  if (!status || !error || !world) return MI_BA_ERR_INVALID_ARGUMENT;
  if (!S->has_raster[image1] || !S->has_raster[image2]) return MI_BA_ERR_UNSUPPORTED;
  if (n == 0) return MI_BA_OK;
  DevArray<int32_t> d_pix, d_st;
  DevArray<double> d_err, d_w;
  if (d_pix.alloc(4 * n) || d_st.alloc(n) || d_err.alloc(n) || d_w.alloc(3 * n)) return MI_BA_ERR_OUT_OF_MEMORY;
  SemArgs a = make_args(ctx, ctx->dev.qt, ctx->dev.cam);
  hipLaunchKernelGGL(semantic_export_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                     a, (uint32_t)image1, (uint32_t)image2, S->step, nx, n, d_pix.ptr, d_st.ptr, d_err.ptr, d_w.ptr);
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(pixels, d_pix.ptr, 16 * n, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipMemcpyAsync(status, d_st.ptr, 4 * n, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipMemcpyAsync(error, d_err.ptr, 8 * n, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipMemcpyAsync(world, d_w.ptr, 24 * n, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    return MI_BA_ERR_HIP;
  return MI_BA_OK;
}

mi_ba_status semantic_set_window_summary(mi_ba_context* ctx, bool on) {
  SemanticState* S = ctx->sem;
  if (!S) return MI_BA_ERR_STATE;
  if (on && !S->wsum.ptr) {
    const int64_t n = S->npix;
    if (n > 0) {
      if (S->wsum.alloc((size_t)n)) {
        (void)hipGetLastError();
        S->use_wsum = false;
        return MI_BA_ERR_OUT_OF_MEMORY;
      }
      hipLaunchKernelGGL(window_summary_kernel, dim3((unsigned)((S->max_plane + 255) / 256), (unsigned)S->nslots),
                         dim3(256), 0, ctx->stream, S->dl.ptr, S->slots.ptr, S->wsum.ptr);
      if (hipGetLastError() != hipSuccess) return MI_BA_ERR_HIP;
    }
  }
  if (!on) S->wsum.release();
  S->use_wsum = on && S->wsum.ptr != nullptr;
  return MI_BA_OK;
}

mi_ba_status semantic_set_label_planes(mi_ba_context* ctx, bool on) {
  SemanticState* S = ctx->sem;
  if (!S) return MI_BA_ERR_STATE;
  if (!on) {
    S->lab8.release();
    S->dtile.release();
    S->pal.release();
    S->use_lp = false;
    return MI_BA_OK;
  }
  if (S->use_lp) return MI_BA_OK;
  const int64_t n = S->npix;
  if (n <= 0) return MI_BA_OK;
  const int64_t nt = S->ntile;
  DevArray<unsigned long long> keys;
  DevArray<unsigned> overflow;
  if (keys.alloc(256) || overflow.alloc(1) || S->lab8.alloc((size_t)n) || S->dtile.alloc((size_t)nt) ||
      S->pal.alloc(256)) {
    (void)hipGetLastError();
    S->lab8.release();
    S->dtile.release();
    S->pal.release();
    return MI_BA_ERR_OUT_OF_MEMORY;
  }
  hipStream_t s = ctx->stream;
  const unsigned g = (unsigned)((n + 255) / 256);
  if (hipMemsetAsync(keys.ptr, 0, keys.bytes(), s) != hipSuccess ||
      hipMemsetAsync(overflow.ptr, 0, overflow.bytes(), s) != hipSuccess)
    return MI_BA_ERR_HIP;
  hipLaunchKernelGGL(label_palette_kernel, dim3(g), dim3(256), 0, s, S->dl.ptr, n, keys.ptr, overflow.ptr);
  unsigned long long hk[256];
  unsigned ov = 0;
  if (hipGetLastError() != hipSuccess || hipMemcpyAsync(hk, keys.ptr, sizeof(hk), hipMemcpyDeviceToHost, s) ||
      hipMemcpyAsync(&ov, overflow.ptr, sizeof(ov), hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
    return MI_BA_ERR_HIP;
  if (ov) {  // more than 256 distinct labels: the flat pass reads the rasters
    S->lab8.release();
    S->dtile.release();
    S->pal.release();
    return MI_BA_OK;
  }
  float hp[256];
  for (int k = 0; k < 256; ++k) {
    const uint32_t b = (uint32_t)(hk[k] & 0xffffffffull);
    std::memcpy(&hp[k], &b, 4);
  }
  hipLaunchKernelGGL(label_index_kernel, dim3(g), dim3(256), 0, s, S->dl.ptr, n, keys.ptr, S->lab8.ptr);
  hipLaunchKernelGGL(depth_tile_kernel, dim3((unsigned)((S->max_tiles + 255) / 256), (unsigned)S->nslots), dim3(256),
                     0, s, S->dl.ptr, S->slots.ptr, S->dtile.ptr);
  if (hipGetLastError() != hipSuccess || hipMemcpyAsync(S->pal.ptr, hp, sizeof(hp), hipMemcpyHostToDevice, s) ||
      hipStreamSynchronize(s))
    return MI_BA_ERR_HIP;
  S->use_lp = true;
  return MI_BA_OK;
}

void semantic_destroy(mi_ba_context* ctx) {
  if (!ctx->sem) return;
  delete ctx->sem;
  ctx->sem = nullptr;
}

// The per-pair stencil tables and the cleared accumulators of one
// linearization (semantic_pair_prep_kernel) on `stream`.
mi_ba_status semantic_pair_prep(mi_ba_context* ctx, hipStream_t stream) {
  SemanticState* S = ctx->sem;
  if (!S || S->ns == 0 || S->npairs == 0) return MI_BA_OK;
  SemArgs a = make_args(ctx, ctx->dev.qt, ctx->dev.cam);
  PairConst* pcs = reinterpret_cast<PairConst*>(S->pconst.ptr);
  hipLaunchKernelGGL(semantic_pair_prep_kernel, dim3((S->npairs + 1) / 2), dim3(64), 0, stream, S->pairs.ptr,
                     S->npairs, a.qt, a.cam, a.img_cam, a.img_flags, a.raster_slot, a.slots, a.rel_step, pcs,
                     S->pair_blk.ptr,
                     kPairStride, ctx->sem_variant == 6 ? S->pair_cnt.ptr : nullptr,
                     ctx->sem_variant == 6 ? S->dcount.ptr : nullptr, kNumModels);
  return hipGetLastError() == hipSuccess ? MI_BA_OK : MI_BA_ERR_HIP;
}

// deferred_stream: when given (two-pass route), the deferred-sample pass is
// launched there instead (after an event on ctx->stream marks the flat pass
// done), and the caller joins it; the cost is complete on ctx->stream.
mi_ba_status semantic_linearize(mi_ba_context* ctx, double* d_cost, bool write_samples, hipStream_t deferred_stream,
                                hipEvent_t flat_done, hipEvent_t timer_start, const double* other_partial,
                                int64_t other_n, double* other_out, double* other_scratch,
                                const std::function<mi_ba_status()>& after_flat, hipEvent_t prep_done) {
  SemanticState* S = ctx->sem;
  hipStream_t s = ctx->stream;
  S->samples_valid = write_samples;
  if (S->ns == 0) {
    if (S->npairs && hipMemsetAsync(S->pair_blk.ptr, 0, S->pair_blk.bytes(), s) != hipSuccess) return MI_BA_ERR_HIP;
    if (other_partial) launch_sum(other_partial, other_n, other_out, s, other_scratch);
    return MI_BA_OK;
  }
  SemArgs a = make_args(ctx, ctx->dev.qt, ctx->dev.cam);
  PairConst* pcs = reinterpret_cast<PairConst*>(S->pconst.ptr);
  hipEvent_t stop;
  timer_begin_after(ctx, "semantic_jacobian", timer_start, &stop);
  if (prep_done) {
    // the pair tables were formed on a side stream beside the reprojection
    // kernel (semantic_pair_prep)
    if (hipStreamWaitEvent(s, prep_done, 0) != hipSuccess) return MI_BA_ERR_HIP;
  } else {
    const mi_ba_status st = semantic_pair_prep(ctx, s);
    if (st != MI_BA_OK) return st;
  }
  const bool split = deferred_stream != nullptr && ctx->sem_variant == 6;
  if (ctx->sem_variant == 6) {
    const int ws = write_samples ? 1 | (ctx->sem_diag ? 2 : 0) | (ctx->sem_diag == 2 ? 4 : 0) : 0;
    auto deferred = [&](hipStream_t ds) -> mi_ba_status {
      // each pair's deferred samples in sample order (pair_cnt, dlist)
      hipLaunchKernelGGL(deferred_order_kernel, dim3(S->npairs), dim3(256), 0, ds, S->dmask.ptr, S->pair_tile0.ptr,
                         S->pairs.ptr, S->pair_cnt.ptr, S->dlist.ptr);
      // the non-empty chunks, then a resident grid per model looping over them
      const int nall = S->model_chunks[kNumModels];
      const bool compact = ctx->sem_compact != 0;
      if (nall > 0 && compact) {
        ModelRanges mr;
        for (int m = 0; m <= kNumModels; ++m) mr.b[m] = S->model_chunks[m];
        // dcount was zeroed by the pair prep kernel (ordered before the flat pass)
        hipLaunchKernelGGL(deferred_compact_kernel, dim3((unsigned)((nall + 255) / 256)), dim3(256), 0, ds,
                           S->chunks.ptr, nall, S->pair_cnt.ptr, mr, S->dchunks.ptr, S->dcount.ptr);
      }
      for (int model = 0; model < kNumModels; ++model) {
        const int c0 = S->model_chunks[model], nc = S->model_chunks[model + 1] - c0;
        if (S->model_tiles[model + 1] == S->model_tiles[model] || nc == 0) continue;
        // compact: a grid of 64-thread workgroups, semantic_deferred_grid per CU
        // (16 resident at 128 VGPRs, LDS would allow 24 at 6.6 KB each; 24
        // measured 6 us faster than 16: the extra ones take the second round's
        // chunks as the first finish); else one per static chunk
        const int grid = compact ? std::min(nc, std::max(1, ctx->sem_dgrid) * S->n_cu) : nc;
        const uint2* list = (compact ? S->dchunks.ptr : S->chunks.ptr) + c0;
        const uint32_t* count = compact ? S->dcount.ptr + model : nullptr;
        dispatch_model(model, [&](auto m) {
          constexpr int M = decltype(m)::value;
          if (ctx->sem_deferred_box)
            hipLaunchKernelGGL((semantic_deferred_kernel<M, true, 4, true>), dim3(grid), dim3(64), 0, ds, a, list,
                               count, pcs, S->pair_cnt.ptr, S->dlist.ptr, S->pair_chunk0.ptr, S->cpart.ptr, S->J.ptr,
                               ws, S->status.ptr);
#ifdef MI_BA_AB_VARIANTS
          // semantic_deferred_variant: 1 NB 2; 2 NB 2 at >= 5 waves per SIMD;
          // 3 NB 4 at >= 5; 4 NB 2 at >= 6 (register spills)
          else if (ctx->sem_dvar == 1)
            hipLaunchKernelGGL((semantic_deferred_kernel<M, true, 2>), dim3(grid), dim3(64), 0, ds, a, list, count,
                               pcs, S->pair_cnt.ptr, S->dlist.ptr, S->pair_chunk0.ptr, S->cpart.ptr, S->J.ptr, ws,
                               S->status.ptr);
          else if (ctx->sem_dvar == 2)
            hipLaunchKernelGGL((semantic_deferred_kernel<M, true, 2, false, 5>), dim3(grid), dim3(64), 0, ds, a,
                               list, count, pcs, S->pair_cnt.ptr, S->dlist.ptr, S->pair_chunk0.ptr, S->cpart.ptr, S->J.ptr,
                               ws, S->status.ptr);
          else if (ctx->sem_dvar == 3)
            hipLaunchKernelGGL((semantic_deferred_kernel<M, true, 4, false, 5>), dim3(grid), dim3(64), 0, ds, a,
                               list, count, pcs, S->pair_cnt.ptr, S->dlist.ptr, S->pair_chunk0.ptr, S->cpart.ptr, S->J.ptr,
                               ws, S->status.ptr);
          else if (ctx->sem_dvar == 4)
            hipLaunchKernelGGL((semantic_deferred_kernel<M, true, 2, false, 6>), dim3(grid), dim3(64), 0, ds, a,
                               list, count, pcs, S->pair_cnt.ptr, S->dlist.ptr, S->pair_chunk0.ptr, S->cpart.ptr, S->J.ptr,
                               ws, S->status.ptr);
#endif
          else
            hipLaunchKernelGGL((semantic_deferred_kernel<M, true, 4>), dim3(grid), dim3(64), 0, ds, a, list, count,
                               pcs, S->pair_cnt.ptr, S->dlist.ptr, S->pair_chunk0.ptr, S->cpart.ptr, S->J.ptr, ws,
                               S->status.ptr);
        });
      }
      // pair blocks from the chunk partials, in chunk order
      hipLaunchKernelGGL(pair_reduce_kernel, dim3(S->npairs), dim3(128), 0, ds, S->pair_cnt.ptr, S->pair_chunk0.ptr,
                         S->cpart.ptr, S->pair_blk.ptr);
      return MI_BA_OK;
    };
    for (int model = 0; model < kNumModels; ++model) {
      const int t0 = S->model_tiles[model], nt = S->model_tiles[model + 1] - t0;
      if (nt == 0) continue;
      dispatch_model(model, [&](auto m) {
        constexpr int M = decltype(m)::value;
        auto launch = [&](auto ws_, auto lp_, auto coarse_) {
          hipLaunchKernelGGL((semantic_flat_kernel<M, true, decltype(ws_)::value, decltype(lp_)::value,
                                                   decltype(coarse_)::value>),
                             dim3(nt), dim3(kBlock), 0, s, a, S->tiles.ptr + t0, pcs,
                             S->dmask.ptr + (size_t)t0 * (kBlock / 64), S->partial.ptr + t0, S->r.ptr, S->status.ptr,
                             S->J.ptr, ws);
        };
        using T = std::true_type;
        using F = std::false_type;
        using C0 = std::integral_constant<int, 0>;
        using C1 = std::integral_constant<int, 1>;
        using C2 = std::integral_constant<int, 2>;
        using C3 = std::integral_constant<int, 3>;
        auto pick = [&](auto ws_, auto lp_) {
          if (ctx->sem_coarse == 3) launch(ws_, lp_, C3{});
          else if (ctx->sem_coarse == 2) launch(ws_, lp_, C2{});
          else if (ctx->sem_coarse == 1) launch(ws_, lp_, C1{});
          else launch(ws_, lp_, C0{});
        };
        if (a.lab8)
          pick(F{}, T{});
        else if (a.wsum)
          pick(T{}, F{});
        else
          pick(F{}, F{});
      });
    }
    if (after_flat) {
      const mi_ba_status st = after_flat();
      if (st != MI_BA_OK) return st;
    }
    if (split) {
      if (hipEventRecord(flat_done, s) != hipSuccess || hipStreamWaitEvent(deferred_stream, flat_done, 0) != hipSuccess)
        return MI_BA_ERR_HIP;
      const mi_ba_status st = deferred(deferred_stream);
      if (st != MI_BA_OK) return st;
    } else {
      const mi_ba_status st = deferred(s);
      if (st != MI_BA_OK) return st;
    }
  }
#ifdef MI_BA_AB_VARIANTS
  // the one-kernel routes (variants 0-5), kept for A/B in the tools build
  for (int model = 0; model < kNumModels && ctx->sem_variant != 6; ++model) {
    const int t0 = S->model_tiles[model], nt = S->model_tiles[model + 1] - t0;
    if (nt == 0) continue;
    dispatch_model(model, [&](auto m) {
      constexpr int M = decltype(m)::value;
      auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(nt), dim3(kBlock), 0, s, a, S->tiles.ptr + t0, pcs, S->pair_blk.ptr,
                           S->partial.ptr + t0, S->r.ptr, S->status.ptr, S->J.ptr,
                           write_samples ? 1 | (ctx->sem_diag ? 2 : 0) | (ctx->sem_diag == 2 ? 4 : 0) : 0);
      };
      switch (ctx->sem_variant) {
        case 0: launch(semantic_linearize_kernel<M, false>); break;
        case 1: launch(semantic_linearize_kernel<M, true>); break;
        case 2: launch(semantic_linearize_kernel<M, true, 1>); break;
        case 3: launch(semantic_linearize_kernel<M, true, 2>); break;
        case 4: launch(semantic_linearize_kernel<M, true, 4>); break;
        default: launch(semantic_linearize_kernel<M, true, 4, true>); break;
      }
    });
  }
#endif
  timer_end(ctx, stop);
  if (other_partial)
    launch_sum2(other_partial, other_n, other_out, other_scratch, S->partial.ptr, S->ntiles, d_cost, s);
  else
    launch_sum(S->partial.ptr, S->ntiles, d_cost, s);
  if (hipGetLastError() != hipSuccess) return MI_BA_ERR_HIP;
  return MI_BA_OK;
}

void semantic_cost(mi_ba_context* ctx, const double* qt, const double* cam, double* d_cost) {
  SemanticState* S = ctx->sem;
  if (S->ns == 0) return;
  SemArgs a = make_args(ctx, qt, cam);
  const unsigned g = (unsigned)((S->ns + kBlock - 1) / kBlock);
  if (ctx->dev.model == kMixedModels) {
    hipLaunchKernelGGL(semantic_cost_kernel<kMixedModels>, dim3(g), dim3(kBlock), 0, ctx->stream, a, S->partial.ptr);
  } else {
    dispatch_model(ctx->dev.model, [&](auto m) {
      constexpr int M = decltype(m)::value;
      hipLaunchKernelGGL(semantic_cost_kernel<M>, dim3(g), dim3(kBlock), 0, ctx->stream, a, S->partial.ptr);
    });
  }
  launch_sum(S->partial.ptr, g, d_cost, ctx->stream);
}

void semantic_add_fblock(mi_ba_context* ctx) {
  SemanticState* S = ctx->sem;
  const int I = ctx->dev.num_images;
  if (!S->npairs || I == 0) return;
  hipLaunchKernelGGL(semantic_fblock_kernel, dim3(I), dim3(64), 0, ctx->stream, S->pairs.ptr, S->img_pairs_off.ptr,
                     S->img_pairs.ptr, S->pair_blk.ptr, ctx->pose_blk.ptr, ctx->bvec.ptr, ctx->udiag.ptr);
}

void semantic_add_gradient(mi_ba_context* ctx, double* g) {
  SemanticState* S = ctx->sem;
  const int I = ctx->dev.num_images;
  if (!S->npairs || I == 0) return;
  hipLaunchKernelGGL(semantic_gradient_kernel, dim3(I), dim3(64), 0, ctx->stream, S->pairs.ptr, S->img_pairs_off.ptr,
                     S->img_pairs.ptr, S->pair_blk.ptr, g);
}

void semantic_schur_product(mi_ba_context* ctx, const double* x, double* y) {
  SemanticState* S = ctx->sem;
  const int I = ctx->dev.num_images;
  if (!S->npairs || I == 0) return;
  hipLaunchKernelGGL(semantic_product_kernel, dim3(I), dim3(64), 0, ctx->stream, S->pairs.ptr, S->img_pairs_off.ptr,
                     S->img_pairs.ptr, S->pair_blk.ptr, x, y);
}

void semantic_add_dense(mi_ba_context* ctx, double* S) {
  SemanticState* S_ = ctx->sem;
  if (!S_->npairs || S_->nsblk == 0) return;
  hipLaunchKernelGGL(semantic_dense_kernel, dim3(S_->nsblk), dim3(64), 0, ctx->stream, S_->pairs.ptr, S_->sblk.ptr,
                     S_->sblk_off.ptr, S_->sblk_ent.ptr, S_->pair_blk.ptr, ctx->dev.lds, S);
}

void semantic_model_cost(mi_ba_context* ctx, const double* df, double* d_out) {
  SemanticState* S = ctx->sem;
  if (!S->npairs) return;
  const int nw = (S->npairs + 63) / 64;
  hipLaunchKernelGGL(semantic_model_kernel, dim3(nw), dim3(64), 0, ctx->stream, S->pairs.ptr, S->npairs,
                     S->pair_blk.ptr, df, S->mpart.ptr);
  launch_sum(S->mpart.ptr, nw, d_out, ctx->stream);
}

}  // namespace miba
