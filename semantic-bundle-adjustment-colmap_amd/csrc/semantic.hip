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
// Samples are grouped by image pair, so J'J, J'r reduce per pair in
// pair-aligned tiles (one atomic flush per tile).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>

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
  const uint32_t* img_flags;
  const uint32_t* raster_slot;
  const float* depth;
  const float* label;
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

// compute_semantic_error (semantic_cost_functions.h:87-208).
template <int M>
__device__ inline double semantic_error(const SemArgs& a, const double pc1[3], float label1, const double* q1,
                                        const double* t1, const double* q2, const double* t2, const double* K2,
                                        const float* depth2, const float* label2, int* status) {
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
  if (px < 0 || px >= a.W || py < 0 || py >= a.H) {
    *status = MI_BA_OUT_OF_BOUNDS;
    return 0.0;
  }
  const size_t off = (size_t)py * a.W + px;
  const double depth_2 = (double)depth2[off];
  if (fabs(depth_2 - measured_depth_2) > a.threshold) {
    *status = MI_BA_INVALID_DEPTH;
    return 0.0;
  }
  *status = MI_BA_VALID;
  return (label1 == label2[off]) ? 0.0 : 1.0;
}

// ---------------------------------------------------------------------------
// The same evaluation split into its pose-1 / pose-2 stages so the CENTRAL
// stencil recomputes only what the perturbed parameter feeds.  Each stage is
// exactly the operation sequence of semantic_error above, so every stencil
// value is bitwise the one the unsplit evaluation (and the CPU reference)
// produces.
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

// P_w = rot + t_inv with t_inv = -(R t1)
__device__ inline void pose1_world(const Pose1Stage& s, const double* t1, double pw[3]) {
  const double ti0 = -(s.R[0] * t1[0] + s.R[1] * t1[1] + s.R[2] * t1[2]);
  const double ti1 = -(s.R[3] * t1[0] + s.R[4] * t1[1] + s.R[5] * t1[2]);
  const double ti2 = -(s.R[6] * t1[0] + s.R[7] * t1[1] + s.R[8] * t1[2]);
  pw[0] = s.rot[0] + ti0;
  pw[1] = s.rot[1] + ti1;
  pw[2] = s.rot[2] + ti2;
}

__device__ inline void unit_quat(const double* q, double u[4]) {
  const double scale = 1.0 / sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  u[0] = scale * q[0];
  u[1] = scale * q[1];
  u[2] = scale * q[2];
  u[3] = scale * q[3];
}

struct PixelCache {   // the centre evaluation's raster reads
  int px, py;
  float depth, label;
  bool valid;
};

// Projection into image 2 and the raster tests (semantic_cost_functions.h:141-205).
template <int M>
__device__ inline double project_test(const SemArgs& a, const double p2[3], float label1, const double* K2,
                                      const float* depth2, const float* label2, PixelCache& pc, bool centre,
                                      int* status) {
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
  float d2, l2;
  if (!centre && pc.valid && px == pc.px && py == pc.py) {
    d2 = pc.depth;
    l2 = pc.label;
  } else {
    const size_t off = (size_t)py * a.W + px;
    d2 = depth2[off];
    l2 = label2[off];
    if (centre) {
      pc.px = px; pc.py = py; pc.depth = d2; pc.label = l2; pc.valid = true;
    }
  }
  if (fabs((double)d2 - measured_depth_2) > a.threshold) {
    *status = MI_BA_INVALID_DEPTH;
    return 0.0;
  }
  *status = MI_BA_VALID;
  return (label1 == l2) ? 0.0 : 1.0;
}

template <int M>
__global__ __launch_bounds__(kBlock) void semantic_jacobian_kernel(SemArgs a, double* __restrict__ r_out,
                                                                    int32_t* __restrict__ status_out,
                                                                    double* __restrict__ J_out) {
  const int64_t n = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (n >= a.ns) return;
  const SemSample smp = a.samples[n];
  const SemPair pr = a.pairs[smp.pair];
  const double* qt1 = a.qt + 8 * (size_t)pr.i;
  const double* qt2 = a.qt + 8 * (size_t)pr.j;
  double q1[4], t1[3], q2[4], t2[3];
#pragma unroll
  for (int m = 0; m < 4; ++m) { q1[m] = qt1[m]; q2[m] = qt2[m]; }
#pragma unroll
  for (int m = 0; m < 3; ++m) { t1[m] = qt1[4 + m]; t2[m] = qt2[4 + m]; }
  constexpr int np = Model<M>::kNumParams;
  double K2[np];
  const double* kc = a.cam + 8 * (size_t)a.img_cam[pr.j];
#pragma unroll
  for (int m = 0; m < np; ++m) K2[m] = kc[m];
  const size_t slot = a.raster_slot[pr.j];
  const float* depth2 = a.depth + slot * a.H * a.W;
  const float* label2 = a.label + slot * a.H * a.W;
  PixelCache pc;
  pc.valid = false;
  pc.px = pc.py = 0;
  pc.depth = pc.label = 0.f;
  // centre
  Pose1Stage s1;
  pose1_stage(q1, smp.pc1, s1);
  double pw[3];
  pose1_world(s1, t1, pw);
  double u2[4];
  unit_quat(q2, u2);
  double rot2[3];
  unit_quat_rotate(u2, pw, rot2);
  double p2[3] = {rot2[0] + t2[0], rot2[1] + t2[1], rot2[2] + t2[2]};
  int st = 0, st2 = 0;
  const double r = project_test<M>(a, p2, smp.label1, K2, depth2, label2, pc, true, &st);
  double Jamb[14];
#pragma unroll
  for (int m = 0; m < 14; ++m) Jamb[m] = 0.0;
  if (pr.var1) {
    // q1 stencil: pose-1 stage recomputed, normalised q2 reused
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const double orig = q1[m];
      const double delta = fmax(kMinStep, fabs(orig) * a.rel_step);
      double f[2];
#pragma unroll
      for (int sgn = 0; sgn < 2; ++sgn) {
        double qq[4] = {q1[0], q1[1], q1[2], q1[3]};
        qq[m] = sgn == 0 ? orig + delta : orig - delta;
        Pose1Stage s;
        pose1_stage(qq, smp.pc1, s);
        double w[3], rr[3];
        pose1_world(s, t1, w);
        unit_quat_rotate(u2, w, rr);
        const double pp[3] = {rr[0] + t2[0], rr[1] + t2[1], rr[2] + t2[2]};
        f[sgn] = project_test<M>(a, pp, smp.label1, K2, depth2, label2, pc, false, &st2);
      }
      double one_over_delta = 1.0 / delta;
      one_over_delta /= 2;
      Jamb[m] = (f[0] - f[1]) * one_over_delta;
    }
    // t1 stencil: rotation stage of pose 1 reused
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const double orig = t1[m];
      const double delta = fmax(kMinStep, fabs(orig) * a.rel_step);
      double f[2];
#pragma unroll
      for (int sgn = 0; sgn < 2; ++sgn) {
        double tt[3] = {t1[0], t1[1], t1[2]};
        tt[m] = sgn == 0 ? orig + delta : orig - delta;
        double w[3], rr[3];
        pose1_world(s1, tt, w);
        unit_quat_rotate(u2, w, rr);
        const double pp[3] = {rr[0] + t2[0], rr[1] + t2[1], rr[2] + t2[2]};
        f[sgn] = project_test<M>(a, pp, smp.label1, K2, depth2, label2, pc, false, &st2);
      }
      double one_over_delta = 1.0 / delta;
      one_over_delta /= 2;
      Jamb[4 + m] = (f[0] - f[1]) * one_over_delta;
    }
  }
  if (pr.var2) {
    // q2 stencil: world point reused
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const double orig = q2[m];
      const double delta = fmax(kMinStep, fabs(orig) * a.rel_step);
      double f[2];
#pragma unroll
      for (int sgn = 0; sgn < 2; ++sgn) {
        double qq[4] = {q2[0], q2[1], q2[2], q2[3]};
        qq[m] = sgn == 0 ? orig + delta : orig - delta;
        double uu[4], rr[3];
        unit_quat(qq, uu);
        unit_quat_rotate(uu, pw, rr);
        const double pp[3] = {rr[0] + t2[0], rr[1] + t2[1], rr[2] + t2[2]};
        f[sgn] = project_test<M>(a, pp, smp.label1, K2, depth2, label2, pc, false, &st2);
      }
      double one_over_delta = 1.0 / delta;
      one_over_delta /= 2;
      Jamb[7 + m] = (f[0] - f[1]) * one_over_delta;
    }
    // t2 stencil: rotated point reused
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const double orig = t2[m];
      const double delta = fmax(kMinStep, fabs(orig) * a.rel_step);
      double f[2];
#pragma unroll
      for (int sgn = 0; sgn < 2; ++sgn) {
        double pp[3] = {rot2[0] + t2[0], rot2[1] + t2[1], rot2[2] + t2[2]};
        pp[m] = rot2[m] + (sgn == 0 ? orig + delta : orig - delta);
        f[sgn] = project_test<M>(a, pp, smp.label1, K2, depth2, label2, pc, false, &st2);
      }
      double one_over_delta = 1.0 / delta;
      one_over_delta /= 2;
      Jamb[11 + m] = (f[0] - f[1]) * one_over_delta;
    }
  }
  double Jt[12];
  const double xq[2][4] = {{q1[0], q1[1], q1[2], q1[3]}, {q2[0], q2[1], q2[2], q2[3]}};
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const uint32_t img = blk == 0 ? pr.i : pr.j;
    const uint32_t mask = (a.img_flags[img] >> 1) & 7u;
    const bool var = blk == 0 ? pr.var1 != 0 : pr.var2 != 0;
    if (!var) {
#pragma unroll
      for (int m = 0; m < 6; ++m) Jt[blk * 6 + m] = 0.0;
      continue;
    }
    double PJ[12];
    quat_plus_jacobian(xq[blk], PJ);
#pragma unroll
    for (int col = 0; col < 3; ++col) {
      double acc = 0.0;
#pragma unroll
      for (int m = 0; m < 4; ++m) acc += Jamb[blk * 7 + m] * PJ[m * 3 + col];
      Jt[blk * 6 + col] = acc;
    }
#pragma unroll
    for (int col = 0; col < 3; ++col) Jt[blk * 6 + 3 + col] = ((mask >> col) & 1u) ? 0.0 : Jamb[blk * 7 + 4 + col];
  }
  r_out[n] = r;
  status_out[n] = st;
  double2* jo = reinterpret_cast<double2*>(J_out + 12 * n);
#pragma unroll
  for (int m = 0; m < 6; ++m) jo[m] = make_double2(Jt[2 * m], Jt[2 * m + 1]);
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
    const double* kc = a.cam + 8 * (size_t)a.img_cam[pr.j];
#pragma unroll
    for (int m = 0; m < np; ++m) K2[m] = kc[m];
    const size_t slot = a.raster_slot[pr.j];
    int st;
    const double r = semantic_error<M>(a, smp.pc1, smp.label1, q1, t1, q2, t2, K2, a.depth + slot * a.H * a.W,
                                       a.label + slot * a.H * a.W, &st);
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

// Per-pair tile reduction of the loss-corrected J'J (packed 12x12 upper, 78)
// and J'r (12), plus the cost.
constexpr int kPairVals = 78 + 12;
constexpr int kPairStride = 96;  // padded record per pair

__global__ __launch_bounds__(kBlock) void semantic_reduce_kernel(const SemTile* __restrict__ tiles,
                                                                  const double* __restrict__ r_in,
                                                                  const double* __restrict__ J_in, int loss_type,
                                                                  double loss_scale, double weight,
                                                                  double* __restrict__ pair_blk,
                                                                  double* __restrict__ cost_partial) {
  __shared__ double sred[4 * (kPairVals + 1)];
  const SemTile t = tiles[blockIdx.x];
  double acc[kPairVals + 1];
#pragma unroll
  for (int k = 0; k < kPairVals + 1; ++k) acc[k] = 0.0;
  for (uint32_t k = threadIdx.x; k < t.count; k += kBlock) {
    const int64_t n = (int64_t)t.start + k;
    double r = r_in[n];
    double J[12];
#pragma unroll
    for (int m = 0; m < 12; ++m) J[m] = J_in[12 * n + m];
    double rho[3];
    loss_eval(loss_type, loss_scale, r * r, rho);
    acc[kPairVals] += 0.5 * (weight * rho[0]);
    // ScaledLoss(w) Corrector, rho'' <= 0 branch: sqrt(w * rho')
    const double sc = sqrt(weight * rho[1]);
    r *= sc;
#pragma unroll
    for (int m = 0; m < 12; ++m) J[m] *= sc;
    int o = 0;
#pragma unroll
    for (int a = 0; a < 12; ++a)
#pragma unroll
      for (int b = a; b < 12; ++b, ++o) acc[o] += J[a] * J[b];
#pragma unroll
    for (int a = 0; a < 12; ++a) acc[78 + a] += J[a] * r;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kPairVals + 1; ++k) {
    double v = acc[k];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) sred[wid * (kPairVals + 1) + k] = v;
  }
  __syncthreads();
  const int k = threadIdx.x;
  if (k < kPairVals + 1) {
    const double v = sred[k] + sred[(kPairVals + 1) + k] + sred[2 * (kPairVals + 1) + k] + sred[3 * (kPairVals + 1) + k];
    if (k < kPairVals) {
      atomicAdd(pair_blk + (size_t)t.pair * kPairStride + k, v);
    } else {
      cost_partial[blockIdx.x] = v;
    }
  }
}

__device__ inline int sym12(int a, int b) {  // a <= b
  return a * 12 - (a * (a - 1)) / 2 + (b - a);
}

// Fold pair blocks into the per-image Schur-Jacobi blocks, b, diag(U).
__global__ void semantic_fblock_kernel(const SemPair* __restrict__ pairs, int npairs,
                                       const double* __restrict__ pair_blk, double* __restrict__ pose_blk,
                                       double* __restrict__ bvec, double* __restrict__ udiag) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= npairs) return;
  const SemPair pr = pairs[k];
  const double* B = pair_blk + (size_t)k * kPairStride;
  for (int side = 0; side < 2; ++side) {
    if (!(side == 0 ? pr.var1 : pr.var2)) continue;
    const uint32_t img = side == 0 ? pr.i : pr.j;
    const int base = side * 6;
    int o = 0;
    for (int a = 0; a < 6; ++a)
      for (int b = a; b < 6; ++b, ++o) atomicAdd(pose_blk + 21 * (size_t)img + o, B[sym12(base + a, base + b)]);
    for (int a = 0; a < 6; ++a) {
      atomicAdd(bvec + 6 * (size_t)img + a, B[78 + base + a]);
      atomicAdd(udiag + 6 * (size_t)img + a, B[sym12(base + a, base + a)]);
    }
  }
}

// y += M x over the pair's two poses.
__global__ void semantic_product_kernel(const SemPair* __restrict__ pairs, int npairs,
                                        const double* __restrict__ pair_blk, const double* __restrict__ x,
                                        double* __restrict__ y) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= npairs) return;
  const SemPair pr = pairs[k];
  const double* B = pair_blk + (size_t)k * kPairStride;
  double xv[12];
  for (int m = 0; m < 6; ++m) {
    xv[m] = pr.var1 ? x[6 * (size_t)pr.i + m] : 0.0;
    xv[6 + m] = pr.var2 ? x[6 * (size_t)pr.j + m] : 0.0;
  }
  for (int a = 0; a < 12; ++a) {
    if (!(a < 6 ? pr.var1 : pr.var2)) continue;
    double s = 0.0;
    for (int b = 0; b < 12; ++b) s += B[a <= b ? sym12(a, b) : sym12(b, a)] * xv[b];
    const uint32_t img = a < 6 ? pr.i : pr.j;
    atomicAdd(y + 6 * (size_t)img + (a % 6), s);
  }
}

// Pair blocks into the explicit reduced camera system (both triangles).
__global__ void semantic_dense_kernel(const SemPair* __restrict__ pairs, int npairs,
                                      const double* __restrict__ pair_blk, int64_t nf, double* __restrict__ S) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)npairs * 144) return;
  const int k = (int)(t / 144), e = (int)(t % 144);
  const int a = e / 12, b = e % 12;
  const SemPair pr = pairs[k];
  const bool va = a < 6 ? pr.var1 : pr.var2, vb = b < 6 ? pr.var1 : pr.var2;
  if (!va || !vb) return;
  const double v = pair_blk[(size_t)k * kPairStride + (a <= b ? sym12(a, b) : sym12(b, a))];
  const int64_t ra = 6 * (int64_t)(a < 6 ? pr.i : pr.j) + a % 6;
  const int64_t rb = 6 * (int64_t)(b < 6 ? pr.i : pr.j) + b % 6;
  atomicAdd(S + ra * nf + rb, v);
}

__global__ void semantic_model_kernel(const SemPair* __restrict__ pairs, int npairs,
                                      const double* __restrict__ pair_blk, const double* __restrict__ df,
                                      double* __restrict__ out) {
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
  if ((threadIdx.x & 63) == 0) atomicAdd(out, v);
}

SemArgs make_args(mi_ba_context* ctx, const double* qt, const double* cam) {
  SemanticState* S = ctx->sem;
  SemArgs a;
  a.samples = S->samples.ptr;
  a.pairs = S->pairs.ptr;
  a.qt = qt;
  a.cam = cam;
  a.img_cam = ctx->dev.img_cam;
  a.img_flags = ctx->dev.img_flags;
  a.raster_slot = S->raster_slot.ptr;
  a.depth = S->depth.ptr;
  a.label = S->label.ptr;
  a.H = S->H;
  a.W = S->W;
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
  if (sem->height <= 0 || sem->width <= 0 || !sem->depth || !sem->label || sem->num_pairs < 0 ||
      (sem->num_pairs > 0 && !sem->pairs) || sem->pixel_step <= 0)
    return MI_BA_ERR_INVALID_ARGUMENT;
  auto* S = new SemanticState();
  ctx->sem = S;
  S->H = sem->height;
  S->W = sem->width;
  S->depth_threshold = sem->depth_error_threshold;
  S->rel_step = sem->numeric_relative_step_size;
  const int H = S->H, W = S->W, I = p->num_images;
  const int np = num_params(p->camera_model);
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
    const double* K1 = p->camera_params + (size_t)np * p->image_camera[i];
    const float* d1 = sem->depth + (size_t)i * H * W;
    const float* l1 = sem->label + (size_t)i * H * W;
    const uint32_t pair_idx = (uint32_t)S->pairs_host.size();
    // pixel grid: y outer, x inner (:796-799); skip depth < 1e-4 (:806-814)
    for (int y = 0; y < H; y += sem->pixel_step) {
      for (int x = 0; x < W; x += sem->pixel_step) {
        const float depth = d1[(size_t)y * W + x];
        if (depth < 1e-4) continue;
        double u1 = 0, v1 = 0;
        dispatch_model(p->camera_model, [&](auto m) {
          constexpr int M = decltype(m)::value;
          image_to_world<M>(K1, (double)x, (double)y, &u1, &v1);
        });
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
    for (uint32_t t0 = 0; t0 < pr.count; t0 += kTileObs) {
      SemTile t;
      t.pair = pair_idx;
      t.start = pr.start + t0;
      t.count = std::min<uint32_t>(kTileObs, pr.count - t0);
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
  const size_t plane = (size_t)H * W;
  std::vector<uint32_t> slot_u(I, 0);
  for (int i = 0; i < I; ++i) slot_u[i] = slot[i] < 0 ? 0u : (uint32_t)slot[i];
  S->ntiles = (int)tiles.size();
  if (S->samples.alloc(S->ns) || S->pairs.alloc(S->npairs) || S->raster_slot.alloc(I) ||
      S->depth.alloc(plane * std::max<size_t>(1, slot_images.size())) ||
      S->label.alloc(plane * std::max<size_t>(1, slot_images.size())) || S->r.alloc(S->ns) ||
      S->status.alloc(S->ns) || S->J.alloc(12 * S->ns) ||
      S->pair_blk.alloc((size_t)kPairStride * std::max(1, S->npairs)) || S->tiles.alloc(tiles.size()))
    return MI_BA_ERR_OUT_OF_MEMORY;
  S->npartial = std::max<int64_t>({(int64_t)tiles.size(), (S->ns + kBlock - 1) / kBlock, (int64_t)1});
  if (S->partial.alloc(S->npartial)) return MI_BA_ERR_OUT_OF_MEMORY;
  if ((S->ns && hipMemcpy(S->samples.ptr, samples.data(), S->ns * sizeof(SemSample), hipMemcpyHostToDevice)) ||
      (S->npairs &&
       hipMemcpy(S->pairs.ptr, S->pairs_host.data(), S->npairs * sizeof(SemPair), hipMemcpyHostToDevice)) ||
      (I && hipMemcpy(S->raster_slot.ptr, slot_u.data(), I * 4, hipMemcpyHostToDevice)) ||
      (!tiles.empty() &&
       hipMemcpy(S->tiles.ptr, tiles.data(), tiles.size() * sizeof(SemTile), hipMemcpyHostToDevice)))
    return MI_BA_ERR_HIP;
  for (size_t s = 0; s < slot_images.size(); ++s) {
    const int j = slot_images[s];
    if (hipMemcpy(S->depth.ptr + s * plane, sem->depth + (size_t)j * plane, plane * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(S->label.ptr + s * plane, sem->label + (size_t)j * plane, plane * 4, hipMemcpyHostToDevice))
      return MI_BA_ERR_HIP;
  }
  return MI_BA_OK;
}

void semantic_destroy(mi_ba_context* ctx) {
  if (!ctx->sem) return;
  delete ctx->sem;
  ctx->sem = nullptr;
}

mi_ba_status semantic_linearize(mi_ba_context* ctx, double* d_cost, bool write_samples) {
  (void)write_samples;
  SemanticState* S = ctx->sem;
  hipStream_t s = ctx->stream;
  if (S->npairs && hipMemsetAsync(S->pair_blk.ptr, 0, S->pair_blk.bytes(), s) != hipSuccess) return MI_BA_ERR_HIP;
  if (S->ns == 0) return MI_BA_OK;
  SemArgs a = make_args(ctx, ctx->dev.qt, ctx->dev.cam);
  hipEvent_t stop;
  timer_begin(ctx, "semantic_jacobian", &stop);
  dispatch_model(ctx->dev.model, [&](auto m) {
    constexpr int M = decltype(m)::value;
    hipLaunchKernelGGL(semantic_jacobian_kernel<M>, dim3((unsigned)((S->ns + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, s, a, S->r.ptr, S->status.ptr, S->J.ptr);
  });
  timer_end(ctx, stop);
  if (S->ntiles) {
    hipLaunchKernelGGL(semantic_reduce_kernel, dim3(S->ntiles), dim3(kBlock), 0, s, S->tiles.ptr,
                       S->r.ptr, S->J.ptr, a.loss_type, a.loss_scale, a.weight, S->pair_blk.ptr, S->partial.ptr);
    launch_sum(S->partial.ptr, S->ntiles, d_cost, s);
  }
  if (hipGetLastError() != hipSuccess) return MI_BA_ERR_HIP;
  return MI_BA_OK;
}

void semantic_cost(mi_ba_context* ctx, const double* qt, const double* cam, double* d_cost) {
  SemanticState* S = ctx->sem;
  if (S->ns == 0) return;
  SemArgs a = make_args(ctx, qt, cam);
  const unsigned g = (unsigned)((S->ns + kBlock - 1) / kBlock);
  dispatch_model(ctx->dev.model, [&](auto m) {
    constexpr int M = decltype(m)::value;
    hipLaunchKernelGGL(semantic_cost_kernel<M>, dim3(g), dim3(kBlock), 0, ctx->stream, a, S->partial.ptr);
  });
  launch_sum(S->partial.ptr, g, d_cost, ctx->stream);
}

void semantic_add_fblock(mi_ba_context* ctx) {
  SemanticState* S = ctx->sem;
  if (!S->npairs) return;
  hipLaunchKernelGGL(semantic_fblock_kernel, dim3((S->npairs + 63) / 64), dim3(64), 0, ctx->stream, S->pairs.ptr,
                     S->npairs, S->pair_blk.ptr, ctx->pose_blk.ptr, ctx->bvec.ptr, ctx->udiag.ptr);
}

void semantic_schur_product(mi_ba_context* ctx, const double* x, double* y) {
  SemanticState* S = ctx->sem;
  if (!S->npairs) return;
  hipLaunchKernelGGL(semantic_product_kernel, dim3((S->npairs + 63) / 64), dim3(64), 0, ctx->stream, S->pairs.ptr,
                     S->npairs, S->pair_blk.ptr, x, y);
}

void semantic_add_dense(mi_ba_context* ctx, double* S) {
  SemanticState* S_ = ctx->sem;
  if (!S_->npairs) return;
  const int64_t n = (int64_t)S_->npairs * 144;
  hipLaunchKernelGGL(semantic_dense_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream,
                     S_->pairs.ptr, S_->npairs, S_->pair_blk.ptr, ctx->dev.nf, S);
}

void semantic_model_cost(mi_ba_context* ctx, const double* df, double* d_out) {
  SemanticState* S = ctx->sem;
  if (!S->npairs) return;
  hipLaunchKernelGGL(semantic_model_kernel, dim3((S->npairs + 63) / 64), dim3(64), 0, ctx->stream, S->pairs.ptr,
                     S->npairs, S->pair_blk.ptr, df, d_out);
}

}  // namespace miba
