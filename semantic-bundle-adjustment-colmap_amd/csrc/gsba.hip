// gsba.hip — geometric-semantic BA (GSBA) cylinder IoU term (product code;
// see gsba.h).
//
// Restates for gfx950:
//   Cylinder::ComputeSemanticIoU / ProjectToMask / ProjectToQuadrilateral /
//   GetEdgePoints       src/util/cylinder.h:270-540
//   drawQuadrilateral   src/util/cylinder.h:21-117 (as a per-pixel predicate)
//   XYWH                src/util/xywh.h
//   simplePinholeProject src/util/utils.h:22-54
//   GSBA cost functions src/base/geometric_semantic_cost_functions.h:33-165
//   Ceres 2.1 AngleAxisRotatePoint, NumericDiffCostFunction CENTRAL,
//   QuaternionManifold (3rd party, restated)
// Built with -ffp-contract=off: the pixel predicates compare products of
// doubles against 0 exactly as the reference's x86-64 (no FMA) build does.
//
// Layout and roofline: one workgroup (4 waves) per IoU evaluation; waves take
// rows of the quadrilateral's bounding box, lanes consecutive pixels (1-byte
// trunk mask loads, coalesced along x).  Per pixel: <= 4 edge tests (2 FP64
// multiplies) and <= 4 rectangle tests; the 33 evaluations of a block scan
// nearly the same box, so the mask stays in L2 — the kernel is bound by FP64
// VALU issue, not HBM.
#include "gsba.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>

#include "ba_math.h"
#include "kernels.h"

namespace miba {

namespace {

constexpr int kGsbaFull = 0, kGsbaConstantPose = 1, kGsbaConstantCylinder = 2;
constexpr int kTB = 256;

struct Box {
  int x, y, w, h;
  __device__ int x_end() const { return x + w - 1; }
  __device__ int y_end() const { return y + h - 1; }
};

__device__ inline Box bound2(double ax, double ay, double bx, double by) {
  const double min_x = fmin(ax, bx), max_x = fmax(ax, bx);
  const double min_y = fmin(ay, by), max_y = fmax(ay, by);
  Box b;
  b.x = cast_to_int_x86(floor(min_x));
  b.y = cast_to_int_x86(floor(min_y));
  b.w = cast_to_int_x86(ceil(max_x)) - b.x + 1;
  b.h = cast_to_int_x86(ceil(max_y)) - b.y + 1;
  return b;
}

// XYWH::shrinkToFitInToFitIn(XYWH(0, 0, W, H)); the empty box is (0,0,0,0)
__device__ inline Box shrink(Box b, int W, int H) {
  const int x0 = max(b.x, 0), y0 = max(b.y, 0);
  const int x1 = min(b.x_end(), W - 1), y1 = min(b.y_end(), H - 1);
  Box o{0, 0, 0, 0};
  if (x1 < x0 || y1 < y0) return o;
  o.x = x0;
  o.y = y0;
  o.w = x1 - x0 + 1;
  o.h = y1 - y0 + 1;
  return o;
}

// QuaternionRotatePoint (normalising) + t
__device__ inline void pose_transform(const double q[4], const double t[3], const double pt[3], double r[3]) {
  const double scale = 1.0 / sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const double u[4] = {scale * q[0], scale * q[1], scale * q[2], scale * q[3]};
  unit_quat_rotate(u, pt, r);
  r[0] += t[0];
  r[1] += t[1];
  r[2] += t[2];
}

// PoseInverse (rotation_extension.h:43-79): QuaternionInverseRotation, then
// t_inv = -R(q_inv) t with QuaternionToRotation's 1 / |q|^2 normaliser.
__device__ inline void pose_inverse(const double q[4], const double t[3], double qi[4], double ti[3]) {
  const double scale = 1.0 / sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  qi[0] = scale * q[0];
  qi[1] = -(scale * q[1]);
  qi[2] = -(scale * q[2]);
  qi[3] = -(scale * q[3]);
  const double a = qi[0], b = qi[1], c = qi[2], d = qi[3];
  const double aa = a * a, ab = a * b, ac = a * c, ad = a * d;
  const double bb = b * b, bc = b * c, bd = b * d;
  const double cc = c * c, cd = c * d, dd = d * d;
  double R[9] = {aa + bb - cc - dd, 2.0 * (bc - ad), 2.0 * (ac + bd),
                 2.0 * (ad + bc),  aa - bb + cc - dd, 2.0 * (cd - ab),
                 2.0 * (bd - ac),  2.0 * (ab + cd),  aa - bb - cc + dd};
  double normalizer = a * a + b * b + c * c + d * d;
  normalizer = 1.0 / normalizer;
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] *= normalizer;
  ti[0] = -(R[0] * t[0] + R[1] * t[1] + R[2] * t[2]);
  ti[1] = -(R[3] * t[0] + R[4] * t[1] + R[5] * t[2]);
  ti[2] = -(R[6] * t[0] + R[7] * t[1] + R[8] * t[2]);
}

// Ceres 2.1 AngleAxisRotatePoint
__device__ inline void angle_axis_rotate(const double aa[3], const double pt[3], double r[3]) {
  const double theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta2 > DBL_EPSILON) {
    const double theta = sqrt(theta2);
    const double costheta = cos(theta);
    const double sintheta = sin(theta);
    const double theta_inverse = 1.0 / theta;
    const double w[3] = {aa[0] * theta_inverse, aa[1] * theta_inverse, aa[2] * theta_inverse};
    const double wx[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2], w[0] * pt[1] - w[1] * pt[0]};
    const double tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (1.0 - costheta);
    r[0] = pt[0] * costheta + wx[0] * sintheta + w[0] * tmp;
    r[1] = pt[1] * costheta + wx[1] * sintheta + w[1] * tmp;
    r[2] = pt[2] * costheta + wx[2] * sintheta + w[2] * tmp;
  } else {
    const double wx[3] = {aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2], aa[0] * pt[1] - aa[1] * pt[0]};
    r[0] = pt[0] + wx[0];
    r[1] = pt[1] + wx[1];
    r[2] = pt[2] + wx[2];
  }
}

// CylinderBy2Points (src/util/cylinder_by_2_points.h:26-155).  The
// parameters y = tvec_1(3) tvec_2(3) radius; ToCylinder (:95-117) gives the
// evaluated Cylinder (qvec, tvec_1, radius, |tvec_1 - tvec_2|): the axis
// direction d = (t2 - t1) / |t2 - t1|, rotation z -> d as the angle-axis
// acos(z . d) * (z x d) / |z x d| ((1, 0, 0) when |z x d| < 1e-10) through
// Ceres 2.1 AngleAxisToQuaternion.  Eigen's fixed-size-3 norms and dot
// products sum left to right; the constructor's Check clamps a radius <= 0 to
// 1e-4 (and Cylinder's a height <= 0).  out = q(4) t(3) r h.
MI_HD void by2_to_cylinder(const double* y, double out[9]) {
  const double radius = y[6] <= 0 ? 1e-4 : y[6];
  double d[3] = {y[3] - y[0], y[4] - y[1], y[5] - y[2]};
  const double dn = sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
  d[0] /= dn;
  d[1] /= dn;
  d[2] /= dn;
  double axis[3] = {0.0 * d[2] - 1.0 * d[1], 1.0 * d[0] - 0.0 * d[2], 0.0 * d[1] - 0.0 * d[0]};
  const double an = sqrt((axis[0] * axis[0] + axis[1] * axis[1]) + axis[2] * axis[2]);
  if (fabs(an) < 1e-10) {
    axis[0] = 1.0;
    axis[1] = 0.0;
    axis[2] = 0.0;
  } else {
    axis[0] /= an;
    axis[1] /= an;
    axis[2] /= an;
  }
  const double angle = acos((0.0 * d[0] + 0.0 * d[1]) + 1.0 * d[2]);
  const double aa[3] = {angle * axis[0], angle * axis[1], angle * axis[2]};
  // Ceres 2.1 AngleAxisToQuaternion
  const double theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta2 > 0.0) {
    const double theta = sqrt(theta2);
    const double half = theta * 0.5;
    const double k = sin(half) / theta;
    out[0] = cos(half);
    out[1] = aa[0] * k;
    out[2] = aa[1] * k;
    out[3] = aa[2] * k;
  } else {
    out[0] = 1.0;
    out[1] = aa[0] * 0.5;
    out[2] = aa[1] * 0.5;
    out[3] = aa[2] * 0.5;
  }
  out[4] = y[0];
  out[5] = y[1];
  out[6] = y[2];
  const double e0 = y[0] - y[3], e1 = y[1] - y[4], e2 = y[2] - y[5];
  const double height = sqrt((e0 * e0 + e1 * e1) + e2 * e2);
  out[7] = radius;
  out[8] = height <= 0 ? 1e-4 : height;
}

// CylinderBy2Points(const Cylinder&) (cylinder_by_2_points.h:44-48): tvec_1 =
// the lower circle centre, tvec_2 = GetEigUpperTvec() (PoseTransformPoint of
// (0, 0, height), cylinder.h:567-577), the radius; y = t1(3) t2(3) r, 0, 0.
inline void cylinder_to_by2(const mi_ba_cylinder& c, double y[9]) {
  const double* q = c.qvec;
  const double scale = 1.0 / sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const double u[4] = {scale * q[0], scale * q[1], scale * q[2], scale * q[3]};
  const double top[3] = {0, 0, c.height};
  double r[3];
  unit_quat_rotate(u, top, r);
  for (int m = 0; m < 3; ++m) {
    y[m] = c.tvec[m];
    y[3 + m] = r[m] + c.tvec[m];
  }
  y[6] = c.radius;
  y[7] = 0.0;
  y[8] = 0.0;
}

// ProjectToQuadrilateral + GetEdgePoints; false where the reference throws
// (ComputeSemanticIoU then returns 0).
__device__ inline bool project_quad(const double* x, const double K[3], double p[4][2]) {
  const double* cq = x;
  const double* ct = x + 4;
  const double* yq = x + 7;
  const double* yt = x + 11;
  double radius = x[14], height = x[15];
  if (radius <= 0) radius = 1e-4;  // Cylinder::Check on the evaluated copy
  if (height <= 0) height = 1e-4;
  double cwq[4], cwt[3];
  pose_inverse(cq, ct, cwq, cwt);
  double qi[4], ti[3];
  pose_inverse(yq, yt, qi, ti);
  double c[3];
  pose_transform(qi, ti, cwt, c);
  c[2] = 0;
  const double dist = sqrt(c[0] * c[0] + c[1] * c[1]);
  if (dist <= radius) return false;
  const double dir[3] = {c[0] / dist * radius, c[1] / dist * radius, 0};
  const double beta = acos(radius / dist);
  const double aap[3] = {0, 0, beta}, aan[3] = {0, 0, -beta};
  double e[4][3];
  angle_axis_rotate(aap, dir, e[0]);
  angle_axis_rotate(aan, dir, e[1]);
  e[2][0] = e[1][0]; e[2][1] = e[1][1]; e[2][2] = e[1][2] + height;
  e[3][0] = e[0][0]; e[3][1] = e[0][1]; e[3][2] = e[0][2] + height;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double w[3], pc[3];
    pose_transform(yq, yt, e[k], w);
    pose_transform(cq, ct, w, pc);
    if (pc[2] <= 0) return false;
    pc[0] /= pc[2];
    pc[1] /= pc[2];
    p[k][0] = K[0] * pc[0] + K[1];
    p[k][1] = K[0] * pc[1] + K[2];
  }
  const double v0x = p[1][0] - p[0][0], v0y = p[1][1] - p[0][1];
  const double v1x = p[2][0] - p[0][0], v1y = p[2][1] - p[0][1];
  if (v0x * v1y - v0y * v1x < 0) {
    double t0 = p[1][0], t1 = p[1][1];
    p[1][0] = p[3][0]; p[1][1] = p[3][1];
    p[3][0] = t0; p[3][1] = t1;
  }
  return true;
}

struct GsbaArgs {
  const GsbaBlock* blocks;
  const double* qt;        // [I][8] poses (current or candidate)
  const double* cam;       // [C][8]
  const uint32_t* img_cam;
  const double* cyl;       // [ncyl][9]
  const GsbaSlot* slots;   // [slot] each mask's plane offsets and size
  const uint8_t* masks;    // slot planes [H][W] (per-pixel kernel, tools build)
  const uint64_t* mask_bits;  // slot planes [H][words]: bit x % 64 of word x / 64 = mask pixel (y, x) != 0
  const int64_t* sem_total;
  double rel_step;
  int by2;                 // MI_BA_CYLINDER_BY_2_POINTS: cyl rows are t1(3) t2(3) r, 0, 0
};

// Ambient parameter vector of a block: camera q(4) t(3), then the cylinder's
// 9 stored values — q(4) t(3) r h, or by_2_points t1(3) t2(3) r (+ 2 unused).
__device__ inline void load_params(const GsbaArgs& a, const GsbaBlock& b, double x[16]) {
  const double* qt = a.qt + 8 * (size_t)b.img;
#pragma unroll
  for (int m = 0; m < 7; ++m) x[m] = qt[m];
  const double* y = a.cyl + 9 * (size_t)b.cyl;
#pragma unroll
  for (int m = 0; m < 9; ++m) x[7 + m] = y[m];
}

// numeric_diff.h: delta = max(sqrt(eps), |x| * relative_step_size)
__device__ inline double step_of(double xj, double rel) {
  return fmax(sqrt(DBL_EPSILON), fabs(xj) * rel);
}

// The projected quadrilateral of one IoU evaluation (the evaluation's
// parameter perturbed): drawQuadrilateral's bounding box, the four edges'
// boxes and directions, and the four corner rectangles it clears.
struct QuadGeom {
  bool ok;
  double p[4][2];
  double dy[4], dx[4];
  Box box, eb[4], rb[4];
};

__device__ inline QuadGeom quad_geom(const GsbaArgs& a, const GsbaEval& ev, const GsbaBlock& b) {
  QuadGeom g;
  double x[16];
  load_params(a, b, x);
  if (ev.param >= 0) {
    const double orig = x[ev.param];
    const double delta = step_of(orig, a.rel_step);
    x[ev.param] = ev.sign > 0 ? orig + delta : orig - delta;
  }
  const double* kc = a.cam + 8 * (size_t)a.img_cam[b.img];
  const double K[3] = {kc[0], kc[1], kc[2]};
  if (a.by2) {
    double cyl[9];
    by2_to_cylinder(x + 7, cyl);
#pragma unroll
    for (int m = 0; m < 9; ++m) x[7 + m] = cyl[m];
  }
  g.ok = project_quad(x, K, g.p);
  g.box = Box{0, 0, 0, 0};
  if (!g.ok) return g;
  const int H = a.slots[b.slot].H, W = a.slots[b.slot].W;  // the image's own semantic map size
  const double(&p)[4][2] = g.p;
  // drawQuadrilateral as a predicate over the shrunk bounding box
  double min_x = p[0][0], min_y = p[0][1], max_x = p[0][0], max_y = p[0][1];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    min_x = fmin(min_x, p[k][0]);
    max_x = fmax(max_x, p[k][0]);
    min_y = fmin(min_y, p[k][1]);
    max_y = fmax(max_y, p[k][1]);
  }
  Box box;
  box.x = cast_to_int_x86(floor(min_x));
  box.y = cast_to_int_x86(floor(min_y));
  box.w = cast_to_int_x86(ceil(max_x)) - box.x + 1;
  box.h = cast_to_int_x86(ceil(max_y)) - box.y + 1;
  box = shrink(box, W, H);
  g.box = box;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int n = (e + 1) & 3;
    g.eb[e] = shrink(bound2(p[e][0], p[e][1], p[n][0], p[n][1]), W, H);
    g.dy[e] = p[n][1] - p[e][1];
    g.dx[e] = p[n][0] - p[e][0];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    g.rb[k] = Box{0, 0, 0, 0};
    const double qx = p[k][0], qy = p[k][1];
    if (qx - box.x < 1 || box.x_end() - qx < 1 || qy - box.y < 1 || box.y_end() - qy < 1) continue;
    const int cx[4] = {box.x, box.x_end(), box.x_end(), box.x};
    const int cy[4] = {box.y, box.y, box.y_end(), box.y_end()};
    int best = 0;
    double bd = 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const double ddx = qx - (double)cx[m], ddy = qy - (double)cy[m];
      const double d = sqrt(ddx * ddx + ddy * ddy);
      if (m == 0 || d < bd) { best = m; bd = d; }
    }
    g.rb[k] = shrink(bound2((double)cx[best], (double)cy[best], qx, qy), W, H);
  }
  return g;
}

// IoU = TP / (TP + FP + FN) from the workgroup's per-thread counts (thread 0
// writes it; FN = the mask's pixel total - TP).
__device__ inline void iou_reduce(int64_t tp, int64_t fp, bool ok, int64_t total, double* out) {
  __shared__ int64_t red[2][kTB / 64];
  for (int off = 32; off > 0; off >>= 1) {
    tp += __shfl_xor(tp, off, 64);
    fp += __shfl_xor(fp, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = tp;
    red[1][threadIdx.x >> 6] = fp;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double iou = 0.0;
    if (ok) {
      int64_t T = 0, F = 0;
#pragma unroll
      for (int w = 0; w < kTB / 64; ++w) {
        T += red[0][w];
        F += red[1][w];
      }
      const int64_t fn = total - T;
      double den = (double)T * 1.;
      den = den + (double)F;
      den = den + (double)fn;
      iou = (double)T / den;
    }
    *out = iou;
  }
}

#ifdef MI_BA_AB_VARIANTS
// One IoU evaluation per workgroup, a per-pixel predicate (tools build,
// gsba_variant 1; the round-2 kernel): waves take rows of the box, lanes
// consecutive pixels of the byte mask.
__global__ __launch_bounds__(kTB) void gsba_iou_kernel(GsbaArgs a, const GsbaEval* __restrict__ evals,
                                                       double* __restrict__ iou_out) {
  const GsbaEval ev = evals[blockIdx.x];
  const GsbaBlock b = a.blocks[ev.block];
  const QuadGeom g = quad_geom(a, ev, b);
  const int W = a.slots[b.slot].W;
  int64_t tp = 0, fp = 0;
  if (g.ok) {
    const Box box = g.box;
    const uint8_t* sem = a.masks + a.slots[b.slot].moff;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int y = box.y + wave; y <= box.y_end(); y += kTB / 64) {
      const uint8_t* srow = sem + (size_t)y * W;
      for (int xx = box.x + lane; xx <= box.x_end(); xx += 64) {
        bool m = true;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (xx >= g.eb[e].x && xx <= g.eb[e].x_end() && y >= g.eb[e].y && y <= g.eb[e].y_end()) {
            const double cross = ((double)xx - g.p[e][0]) * g.dy[e] - ((double)y - g.p[e][1]) * g.dx[e];
            if (cross > 0) m = false;
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (xx >= g.rb[k].x && xx <= g.rb[k].x_end() && y >= g.rb[k].y && y <= g.rb[k].y_end()) m = false;
        if (m) {
          if (srow[xx]) ++tp;
          else ++fp;
        }
      }
    }
  }
  iou_reduce(tp, fp, g.ok, a.sem_total[b.slot], iou_out + blockIdx.x);
}
#endif

// Bits lo..hi (0 <= lo, hi <= 63) of a word; 0 when lo > hi.
__device__ inline uint64_t bit_range(int lo, int hi) {
  lo = max(lo, 0);
  hi = min(hi, 63);
  if (lo > hi) return 0ull;
  return (~0ull >> (63 - hi)) & (~0ull << lo);
}

// One IoU evaluation per workgroup by row spans over the bit-packed mask (the
// default).  In row y the pixels drawQuadrilateral clears are <= 8 intervals:
// per edge e, the pixels of its box with cross_e > 0, and the corner
// rectangles.  The computed cross_e(x) = fl(fl(fl(x - p_e.x) dy_e) -
// fl(fl(y - p_e.y) dx_e)) is monotone in x (every rounding step is monotone;
// the sign of dy_e gives the direction), so {x : cross_e(x) > 0} is a half-line
// and a binary search with the per-pixel predicate itself finds its end: the
// spans are exactly the per-pixel kernel's pixels.  TP / FP are popcounts of
// the kept bits of each 64-pixel word against the mask bits.  One thread per
// row; per row about 4 x 11 predicate evaluations + 2 popcounts per word,
// where the per-pixel kernel evaluated up to 4 predicates per pixel.
__global__ __launch_bounds__(kTB) void gsba_iou_span_kernel(GsbaArgs a, const GsbaEval* __restrict__ evals,
                                                            double* __restrict__ iou_out) {
  const GsbaEval ev = evals[blockIdx.x];
  const GsbaBlock b = a.blocks[ev.block];
  const QuadGeom g = quad_geom(a, ev, b);
  int64_t tp = 0, fp = 0;
  if (g.ok && g.box.w > 0) {
    const Box box = g.box;
    const GsbaSlot si = a.slots[b.slot];
    const uint64_t* bits = a.mask_bits + si.boff;
    for (int y = box.y + (int)threadIdx.x; y <= box.y_end(); y += kTB) {
      int lo[8], hi[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        lo[e] = 1;
        hi[e] = 0;
        const Box& eb = g.eb[e];
        if (eb.w <= 0 || y < eb.y || y > eb.y_end()) continue;
        const int l = max(eb.x, box.x), h = min(eb.x_end(), box.x_end());
        if (l > h) continue;
        const double px = g.p[e][0], dy = g.dy[e];
        const double cy = ((double)y - g.p[e][1]) * g.dx[e];
        auto clear = [&](int xx) { return ((double)xx - px) * dy - cy > 0; };
        if (dy > 0) {  // cleared: [first x with cross > 0, h]
          int u = l, v = h + 1;
          while (u < v) {
            const int mid = (u + v) >> 1;
            if (clear(mid)) v = mid; else u = mid + 1;
          }
          lo[e] = u;
          hi[e] = h;
        } else if (dy < 0) {  // cleared: [l, last x with cross > 0]
          int u = l - 1, v = h;
          while (u < v) {
            const int mid = (u + v + 1) >> 1;
            if (clear(mid)) u = mid; else v = mid - 1;
          }
          lo[e] = l;
          hi[e] = u;
        } else if (clear(l)) {  // constant in x
          lo[e] = l;
          hi[e] = h;
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const Box& rb = g.rb[k];
        const bool in = rb.w > 0 && y >= rb.y && y <= rb.y_end();
        lo[4 + k] = in ? rb.x : 1;
        hi[4 + k] = in ? rb.x_end() : 0;
      }
      const uint64_t* row = bits + (size_t)y * si.words;
      for (int w = box.x >> 6; w <= (box.x_end() >> 6); ++w) {
        const int w0 = 64 * w;
        uint64_t keep = bit_range(box.x - w0, box.x_end() - w0);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (lo[i] <= hi[i]) keep &= ~bit_range(lo[i] - w0, hi[i] - w0);
        const uint64_t mb = row[w];
        tp += __popcll(keep & mb);
        fp += __popcll(keep & ~mb);
      }
    }
  }
  iou_reduce(tp, fp, g.ok, a.sem_total[b.slot], iou_out + blockIdx.x);
}

// Ceres 2.1 QuaternionManifold::PlusJacobian (4 x 3 row-major)
__device__ inline void quat_plus_jac(const double q[4], double J[12]) {
  J[0] = -q[1]; J[1] = -q[2];  J[2] = -q[3];
  J[3] = q[0];  J[4] = q[3];   J[5] = -q[2];
  J[6] = -q[3]; J[7] = q[0];   J[8] = q[1];
  J[9] = q[2];  J[10] = -q[1]; J[11] = q[0];
}

// Per block: residual, ambient CENTRAL Jacobian, tangent rows with the
// manifolds (camera / cylinder quaternions, constant tvec coordinates) and
// the ScaledLoss(weight) Corrector (r, J *= sqrt(weight)).
__global__ void gsba_block_kernel(GsbaArgs a, int nblocks, const uint32_t* __restrict__ img_flags,
                                  const double* __restrict__ iou, double weight, double* __restrict__ r_out,
                                  double* __restrict__ J_out, double* __restrict__ J16_out,
                                  double* __restrict__ r_raw_out, double* __restrict__ cost) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= nblocks) return;
  const GsbaBlock b = a.blocks[k];
  double x[16];
  load_params(a, b, x);
  const double* f = iou + b.eval0;
  double r = 1.0 - f[0];
  const int lo = b.variant == kGsbaConstantPose ? 7 : 0;
  const int hi = b.variant == kGsbaConstantCylinder ? 7 : (a.by2 ? 14 : 16);
  double J16[16];
  int e = 1;
  for (int j = 0; j < 16; ++j) {
    J16[j] = 0.0;
    if (j < lo || j >= hi) continue;
    const double delta = step_of(x[j], a.rel_step);
    const double fp = 1.0 - f[e], fm = 1.0 - f[e + 1];
    e += 2;
    double one_over_delta = 1.0 / delta;
    one_over_delta /= 2;
    J16[j] = (fp - fm) * one_over_delta;
  }
  if (J16_out) {
#pragma unroll
    for (int j = 0; j < 16; ++j) J16_out[16 * (size_t)k + j] = J16[j];
    r_raw_out[k] = r;
  }
  double Jt[14], PJ[12];
  quat_plus_jac(x, PJ);
  for (int col = 0; col < 3; ++col) {
    double acc = 0.0;
    for (int m = 0; m < 4; ++m) acc += J16[m] * PJ[m * 3 + col];
    Jt[col] = acc;
  }
  const uint32_t flags = img_flags[b.img];
  for (int col = 0; col < 3; ++col) Jt[3 + col] = ((flags >> (1 + col)) & 1u) ? 0.0 : J16[4 + col];
  if (a.by2) {
    // by_2_points: Euclidean t1, t2, radius (no manifold); column 13 unused
    for (int col = 0; col < 7; ++col) Jt[6 + col] = J16[7 + col];
    Jt[13] = 0.0;
  } else {
    quat_plus_jac(x + 7, PJ);
    for (int col = 0; col < 3; ++col) {
      double acc = 0.0;
      for (int m = 0; m < 4; ++m) acc += J16[7 + m] * PJ[m * 3 + col];
      Jt[6 + col] = acc;
    }
    for (int col = 0; col < 5; ++col) Jt[9 + col] = J16[11 + col];
  }
  // ScaledLoss corrector: rho = (w s, w, 0)
  cost[k] = 0.5 * (weight * (r * r));
  const double sqrt_rho1 = sqrt(weight);
  for (int col = 0; col < 14; ++col) J_out[14 * (size_t)k + col] = Jt[col] * sqrt_rho1;
  r_out[k] = r * sqrt_rho1;
}

__global__ void gsba_cost_kernel(const GsbaBlock* __restrict__ blocks, int nblocks, const double* __restrict__ iou,
                                 double weight, double* __restrict__ cost) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= nblocks) return;
  const double r = 1.0 - iou[k];
  (void)blocks;
  cost[k] = 0.5 * (weight * (r * r));
}

// Slots of a block's tangent columns: pose 6 (or -1), cylinder cw (or -1):
// cw = 8 (q 3, t 3, radius, height) or 7 (by_2_points: t1 3, t2 3, radius).
__device__ inline int64_t gsba_slot(const GsbaBlock& b, int m, int64_t cyl0, int cyl_var, uint32_t pose_var,
                                    int cw) {
  if (m < 6) return (b.variant != kGsbaConstantPose && pose_var) ? 6 * (int64_t)b.img + m : -1;
  return (b.variant != kGsbaConstantCylinder && cyl_var && m - 6 < cw) ? cyl0 + cw * (int64_t)b.cyl + (m - 6) : -1;
}

__device__ inline int sym6(int a, int c) { return a * 6 - (a * (a - 1)) / 2 + (c - a); }   // a <= c < 6
// packed upper index of (a, c), a <= c < n
__device__ inline int symn(int n, int a, int c) { return a * n - (a * (a - 1)) / 2 + (c - a); }





// Ceres 2.1 QuaternionManifold::Plus on the cylinder qvec, Euclidean t, r,
// h; the radius is projected onto its lower bound 0 (ParameterBlock::Plus).
__global__ void gsba_plus_kernel(int ncyl, const double* __restrict__ cyl, const double* __restrict__ df,
                                 double* __restrict__ out) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= ncyl) return;
  const double* y = cyl + 9 * (size_t)k;
  const double* d = df + 8 * (size_t)k;
  double* o = out + 9 * (size_t)k;
  const double q[4] = {y[0], y[1], y[2], y[3]};
  const double dr[3] = {d[0], d[1], d[2]};
  double qn[4];
  quat_plus(q, dr, qn);
  o[0] = qn[0]; o[1] = qn[1]; o[2] = qn[2]; o[3] = qn[3];
  o[4] = y[4] + d[3];
  o[5] = y[5] + d[4];
  o[6] = y[6] + d[5];
  o[7] = fmax(y[7] + d[6], 0.0);
  o[8] = y[8] + d[7];
}

// by_2_points: Euclidean t1, t2; the radius projected onto its lower bound 0
// (SetUpCylinderManifolds, :1185-1213; ParameterBlock::Plus).
__global__ void gsba_plus_by2_kernel(int ncyl, const double* __restrict__ cyl, const double* __restrict__ df,
                                     double* __restrict__ out) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= ncyl) return;
  const double* y = cyl + 9 * (size_t)k;
  const double* d = df + 7 * (size_t)k;
  double* o = out + 9 * (size_t)k;
#pragma unroll
  for (int m = 0; m < 6; ++m) o[m] = y[m] + d[m];
  o[6] = fmax(y[6] + d[6], 0.0);
  o[7] = 0.0;
  o[8] = 0.0;
}


__device__ inline void gsba_atomic_max(double* out, double v) {
  if (v > 0.0) atomicMax(reinterpret_cast<unsigned long long*>(out), (unsigned long long)__double_as_longlong(v));
}

// |y - Plus(y, -g)|_inf of every cylinder (qvec on the QuaternionManifold,
// the radius projected onto its bound 0; by two points Euclidean + radius).
__global__ void gsba_grad_max_kernel(int ncyl, int by2, const double* __restrict__ cyl, const double* __restrict__ g,
                                     double* out) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= ncyl) return;
  const double* y = cyl + 9 * (size_t)k;
  double mx = 0.0;
  if (by2) {
    const double* gc = g + 7 * (size_t)k;
    for (int m = 0; m < 6; ++m) mx = fmax(mx, fabs(y[m] - (y[m] + -gc[m])));
    mx = fmax(mx, fabs(y[6] - fmax(y[6] + -gc[6], 0.0)));
  } else {
    const double* gc = g + 8 * (size_t)k;
    const double q[4] = {y[0], y[1], y[2], y[3]};
    const double d[3] = {-gc[0], -gc[1], -gc[2]};
    double qn[4];
    quat_plus(q, d, qn);
    for (int m = 0; m < 4; ++m) mx = fmax(mx, fabs(q[m] - qn[m]));
    for (int m = 0; m < 3; ++m) mx = fmax(mx, fabs(y[4 + m] - (y[4 + m] + -gc[3 + m])));
    mx = fmax(mx, fabs(y[7] - fmax(y[7] + -gc[6], 0.0)));
    mx = fmax(mx, fabs(y[8] - (y[8] + -gc[7])));
  }
  gsba_atomic_max(out, mx);
}


// ---------------------------------------------------------------------------
// Deterministic per-owner sums.  Blocks are image-major, one per (image,
// cylinder): image rank r owns blocks [r ncyl, (r + 1) ncyl), cylinder c owns
// blocks c, c + ncyl, ...  One workgroup per owner (images first, then
// cylinders), one thread per output value, the owner's blocks summed in block
// order; each output is added once.
// ---------------------------------------------------------------------------
__device__ inline void sym_pair(int n, int k, int* a, int* c) {
  int aa = 0, rem = k;
  while (rem >= n - aa) { rem -= n - aa; ++aa; }
  *a = aa;
  *c = aa + rem;
}

struct GsbaOwn {
  const GsbaBlock* blocks;
  const uint32_t* img_flags;
  const double* J;
  int nblocks, ncyl, nimg;  // nimg: images with blocks (nblocks / ncyl)
  int64_t cyl0;
  int cyl_var, cw;
  __device__ int first(int o) const { return o < nimg ? o * ncyl : o - nimg; }
  __device__ int step(int o) const { return o < nimg ? 1 : ncyl; }
  __device__ int count(int o) const { return o < nimg ? ncyl : nimg; }
  __device__ bool valid(int k, bool cyl_side) const {
    const GsbaBlock b = blocks[k];
    return gsba_slot(b, cyl_side ? 6 : 0, cyl0, cyl_var, img_flags[b.img] & 1u, cw) >= 0;
  }
};

// f-blocks: the image's pose Schur-Jacobi block (21), b (6), diag U (6); the
// cylinder's block (cw (cw + 1) / 2), b (cw), diag U (cw).
__global__ void gsba_fblock_owner_kernel(GsbaOwn w, const double* __restrict__ r, double* __restrict__ pose_blk,
                                         double* __restrict__ cyl_blk, double* __restrict__ bvec,
                                         double* __restrict__ udiag) {
  const int o = blockIdx.x;
  const bool cs = o >= w.nimg;
  const int n = cs ? w.cw : 6, ns = n * (n + 1) / 2;
  const int v = threadIdx.x;
  if (v >= ns + 2 * n) return;
  const int off = cs ? 6 : 0;
  int a = 0, c = 0, kind = 0;  // 0 block entry (a, c), 1 b[a], 2 diag[a]
  if (v < ns) {
    sym_pair(n, v, &a, &c);
  } else {
    kind = v < ns + n ? 1 : 2;
    a = v - ns - (kind == 1 ? 0 : n);
  }
  double acc = 0.0;
  bool any = false;
  const int k0 = w.first(o), st = w.step(o), cnt = w.count(o);
  for (int q = 0; q < cnt; ++q) {
    const int k = k0 + q * st;
    if (!w.valid(k, cs)) continue;
    any = true;
    const double* Jr = w.J + 14 * (size_t)k;
    const double ja = Jr[off + a];
    acc += kind == 0 ? ja * Jr[off + c] : (kind == 1 ? ja * r[k] : ja * ja);
  }
  if (!any) return;
  if (!cs) {
    const int img = w.blocks[k0].img;
    if (kind == 0) pose_blk[21 * (size_t)img + sym6(a, c)] += acc;
    else if (kind == 1) bvec[6 * (size_t)img + a] += acc;
    else udiag[6 * (size_t)img + a] += acc;
  } else {
    const int cyl = o - w.nimg;
    const int64_t s0 = w.cyl0 + w.cw * (int64_t)cyl;
    if (kind == 0) cyl_blk[ns * (size_t)cyl + symn(n, a, c)] += acc;
    else if (kind == 1) bvec[s0 + a] += acc;
    else udiag[s0 + a] += acc;
  }
}

// e_k = J_k x over the block's slots (the product's first half).
__global__ void gsba_jx_kernel(GsbaOwn w, const double* __restrict__ x, double* __restrict__ e) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= w.nblocks) return;
  const GsbaBlock b = w.blocks[k];
  const double* Jr = w.J + 14 * (size_t)k;
  const uint32_t pv = w.img_flags[b.img] & 1u;
  double s = 0.0;
  for (int m = 0; m < 14; ++m) {
    const int64_t sl = gsba_slot(b, m, w.cyl0, w.cyl_var, pv, w.cw);
    if (sl >= 0) s += Jr[m] * x[sl];
  }
  e[k] = s;
}

// y[slot] += sum over the owner's blocks of J_k[m] e_k (J'(J x) with e = J x,
// the gradient J'r with e = r).
__global__ void gsba_jte_owner_kernel(GsbaOwn w, const double* __restrict__ e, double* __restrict__ y) {
  const int o = blockIdx.x;
  const bool cs = o >= w.nimg;
  const int m = threadIdx.x;
  if (m >= (cs ? w.cw : 6)) return;
  const int off = cs ? 6 : 0;
  double acc = 0.0;
  bool any = false;
  const int k0 = w.first(o), st = w.step(o), cnt = w.count(o);
  for (int q = 0; q < cnt; ++q) {
    const int k = k0 + q * st;
    if (!w.valid(k, cs)) continue;
    any = true;
    acc += w.J[14 * (size_t)k + off + m] * e[k];
  }
  if (!any) return;
  if (!cs) y[6 * (size_t)w.blocks[k0].img + m] += acc;
  else y[w.cyl0 + w.cw * (int64_t)(o - w.nimg) + m] += acc;
}

// S += J'J: the owners' diagonal blocks (upper triangle), then one thread per
// (block, pose column, cylinder column) for the pose-cylinder entries (each
// block is the only one of its (image, cylinder) pair: one writer each).
__global__ void gsba_dense_owner_kernel(GsbaOwn w, int64_t lds, double* __restrict__ S) {
  const int o = blockIdx.x;
  const bool cs = o >= w.nimg;
  const int n = cs ? w.cw : 6, ns = n * (n + 1) / 2;
  const int v = threadIdx.x;
  if (v >= ns) return;
  int a, c;
  sym_pair(n, v, &a, &c);
  const int off = cs ? 6 : 0;
  double acc = 0.0;
  bool any = false;
  const int k0 = w.first(o), st = w.step(o), cnt = w.count(o);
  for (int q = 0; q < cnt; ++q) {
    const int k = k0 + q * st;
    if (!w.valid(k, cs)) continue;
    any = true;
    const double* Jr = w.J + 14 * (size_t)k;
    acc += Jr[off + a] * Jr[off + c];
  }
  if (!any) return;
  const int64_t s0 = cs ? w.cyl0 + w.cw * (int64_t)(o - w.nimg) : 6 * (int64_t)w.blocks[k0].img;
  S[(s0 + a) * lds + (s0 + c)] += acc;
}

__global__ void gsba_dense_cross_kernel(GsbaOwn w, int64_t lds, double* __restrict__ S) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)w.nblocks * 6 * w.cw) return;
  const int k = (int)(t / (6 * w.cw)), e = (int)(t % (6 * w.cw));
  const int a = e / w.cw, c = e % w.cw;
  const GsbaBlock b = w.blocks[k];
  const uint32_t pv = w.img_flags[b.img] & 1u;
  const int64_t ra = gsba_slot(b, a, w.cyl0, w.cyl_var, pv, w.cw), rc = gsba_slot(b, 6 + c, w.cyl0, w.cyl_var, pv, w.cw);
  if (ra < 0 || rc < 0) return;
  const double* Jr = w.J + 14 * (size_t)k;
  S[ra * lds + rc] += Jr[a] * Jr[6 + c];
}

// per-block model term -(e (r + e / 2)), e = J df
__global__ void gsba_model_terms_kernel(GsbaOwn w, const double* __restrict__ r, const double* __restrict__ df,
                                        double* __restrict__ out) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= w.nblocks) return;
  const GsbaBlock b = w.blocks[k];
  const double* Jr = w.J + 14 * (size_t)k;
  const uint32_t pv = w.img_flags[b.img] & 1u;
  double e = 0.0;
  for (int m = 0; m < 14; ++m) {
    const int64_t s = gsba_slot(b, m, w.cyl0, w.cyl_var, pv, w.cw);
    if (s >= 0) e += Jr[m] * df[s];
  }
  out[k] = -(e * (r[k] + e / 2.0));
}

// per-cylinder |y|^2 and |y - y_c|^2 into part[k], part[ncyl + k]
__global__ void gsba_state_terms_kernel(int ncyl, int by2, const double* __restrict__ cyl,
                                        const double* __restrict__ cyl_c, double* __restrict__ part) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= ncyl) return;
  const int n = by2 ? 7 : 9;
  double vx = 0.0, vd = 0.0;
  for (int m = 0; m < n; ++m) {
    const double a = cyl[9 * (size_t)k + m], d = a - cyl_c[9 * (size_t)k + m];
    vx += a * a;
    vd += d * d;
  }
  part[k] = vx;
  part[ncyl + k] = vd;
}

// out[j] += the n values of part + j n summed in index order (one workgroup)
__global__ __launch_bounds__(256) void gsba_ordered_add_kernel(const double* __restrict__ part, int n, int nout,
                                                               double* __restrict__ out) {
  __shared__ double s[256];
  for (int j = 0; j < nout; ++j) {
    double v = 0.0;
    for (int k = threadIdx.x; k < n; k += 256) v += part[(size_t)j * n + k];
    s[threadIdx.x] = v;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if ((int)threadIdx.x < h) s[threadIdx.x] += s[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) out[j] += s[0];
    __syncthreads();
  }
}

GsbaArgs make_args(mi_ba_context* ctx, const double* qt, const double* cyl) {
  GsbaState* G = ctx->gsba;
  GsbaArgs a;
  a.blocks = G->blocks.ptr;
  a.qt = qt;
  a.cam = ctx->dev.cam;
  a.img_cam = ctx->dev.img_cam;
  a.cyl = cyl;
  a.slots = G->slots.ptr;
  a.masks = G->masks.ptr;
  a.mask_bits = G->mask_bits.ptr;
  a.sem_total = G->sem_total.ptr;
  a.rel_step = G->rel_step;
  a.by2 = G->by2 ? 1 : 0;
  return a;
}

unsigned grid64(int64_t n) { return (unsigned)((n + 63) / 64); }

GsbaOwn owners(mi_ba_context* ctx) {
  const GsbaState* G = ctx->gsba;
  GsbaOwn w;
  w.blocks = G->blocks.ptr;
  w.img_flags = ctx->dev.img_flags;
  w.J = G->J.ptr;
  w.nblocks = G->nblocks;
  w.ncyl = G->ncyl;
  w.nimg = G->ncyl > 0 ? G->nblocks / G->ncyl : 0;
  w.cyl0 = ctx->dev.cyl0;
  w.cyl_var = ctx->dev.cyl_var;
  w.cw = G->cw;
  return w;
}

}  // namespace

int gsba_cylinder_slots(const mi_ba_options& o, const mi_ba_problem* p, const mi_ba_gsba* g) {
  (void)o;
  if (!g || !g->refine_geometry || g->num_cylinders <= 0) return 0;
  int ncfg = 0;
  for (int i = 0; i < p->num_images; ++i) ncfg += p->image_in_config ? (p->image_in_config[i] != 0) : 1;
  const int cw = g->cylinder_parametrization == MI_BA_CYLINDER_BY_2_POINTS ? 7 : 8;
  return ncfg > 0 ? cw * g->num_cylinders : 0;
}

mi_ba_status gsba_create(mi_ba_context* ctx, const mi_ba_gsba* g) {
  const mi_ba_problem* p = &ctx->problem;
  const mi_ba_options& o = ctx->options;
  const bool per_image = g->image_height || g->image_width;
  if ((per_image && !(g->image_height && g->image_width)) || (!per_image && (g->height <= 0 || g->width <= 0)) ||
      !g->trunk_mask || g->num_cylinders < 0 ||
      (g->num_cylinders > 0 && !g->cylinders) || !(g->numeric_relative_step_size > 0) ||
      (g->cylinder_parametrization != MI_BA_CYLINDER_DEFAULT &&
       g->cylinder_parametrization != MI_BA_CYLINDER_BY_2_POINTS))
    return MI_BA_ERR_INVALID_ARGUMENT;
  HostSetup& s = ctx->setup;
  const int I = p->num_images;
  auto in_cfg = [&](int i) { return p->image_in_config ? p->image_in_config[i] != 0 : true; };
  // each image's mask size and plane (ABI 4: per-image sizes, planes back to back)
  std::vector<int32_t> img_h(I), img_w(I);
  std::vector<size_t> img_off(I);
  {
    size_t off = 0;
    for (int i = 0; i < I; ++i) {
      img_h[i] = per_image ? g->image_height[i] : g->height;
      img_w[i] = per_image ? g->image_width[i] : g->width;
      if (img_h[i] < 0 || img_w[i] < 0 || (in_cfg(i) && (img_h[i] == 0 || img_w[i] == 0)))
        return MI_BA_ERR_INVALID_ARGUMENT;
      img_off[i] = off;
      off += (size_t)img_h[i] * img_w[i];
    }
  }
  // GeometricSemanticBundleAdjuster::Assert (:664-712)
  int ncfg = 0;
  for (int i = 0; i < I; ++i) {
    if (!in_cfg(i)) continue;
    ++ncfg;
    const int cam = p->image_camera[i];
    if (!(p->camera_constant && p->camera_constant[cam])) return MI_BA_ERR_UNSUPPORTED;
    if (s.cam_model[cam] != kSimplePinhole) return MI_BA_ERR_UNSUPPORTED;
  }
  auto* G = new GsbaState();
  ctx->gsba = G;
  G->host = g;
  G->ncyl = g->num_cylinders;
  G->rel_step = g->numeric_relative_step_size;
  G->weight = ncfg > 0 ? 1. / (double)ncfg : 1.0;
  G->by2 = g->cylinder_parametrization == MI_BA_CYLINDER_BY_2_POINTS;
  G->cw = G->by2 ? 7 : 8;
  // blocks (AddImageToProblem, :835-909): config images in problem order
  std::vector<int32_t> slot(I, -1);
  std::vector<int> slot_images;
  std::vector<GsbaEval> evals, centres;
  for (int i = 0; i < I; ++i) {
    if (!in_cfg(i)) continue;
    const bool constant_pose = !o.refine_extrinsics || (p->image_constant_pose && p->image_constant_pose[i]);
    if (constant_pose && !g->refine_geometry) continue;
    for (int c = 0; c < g->num_cylinders; ++c) {
      GsbaBlock b{};
      b.img = i;
      b.cyl = c;
      b.variant = constant_pose ? kGsbaConstantPose : g->refine_geometry ? kGsbaFull : kGsbaConstantCylinder;
      if (slot[i] < 0) {
        slot[i] = (int32_t)slot_images.size();
        slot_images.push_back(i);
      }
      b.slot = slot[i];
      b.eval0 = (int32_t)evals.size();
      const int32_t kb = (int32_t)G->blocks_host.size();
      evals.push_back(GsbaEval{kb, -1, 1});
      centres.push_back(GsbaEval{kb, -1, 1});
      const int lo = b.variant == kGsbaConstantPose ? 7 : 0;
      const int hi = b.variant == kGsbaConstantCylinder ? 7 : (G->by2 ? 14 : 16);
      for (int j = lo; j < hi; ++j) {
        evals.push_back(GsbaEval{kb, (int16_t)j, 1});
        evals.push_back(GsbaEval{kb, (int16_t)j, -1});
      }
      b.nevals = (int32_t)evals.size() - b.eval0;
      G->blocks_host.push_back(b);
      // poses of GSBA blocks are variable parameter blocks (SetUpManifolds)
      if (b.variant != kGsbaConstantPose && !s.img_var[i]) {
        s.img_var[i] = 1;
        s.img_tvec_mask[i] = p->image_constant_tvec ? p->image_constant_tvec[i] : 0;
        int masked = 0;
        for (int m = 0; m < 3; ++m) masked += (s.img_tvec_mask[i] >> m) & 1;
        s.num_effective_parameters_reduced += 6 - masked;
      }
    }
  }
  G->nblocks = (int)G->blocks_host.size();
  G->nevals = (int64_t)evals.size();
  if (ctx->dev.cyl_var) s.num_effective_parameters_reduced += G->cw * (int64_t)G->ncyl;
  std::vector<int64_t> totals(slot_images.size(), 0);
  G->slots_host.resize(slot_images.size());
  size_t mtot = 0, btot = 0;
  for (size_t k = 0; k < slot_images.size(); ++k) {
    const int i = slot_images[k];
    GsbaSlot& si = G->slots_host[k];
    si.H = img_h[i];
    si.W = img_w[i];
    si.words = (si.W + 63) / 64;
    si.pad = 0;
    si.moff = mtot;
    si.boff = btot;
    const size_t plane = (size_t)si.H * si.W;
    mtot += plane;
    btot += (size_t)si.H * si.words;
    const uint8_t* m = g->trunk_mask + img_off[i];
    int64_t t = 0;
    for (size_t q = 0; q < plane; ++q) t += m[q] != 0;
    totals[k] = t;
  }
  std::vector<double> cyl(9 * (size_t)std::max(1, G->ncyl), 0.0);
  for (int c = 0; c < G->ncyl; ++c) {
    const mi_ba_cylinder& y = g->cylinders[c];
    if (G->by2) {
      cylinder_to_by2(y, &cyl[9 * c]);
      continue;
    }
    for (int m = 0; m < 4; ++m) cyl[9 * c + m] = y.qvec[m];
    for (int m = 0; m < 3; ++m) cyl[9 * c + 4 + m] = y.tvec[m];
    cyl[9 * c + 7] = y.radius;
    cyl[9 * c + 8] = y.height;
  }
  const int nb = std::max(1, G->nblocks);
  if (G->blocks.alloc(nb) || G->evals.alloc(std::max<int64_t>(1, G->nevals)) || G->centres.alloc(nb) ||
      G->masks.alloc(std::max<size_t>(1, mtot)) || G->slots.alloc(std::max<size_t>(1, slot_images.size())) ||
      G->sem_total.alloc(std::max<size_t>(1, slot_images.size())) || G->cyl.alloc(cyl.size()) ||
      G->cyl_c.alloc(cyl.size()) || G->iou.alloc(std::max<int64_t>(1, G->nevals)) || G->r.alloc(nb) ||
      G->J.alloc(14 * (size_t)nb) || G->cyl_blk.alloc(36 * (size_t)std::max(1, G->ncyl)) ||
      G->prec_cyl.alloc(64 * (size_t)std::max(1, G->ncyl)) || G->partial.alloc(nb) || G->ework.alloc(nb) ||
      G->cstate.alloc(2 * (size_t)std::max(1, G->ncyl)))
    return MI_BA_ERR_OUT_OF_MEMORY;
  if ((G->nblocks &&
       (hipMemcpy(G->blocks.ptr, G->blocks_host.data(), G->nblocks * sizeof(GsbaBlock), hipMemcpyHostToDevice) ||
        hipMemcpy(G->evals.ptr, evals.data(), evals.size() * sizeof(GsbaEval), hipMemcpyHostToDevice) ||
        hipMemcpy(G->centres.ptr, centres.data(), centres.size() * sizeof(GsbaEval), hipMemcpyHostToDevice))) ||
      hipMemcpy(G->cyl.ptr, cyl.data(), cyl.size() * 8, hipMemcpyHostToDevice) ||
      (!slot_images.empty() &&
       (hipMemcpy(G->sem_total.ptr, totals.data(), totals.size() * 8, hipMemcpyHostToDevice) ||
        hipMemcpy(G->slots.ptr, G->slots_host.data(), G->slots_host.size() * sizeof(GsbaSlot),
                  hipMemcpyHostToDevice))))
    return MI_BA_ERR_HIP;
  for (size_t k = 0; k < slot_images.size(); ++k) {
    const GsbaSlot& si = G->slots_host[k];
    if (hipMemcpy(G->masks.ptr + si.moff, g->trunk_mask + img_off[slot_images[k]], (size_t)si.H * si.W,
                  hipMemcpyHostToDevice))
      return MI_BA_ERR_HIP;
  }
#ifdef MI_BA_AB_VARIANTS
  // tools build: MI_BA_GSBA_VARIANT=1 selects the per-pixel kernel (the GSBA
  // entry points create their contexts internally, out of mi_ba_set_tuning's reach)
  if (const char* v = std::getenv("MI_BA_GSBA_VARIANT")) G->iou_variant = std::atoi(v) == 1 ? 1 : 0;
#endif
  // bit-packed masks (row-major, whole 64-bit words per row) for the span kernel
  {
    if (G->mask_bits.alloc(std::max<size_t>(1, btot))) return MI_BA_ERR_OUT_OF_MEMORY;
    std::vector<uint64_t> wb;
    for (size_t k = 0; k < slot_images.size(); ++k) {
      const GsbaSlot& si = G->slots_host[k];
      const size_t wplane = (size_t)si.H * si.words;
      const uint8_t* m = g->trunk_mask + img_off[slot_images[k]];
      wb.assign(wplane, 0ull);
      for (int y = 0; y < si.H; ++y)
        for (int x = 0; x < si.W; ++x)
          if (m[(size_t)y * si.W + x]) wb[(size_t)y * si.words + (x >> 6)] |= 1ull << (x & 63);
      if (hipMemcpy(G->mask_bits.ptr + si.boff, wb.data(), wplane * 8, hipMemcpyHostToDevice)) return MI_BA_ERR_HIP;
    }
  }
  // refresh image flags (poses made variable by the GSBA term)
  std::vector<uint32_t> fl(I);
  for (int i = 0; i < I; ++i) fl[i] = (s.img_var[i] ? 1u : 0u) | ((uint32_t)s.img_tvec_mask[i] << 1);
  if (I && hipMemcpy(ctx->img_flags.ptr, fl.data(), I * 4, hipMemcpyHostToDevice) != hipSuccess) return MI_BA_ERR_HIP;
  return MI_BA_OK;
}

void gsba_destroy(mi_ba_context* ctx) {
  if (!ctx->gsba) return;
  delete ctx->gsba;
  ctx->gsba = nullptr;
}

namespace {
// The IoU evaluations: row spans over the bit-packed masks (default), or the
// per-pixel predicate over the byte masks (tools build, gsba_variant 1).
void launch_iou(mi_ba_context* ctx, const GsbaArgs& a, const GsbaEval* evals, int64_t n, double* out,
                hipStream_t s) {
  if (n <= 0) return;
#ifdef MI_BA_AB_VARIANTS
  if (ctx->gsba->iou_variant == 1) {
    hipLaunchKernelGGL(gsba_iou_kernel, dim3((unsigned)n), dim3(kTB), 0, s, a, evals, out);
    return;
  }
#else
  (void)ctx;
#endif
  hipLaunchKernelGGL(gsba_iou_span_kernel, dim3((unsigned)n), dim3(kTB), 0, s, a, evals, out);
}

mi_ba_status eval_blocks(mi_ba_context* ctx, double* d_cost, double* J16, double* r_raw) {
  GsbaState* G = ctx->gsba;
  if (!G->nblocks) return MI_BA_OK;
  hipStream_t s = ctx->stream;
  GsbaArgs a = make_args(ctx, ctx->dev.qt, G->cyl.ptr);
  hipEvent_t stop;
  timer_begin(ctx, "gsba_iou", &stop);
  launch_iou(ctx, a, G->evals.ptr, G->nevals, G->iou.ptr, s);
  timer_end(ctx, stop);
  hipLaunchKernelGGL(gsba_block_kernel, dim3(grid64(G->nblocks)), dim3(64), 0, s, a, G->nblocks, ctx->dev.img_flags,
                     G->iou.ptr, G->weight, G->r.ptr, G->J.ptr, J16, r_raw, G->partial.ptr);
  launch_sum(G->partial.ptr, G->nblocks, d_cost, s);
  return hipGetLastError() == hipSuccess ? MI_BA_OK : MI_BA_ERR_HIP;
}
}  // namespace

mi_ba_status gsba_linearize(mi_ba_context* ctx, double* d_cost) { return eval_blocks(ctx, d_cost, nullptr, nullptr); }

void gsba_cost(mi_ba_context* ctx, const double* qt, const double* cyl, double* d_cost) {
  GsbaState* G = ctx->gsba;
  if (!G->nblocks) return;
  hipStream_t s = ctx->stream;
  GsbaArgs a = make_args(ctx, qt, cyl);
  launch_iou(ctx, a, G->centres.ptr, G->nblocks, G->iou.ptr, s);
  hipLaunchKernelGGL(gsba_cost_kernel, dim3(grid64(G->nblocks)), dim3(64), 0, s, G->blocks.ptr, G->nblocks,
                     G->iou.ptr, G->weight, G->partial.ptr);
  launch_sum(G->partial.ptr, G->nblocks, d_cost, s);
}

void gsba_add_fblock(mi_ba_context* ctx) {
  GsbaState* G = ctx->gsba;
  hipStream_t s = ctx->stream;
  (void)hipMemsetAsync(G->cyl_blk.ptr, 0, G->cyl_blk.bytes(), s);
  if (!G->nblocks) return;
  const GsbaOwn w = owners(ctx);
  hipLaunchKernelGGL(gsba_fblock_owner_kernel, dim3(w.nimg + w.ncyl), dim3(64), 0, s, w, G->r.ptr, ctx->pose_blk.ptr,
                     G->cyl_blk.ptr, ctx->bvec.ptr, ctx->udiag.ptr);
}

void gsba_finalize(mi_ba_context* ctx, int first, int reuse_diag, double radius) {
  GsbaState* G = ctx->gsba;
  if (!ctx->dev.cyl_var || G->ncyl == 0) return;
  const int64_t o = ctx->dev.cyl0;
  launch_finalize_n(G->cw, G->ncyl, G->cyl_blk.ptr, ctx->udiag.ptr + o, ctx->scale_f.ptr + o, ctx->diag_f.ptr + o,
                    ctx->lambda_f.ptr + o, G->prec_cyl.ptr, ctx->bvec.ptr + o, 1, first, reuse_diag, radius,
                    ctx->stream);
}

void gsba_schur_product(mi_ba_context* ctx, const double* x, double* y) {
  GsbaState* G = ctx->gsba;
  if (!G->nblocks) return;
  const GsbaOwn w = owners(ctx);
  hipLaunchKernelGGL(gsba_jx_kernel, dim3(grid64(G->nblocks)), dim3(64), 0, ctx->stream, w, x, G->ework.ptr);
  hipLaunchKernelGGL(gsba_jte_owner_kernel, dim3(w.nimg + w.ncyl), dim3(64), 0, ctx->stream, w, G->ework.ptr, y);
}

void gsba_precond(mi_ba_context* ctx, const double* r, double* z) {
  GsbaState* G = ctx->gsba;
  if (!ctx->dev.cyl_var || G->ncyl == 0) return;
  const int64_t o = ctx->dev.cyl0;
  launch_precond_n(G->cw, G->ncyl, G->prec_cyl.ptr, r + o, z + o, ctx->stream);
}

void gsba_add_dense(mi_ba_context* ctx, double* S) {
  GsbaState* G = ctx->gsba;
  if (!G->nblocks) return;
  const GsbaOwn w = owners(ctx);
  hipLaunchKernelGGL(gsba_dense_owner_kernel, dim3(w.nimg + w.ncyl), dim3(64), 0, ctx->stream, w, ctx->dev.lds, S);
  const int64_t n = (int64_t)G->nblocks * 6 * G->cw;
  hipLaunchKernelGGL(gsba_dense_cross_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, w,
                     ctx->dev.lds, S);
}

void gsba_model_cost(mi_ba_context* ctx, const double* df, double* d_out) {
  GsbaState* G = ctx->gsba;
  if (!G->nblocks) return;
  const GsbaOwn w = owners(ctx);
  hipLaunchKernelGGL(gsba_model_terms_kernel, dim3(grid64(G->nblocks)), dim3(64), 0, ctx->stream, w, G->r.ptr, df,
                     G->ework.ptr);
  hipLaunchKernelGGL(gsba_ordered_add_kernel, dim3(1), dim3(256), 0, ctx->stream, G->ework.ptr, G->nblocks, 1, d_out);
}

void gsba_plus(mi_ba_context* ctx, const double* df) {
  GsbaState* G = ctx->gsba;
  if (G->ncyl == 0) return;
  if (!ctx->dev.cyl_var) {
    (void)hipMemcpyAsync(G->cyl_c.ptr, G->cyl.ptr, G->cyl.bytes(), hipMemcpyDeviceToDevice, ctx->stream);
    return;
  }
  if (G->by2)
    hipLaunchKernelGGL(gsba_plus_by2_kernel, dim3(grid64(G->ncyl)), dim3(64), 0, ctx->stream, G->ncyl, G->cyl.ptr,
                       df + ctx->dev.cyl0, G->cyl_c.ptr);
  else
    hipLaunchKernelGGL(gsba_plus_kernel, dim3(grid64(G->ncyl)), dim3(64), 0, ctx->stream, G->ncyl, G->cyl.ptr,
                       df + ctx->dev.cyl0, G->cyl_c.ptr);
}

void gsba_add_gradient(mi_ba_context* ctx, double* g) {
  GsbaState* G = ctx->gsba;
  if (!G->nblocks) return;
  const GsbaOwn w = owners(ctx);
  hipLaunchKernelGGL(gsba_jte_owner_kernel, dim3(w.nimg + w.ncyl), dim3(64), 0, ctx->stream, w, G->r.ptr, g);
}

void gsba_grad_max(mi_ba_context* ctx, const double* g, double* out) {
  GsbaState* G = ctx->gsba;
  if (!ctx->dev.cyl_var || G->ncyl == 0) return;
  hipLaunchKernelGGL(gsba_grad_max_kernel, dim3(grid64(G->ncyl)), dim3(64), 0, ctx->stream, G->ncyl, G->by2 ? 1 : 0,
                     G->cyl.ptr, g + ctx->dev.cyl0, out);
}

void gsba_state_norms(mi_ba_context* ctx, double* out) {
  GsbaState* G = ctx->gsba;
  if (!ctx->dev.cyl_var || G->ncyl == 0) return;
  hipLaunchKernelGGL(gsba_state_terms_kernel, dim3(grid64(G->ncyl)), dim3(64), 0, ctx->stream, G->ncyl, G->by2 ? 1 : 0,
                     G->cyl.ptr, G->cyl_c.ptr, G->cstate.ptr);
  hipLaunchKernelGGL(gsba_ordered_add_kernel, dim3(1), dim3(256), 0, ctx->stream, G->cstate.ptr, G->ncyl, 2, out);
}

void gsba_accept(mi_ba_context* ctx) {
  GsbaState* G = ctx->gsba;
  std::swap(G->cyl.ptr, G->cyl_c.ptr);
}

mi_ba_status gsba_writeback(mi_ba_context* ctx) {
  GsbaState* G = ctx->gsba;
  if (!G->ncyl) return MI_BA_OK;
  std::vector<double> cyl(9 * (size_t)G->ncyl);
  if (hipStreamSynchronize(ctx->stream) != hipSuccess ||
      hipMemcpy(cyl.data(), G->cyl.ptr, cyl.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return MI_BA_ERR_HIP;
  if (!ctx->dev.cyl_var) return MI_BA_OK;
  for (int c = 0; c < G->ncyl; ++c) {
    mi_ba_cylinder& y = G->host->cylinders[c];
    if (G->by2) {
      // exportCylindersToText writes ToCylinder() (cylinder_by_2_points.h:134-143)
      double e[9];
      by2_to_cylinder(&cyl[9 * c], e);
      for (int m = 0; m < 4; ++m) y.qvec[m] = e[m];
      for (int m = 0; m < 3; ++m) y.tvec[m] = e[4 + m];
      y.radius = e[7];
      y.height = e[8];
      continue;
    }
    for (int m = 0; m < 4; ++m) y.qvec[m] = cyl[9 * c + m];
    for (int m = 0; m < 3; ++m) y.tvec[m] = cyl[9 * c + 4 + m];
    y.radius = cyl[9 * c + 7];
    y.height = cyl[9 * c + 8];
  }
  return MI_BA_OK;
}

mi_ba_status gsba_download(mi_ba_context* ctx, int32_t* ids, double* residuals, double* jacobians) {
  GsbaState* G = ctx->gsba;
  const int nb = G->nblocks;
  if (!nb) return MI_BA_OK;
  DevArray<double> J16, rr;
  DevArray<double> cost;
  if (J16.alloc(16 * (size_t)nb) || rr.alloc(nb) || cost.alloc(1)) return MI_BA_ERR_OUT_OF_MEMORY;
  if (hipMemsetAsync(cost.ptr, 0, 8, ctx->stream) != hipSuccess) return MI_BA_ERR_HIP;
  mi_ba_status st = eval_blocks(ctx, cost.ptr, J16.ptr, rr.ptr);
  if (st != MI_BA_OK) return st;
  if (hipStreamSynchronize(ctx->stream) != hipSuccess ||
      hipMemcpy(jacobians, J16.ptr, 16 * (size_t)nb * 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(residuals, rr.ptr, (size_t)nb * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return MI_BA_ERR_HIP;
  for (int k = 0; k < nb; ++k) {
    ids[2 * k] = G->blocks_host[k].img;
    ids[2 * k + 1] = G->blocks_host[k].cyl;
  }
  return MI_BA_OK;
}

}  // namespace miba
