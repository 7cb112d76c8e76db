// oracle_gsba.h — TEST INFRASTRUCTURE ONLY (the CPU oracle; never linked by
// the product).  Restatement of the geometric-semantic BA (GSBA) cylinder
// IoU residual of AlainSchoebi/semantic-bundle-adjustment-colmap:
//
//   ComputeSemanticIoU / ProjectToMask / ProjectToQuadrilateral /
//   GetEdgePoints      src/util/cylinder.h:270-540
//   drawQuadrilateral  src/util/cylinder.h:21-117
//   XYWH               src/util/xywh.h (bound points, shrink, corners)
//   simplePinholeProject src/util/utils.h:22-54
//   GSBACostFunction / ConstantPoseGSBACostFunction /
//   ConstantCylinderGSBACostFunction  src/base/geometric_semantic_cost_functions.h:33-165
//   Ceres 2.1 AngleAxisRotatePoint (rotation.h) and NumericDiffCostFunction
//   CENTRAL (numeric_diff.h): 3rd party, not vendored, restated.
//
// Parity unpinned: the reference has no GSBA tests or data.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

#include "oracle_math.h"

namespace oracle {

struct GsbaBox {  // XYWH
  int x = 0, y = 0, w = 0, h = 0;
  int x_end() const { return x + w - 1; }
  int y_end() const { return y + h - 1; }
  int npix() const { return w * h; }
};

// XYWH::setToBoundPoints: floor of the minima, ceil of the maxima.
inline GsbaBox GsbaBound(const double (*p)[2], int n) {
  double min_x = p[0][0], min_y = p[0][1], max_x = p[0][0], max_y = p[0][1];
  for (int k = 0; k < n; ++k) {
    min_x = std::min<double>(min_x, p[k][0]);
    max_x = std::max<double>(max_x, p[k][0]);
    min_y = std::min<double>(min_y, p[k][1]);
    max_y = std::max<double>(max_y, p[k][1]);
  }
  GsbaBox b;
  b.x = CastToIntX86(std::floor(min_x));
  b.y = CastToIntX86(std::floor(min_y));
  b.w = CastToIntX86(std::ceil(max_x)) - b.x + 1;
  b.h = CastToIntX86(std::ceil(max_y)) - b.y + 1;
  return b;
}

// XYWH::shrinkToFitInToFitIn(XYWH(0, 0, W, H))
inline GsbaBox GsbaShrink(GsbaBox b, int W, int H) {
  const int x0 = std::max(b.x, 0), y0 = std::max(b.y, 0);
  const int x1 = std::min(b.x_end(), W - 1), y1 = std::min(b.y_end(), H - 1);
  GsbaBox o;
  if (x1 < x0 || y1 < y0) return o;
  o.x = x0;
  o.y = y0;
  o.w = x1 - x0 + 1;
  o.h = y1 - y0 + 1;
  return o;
}

// Ceres 2.1 AngleAxisRotatePoint (rotation.h), restated.
inline void AngleAxisRotatePoint(const double aa[3], const double pt[3], double r[3]) {
  const double theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta2 > std::numeric_limits<double>::epsilon()) {
    const double theta = std::sqrt(theta2);
    const double costheta = std::cos(theta);
    const double sintheta = std::sin(theta);
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

// simplePinholeProject (utils.h:22-54): false where the reference throws
// (point behind the camera).
inline bool GsbaProject(const double cq[4], const double ct[3], const double K[3], const double X[3], double out[2]) {
  double pc[3];
  PoseTransformPoint(cq, ct, X, pc);
  if (pc[2] <= 0) return false;
  pc[0] /= pc[2];
  pc[1] /= pc[2];
  out[0] = K[0] * pc[0] + K[1];
  out[1] = K[0] * pc[1] + K[2];
  return true;
}

// Cylinder::ProjectToQuadrilateral (cylinder.h:356-402) with GetEdgePoints
// (:286-354): false where the reference throws (camera inside the infinite
// cylinder, an edge point behind the camera) — ComputeSemanticIoU then
// returns 0.
inline bool GsbaQuad(const double cq[4], const double ct[3], const double K[3], const double yq[4],
                     const double yt[3], double radius, double height, double p2d[4][2]) {
  double cwq[4], cwt[3];
  PoseInverse(cq, ct, cwq, cwt);
  double qi[4], ti[3];
  PoseInverse(yq, yt, qi, ti);
  double c[3];
  PoseTransformPoint(qi, ti, cwt, c);
  c[2] = 0;
  const double dist = std::sqrt(c[0] * c[0] + c[1] * c[1]);
  if (dist <= radius) return false;
  const double dir[3] = {c[0] / dist * radius, c[1] / dist * radius, 0};
  const double beta = std::acos(radius / dist);
  const double aap[3] = {0, 0, beta}, aan[3] = {0, 0, -beta};
  double p[4][3];
  AngleAxisRotatePoint(aap, dir, p[0]);
  AngleAxisRotatePoint(aan, dir, p[1]);
  p[2][0] = p[1][0]; p[2][1] = p[1][1]; p[2][2] = p[1][2] + height;
  p[3][0] = p[0][0]; p[3][1] = p[0][1]; p[3][2] = p[0][2] + height;
  for (int k = 0; k < 4; ++k) {
    double w[3];
    PoseTransformPoint(yq, yt, p[k], w);
    if (!GsbaProject(cq, ct, K, w, p2d[k])) return false;
  }
  // order the edge points (image y-axis down): reverse if v0 x v1 < 0
  const double v0x = p2d[1][0] - p2d[0][0], v0y = p2d[1][1] - p2d[0][1];
  const double v1x = p2d[2][0] - p2d[0][0], v1y = p2d[2][1] - p2d[0][1];
  if (v0x * v1y - v0y * v1x < 0) {
    std::swap(p2d[1][0], p2d[3][0]);
    std::swap(p2d[1][1], p2d[3][1]);
  }
  return true;
}

// drawQuadrilateral (cylinder.h:21-117) restricted to its shrunk bounding
// box: the box is set, each edge clears the pixels of its own bounding box
// strictly on its outer side, and a vertex strictly inside the box clears the
// rectangle between it and the nearest box corner.  mask = box.w x box.h.
inline void GsbaDraw(const double p[4][2], int W, int H, GsbaBox* out_box, std::vector<uint8_t>* out_mask) {
  const GsbaBox box = GsbaShrink(GsbaBound(p, 4), W, H);
  std::vector<uint8_t>& mask = *out_mask;
  mask.assign((size_t)std::max(0, box.npix()), 1);
  auto at = [&](int x, int y) -> uint8_t& { return mask[(size_t)(y - box.y) * box.w + (x - box.x)]; };
  for (int e = 0; e < 4; ++e) {
    const double* a = p[e];
    const double* b = p[(e + 1) % 4];
    const double ab[2][2] = {{a[0], a[1]}, {b[0], b[1]}};
    const GsbaBox eb = GsbaShrink(GsbaBound(ab, 2), W, H);
    if (eb.npix() == 0) continue;
    for (int y = eb.y; y <= eb.y_end(); ++y)
      for (int x = eb.x; x <= eb.x_end(); ++x) {
        const double cross = ((double)x - a[0]) * (b[1] - a[1]) - ((double)y - a[1]) * (b[0] - a[0]);
        if (cross > 0) at(x, y) = 0;  // eb lies inside box
      }
  }
  for (int k = 0; k < 4; ++k) {
    const double* q = p[k];
    if (q[0] - box.x < 1 || box.x_end() - q[0] < 1 || q[1] - box.y < 1 || box.y_end() - q[1] < 1) continue;
    const int cx[4] = {box.x, box.x_end(), box.x_end(), box.x};  // TL, TR, BR, BL
    const int cy[4] = {box.y, box.y, box.y_end(), box.y_end()};
    int best = 0;
    double bd = 0.0;
    for (int m = 0; m < 4; ++m) {
      const double dx = q[0] - (double)cx[m], dy = q[1] - (double)cy[m];
      const double d = std::sqrt(dx * dx + dy * dy);
      if (m == 0 || d < bd) { best = m; bd = d; }
    }
    const double cb[2][2] = {{(double)cx[best], (double)cy[best]}, {q[0], q[1]}};
    const GsbaBox rb = GsbaShrink(GsbaBound(cb, 2), W, H);
    for (int y = rb.y; y <= rb.y_end(); ++y)
      for (int x = rb.x; x <= rb.x_end(); ++x) at(x, y) = 0;
  }
  *out_box = box;
}

// Cylinder::ComputeSemanticIoU (cylinder.h:496-540) over the boolean map
// `sem` (row-major H x W, 1 = trunk class); sem_total = its count.
inline double GsbaIoU(const double cq[4], const double ct[3], const double K[3], const double yq[4],
                      const double yt[3], double radius, double height, const uint8_t* sem, int H, int W,
                      int64_t sem_total) {
  // Cylinder::Check on the evaluated copy
  if (radius <= 0) radius = 1e-4;
  if (height <= 0) height = 1e-4;
  double p[4][2];
  if (!GsbaQuad(cq, ct, K, yq, yt, radius, height, p)) return 0.0;
  GsbaBox box;
  std::vector<uint8_t> mask;
  GsbaDraw(p, W, H, &box, &mask);
  auto at = [&](int x, int y) { return mask[(size_t)(y - box.y) * box.w + (x - box.x)]; };
  int64_t tp = 0, fp = 0;
  for (int y = box.y; y <= box.y_end(); ++y)
    for (int x = box.x; x <= box.x_end(); ++x) {
      if (!at(x, y)) continue;
      if (sem[(size_t)y * W + x]) ++tp;
      else ++fp;
    }
  // fn = sem_pos_outside + (npix - count(select(sem, mask, true))) = sem_total - tp
  const int64_t fn = sem_total - tp;
  double den = (double)tp * 1.;
  den = den + (double)fp;
  den = den + (double)fn;
  return (double)tp / den;
}

// CylinderBy2Points::ToCylinder (src/util/cylinder_by_2_points.h:95-117) on
// y = tvec_1(3) tvec_2(3) radius, through the constructor's Check (radius
// <= 0 -> 1e-4, :38-42) and Cylinder's (height <= 0 -> 1e-4): d = (t2 - t1)
// / |t2 - t1| (Eigen: norms and dot products of 3-vectors summed left to
// right, division per element), axis = z x d normalised ((1, 0, 0) when its
// norm < 1e-10), angle = acos(z . d), Ceres 2.1 AngleAxisToQuaternion(angle *
// axis); tvec = t1, height = |t1 - t2|.
inline void GsbaBy2ToCylinder(const double* y, double q[4], double t[3], double* radius, double* height) {
  *radius = y[6] <= 0 ? 1e-4 : y[6];
  double d[3] = {y[3] - y[0], y[4] - y[1], y[5] - y[2]};
  const double dn = std::sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
  for (double& v : d) v /= dn;
  double axis[3] = {0.0 * d[2] - 1.0 * d[1], 1.0 * d[0] - 0.0 * d[2], 0.0 * d[1] - 0.0 * d[0]};
  const double an = std::sqrt((axis[0] * axis[0] + axis[1] * axis[1]) + axis[2] * axis[2]);
  if (std::fabs(an) < 1e-10) {
    axis[0] = 1.0;
    axis[1] = 0.0;
    axis[2] = 0.0;
  } else {
    for (double& v : axis) v /= an;
  }
  const double angle = std::acos((0.0 * d[0] + 0.0 * d[1]) + 1.0 * d[2]);
  const double aa[3] = {angle * axis[0], angle * axis[1], angle * axis[2]};
  const double theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta2 > 0.0) {
    const double theta = std::sqrt(theta2);
    const double half = theta * 0.5;
    const double k = std::sin(half) / theta;
    q[0] = std::cos(half);
    q[1] = aa[0] * k;
    q[2] = aa[1] * k;
    q[3] = aa[2] * k;
  } else {
    q[0] = 1.0;
    q[1] = aa[0] * 0.5;
    q[2] = aa[1] * 0.5;
    q[3] = aa[2] * 0.5;
  }
  for (int m = 0; m < 3; ++m) t[m] = y[m];
  const double e0 = y[0] - y[3], e1 = y[1] - y[4], e2 = y[2] - y[5];
  const double h = std::sqrt((e0 * e0 + e1 * e1) + e2 * e2);
  *height = h <= 0 ? 1e-4 : h;
}

// CylinderBy2Points(const Cylinder&) (:44-48): tvec_1 = tvec, tvec_2 =
// GetEigUpperTvec() = PoseTransformPoint(q, t, (0, 0, height)) (cylinder.h:
// 567-577), radius.
inline void GsbaCylinderToBy2(const double q[4], const double t[3], double radius, double height, double y[7]) {
  const double top[3] = {0, 0, height};
  double u[3];
  PoseTransformPoint(q, t, top, u);
  for (int m = 0; m < 3; ++m) {
    y[m] = t[m];
    y[3 + m] = u[m];
  }
  y[6] = radius;
}

// GSBA residual block variants (geometric_semantic_bundle_adjustment.cc:853-909).
enum { kGsbaFull = 0, kGsbaConstantPose = 1, kGsbaConstantCylinder = 2 };

// Residual 1 - IoU and the ambient CENTRAL numeric-diff Jacobian of one
// block, columns [camera q(4), camera t(3), cylinder q(4), t(3), radius,
// height] (columns of constant blocks zero), Ceres 2.1 numeric_diff.h:
// delta_j = max(sqrt(eps), |x_j| * relative_step_size),
// J_j = (f(x + delta e_j) - f(x - delta e_j)) * ((1 / delta) / 2).
//
// by2 (CylinderBy2Points, GSBACostFunctionBy2Points and its constant-pose /
// constant-cylinder variants, geometric_semantic_cost_functions.h:167-348):
// yq = nullptr and yt = the 7 parameters tvec_1, tvec_2, radius; the
// cylinder columns are then [tvec_1, tvec_2, radius, 0, 0].
inline double GsbaEvalBlock(int variant, const double cq[4], const double ct[3], const double K[3],
                            const double yq[4], const double yt[3], double radius, double height,
                            const uint8_t* sem, int H, int W, int64_t sem_total, double rel_step, double* J16) {
  const bool by2 = yq == nullptr;
  double x[16];
  for (int m = 0; m < 4; ++m) x[m] = cq[m];
  for (int m = 0; m < 3; ++m) x[4 + m] = ct[m];
  if (by2) {
    for (int m = 0; m < 7; ++m) x[7 + m] = yt[m];
    x[14] = x[15] = 0.0;
  } else {
    for (int m = 0; m < 4; ++m) x[7 + m] = yq[m];
    for (int m = 0; m < 3; ++m) x[11 + m] = yt[m];
    x[14] = radius;
    x[15] = height;
  }
  auto f = [&]() {
    if (!by2) return 1.0 - GsbaIoU(&x[0], &x[4], K, &x[7], &x[11], x[14], x[15], sem, H, W, sem_total);
    double q[4], t[3], r, h;
    GsbaBy2ToCylinder(&x[7], q, t, &r, &h);
    return 1.0 - GsbaIoU(&x[0], &x[4], K, q, t, r, h, sem, H, W, sem_total);
  };
  const double r = f();
  if (!J16) return r;
  const int lo = variant == kGsbaConstantPose ? 7 : 0;
  const int hi = variant == kGsbaConstantCylinder ? 7 : (by2 ? 14 : 16);
  const double min_step = std::sqrt(std::numeric_limits<double>::epsilon());
  for (int j = 0; j < 16; ++j) {
    J16[j] = 0.0;
    if (j < lo || j >= hi) continue;
    const double orig = x[j];
    const double delta = std::max(min_step, std::fabs(orig) * rel_step);
    x[j] = orig + delta;
    const double fp = f();
    x[j] = orig - delta;
    const double fm = f();
    x[j] = orig;
    double one_over_delta = 1.0 / delta;
    one_over_delta /= 2;
    J16[j] = (fp - fm) * one_over_delta;
  }
  return r;
}

}  // namespace oracle
