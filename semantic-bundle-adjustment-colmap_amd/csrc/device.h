// device.h — device-side data layout of a resident BA problem (product code).
//
// HBM layout (all f64 unless noted), chosen for the MI355X path:
//   blocks (reduced residual blocks, POINT-MAJOR order: all observations of a
//   point are contiguous, so point-block reductions are wave-local):
//     obs_xy   double2[nb]     observed pixel (Point2D::XY)
//     obs_img  u32[nb]         image index
//     obs_pt   u32[nb]         point index
//     r        double2[nb]     corrected residual
//     J        double[nb][2][W] corrected tangent Jacobian, W = 9 + c,
//                              columns rot(3) trans(3) point(3) cam(c)
//   images     qt[I][8]        q(4) t(3) pad — one 64-B line per image
//              img_flags u32[I] bit0 variable pose, bits1..3 constant tvec
//   cameras    cam[C][8]       params, padded to 8
//   img_rec    double[I][kImgRec] q t meta cam R unit-q: the Jacobian kernel's per-image
//                              record (two 128-B lines), packed per linearization;
//                              meta = img_flags | cam_var << 8 | model << 16
//   points     X[P][3]
// Camera-side reductions run over cm_perm (blocks sorted by image) in tiles
// that never straddle an image, so each tile folds into one atomic flush.
#pragma once

#include <cstdint>

namespace miba {

constexpr int kMaxCamTangent = 8;
constexpr int kBlock = 256;          // threads per workgroup (4 waves)
constexpr int kTileObs = 1024;       // camera-major tile (4 obs per thread)

struct DevTile {
  uint32_t image;
  uint32_t start;  // offset into cm_perm
  uint32_t count;
  uint32_t pad;
};

struct DevPoint {      // variable point with its contiguous block range
  uint32_t point;
  uint32_t start;
  uint32_t count;
  uint32_t pad;
};

struct DevPairTile {   // image-pair tile of the explicit Schur build
  uint32_t ia, ib;     // images of the pairs' first / second block (ia <= ib)
  uint32_t start;      // offset into the pair list
  uint32_t count : 31; // pairs (<= kPairTile)
  uint32_t self : 1;   // pairs (a, a) of one observation
};
constexpr int kPairTile = 256;

// doubles per packed image record (kernels.hip pack_images_kernel)
constexpr int kImgRec = 32;

struct DevProblem {
  int model;           // camera model of every camera, or kMixedModels (per-camera cam_model)
  int np;              // camera params per camera (largest)
  int ct;              // refined intrinsics slots per camera (largest; a camera with fewer
                       // refined intrinsics has zero Jacobian columns in the rest)
  int W;               // 9 + ct
  int cam_tan_idx[kMaxCamTangent];
  int64_t nb;          // reduced geometric blocks
  int num_images, num_cameras;
  int64_t num_points;
  int64_t nf;          // f-vector length: 6*I + ct*C (+ 8 per GSBA cylinder: fixed slots, masked)
  int64_t lds;         // leading dimension of the explicit S (row-major upper = column-major lower): nf + 1
                       // rounded to 16 on the exact path, whose extra column-major row n carries the
                       // right-hand side through the factorisation (forward solve fused), else nf
  int64_t cyl0;        // first GSBA cylinder slot (= 6*I + ct*C)
  int cyl_var;         // GSBA cylinders are parameters (refine_geometry)
  int loss_type;
  double loss_scale;
  int refine_mask;     // bit0 focal, bit1 principal point, bit2 extra params
  int jvariant;        // Jacobian store path (kernels.hip reproj_jacobian_kernel V)
  int svariant;        // explicit Schur pair kernel (kernels.hip launch_dense_schur)
  int fvariant;        // fblock kernels: 0 default; 1 exact path LDS-staged MFMA, 2 PCG path one lane per block (tools build)
  // inputs
  const double2* obs_xy;
  const uint32_t* obs_img;
  const uint32_t* obs_pt;
  const uint32_t* img_flags;
  const uint32_t* img_cam;
  const uint8_t* cam_var;
  const uint8_t* cam_model;  // [C] model id per camera
  const uint8_t* pt_var;
  // parameters (current)
  double* qt;   // [I][8]
  double* cam;  // [C][8]
  double* X;    // [P][3]
  double* img_rec;  // [I][kImgRec] q(4) t(3) meta cam(8) R(9) unit-q: packed by launch_pack_images
};

}  // namespace miba
