// device.h — device-side data layout of a resident BA problem (product code).
//
// HBM layout (all f64 unless noted), chosen for the MI355X path:
//   blocks (reduced residual blocks, POINT-MAJOR order: all observations of a
//   point are contiguous, so point-block reductions are wave-local):
//     obs_xy   double2[nb]     observed pixel (Point2D::XY)
//     obs_img  u32[nb]         image index
//     obs_pt   u32[nb]         point index
//     obs_ids  u32[nb], wave_pt0 u32[nb/64]: the same ids packed (the
//                              reprojection kernel's reads)
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
// that never straddle an image; each tile's sums are flushed per image /
// camera in a fixed order (TileOwners, deterministic).
#pragma once

#include <hip/hip_runtime.h>

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

// Owners of the camera-side tile sums (the deterministic flush,
// kernels.hip owner_flush_kernel): the tiles of image i are
// [img_tile_off[i], img_tile_off[i + 1]) (tiles are image-sorted); the tiles
// of camera c are cam_tiles[cam_tile_off[c] .. cam_tile_off[c + 1]) in image
// then tile order.  part: per-tile block sums, [tile][stride].
struct TileOwners {
  const uint32_t* img_tile_off;
  const uint32_t* cam_tile_off;
  const uint32_t* cam_tiles;
  double* part;
  int stride;  // capacity per tile (kTilePartStride)
};
constexpr int kTilePartStride = 120;  // >= the widest per-tile flush (fblock_dense at 8 intrinsics: 105 + 14)

// Deterministic Schur pair sums (kernels.hip schur_pairs_kernel with pslot):
// a pair tile whose S block no other tile writes (an off-diagonal image
// pair's only tile, cameras not shared between images) subtracts its block
// from S directly; every other tile (a diagonal block's self / same-image
// tiles, an image pair of more than one tile) writes its 16 x 16 accumulator
// to part[pslot[t]] and schur_pairs_flush_kernel sums each such block's
// tiles in list order.  pslot null: float-atomic flushes.
struct PairFlush {
  const int32_t* pslot;  // [ntiles] partial slot, -1: direct
  double* part;          // [nslots][256]
  const uint4* dest;     // [ndest] (ia, ib, first slot, slot count)
  const uint8_t* self;   // [nslots] the slot's tile holds self pairs (a == b)
  int ndest;
  // Shared cameras (several images per camera): every tile's accumulator
  // goes to part[tile] and the S blocks are summed per owner pair instead
  // (schur_owner_chunk_kernel + schur_owner_flush_kernel).  An owner is a
  // pose (image i: kOwnerPose | i) or a camera (kOwnerCam | c); a tile (ia,
  // ib) holds the four owner-pair quadrants (pose ia | cam of ia) x (pose ib
  // | cam of ib).  oent: (tile << 4 | quadrant << 2 | swapped << 1 | self),
  // tile order per owner pair; ochunk: (owner pair, first entry, entries) in
  // runs of <= 256, summed into opart[chunk][64]; odest: (X, Y, first chunk,
  // chunks), X before Y in S's slot order.  odest null: the route above.
  const uint4* odest;
  const uint4* ochunk;
  const uint32_t* oent;
  double* opart;
  int nodest, nochunk;
};
constexpr uint32_t kOwnerCam = 1u << 31;

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
  int sself1;          // schur_pairs_kernel: self tiles with one Z load per pair (1) or two (0)
  int zorder;          // Schur factors Z: 0 rows in block order, 1 in image (cm_perm) order with pairs in positions
  // inputs
  const double2* obs_xy;
  const uint32_t* obs_img;
  const uint32_t* obs_pt;
  // packed ids of the reprojection kernel (reproj_jacobian_kernel D & 8192):
  // obs_ids[b] = image | (point - wave_pt0[b / 64]) << 16, one 4-B read per
  // block instead of two (point-major order keeps a wave's points within a
  // few of each other); null (the kernel reads obs_img / obs_pt) above 65536
  // images or when a wave's points span more than 65535
  const uint32_t* obs_ids;
  const uint32_t* wave_pt0;
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
