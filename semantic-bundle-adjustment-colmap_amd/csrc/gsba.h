// gsba.h — the geometric-semantic BA (GSBA) cylinder IoU term of a resident
// context (product code; kernels in gsba.hip).
//
// Blocks: one per (config image, cylinder) (geometric_semantic_bundle_
// adjustment.cc:835-909), variants full / constant pose / constant cylinder.
// Each block's residual 1 - IoU and its CENTRAL numeric derivatives take 1 +
// 2 * (ambient parameters) IoU evaluations (33 / 17 / 15); every evaluation
// is one workgroup that projects the perturbed cylinder to its quadrilateral
// and scans the quadrilateral's bounding box in the image's trunk mask.
// Tangent Jacobian rows (pose 6, cylinder 8) then feed the same normal
// equation hooks as the semantic term.
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/mi_ba.h"
#include "context.h"

namespace miba {

struct GsbaBlock {     // device block descriptor
  int32_t img, cyl, variant, slot;   // slot: trunk mask of the image
  int32_t eval0, nevals, pad0, pad1; // evaluations [eval0, eval0 + nevals)
};
// One image's trunk mask (its own size, ABI 4): its plane in the byte masks
// (moff) and in the bit-packed masks (boff, words per row).
struct GsbaSlot {
  uint64_t moff, boff;
  int32_t H, W, words, pad;
};
struct GsbaEval {      // one IoU evaluation: block, perturbed parameter (-1 = none), sign
  int32_t block;
  int16_t param;
  int16_t sign;
};

struct GsbaState {
  const mi_ba_gsba* host = nullptr;  // caller's struct (cylinders written back)
  int ncyl = 0, nblocks = 0;
  int64_t nevals = 0;
  double rel_step = 1e-3;
  double weight = 1.0;               // ScaledLoss(1 / #config images)
  bool by2 = false;                  // MI_BA_CYLINDER_BY_2_POINTS (CylinderBy2Points)
  int cw = 8;                        // cylinder tangent width: 8, or 7 by 2 points
  std::vector<GsbaBlock> blocks_host;
  DevArray<GsbaBlock> blocks;
  DevArray<GsbaEval> evals;          // linearization: every evaluation
  DevArray<GsbaEval> centres;        // cost: one per block
  std::vector<GsbaSlot> slots_host;  // [slot] the masks' planes and sizes
  DevArray<GsbaSlot> slots;
  DevArray<uint8_t> masks;           // slot planes [H_s][W_s]
  DevArray<uint64_t> mask_bits;      // slot planes [H_s][words_s] bit-packed masks (span kernel)
  int iou_variant = 0;               // 0 row spans over mask_bits, 1 per-pixel predicate (tools build)
  DevArray<int64_t> sem_total;       // [slot]
  DevArray<double> cyl, cyl_c;       // [ncyl][9] q(4) t(3) radius height (by 2 points: t1(3) t2(3) radius 0 0):
                                     // current, candidate
  DevArray<double> iou;              // [nevals]
  DevArray<double> r;                // [nblocks] corrected residual
  DevArray<double> J;                // [nblocks][14] corrected tangent rows: pose(6) cylinder(cw)
  DevArray<double> cyl_blk;          // [ncyl][cw (cw + 1) / 2] cylinder Schur-Jacobi blocks (packed upper)
  DevArray<double> prec_cyl;         // [ncyl][64]
  DevArray<double> partial;          // per-block cost
  // deterministic sums: blocks are image-major with every cylinder once per
  // image (block = image rank * ncyl + cylinder), so an image's blocks are
  // contiguous and a cylinder's are strided; the per-owner kernels sum them
  // in block order (no float atomics)
  DevArray<double> ework;            // [nblocks] per-block scalar (J x, residual, model term)
  DevArray<double> cstate;           // [2][ncyl] per-cylinder |y|^2, |y - y_c|^2
};

// Number of cylinder parameter slots the context must reserve (8 per
// cylinder when they are refined, 7 by 2 points).
int gsba_cylinder_slots(const mi_ba_options& o, const mi_ba_problem* p, const mi_ba_gsba* g);
// Validates (GeometricSemanticBundleAdjuster::Assert), builds blocks, uploads
// masks and cylinders, marks GSBA poses variable.  Called at the end of
// context creation.
mi_ba_status gsba_create(mi_ba_context* ctx, const mi_ba_gsba* g);
void gsba_destroy(mi_ba_context* ctx);
// Residuals + tangent Jacobians of every block at the current parameters;
// cost (0.5 * w * sum r^2) into *d_cost.
mi_ba_status gsba_linearize(mi_ba_context* ctx, double* d_cost);
// Cost at candidate poses qt and candidate cylinders.
void gsba_cost(mi_ba_context* ctx, const double* qt, const double* cyl, double* d_cost);
void gsba_add_fblock(mi_ba_context* ctx);
void gsba_finalize(mi_ba_context* ctx, int first, int reuse_diag, double radius);
void gsba_schur_product(mi_ba_context* ctx, const double* x, double* y);
void gsba_precond(mi_ba_context* ctx, const double* r, double* z);
void gsba_add_dense(mi_ba_context* ctx, double* S);
void gsba_model_cost(mi_ba_context* ctx, const double* df, double* d_out);
// candidate cylinders from the step df (QuaternionManifold, radius >= 0)
void gsba_plus(mi_ba_context* ctx, const double* df);
void gsba_accept(mi_ba_context* ctx);
// gradient tolerance: g += J'r of every block; |y - Plus(y, -g)|_inf of the
// cylinders max-ed into *out (bit pattern, atomicMax)
void gsba_add_gradient(mi_ba_context* ctx, double* g);
void gsba_grad_max(mi_ba_context* ctx, const double* g, double* out);
// parameter tolerance: |y|^2, |y - y_c|^2 of the cylinders added into out[0..1]
void gsba_state_norms(mi_ba_context* ctx, double* out);
mi_ba_status gsba_writeback(mi_ba_context* ctx);
// every block's residual (1 - IoU) and ambient Jacobian [16] (mi_ba_gsba_evaluate)
mi_ba_status gsba_download(mi_ba_context* ctx, int32_t* ids, double* residuals, double* jacobians);

}  // namespace miba
