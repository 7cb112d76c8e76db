// semantic.h — semantic-label residual term on the GPU (product code).
//
// Replaces the Ceres NumericDiff evaluation of the
// {,ConstantFirstPose,ConstantSecondPose}SemanticBACostFunction blocks
// (src/base/semantic_cost_functions.h:87-404) that
// SemanticBundleAdjuster::AddImagePairToProblem creates per sampled pixel
// (src/optim/semantic_bundle_adjustment.cc:699-906).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>

#include "../../include/mi_ba.h"
#include "ba_math.h"
#include "context.h"

namespace miba {

struct SemSample {      // 32 B, one per sampled pixel
  double pc1[3];        // P_c1 = (u1*d1, v1*d1, d1) (semantic_cost_functions.h:103-118)
  float label1;         // semantic_1_
  uint32_t pair;        // index into the pair table
};

struct SemTile {       // pair-aligned tile of samples
  uint32_t pair, start, count, pad;
};

struct SemPair {
  uint32_t i, j;        // image indices
  uint32_t var1, var2;  // pose i / pose j variable
  uint32_t start, count;
};

// One raster slot (an image used as the second image of a pair): its plane
// in the rasters / label plane / window summaries (off, pixels) and in the
// tile depth ranges (toff, 8 x 8 tiles), its own size (ABI 4: every image
// has its own H x W, semantic_bundle_adjustment.cc:792-793,
// semantic_cost_functions.h:163) and tiles per row.
struct SlotInfo {
  uint64_t off, toff;
  int32_t H, W, TW, pad;
};

struct SemanticState {
  std::vector<int32_t> img_h, img_w;       // [I] each image's raster size
  std::vector<SlotInfo> slots_host;        // [nslots]
  DevArray<SlotInfo> slots;
  int64_t npix = 0;                        // pixels of every slot's plane
  int64_t ntile = 0;                       // 8 x 8 tiles of every slot
  int max_plane = 0, max_tiles = 0;        // largest slot plane / tile grid
  double depth_threshold = 2.0;
  double rel_step = 1e-3;
  int step = 1;          // pixel grid step (error_computation_pixel_step)
  std::vector<uint8_t> has_raster;         // [I] image has a raster slot
  int64_t ns = 0;        // samples
  int npairs = 0;
  std::vector<SemPair> pairs_host;
  std::vector<int32_t> sample_pixel_host;  // [ns][3]
  DevArray<SemSample> samples;
  DevArray<SemPair> pairs;
  DevArray<float2> dl;                     // slot planes [H_s][W_s] (depth, label) of images used as j
  int nslots = 0;
  DevArray<float4> wsum;                   // slot planes: 3x3 window summaries ("semantic_window_summary")
  bool use_wsum = false;
  // label planes ("semantic_label_planes"): the flat pass's first reads.
  // lab8 = each raster pixel's label as an index into pal (the rasters'
  // distinct label bit patterns, <= 256), dtile = (min, max) depth over each
  // 8 x 8 pixel tile extended by 2 pixels right and down (every 3 x 3 box
  // whose top-left pixel lies in the tile), NaN when a depth in it is NaN
  DevArray<uint8_t> lab8;                  // slot planes [H_s][W_s]
  DevArray<float2> dtile;                  // slot tile planes [ceil(H_s/8)][ceil(W_s/8)]
  DevArray<float> pal;                     // [256]
  bool use_lp = false;
  DevArray<uint32_t> raster_slot;          // image -> raster slot
  DevArray<double> r;                      // [ns]
  DevArray<int32_t> status;                // [ns]
  DevArray<double> J;                      // [ns][12]
  DevArray<double> pconst;                 // [npairs] PairConst (semantic.hip), per linearization
  bool samples_valid = false;              // r / status / J hold the last evaluation
  DevArray<double> pair_blk;               // [npairs][12*12 + 12]: M = J'J (full) and g = J'r
  DevArray<double> partial;
  int64_t npartial = 0;
  DevArray<SemTile> tiles;                 // grouped by the model of the pair's second camera
  int ntiles = 0;
  int model_tiles[kNumModels + 1] = {};    // tile range of each camera model
  // two-pass linearization (semantic_variant 6): per-pair deferred lists
  DevArray<uint32_t> pair_cnt;             // [npairs] deferred samples of the pair
  DevArray<uint32_t> dlist;                // [ns] deferred samples (offset in pair), pair regions
  DevArray<uint2> chunks;                  // (pair, first entry): 64-entry chunks of every pair region
  DevArray<uint2> dchunks;                 // the chunks the flat pass filled (deferred_compact_kernel), same regions
  DevArray<uint32_t> dcount;               // [model] their number
  int n_cu = 256;                          // compute units (the deferred pass's resident grid)
  int model_chunks[kNumModels + 1] = {};   // chunk range of each camera model
  // deterministic sums: the flat pass's deferral masks ([tile][4] words),
  // each pair's first tile and first static chunk, the deferred pass's chunk
  // partials; the pairs of each image ((pair << 1) | side, pair order) and
  // the pair-block contributions to each explicit S block
  DevArray<unsigned long long> dmask;
  DevArray<uint32_t> pair_tile0, pair_chunk0;
  DevArray<double> cpart;                  // [static chunk][kPairVals]
  DevArray<uint32_t> img_pairs_off, img_pairs;
  DevArray<uint2> sblk;                    // S blocks (i <= j) the pairs touch
  DevArray<uint32_t> sblk_off, sblk_ent;   // their contributions ((pair << 1) | i-is-second)
  int nsblk = 0;
  DevArray<double> mpart;                  // per-wave partials of the model cost change
};

mi_ba_status semantic_create(mi_ba_context* ctx, const mi_ba_semantic* sem);
void semantic_destroy(mi_ba_context* ctx);
// Evaluate residuals + numeric-diff Jacobians of every sample; store r/J and
// reduce into per-pair blocks; cost (0.5 * w * sum rho) into *d_cost.
// deferred_stream (nullable): run the two-pass route's deferred-sample pass
// there, ordered after the flat pass by flat_done; the caller joins it.
// timer_start: the semantic timer starts at this recorded event (the
// previous phase's stop).  other_partial / other_n / other_out / other_scratch:
// a second cost sum (the reprojection partials) launched together with the
// semantic one.  after_flat (optional): called once the flat pass is
// enqueued, before the deferred pass (the input warm-up's launch point).
mi_ba_status semantic_linearize(mi_ba_context* ctx, double* d_cost, bool write_samples,
                                hipStream_t deferred_stream = nullptr, hipEvent_t flat_done = nullptr,
                                hipEvent_t timer_start = nullptr, const double* other_partial = nullptr,
                                int64_t other_n = 0, double* other_out = nullptr, double* other_scratch = nullptr,
                                const std::function<mi_ba_status()>& after_flat = nullptr,
                                hipEvent_t prep_done = nullptr);
// The pair tables of one linearization on `stream` (semantic_linearize does
// it itself unless given prep_done, the event after an earlier call).
mi_ba_status semantic_pair_prep(mi_ba_context* ctx, hipStream_t stream);
// ExportSemanticErrorToCSV rows of the ordered image pair (image1, image2) at
// the current parameters (mi_ba_semantic_export).
mi_ba_status semantic_export(mi_ba_context* ctx, int32_t image1, int32_t image2, int64_t* count, int32_t* pixels,
                             int32_t* status, double* error, double* world);
// Build (on) or drop (off) the rasters' 3x3 window summaries the flat pass
// decides most samples from without reading the raster.
mi_ba_status semantic_set_window_summary(mi_ba_context* ctx, bool on);
// Build (on) or drop (off) the label planes (an 8-bit label index plane with
// its palette, and 8 x 8 tile depth ranges) the flat pass reads first: on
// with more than 256 distinct labels leaves them off (MI_BA_OK).
mi_ba_status semantic_set_label_planes(mi_ba_context* ctx, bool on);
// Cost only, at parameters qt (candidate evaluation).
void semantic_cost(mi_ba_context* ctx, const double* qt, const double* cam, double* d_cost);
// Fold the pair blocks into the Schur-Jacobi pose blocks, b and diag(U).
void semantic_add_fblock(mi_ba_context* ctx);
// g += the pair blocks' J'r on their poses (gradient tolerance test).
void semantic_add_gradient(mi_ba_context* ctx, double* g);
// y += M_pair x (implicit Schur product).
void semantic_schur_product(mi_ba_context* ctx, const double* x, double* y);
// Add the pair blocks M into the explicit reduced camera system S.
void semantic_add_dense(mi_ba_context* ctx, double* S);
// Model cost change contribution -(g'd + d'Md/2) into *d_out.
void semantic_model_cost(mi_ba_context* ctx, const double* df, double* d_out);

}  // namespace miba
