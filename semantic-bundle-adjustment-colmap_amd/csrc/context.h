// context.h — device-resident problem and LM driver (product code).
#pragma once

#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rccl/rccl.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/mi_ba.h"
#include "cholesky.h"
#include "device.h"
#include "setup.h"

namespace miba {

// RAII device allocation.  alloc() keeps an allocation that is large
// enough (a recycled context re-sizes without hipMalloc / hipFree, which
// synchronise the device), so n is the live size and cap the allocated one.
template <typename T>
struct DevArray {
  T* ptr = nullptr;
  size_t n = 0;
  size_t cap = 0;
  DevArray() = default;
  DevArray(const DevArray&) = delete;
  DevArray& operator=(const DevArray&) = delete;
  ~DevArray() { release(); }
  hipError_t alloc(size_t count) {
    if (ptr && count <= cap) {
      n = count;
      return hipSuccess;
    }
    release();
    n = count;
    if (count == 0) return hipSuccess;
    const hipError_t e = hipMalloc(&ptr, sizeof(T) * count);
    if (e == hipSuccess) cap = count;
    else ptr = nullptr;
    return e;
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    n = 0;
    cap = 0;
  }
  size_t bytes() const { return sizeof(T) * n; }
};

struct SemanticState;  // semantic.h
struct GsbaState;      // gsba.h

struct KernelTimer {
  std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<hipEvent_t> pool;
  std::vector<hipEvent_t> borrowed;  // start events shared with the previous pending entry (pooled once)
  std::map<std::string, std::pair<double, int64_t>> totals;
};

}  // namespace miba

struct mi_ba_context {
  mi_ba_options options;
  mi_ba_problem problem;         // host arrays (caller-owned) for write-back
  miba::HostSetup setup;
  miba::DevProblem dev;
  hipStream_t stream = nullptr;
  int device = 0;

  // geometric blocks (point-major)
  std::vector<int64_t> block_obs;          // host: observation index per device block
  miba::DevArray<double2> obs_xy;
  miba::DevArray<uint32_t> obs_img, obs_pt;
  miba::DevArray<uint32_t> obs_ids, wave_pt0;  // packed ids (device.h DevProblem::obs_ids)
  miba::DevArray<uint32_t> img_flags, img_cam;
  miba::DevArray<uint8_t> cam_var, cam_model, pt_var;
  miba::DevArray<double> qt, cam, X;       // current parameters
  miba::DevArray<double> qt_c, cam_c, X_c; // candidate parameters
  miba::DevArray<double> img_rec;          // [I][kImgRec] packed image records
  miba::DevArray<uint32_t> cm_perm;
  miba::DevArray<uint32_t> cm_ptv;  // [nb] camera-major: the block's point if variable, else 0xffffffff
  miba::DevArray<miba::DevTile> tiles;
  int ntiles = 0;
  // deterministic camera-side sums (owner_flush_kernel): the tiles of each
  // image and camera, and the per-tile partials
  miba::DevArray<uint32_t> img_tile_off, cam_tile_off, cam_tiles;
  miba::DevArray<double> tpart;            // [ntiles][kTilePartStride]
  bool det_sums = true;                    // "deterministic_sums" (0: float-atomic flushes)
  const miba::TileOwners* owners() const { return det_sums && tpart.ptr ? &owners_ : nullptr; }
  miba::TileOwners owners_{};
  miba::DevArray<miba::DevPoint> vpoints;
  int64_t npv = 0;
  int64_t nb_const = 0;  // reduced blocks of constant points
  miba::DevArray<uint32_t> pchunks;  // [npchunks + 1] point-chunk boundaries (backsub_chunk_kernel)
  int npchunks = 0;
  miba::DevArray<double> sum_ws;      // [kSumScratch] stage + ticket of launch_sum's many-workgroup pass
  int lin_overlap = 0;                 // 1 semantic kernels on lin_side beside the reprojection kernel,
                                       // 2 flat pass first, deferred pass on lin_side beside it
  int lin_warm = 15;                   // "linearize_warm_inputs": range mask read right before the reprojection kernel
                                       // (1 observations, 2 image ids, 4 point ids, 8 points; 0 off)
  int lin_warm_conc = 0;               // "linearize_warm_concurrent" (tools): that read beside the semantic deferred pass
  int warm_unroll = 4;                 // "warm_unroll": loads in flight per lane of the warm-up (4 or 8)
  int warm_wgs = 2048;                 // workgroups of the warm-up kernel (0: one per CU)
  int lin_order = 0;                   // 0 reprojection kernel first, 1 semantic pass first
  hipStream_t lin_side = nullptr;
  hipEvent_t lin_ev[2] = {nullptr, nullptr};
  int sem_diag = 0;      // "semantic_diag" 1: downloaded status is offset by +0x1000 for samples the flat test
                         // deferred; 2: also by +0x4000 for samples a window summary decided
  bool sem_deferred_box = false;  // "semantic_deferred_box": the deferred pass reads each sample's 3x3 box once
  int sem_prep_early = 0; // "semantic_prep_early": pair tables on the side stream beside the reprojection kernel
                          // (measured slower: 0.823 vs 0.808 ms per step, it slows the warm-up beside it)
  int sem_dgrid = 24;    // "semantic_deferred_grid": resident deferred-pass workgroups per CU
  int sem_dvar = 0;      // "semantic_deferred_variant" (tools build): stencil batch / occupancy variants
  int sem_compact = 1;   // "semantic_deferred_compact": the deferred pass over the filled chunks only (resident grid)
  int sem_coarse = 2;    // "semantic_flat_coarse": the flat pass's box from a rotation and a translation group
                         // of the stencil classes (2 default: exact A; 1 |A| from the radius; 3 groups
                         // bounded apart; 0 the per-class bounds)
  int sem_variant = 6;   // semantic kernel ("semantic_variant"): 6 flat pass + deferred-sample pass (0.42 ms at C4), 5 flat test + in-tile gather, 4/3/2 batched stencil with 4/2/1 parameters per step (0.70 ms), 1 per-point FMA route (0.82 ms), 0 per-point uncontracted (0.92 ms); all bitwise equal

  // linearization
  miba::DevArray<double2> r;
  miba::DevArray<double> J;
  miba::DevArray<double> Jcm;  // PCG path: J's rows in camera-major (cm_perm) order
  bool jcm_stale = true;       // J re-linearized since Jcm was built
  miba::DevArray<double> Vg;               // [P][9]
  miba::DevArray<double> partial;          // per-workgroup partial sums
  int64_t npartial = 0;
  // LM state
  miba::DevArray<double> scale_p, diag_p, Vinv;
  miba::DevArray<double> pose_blk, cam_blk, bvec, udiag;
  miba::DevArray<double> scale_f, diag_f, lambda_f, prec_pose, prec_cam;
  miba::DevArray<double> cg_x, cg_r, cg_z, cg_p, cg_q, cg_w, dX;
  miba::DevArray<double> scalars;          // device scalars
  miba::DevArray<double> red;              // per-workgroup partials of the multi-workgroup reductions
  miba::DevArray<double> aux;              // [world + 2] gradient max norms: per-rank point part, camera part
  double* host_scalars = nullptr;          // pinned
  int32_t* host_info = nullptr;            // pinned: the factor's per-block info + the flag-wait error word
  int host_info_cap = 0;
  bool chol_pending = false;               // host_info enqueued, not yet checked (dense_solve, single rank)
  int chol_leaves = 0;

  // explicit reduced camera system (exact Schur solve, rocSOLVER Cholesky)
  bool dense = false;
  rocblas_handle blas = nullptr;
  miba::DevArray<double> S;
  miba::DevArray<double> Linv, Z;          // [P][6] inverse point factors, [nb][3F] Schur factors
  miba::DevArray<miba::DevPairTile> ptiles;
  miba::DevArray<miba::DevPairTile> ptiles_blk;  // the same tiles in image-block order (schur_pairs_variant 4, default)
  std::vector<miba::DevPairTile> ptiles_host;    // first-image order, kept to re-order on "schur_block_images"
  miba::DevArray<miba::DevPairTile> ptiles_xcd;  // XCD-interleaved order (schur_pairs_variant 5), empty-tile padded
  int nptiles_xcd = 0;
  int schur_block = 8;                            // images per block edge of ptiles_blk (8: schur_build 3.26 ms
                                                  // vs 3.32 / 3.42 / 3.64 at 16 / 32 / 64, profiles/r3_ab_schur_block.jsonl)
  // deterministic Schur pair sums (PairFlush; cameras not shared between images)
  miba::DevArray<int32_t> pslot;           // [nptiles] of ptiles_blk: partial slot or -1
  miba::DevArray<double> spart;            // [nslots][256]
  miba::DevArray<uint4> pdest;             // [ndest] (ia, ib, first slot, slots)
  miba::DevArray<uint8_t> pself;           // [nslots]
  int npdest = 0;
  bool pflush_ok = false;
  miba::DevArray<uint4> podest, pochunk;   // shared cameras: owner pairs, their entry runs (PairFlush)
  miba::DevArray<uint32_t> poent;
  miba::DevArray<double> popart;           // [nochunk][64]
  int npodest = 0, npochunk = 0;
  miba::DevArray<uint2> pairs;             // (a, b) block pairs bucketed by image pair
  miba::DevArray<uint2> pairs_pos;         // the same pairs as camera-major positions (Z rows of zorder 1)
  int nptiles = 0;
  miba::DevArray<int32_t> info;
  miba::CholConfig chol;                   // factorisation variant (mi_ba_set_tuning)
  bool fused_rhs = true;                   // forward solve carried through the factorisation (S's spare row)
  // PCG product matrix-free ("pcg_matrix_free"): both passes recompute the
  // blocks' Jacobian rows (no Jcm copy, no J read per product); Xcm / obs_cm
  // the camera-major copies of the blocks' points / observations
  bool pcg_mf = false;
  miba::DevArray<double> Xcm;
  miba::DevArray<double2> obs_cm;
  bool xcm_stale = true;
  int pcg_jcm = 2;  // PCG camera-side passes on the camera-major J copy, f pass staged through LDS (1: per-lane rows, 0: row gathers; tools build)
  bool pn_chunks = true;  // point blocks (V_p, g_p) on the point chunks (0: one lane per point, tools build)
  bool pp_chunks = true;                   // PCG Schur product's point pass on the point chunks (0: per point, tools build)
  bool schur_overlap = false;              // one rank: Schur terms on lm_side beside the camera-block pass
                                           // (measured slower: BA iteration 28.5 vs 27.1 ms at C4; tools build)
  hipStream_t lm_side = nullptr;
  hipEvent_t lm_ev[2] = {nullptr, nullptr};
  miba::CholWorkspace cholws;              // side stream / handle / events / scratch of this context

  double fixed_cost = 0.0;
  miba::SemanticState* sem = nullptr;
  miba::GsbaState* gsba = nullptr;        // geometric-semantic (cylinder IoU) term

  bool timing = false;
  miba::KernelTimer timer;
  bool solved = false;

  // multi-rank LM (mi_ba_context_set_comm / _set_host_reducer)
  int rank = 0, world = 1;
  ncclComm_t comm = nullptr;       // non-blocking RCCL communicator (every call polled with a deadline)
  bool comm_failed = false;        // the communicator was aborted: every later collective fails
  int comm_timeout_ms = 300000;    // deadline of one collective / of the communicator set-up ("comm_timeout_ms")
  double comm_due = 0.0;           // collectives enqueued since the last host wait: their latest deadline (0: none)
  int fail_factorizations = 0;     // test hook ("test_fail_factorizations"): the next n factorisations report a
                                   // non-positive pivot (the LM's invalid-step path)
  int comm_stall_ms = 0;           // test hook ("comm_stall_ms"): a kernel that holds the stream this long
                                   // ahead of every collective (a peer that never arrives, seen locally)
  int* stall_flag = nullptr;       // pinned release flag of that kernel
  mi_ba_host_allreduce_fn host_reduce = nullptr;
  void* host_reduce_user = nullptr;
  std::vector<double> reduce_buf;
  // Sums go over the ranks whenever a reducer is installed, a 1-rank RCCL
  // communicator included (the multi-rank code path at world 1).
  bool distributed() const { return world > 1 || comm != nullptr || comm_failed || host_reduce != nullptr; }
};

namespace miba {
mi_ba_status context_create(const mi_ba_options* o, const mi_ba_problem* p, const mi_ba_semantic* sem,
                            mi_ba_context** out);
// As context_create, reusing `old` (may be null) when it lives on the same
// device: its stream, rocBLAS handles, Cholesky workspace, pinned scalars and
// device arrays (re-sized in place when large enough) carry over, the problem
// state is replaced.  On failure `old` is destroyed and *out is null.
mi_ba_status context_recycle(mi_ba_context* old, const mi_ba_options* o, const mi_ba_problem* p,
                             const mi_ba_semantic* sem, mi_ba_context** out, const mi_ba_gsba* gsba = nullptr);
void context_destroy(mi_ba_context* ctx);
mi_ba_status context_linearize(mi_ba_context* ctx, double* cost_out);
mi_ba_status context_solve(mi_ba_context* ctx, mi_ba_summary* sum);
mi_ba_status context_writeback(mi_ba_context* ctx);
void timer_begin(mi_ba_context* ctx, const char* name, hipEvent_t* stop_out);
void timer_end(mi_ba_context* ctx, hipEvent_t stop);
// As timer_begin, starting at an already recorded event (the previous
// measurement's stop): one event record fewer between back-to-back phases.
void timer_begin_after(mi_ba_context* ctx, const char* name, hipEvent_t start, hipEvent_t* stop_out);
}  // namespace miba
