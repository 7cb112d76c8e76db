// cholesky.h — dense Cholesky of the reduced camera system (product code).
//
// The exact Schur path factors S (nf x nf f64, column-major lower) every LM
// iteration.  rocSOLVER's dpotrf runs ~10 TF/s and dpotrs ~0.1 s at
// nf = 12 000 (measured on MI355X), while rocBLAS' MFMA dgemm/dsyrk run
// 40-65 TF/s.  Two factorisations are provided, both with all their work in
// rocBLAS level-3 calls and dpotrf only on small diagonal blocks:
//   panel == 0: recursive left/right split (half the flops in dtrsm);
//   panel  > 0: right-looking blocked with panel width `panel` (dtrsm on the
//               panel only, the trailing update as dsyrk, or as dgemm on
//               block columns of the lower triangle when `gemm_update`).
// The solve recurses the same way (dtrsv leaves + dgemv).
#pragma once

#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <vector>

namespace miba {

// Default: right-looking, 512-wide panels, dgemm trailing update (48 ms vs
// 62 ms for the recursive split at nf = 12 000 on MI355X; profiles/r1/
// chol_variants.txt).
struct CholConfig {
  int panel = 512;        // 0: recursive split; > 0: right-looking panel width
  // non-uniform panel schedule (chol_panel_starts): panels of head_panel
  // columns while the panel starts before column head_cols, of tail_panel
  // columns once at most tail_cols columns remain; 0 = off
  int head_panel = 0, head_cols = 0;
  int tail_panel = 0, tail_cols = 0;
  // look-ahead side stream confined to this many CUs (spread over the chip)
  // so the panel factor's waiting workgroups leave the rest to the trailing
  // dgemm; 0: all CUs at high priority (tools build: cholesky_panel_cus)
  int side_cus = 0;
  // split head: while the panel starts before column split_cols, the
  // look-ahead's panel factor runs on split_cus CUs (spread over the chip) and
  // the trailing dgemm on the complement, so the panel's resident workgroups
  // (76 KB LDS, 342 VGPRs per lane) do not halve the dgemm's occupancy on the
  // CUs they share; 0 = off
  int split_cus = 0, split_cols = 0;
  // split tail (own_diag 6, look-ahead): for the panels starting within the
  // last split_tail_cols columns, the next panel's block column is updated in
  // two dgemms — its diagonal block's rows first, so the diagonal-block rows of
  // the panel factor start on the side stream, the rows below second — and the
  // panel's below-diagonal rows run as a second launch on a second side stream
  // once they are updated; factor_blocked makes the same two dgemms (bitwise
  // equal factors); 0 = off.  Tools build: measured slower, the second side
  // stream takes a fourth hardware queue (profiles/r5ag_ab_cholesky_split_tail.jsonl)
  int split_tail_cols = 0;
  // serial head (tools build): the panels starting before serial_head_cols
  // are factored after the previous panel's whole trailing update instead of
  // beside it (the panel's resident workgroups then never share CUs with the
  // dgemm); 0 = off
  int serial_head_cols = 0;
  // split panel: the panels starting before split_panel_cols are factored in
  // two launches on the look-ahead side stream — the diagonal block's row
  // tiles (the serial chain of 64x64 tile factors: kb / 64 workgroups), then,
  // with every flag already set, the rows below it — so that while the chain
  // runs only kb / 64 CUs are held instead of one per row tile of the panel
  // (the trailing dgemm beside it gets the others).  0: one launch.  Tools
  // build only: slower at every width — Cholesky 14.40 / 14.77-14.93 / 15.76
  // / 16.92 ms splitting the panels before 4096 / 6144 / 8192 / all columns
  // vs 13.95-14.08 ms (profiles/r6c_ab_cholesky_split_panel.jsonl): the
  // panel's latency stays on the critical path, the freed CUs do not make
  // the dgemm beside it faster by as much
  int split_panel_cols = 0;
  // look-ahead dgemm on the side stream: for the panels after the first
  // starting at column >= la_side_from, the next panel's block column is
  // updated on the look-ahead side stream right before the panel factor
  // there (after the previous update's first block-column dgemm, which covers
  // that column), so panel k -> update of k+1 -> panel k+1 chain on one
  // hardware queue without two cross-queue waits per panel, and the update
  // of k+1 no longer queues behind the rest of the previous trailing update;
  // -1 = off (the update on the caller's stream).  Default 0: Cholesky 14.12-
  // 14.31 -> 13.76-13.79 ms in the C4 LM, bitwise equal (from column 2048:
  // 13.75, from 4096: 14.06; profiles/r6l_ab_cholesky_la_side.jsonl)
  int la_side_from = 0;
  // the trailing update's first block column only as wide as the panel after
  // next (the columns the next look-ahead dgemm waits for), the others
  // rest_update-wide; false: all rest_update-wide.  Tools build: within
  // noise (13.67 / 13.77 vs 13.79 / 13.82 ms at C4, bitwise equal,
  // profiles/r6o_ab_cholesky_rest_first_panel.jsonl)
  bool rest_first_panel = false;
  // split tail: the below-rows launch on the second trailing-update stream
  // (rest_streams >= 2; that panel's whole trailing update then on the
  // caller's stream) instead of a fourth stream
  bool split_tail_rest = false;
  // head panel kind: panels starting before column head_own_cols use own_diag
  // head_own (e.g. 2: 64-wide diagonal kernels + rocBLAS dtrsm, no resident
  // spin-waiting workgroups beside the trailing dgemm); 0 = off
  int head_own = 0, head_own_cols = 0;
  // trailing update's block columns (after the next panel's) dealt round-robin
  // over the caller's stream and rest_streams - 1 more (1..4), so one launch's
  // last tiles overlap the next launches' first; 1 = one stream.  Default 2:
  // Cholesky 15.5 -> 14.7-15.1 ms at nf = 11 993; 3 / 4 streams 16.8-20.8 ms
  // (profiles/r4w_ab_cholesky_rest_streams.jsonl, r4x_..._1to4.jsonl)
  int rest_streams = 2;
  // the further update streams created with an all-CU mask (a hardware queue
  // of their own instead of HIP's round-robin share of the process's queues)
  bool rest_cumask = false;
  // the further update streams' priority: 0 normal, 1 the highest (as the
  // look-ahead side stream), 2 the lowest (HIP keeps a queue pool per
  // priority: a low-priority stream never shares the caller's normal-priority
  // hardware queue, whatever other streams the process holds)
  int rest_priority = 0;
  bool gemm_update = true;
  // look-ahead: the trailing update after the next panel's block column,
  // 0 one dgemm per 512-wide block column, 1 one dsyrk, 2 one dgemmt,
  // 3 one dgemm per 1024-wide block column (default: 25.7 -> 25.2 ms at nf =
  // 12 000; dsyrk 38.6 ms, dgemmt 519 ms — profiles/r2_ab_rest_update.jsonl)
  int rest_update = 3;
  // rest_update 4 (tools build, measured slower): the trailing update after
  // the next panel's block column as square batch_tile x batch_tile tiles of
  // the lower triangle, one rocblas_dgemm_batched launch per tile shape
  int batch_tile = 1024;
  // trailing-update dgemm: 0 rocBLAS's default solution, else a Tensile
  // solution index for rocblas_gemm_ex (rocblas_gemm_ex_get_solutions; an
  // index the shape does not accept falls back to the default).  Default: the
  // fastest of the sweep over all 267 solutions of the update's shapes
  // (tools/probes/dgemm_solutions.cpp, profiles/r3_dgemm_solutions.txt: 65-72
  // vs 46-49 TF at M ~ 11 000, N = 512 / 1024, K = 512): Cholesky 17.5 ->
  // 15.8 ms at nf = 12 000 (profiles/r3_ab_gemm_solution.jsonl).
  int gemm_solution = -624952224;
  // panel k+1's diagonal factor + dtrsm on the workspace's side stream under
  // panel k's dgemm (34.6 -> 30.4 ms at nf = 12 000)
  bool lookahead = true;
  // diagonal blocks: hand-written 64-wide sub-panels (eight-wave LDS tile
  // factor + sub-panel solve), 2 blocked by 4 columns per step
  // (diag_panel_blocked_kernel<4>: two barriers per 4 columns; Cholesky 30.7 ->
  // 25.5 ms at nf = 12 000), 3 blocked by 8 (26.7 ms), 1 one column per step
  // (diag_panel_kernel), 0 rocsolver_dpotrf.  (Measured dead ends, DESIGN.md:
  // a four-wave register-resident tile factor with one barrier per pivot ran
  // 80 us per sub-panel vs 69; a fully unrolled one-wave register factor
  // ~300 us, instruction-fetch bound.)
  // 6: one panel_factor_kernel launch per panel for the diagonal block AND the
  // panel's solve below it (no dtrsm; panel <= 512)
  // default 6: 21.5 vs 25.0 ms at nf = 12 000 (profiles/r2_ab_own_diag.jsonl; 16x16-blocked
  // MFMA factor + inverse per diagonal tile, profiles/r2_panel_probe_v3.txt)
  int own_diag = 6;
  // own_diag 6: the diagonal tiles' 64x64 factor + inverse (block columns by
  // register sweeps, pf_chol_inv_fast): 2 pivots by rsq + two Goldschmidt
  // steps (~1 ulp), 1 correctly rounded sqrt + divide.  2: Cholesky 17.3 vs
  // 17.7 ms at nf = 12 000; the previous per-pivot LDS-exchange factor (36 us
  // per tile, 22 ms) is gone (profiles/r3_tile_probe.txt).  3 (default): 2
  // with the diagonal 16x16 inverses' operands loaded ahead of their
  // substitution and the last one overlapped with the inverse's other blocks
  // (bitwise equal to 2; 14.3 vs 15.5 us per tile, profiles/r5x_tile_probe.txt);
  // 4 / 5 the overlap / the loads alone (tools build).
  int tile_factor = 3;
  // own_diag 6: published tiles stored write-through (sc1) and drained before
  // the flag, instead of plain stores + __threadfence()
  bool write_through = true;
  // own_diag 6, panel hand-off waits: 0 every wave polls and acquires, 1 one
  // wave polls and acquires for the workgroup, 2 (default) one wave polls and
  // the handed-off tiles are read by sc1 loads (no acquire), 3 as 2 with the
  // next stage's tiles loaded during the current GEMM (tools build).  Panel alone
  // 320 -> 262 (1) -> 230-245 us (2) at nf = 12 000 (profiles/r5y_*).
  int panel_wait = 2;
  // chol_solve variant 2 / the backward sweep: block results handed over as
  // sc1 stores + relaxed flag, read by sc1 loads (no fences); default
  // (0.82 -> 0.75 ms per solve at C4)
  bool solve_sc1 = true;
  // chol_solve variant: 2 sync-free sweeps (one launch per direction), 1 one
  // launch per 64-wide block column with diagonal-block inverses, 0 recursive
  // rocBLAS dtrsv / dgemv
  int solve = 2;
  // bound of every in-launch flag wait (panel factor, sync-free sweeps):
  // wait_ms of wall-clock time per wait; spin_log2 0 = no polling at all (a
  // wait whose flag is not already set times out at once: the timeout test's
  // hook), any other value = the time bound.  A wait that runs out records
  // kCholErrWait in the workspace's error word (chol_error) instead of
  // returning a silently wrong factor or solution; the solve reports it as a
  // hard error.
  int spin_log2 = 24;
  int wait_ms = 5000;
  // own_diag 6: below-diagonal row tiles per panel workgroup while the rows
  // below the panel number at least panel_group_min_rows (1: one workgroup per
  // row tile throughout).  The resident panel workgroups cost the concurrent
  // trailing dgemm CU time; in the dgemm-bound head the panel has slack.
  int panel_rows_per_group = 1;
  // chol_solve_backward over pairs of 64-row blocks (tools build: measured
  // slower), or per block (trsv_sweep_kernel<false>, the default)
  bool bwd_pairs = false;
  int panel_group_min_rows = 6000;
};

// Error word bits (CholWorkspace::err, read by chol_error).
constexpr unsigned kCholErrWait = 1u;  // a flag wait ran out: the factor / solution is invalid

// Device resources of one factorisation owner (one per mi_ba_context, created
// on the context's device): the look-ahead side stream with its own rocBLAS
// handle, one event pair per panel (no event is re-recorded within a
// factorisation), and a scratch tile per stream for the hand-written diagonal
// factor (the factored 64x64 tile is parked there and copied back by the next
// launch, so no workgroup reads a tile another workgroup is overwriting).
struct CholWorkspace {
  int device = -1;
  hipStream_t side = nullptr;
  rocblas_handle side_h = nullptr;
  std::vector<hipEvent_t> ev;
  std::vector<hipEvent_t> ev_col;  // [panel] the trailing update's first block-column dgemm done (la_side_from)
  int col_rec = -1;                // the panel whose ev_col this factorisation recorded last
  double* scratch = nullptr;  // [2][64*64]: [0] caller's stream, [1] side stream
  double* linv = nullptr;     // [n/64][64*64] inverses of the factor's 64x64 diagonal blocks (chol_solve)
  double* ybuf = nullptr;     // [n] intermediate vector of chol_solve (L y = b)
  unsigned* ctrl = nullptr;   // [2 + n/64] sync-free sweeps: two tickets + per-block solution flags
  unsigned epoch = 0;         // last flag value published (two per chol_solve)
  unsigned* pf_ctrl = nullptr;  // one-launch panel factor: ticket + [16][16] tile flags + second ticket
  double* pf_linv = nullptr;    // [8][64*64] inverses of the panel's diagonal tiles
  unsigned pf_base = 0;         // tickets handed out so far
  unsigned pf_base2 = 0;        // tickets of the below-rows launches (split tail), second counter
  hipStream_t side2 = nullptr;  // split tail: the below-rows launches
  std::vector<hipEvent_t> ev2;  // split tail: [panel][2] below rows updated / factored
  bool ensure_side2(int max_panels, bool stream = true);
  unsigned pf_epoch = 0;        // flag value of the last panel launch
  int tile_factor = 3;          // CholConfig::tile_factor
  bool write_through = false;   // CholConfig::write_through
  int panel_wait = 2;           // CholConfig::panel_wait
  bool solve_sc1 = true;        // CholConfig::solve_sc1
  int linv_rows = 0;
  double* tinv = nullptr;       // own_diag 7: [512*512] inverse of the panel's diagonal block
  double* tbuf = nullptr;       // own_diag 7: [max_n * 512] copy of the panel below it
  int tbuf_rows = 0;
  unsigned* err = nullptr;      // [4] error word (kCholErr* bits) of the in-launch flag waits
  unsigned spin_limit = 0;  // wall-clock ticks per flag wait (CholConfig::wait_ms; 0 = no polling)
  int clock_khz = 0;        // wall-clock rate of the device (hipDeviceAttributeWallClockRate)
  unsigned wait_ticks(int ms) const {
    const uint64_t t = (uint64_t)(ms > 0 ? ms : 1) * (uint64_t)(clock_khz > 0 ? clock_khz : 100000);
    return (unsigned)(t < 0xffffffffull ? t : 0xffffffffull);
  }
  int rows_per_group = 1;          // CholConfig::panel_rows_per_group
  bool bwd_pairs = false;          // CholConfig::bwd_pairs
  int group_min_rows = 6000;       // CholConfig::panel_group_min_rows
  int side_cus = 0;                // CholConfig::side_cus of the current side stream
  bool set_side_cus(int ncu);      // re-create the side stream with that CU mask
  // split head (CholConfig::split_cus): a panel stream on split_cus CUs and a
  // dgemm stream on the others, each with its rocBLAS handle; ev_split orders
  // them against the caller's and the side stream at the regime switches
  hipStream_t split_side = nullptr, split_main = nullptr;
  rocblas_handle split_side_h = nullptr, split_main_h = nullptr;
  hipEvent_t ev_split[4] = {nullptr, nullptr, nullptr, nullptr};
  int split_n = 0;                 // split_cus of the current split streams
  bool set_split_cus(int ncu);
  // CholConfig::rest_streams k > 1: the k - 1 further trailing-update
  // streams with their handles, and per panel a fork event and k - 1 joins
  static constexpr int kMaxRest = 4;
  hipStream_t rest_s[kMaxRest - 1] = {nullptr, nullptr, nullptr};
  rocblas_handle rest_h[kMaxRest - 1] = {nullptr, nullptr, nullptr};
  std::vector<hipEvent_t> ev_rest;  // [panel][kMaxRest]
  int rest_n = 1;
  bool rest_cumask = false;
  int rest_priority = 0;
  bool set_rest_streams(int k, bool cumask = false, int priority = 0);
  // rest_update 4: per panel up to three tile groups (full, bottom row,
  // corner), each A[count], B[count], C[count] pointer arrays at off in bptr
  // (device), made for one (A, n, lda, extra rows, tile, panel schedule)
  struct TileGroup {
    int off, count, m, n;
  };
  std::vector<TileGroup> bgroups;  // [panel][3]
  double** bptr = nullptr;
  size_t bptr_cap = 0;
  std::vector<long long> bkey;

  // Creates the resources on `device` with events for up to `max_panels`
  // panels and diagonal-block inverses for matrices up to max_n; false on any
  // HIP/rocBLAS failure (partially created resources are released by
  // destroy()).
  bool create(int device, int max_panels, int max_n);
  // create() unless the existing resources already cover (device, max_panels, max_n)
  bool ensure(int device, int max_panels, int max_n);
  void destroy();
};

// In-place lower Cholesky of the n x n column-major matrix A (leading
// dimension lda) on h's stream.  info[k] (device, one int per diagonal block,
// count from chol_leaf_count) is 0 for every block of a positive-definite A.
// ws is required for own_diag and for look-ahead; every exit path leaves no
// work of this call pending on the side stream that h's stream does not wait
// for.
// extra_rows > 0 (blocked factorisations only, lda >= n + extra_rows): the
// rows n .. n + extra_rows - 1 below the matrix are carried through the
// factorisation as rows of a trapezoid, so on return they hold B L^-T for the
// B they held on entry — for B = b' the forward solve L y = b (y' in row n)
// comes out of the panel solves and trailing updates at no extra pass.
rocblas_status chol_factor(rocblas_handle h, int n, double* A, int lda, int* info, const CholConfig& cfg,
                           CholWorkspace* ws, int extra_rows = 0);
int chol_leaf_count(int n, const CholConfig& cfg = {});
// First column of every panel of the right-looking factorisation, then n.
std::vector<int> chol_panel_starts(int n, const CholConfig& cfg);
// x := (L L')^-1 x with the factor chol_factor left in A, on h's stream.
// variant 2 (default): sync-free forward / backward sweeps, one launch each
// (per-block solution flags in ws); 1: one launch per 64-wide block column,
// diagonal blocks by their inverses in ws; 0: recursive rocBLAS dtrsv + dgemv
// (ws unused).
rocblas_status chol_solve(rocblas_handle h, int n, const double* A, int lda, double* x, int variant,
                          CholWorkspace* ws);
// x := L'^-1 x (the backward sweep of chol_solve variant 2 alone), after a
// factorisation whose extra row delivered the forward solve.
rocblas_status chol_solve_backward(rocblas_handle h, int n, const double* A, int lda, double* x, CholWorkspace* ws);
// Error word of the factorisations / solves issued on stream s since the last
// call (synchronises s, then clears the word): 0, or kCholErr* bits.  A
// nonzero word means a result of those calls is invalid; callers report it
// as MI_BA_ERR_HIP.  *word = 0 without a workspace.
hipError_t chol_error(CholWorkspace* ws, hipStream_t s, unsigned* word);

}  // namespace miba
