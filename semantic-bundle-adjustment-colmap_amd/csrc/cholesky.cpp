// cholesky.cpp — recursive blocked Cholesky over rocBLAS/rocSOLVER (see cholesky.h).
#define ROCBLAS_BETA_FEATURES_API  // rocblas_gemm_ex_get_solutions
#include "cholesky.h"

#include <hip/hip_runtime.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <atomic>
#include <vector>
#include <array>
#include <map>
#include <mutex>

namespace miba {

namespace {


// ---------------------------------------------------------------------------
// Diagonal-block factor (replaces rocsolver_dpotrf on the panel's diagonal
// block: 1.2 ms per 512-block there, 29 of the 48 ms of an nf = 12 000
// factorisation — profiles/r1/chol_breakdown.txt).  Right-looking over
// 64-wide sub-panels, two launches per sub-panel:
//   diag_panel_kernel:  every workgroup (kPanelWaves waves) factors the 64x64 tile in
//     LDS (lane = row, column-major tile, the pivot column broadcast from a
//     separate LDS vector), workgroup 0
//     writes it back, workgroups 1.. solve 64 rows each of the sub-panel
//     below it (x L' = a, lane = row, L read as LDS broadcasts);
//   diag_update_kernel: the trailing lower triangle of the block, A22 -= P P',
//     one 64x64 tile per 256-thread workgroup, K staged through LDS.
// Widths below 64 are padded with an identity (pivots 1, zero couplings).
constexpr int kSub = 64;
constexpr int kPanelWaves = 8;  // waves per diag_panel_kernel workgroup

__global__ __launch_bounds__(64 * kPanelWaves) void diag_panel_kernel(double* __restrict__ A, int lda, int w, int mrows,
                                                         int* __restrict__ info, double* __restrict__ scratch,
                                                         int koff) {
  // Column-major tiles in LDS, element (r, c) at [c * 64 + r]: lane r's
  // accesses are consecutive across a wave, L[c][j] reads are broadcasts.
  // kPanelWaves waves share the 64 rows: each takes every kPanelWaves-th
  // column of the rank-1 updates (factor) and of the right-looking updates
  // (solve).
  __shared__ double L[kSub * kSub], P[kSub * kSub], col[kSub];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // Loads are unconditional at clamped (in-range) addresses and selected
  // afterwards, so the unrolled loops issue them back to back.
  const double* tile_row = A + std::min(lane, w - 1);
#pragma unroll
  for (int c = wv; c < kSub; c += kPanelWaves) {
    const double v = tile_row[(size_t)std::min(c, w - 1) * lda];
    L[c * kSub + lane] = (lane < w && c < w) ? (lane >= c ? v : 0.0) : (lane == c ? 1.0 : 0.0);
  }
  const int r = (blockIdx.x - 1) * kSub + lane;  // row of the sub-panel below the tile (blocks >= 1)
  const bool solve = blockIdx.x > 0 && r < mrows;
  double* row = A + w + r;  // A points at the tile; the sub-panel rows start w below it
  if (blockIdx.x > 0) {
    const double* src = A + w + std::min(r, mrows - 1);
#pragma unroll
    for (int c = wv; c < kSub; c += kPanelWaves) {
      const double v = src[(size_t)std::min(c, w - 1) * lda];
      P[c * kSub + lane] = (solve && c < w) ? v : 0.0;
    }
  }
  __syncthreads();
  int bad = 0;
  for (int j = 0; j < kSub; ++j) {
    const double d = L[j * kSub + j];
    if (!(d > 0.0) && bad == 0) bad = j + 1;
    const double sd = sqrt(d);
    const double l = lane > j ? L[j * kSub + lane] / sd : (lane == j ? sd : 0.0);
    if (wv == 0) col[lane] = l;  // separate array: the update's broadcast loads cannot alias its stores
    __syncthreads();
    // column j in place only after every wave has read it (before the barrier)
    if (wv == 0 && lane >= j) L[j * kSub + lane] = l;
    // branch-free: entries above the diagonal (c > lane) take garbage, never read
#pragma unroll 2
    for (int c = j + 1 + wv; c < kSub; c += kPanelWaves) L[c * kSub + lane] -= l * col[c];
    __syncthreads();
  }
  if (blockIdx.x == 0) {
    // the factored tile goes to scratch, not over A: the other workgroups of
    // this launch may not have loaded the tile yet (diag_update_kernel's last
    // workgroup copies it back)
#pragma unroll
    for (int c = wv; c < kSub; c += kPanelWaves) scratch[c * kSub + lane] = L[c * kSub + lane];
    // first failing pivot of the block, 1-based (earlier sub-panels' launches
    // have completed; later ones see it set and keep it)
    if (threadIdx.x == 0 && bad != 0 && bad <= w && info[0] == 0) info[0] = koff + bad;
    return;
  }
  // x L' = a, right-looking over the columns of the lane's row; column c's
  // result leaves from the wave that owns it (P[c] is never written again)
  for (int c = 0; c < kSub; ++c) {
    const double x = P[c * kSub + lane] / L[c * kSub + c];
    if (solve && c < w && c % kPanelWaves == wv) row[(size_t)c * lda] = x;
#pragma unroll 2
    for (int t = c + 1 + wv; t < kSub; t += kPanelWaves) P[t * kSub + lane] -= x * L[c * kSub + t];
    __syncthreads();
  }
}

// As diag_panel_kernel, blocked by kStep columns: per step the kStep x kStep
// diagonal block is factored redundantly by every lane (registers), each lane
// forms its row's kStep new entries, and the trailing columns take one
// rank-kStep update — two barriers per kStep columns instead of two per
// column.  The sub-panel solve (x L' = a) steps the same way: each lane forms
// its row's kStep unknowns from the diagonal block, one barrier per step.
template <int kStep, int NW = kPanelWaves>
__global__ __launch_bounds__(64 * NW) void diag_panel_blocked_kernel(double* __restrict__ A, int lda, int w,
                                                                 int mrows, int* __restrict__ info,
                                                                 double* __restrict__ scratch, int koff) {
  __shared__ double L[kSub * kSub], P[kSub * kSub], nb[kStep * kSub];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const double* tile_row = A + std::min(lane, w - 1);
#pragma unroll
  for (int c = wv; c < kSub; c += NW) {
    const double v = tile_row[(size_t)std::min(c, w - 1) * lda];
    L[c * kSub + lane] = (lane < w && c < w) ? (lane >= c ? v : 0.0) : (lane == c ? 1.0 : 0.0);
  }
  const int r = (blockIdx.x - 1) * kSub + lane;
  const bool solve = blockIdx.x > 0 && r < mrows;
  double* row = A + w + r;
  if (blockIdx.x > 0) {
    const double* src = A + w + std::min(r, mrows - 1);
#pragma unroll
    for (int c = wv; c < kSub; c += NW) {
      const double v = src[(size_t)std::min(c, w - 1) * lda];
      P[c * kSub + lane] = (solve && c < w) ? v : 0.0;
    }
  }
  __syncthreads();
  int bad = 0;
  for (int jb = 0; jb < kSub; jb += kStep) {
    // kStep x kStep diagonal block (lower), factored in registers by every lane
    double d[kStep][kStep];
#pragma unroll
    for (int i = 0; i < kStep; ++i)
#pragma unroll
      for (int k = 0; k <= i; ++k) d[i][k] = L[(jb + k) * kSub + jb + i];
#pragma unroll
    for (int k = 0; k < kStep; ++k) {
      const double piv = d[k][k];
      if (!(piv > 0.0) && bad == 0) bad = jb + k + 1;
      d[k][k] = sqrt(piv);
#pragma unroll
      for (int i = k + 1; i < kStep; ++i) d[i][k] /= d[k][k];
#pragma unroll
      for (int i = k + 1; i < kStep; ++i)
#pragma unroll
        for (int m = k + 1; m <= i; ++m) d[i][m] -= d[i][k] * d[m][k];
    }
    // this lane's row of the kStep new columns
    double y[kStep];
    if (lane >= jb + kStep) {
#pragma unroll
      for (int k = 0; k < kStep; ++k) {
        double v = L[(jb + k) * kSub + lane];
#pragma unroll
        for (int m = 0; m < k; ++m) v -= y[m] * d[k][m];
        y[k] = v / d[k][k];
      }
    } else {
      const int i = lane - jb;
#pragma unroll
      for (int k = 0; k < kStep; ++k) {
        double v = 0.0;
#pragma unroll
        for (int ii = k; ii < kStep; ++ii) v = (i == ii) ? d[ii][k] : v;
        y[k] = v;
      }
    }
    if (wv == 0) {
#pragma unroll
      for (int k = 0; k < kStep; ++k) nb[k * kSub + lane] = y[k];
    }
    __syncthreads();
    // every wave has read the block's old columns: store them final, and the
    // trailing columns take the rank-kStep update
    if (wv == 0) {
#pragma unroll
      for (int k = 0; k < kStep; ++k)
        if (lane >= jb + k) L[(jb + k) * kSub + lane] = y[k];
    }
    for (int c = jb + kStep + wv; c < kSub; c += NW) {
      double v = L[c * kSub + lane];
#pragma unroll
      for (int k = 0; k < kStep; ++k) v -= y[k] * nb[k * kSub + c];
      L[c * kSub + lane] = v;
    }
    __syncthreads();
  }
  if (blockIdx.x == 0) {
#pragma unroll
    for (int c = wv; c < kSub; c += NW) scratch[c * kSub + lane] = L[c * kSub + lane];
    if (threadIdx.x == 0 && bad != 0 && bad <= w && info[0] == 0) info[0] = koff + bad;
    return;
  }
  // x L' = a, kStep unknowns per step: the lane's row from the diagonal block
  // (broadcast reads), then the trailing columns of the row (waves by column)
  for (int cb = 0; cb < kSub; cb += kStep) {
    double x[kStep];
#pragma unroll
    for (int k = 0; k < kStep; ++k) {
      double v = P[(cb + k) * kSub + lane];
#pragma unroll
      for (int m = 0; m < k; ++m) v -= x[m] * L[(cb + m) * kSub + cb + k];
      x[k] = v / L[(cb + k) * kSub + cb + k];
    }
#pragma unroll
    for (int k = 0; k < kStep; ++k)
      if (solve && cb + k < w && (cb + k) % NW == wv) row[(size_t)(cb + k) * lda] = x[k];
    for (int t = cb + kStep + wv; t < kSub; t += NW) {
      double v = P[t * kSub + lane];
#pragma unroll
      for (int k = 0; k < kStep; ++k) v -= x[k] * L[(cb + k) * kSub + t];
      P[t * kSub + lane] = v;
    }
    __syncthreads();
  }
}

// A22 (m x m, lower) -= P P', P = the m x w sub-panel left of A22 (column-
// major, P[r + t*lda] = A22[r - w*lda ...]); tile (bi >= bj) per workgroup.
// The workgroup after the last tile copies the factored w x w diagonal tile
// from the scratch diag_panel_kernel parked it in back to `tile` (nothing in
// this launch reads the tile).
__global__ __launch_bounds__(256) void diag_update_kernel(double* __restrict__ A22, const double* __restrict__ P,
                                                          int lda, int m, int w, const double* __restrict__ scratch,
                                                          double* __restrict__ tile) {
  __shared__ double sr[kSub * 33], sc[kSub * 33];
  const int ntiles = ((m + kSub - 1) / kSub) * ((m + kSub - 1) / kSub + 1) / 2;
  if ((int)blockIdx.x == ntiles) {
    for (int e = threadIdx.x; e < kSub * kSub; e += 256) {
      const int r = e & (kSub - 1), c = e / kSub;
      if (r < w && c < w && r >= c) tile[r + (size_t)c * lda] = scratch[e];
    }
    return;
  }
  // lower-triangle tile index -> (bi, bj), bi >= bj
  int t = blockIdx.x, bi = 0;
  while (t > bi) { t -= bi + 1; ++bi; }
  const int bj = t;
  const int r0 = bi * kSub, c0 = bj * kSub;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  double acc[4][4] = {};
  for (int k0 = 0; k0 < w; k0 += 32) {
#pragma unroll
    for (int e = threadIdx.x; e < kSub * 32; e += 256) {
      const int rr = e & 63, kk = e >> 6;
      const int k = k0 + kk;
      const size_t kc = (size_t)std::min(k, w - 1) * lda;  // clamped: loads issue back to back
      const double vr = P[std::min(r0 + rr, m - 1) + kc], vc = P[std::min(c0 + rr, m - 1) + kc];
      sr[rr * 33 + kk] = (r0 + rr < m && k < w) ? vr : 0.0;
      sc[rr * 33 + kk] = (c0 + rr < m && k < w) ? vc : 0.0;
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < 32; ++kk) {
      double x[4], y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = sr[(ty + 16 * i) * 33 + kk];
#pragma unroll
      for (int j = 0; j < 4; ++j) y[j] = sc[(tx + 16 * j) * 33 + kk];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += x[i] * y[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + ty + 16 * i, c = c0 + tx + 16 * j;
      if (r < m && c < m && r >= c) A22[r + (size_t)c * lda] -= acc[i][j];
    }
}

// ---------------------------------------------------------------------------
// Triangular solves L y = b, L' x = y (replace the recursive rocBLAS dtrsv +
// dgemv solve: 134 us dtrsv leaves, ~5.9 ms per solve at nf = 12 000, ~0.2
// TB/s).  The inverses of the 64x64 diagonal blocks are formed once per
// factor (rocblas_dtrtri_strided_batched, into the workspace), so a block's
// solve is a 64x64 mat-vec with no serial dependence.  One launch per block
// column, stepping down (forward) or up (backward); one wave per workgroup,
// 64 rows (forward) / columns (backward) each, so a step spreads over up to
// nf / 64 CUs.  Every workgroup first issues the loads of its share of the
// block column, then forms the block's solution redundantly from L2 (inverse
// block + right-hand side), then applies it to its rows / columns.
// Workgroup 0 publishes the block's solution into the other vector of the
// pair (x -> workspace y on the way down, y -> x on the way up), never into
// the one the launch's workgroups read.  L is read once per direction.
constexpr int kTB = 64;         // block column of the solves (= one wave)

// Linv_kk (col-major 64 x 64, lower) -> T[c * 65 + r]; loads clamped and
// issued back to back, 16 columns per batch.  (An LDS-DMA copy of the block,
// global_load_lds 16 B per lane, measured slower: 7.4 / 8.7 us per step vs
// 6.7 / 7.8.)
__device__ __forceinline__ void load_inv_block(const double* __restrict__ Li, int w, double* T) {
  const int r = threadIdx.x;
  const double* src = Li + min(r, w - 1);
#pragma unroll
  for (int c0 = 0; c0 < kTB; c0 += 16) {
    double v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = src[min(c0 + m, w - 1) * kTB];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int c = c0 + m;
      T[c * (kTB + 1) + r] = (r < w && c < w && r >= c) ? v[m] : 0.0;
    }
  }
}

__global__ __launch_bounds__(kTB) void trsv_fwd_step_kernel(const double* __restrict__ L, int lda, int n, int k0,
                                                            const double* __restrict__ Li, double* __restrict__ x,
                                                            double* __restrict__ yout) {
  __shared__ double T[kTB * (kTB + 1)];
  __shared__ double xs[kTB];
  const int w = min(kTB, n - k0);
  const int lane = threadIdx.x;
  const int r = k0 + w + blockIdx.x * kTB + lane;  // row updated by this lane
  const bool live = r < n;
  const double* Lr = L + (size_t)(live ? r : n - 1) + (size_t)k0 * lda;
  double v[kTB];
#pragma unroll
  for (int c = 0; c < kTB; ++c) v[c] = Lr[(size_t)min(c, w - 1) * lda];
  xs[lane] = lane < w ? x[k0 + lane] : 0.0;
  load_inv_block(Li, w, T);
  __syncthreads();
  // y = Linv_kk x_k: lane = row of the block
  double y = 0.0;
#pragma unroll 16
  for (int c = 0; c < kTB; ++c) y += T[c * (kTB + 1) + lane] * xs[c];
  __syncthreads();
  xs[lane] = lane < w ? y : 0.0;
  // published to a separate vector: other workgroups of this launch may still
  // be reading the block's right-hand side from x
  if (blockIdx.x == 0 && lane < w) yout[k0 + lane] = y;
  __syncthreads();
  if (live) {
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < kTB; ++c) acc += v[c] * xs[c];
    x[r] -= acc;
  }
}

__global__ __launch_bounds__(kTB) void trsv_bwd_step_kernel(const double* __restrict__ L, int lda, int n, int k0,
                                                            const double* __restrict__ Li, double* __restrict__ y,
                                                            double* __restrict__ xout) {
  __shared__ double T[kTB * (kTB + 1)];
  __shared__ double ys[kTB];
  const int w = min(kTB, n - k0);
  const int lane = threadIdx.x;
  const int c = blockIdx.x * kTB + lane;  // column (of L, row of L') updated by this lane
  const bool live = c < k0;
  // L[k0 .. k0 + w, c]: 64 contiguous doubles of column c
  double v[kTB];
  const bool vec = ((k0 & 1) == 0) && ((lda & 1) == 0) && w == kTB;
  if (vec) {
    const double2* Lc = reinterpret_cast<const double2*>(L + (size_t)k0 + (size_t)(live ? c : 0) * lda);
#pragma unroll
    for (int t = 0; t < kTB / 2; ++t) {
      const double2 p = Lc[t];
      v[2 * t] = p.x;
      v[2 * t + 1] = p.y;
    }
  } else {
    const double* Ls = L + (size_t)k0 + (size_t)(live ? c : 0) * lda;
#pragma unroll
    for (int t = 0; t < kTB; ++t) v[t] = Ls[min(t, w - 1)];
  }
  ys[lane] = lane < w ? y[k0 + lane] : 0.0;
  load_inv_block(Li, w, T);
  __syncthreads();
  // x_k = Linv_kk' y_k: lane = row of the block, Linv[t][lane] at T[lane * 65 + t]
  double xk = 0.0;
#pragma unroll 16
  for (int t = 0; t < kTB; ++t) xk += T[lane * (kTB + 1) + t] * ys[t];
  __syncthreads();
  ys[lane] = lane < w ? xk : 0.0;
  if (blockIdx.x == 0 && lane < w) xout[k0 + lane] = xk;
  __syncthreads();
  if (live) {
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < kTB; ++t) acc += v[t] * ys[t];
    y[c] -= acc;
  }
}

// ---------------------------------------------------------------------------
// Sync-free triangular sweeps (chol_solve variant 2): ONE launch per
// direction instead of one per 64-wide block column.  Workgroup t takes row
// block ib (forward: ib = t, backward: ib = nblk-1-t; t from an atomic
// ticket, so a block's producers always started before it and the spin-waits
// below cannot deadlock whatever the dispatch order).  Its waves stream the
// blocks it depends on round-robin — each wave first loads its 64x64 block of
// L into registers, then waits for that block's solution flag, then folds the
// block in — so L is read once per direction, off the critical path.  Wave 0
// then solves the diagonal block by a 64-step register sweep (pivots as
// precomputed reciprocals, the solved entry broadcast with readlane), writes
// the block's solution in place, and publishes it (release fence, flag =
// epoch).  The critical path per block is one flag hand-off + one 64x64
// register solve, with no kernel boundary and no diagonal-block inverses.
//   forward  L y = b: lane = row of the block, dependency blocks L[ib][jb < ib]
//   backward L'x = y: lane = column of the block, dependency blocks L[jb > ib][ib]
// ctrl = {forward ticket, backward ticket, flag[nblk]}.
// Bounded in-launch flag wait (sync-free sweeps, one-launch panel factor).
// The poll is a relaxed (coherent, sc1) load and the acquire fence runs once
// after the flag is seen: an acquire load in the loop would issue an
// agent-scope cache invalidate (buffer_inv sc1) per poll, from every waiting
// workgroup, flushing the XCD's cached tiles under the concurrent trailing
// dgemm.  Bounded by elapsed time, `limit` ticks of the constant-rate wall
// clock (CholWorkspace::wait_ticks, from CholConfig::wait_ms; a poll count
// would drift with the shader clock): a lost flag must not leave waves that
// never finish, and a producer held up for a while (a time-shared GPU, the
// CU-masked side stream) must not fail a factorisation that would complete.
// limit 0 is the no-polling test hook.  A wait that runs out — or that sees
// (every 256 polls) that another wait of the call already ran out, so a broken
// chain drains fast — sets kCholErrWait in the error word and returns; the
// host reads the word (chol_error) and reports the factor / solution invalid
// (a hard error: the solve ends with MI_BA_ERR_HIP) instead of using it.
__device__ __forceinline__ void flag_wait(const unsigned* f, unsigned epoch, unsigned* err, unsigned limit) {
  if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
    const uint64_t t0 = wall_clock64();
    for (unsigned spin = 0;; ++spin) {
      if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) break;
      if (limit == 0u || ((spin & 15u) == 15u && wall_clock64() - t0 >= limit) ||
          ((spin & 255u) == 255u && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
        __hip_atomic_fetch_or(err, kCholErrWait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// Resident workgroups per CU the runtime admits for kern (-1 if unknown): the
// sc1 hand-offs without an acquire are used only where this is 1.
static int blocks_per_cu(const void* kern, int threads) {
  int nb = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, threads, 0) == hipSuccess ? nb : -1;
}

// flag_wait without the acquire: for consumers whose every load of the
// handed-off bytes is an sc1 load of bytes the producer stored sc1 and
// drained before the flag (MI355X_MICROARCH.md §visibility, table row 1)
__device__ __forceinline__ void flag_poll(const unsigned* f, unsigned epoch, unsigned* err, unsigned limit) {
  if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) return;
  const uint64_t t0 = wall_clock64();
  for (unsigned spin = 0;; ++spin) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) return;
    if (limit == 0u || ((spin & 15u) == 15u && wall_clock64() - t0 >= limit) ||
        ((spin & 255u) == 255u && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
      __hip_atomic_fetch_or(err, kCholErrWait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// 8-byte global sc1 load / store (relaxed agent-scope atomics on the global
// address space: global_load/store_dwordx2 sc1)
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(
      (const __attribute__((address_space(1))) unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((__attribute__((address_space(1))) unsigned long long*)p,
                     (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kSweepWaves = 4;
typedef double sweep_dvec2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// SC1: the block results x handed over as sc1 stores drained before a
// relaxed flag, read by sc1 loads after a relaxed poll (no release /
// acquire fences); one workgroup per CU (its u / v registers)
template <bool FWD, bool SC1 = false>
__global__ __launch_bounds__(64 * kSweepWaves) void trsv_sweep_kernel(const double* __restrict__ L, int lda, int n,
                                                                      double* x, unsigned* ctrl, unsigned epoch,
                                                                      unsigned* err, unsigned limit) {
  __shared__ int s_blk;
  __shared__ double part[kSweepWaves][kTB];
  __shared__ double xs[kSweepWaves][kTB];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nblk = (n + kTB - 1) / kTB;
  if (threadIdx.x == 0) s_blk = (int)atomicAdd(ctrl + (FWD ? 0 : 1), 1u);
  __syncthreads();
  const int t = s_blk;
  const int ib = FWD ? t : nblk - 1 - t;
  const int r0 = ib * kTB, w = min(kTB, n - r0);
  unsigned* flag = ctrl + 2;
  const int me = r0 + min(lane, w - 1);  // the lane's row (forward) / column (backward), clamped
  // wave 0: the diagonal block, the pivot reciprocal and the right-hand side
  // are loaded before any waiting (nothing else writes them)
  double u[kTB];
  double dinv = 0.0, z = 0.0;
  if (wv == 0) {
    if (FWD) {
      const double* src = L + me + (size_t)r0 * lda;
#pragma unroll
      for (int c = 0; c < kTB; ++c) u[c] = src[(size_t)min(c, w - 1) * lda];
    } else {
      const double* src = L + r0 + (size_t)me * lda;
#pragma unroll
      for (int r = 0; r < kTB; ++r) u[r] = src[min(r, w - 1)];
    }
    dinv = 1.0 / L[(size_t)me * (lda + 1)];
    z = lane < w ? x[r0 + lane] : 0.0;
  }
  double acc = 0.0;
  const int ndep = FWD ? ib : nblk - 1 - ib;
  for (int q = wv; q < ndep; q += kSweepWaves) {
    const int jb = FWD ? q : nblk - 1 - q;
    const int c0 = jb * kTB, wj = min(kTB, n - c0);
    double v[kTB];
    if (FWD) {
      // row me, columns c0 .. c0+63 (a block left of ib is full width)
      const double* src = L + me + (size_t)c0 * lda;
#pragma unroll
      for (int c = 0; c < kTB; ++c) v[c] = __builtin_nontemporal_load(src + (size_t)c * lda);
    } else {
      // column me, rows c0 .. c0+wj-1 (contiguous)
      const double* src = L + c0 + (size_t)me * lda;
      if (wj == kTB && ((c0 | lda) & 1) == 0) {
        const sweep_dvec2* s2 = reinterpret_cast<const sweep_dvec2*>(src);
#pragma unroll
        for (int r = 0; r < kTB / 2; ++r) {
          const sweep_dvec2 p = __builtin_nontemporal_load(s2 + r);
          v[2 * r] = p.x;
          v[2 * r + 1] = p.y;
        }
      } else {
#pragma unroll
        for (int r = 0; r < kTB; ++r) v[r] = src[min(r, wj - 1)];
      }
    }
    if (SC1) {
      flag_poll(flag + jb, epoch, err, limit);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the poll
      xs[wv][lane] = lane < wj ? ld_sc1(x + c0 + lane) : 0.0;
    } else {
      flag_wait(flag + jb, epoch, err, limit);
      xs[wv][lane] = lane < wj ? x[c0 + lane] : 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
    for (int c = 0; c < kTB; ++c) acc += v[c] * xs[wv][c];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  part[wv][lane] = acc;
  __syncthreads();
  if (wv != 0) return;
#pragma unroll
  for (int k = 0; k < kSweepWaves; ++k) z -= part[k][lane];
  if (lane >= w) z = 0.0;
  // straight-line: past a ragged block's width z is 0 and u, dinv are finite
  // (clamped loads), so those steps leave every live lane unchanged
  if (FWD) {
#pragma unroll
    for (int c = 0; c < kTB; ++c) {
      const double xc = readlane_f64(z, c) * readlane_f64(dinv, c);
      const double zu = z - u[c] * xc;
      z = lane == c ? xc : (lane > c ? zu : z);
    }
  } else {
#pragma unroll
    for (int r = kTB - 1; r >= 0; --r) {
      const double xr = readlane_f64(z, r) * readlane_f64(dinv, r);
      const double zu = z - u[r] * xr;
      z = lane == r ? xr : (lane < r ? zu : z);
    }
  }
  if (SC1) {
    if (lane < w) st_sc1(x + r0 + lane, z);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(flag + ib, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (lane < w) x[r0 + lane] = z;
  __threadfence();
  if (lane == 0) __hip_atomic_store(flag + ib, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// The sweeps' sc1 hand-offs (no fences) only where one workgroup per CU is
// resident (their registers give one; MI355X_MICROARCH.md §visibility).
static bool sweep_sc1_ok() {
  static const bool ok =
      blocks_per_cu(reinterpret_cast<const void*>(&trsv_sweep_kernel<true, true>), 64 * kSweepWaves) == 1 &&
      blocks_per_cu(reinterpret_cast<const void*>(&trsv_sweep_kernel<false, true>), 64 * kSweepWaves) == 1;
  return ok;
}

#ifdef MI_BA_AB_VARIANTS
// Tools build (cholesky_bwd_pairs 1): measured slower, 1.50 vs 0.83 ms at
// nf = 12 000 — with two waves per block each wave streams twice the
// dependency blocks, and the streaming, not the hand-off, then paces the
// deep blocks (profiles/r3_ab_bwd_pairs_schur_xcd.jsonl).
// Backward sweep L'x = y over PAIRS of 64-row blocks (hi, lo = hi - 1): one
// flag hand-off per 128 rows instead of per 64.  Waves 0-1 fold the
// dependencies jb > hi into block hi, waves 2-3 the same jb into block lo;
// wave 0 solves hi, wave 3 folds the local block L[hi][lo]' x_hi, wave 2
// solves lo; both blocks are published under one epoch.  Same arithmetic per
// block as trsv_sweep_kernel<false> except the order in which the dependency
// products are summed (a ragged top block pairs with nothing).
__global__ __launch_bounds__(256) void trsv_bwd_pair_kernel(const double* __restrict__ L, int lda, int n, double* x,
                                                            unsigned* ctrl, unsigned epoch, unsigned* err,
                                                            unsigned limit) {
  __shared__ int s_t;
  __shared__ double part[4][kTB];
  __shared__ double xs[4][kTB];
  __shared__ double xhi[kTB];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nblk = (n + kTB - 1) / kTB;
  if (threadIdx.x == 0) s_t = (int)atomicAdd(ctrl + 1, 1u);
  __syncthreads();
  const int hi = nblk - 1 - 2 * s_t, lo = hi - 1;
  unsigned* flag = ctrl + 2;
  const bool mine_hi = wv < 2;
  const int rb = mine_hi ? hi : lo;  // the block whose column this wave reads
  if (rb < 0) {                      // hi == 0: no lo block; its waves only join the barriers
    __syncthreads();
    __syncthreads();
    __syncthreads();
    __syncthreads();
    return;
  }
  const int r0 = rb * kTB, w = min(kTB, n - r0);
  const int me = r0 + min(lane, w - 1);  // the lane's column, clamped
  double acc = 0.0;
  const int ndep = nblk - 1 - hi;  // blocks jb > hi
  for (int q = (wv & 1); q < ndep; q += 2) {
    const int jb = nblk - 1 - q;
    const int c0 = jb * kTB, wj = min(kTB, n - c0);
    double v[kTB];
    const double* src = L + c0 + (size_t)me * lda;
    if (wj == kTB && ((c0 | lda) & 1) == 0) {
      const sweep_dvec2* s2 = reinterpret_cast<const sweep_dvec2*>(src);
#pragma unroll
      for (int r = 0; r < kTB / 2; ++r) {
        const sweep_dvec2 pv = __builtin_nontemporal_load(s2 + r);
        v[2 * r] = pv.x;
        v[2 * r + 1] = pv.y;
      }
    } else {
#pragma unroll
      for (int r = 0; r < kTB; ++r) v[r] = src[min(r, wj - 1)];
    }
    flag_wait(flag + jb, epoch, err, limit);
    xs[wv][lane] = lane < wj ? x[c0 + lane] : 0.0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
    for (int c = 0; c < kTB; ++c) acc += v[c] * xs[wv][c];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  part[wv][lane] = acc;
  // wave 0: block hi's diagonal; wave 3: the local block L[hi][lo] (column
  // me of lo, rows of hi: contiguous); wave 2: block lo's diagonal
  double u[kTB];
  double dinv = 0.0;
  if (wv == 0 || wv == 2) {
    const double* src = L + r0 + (size_t)me * lda;
#pragma unroll
    for (int r = 0; r < kTB; ++r) u[r] = src[min(r, w - 1)];
    dinv = 1.0 / L[(size_t)me * (lda + 1)];
  } else if (wv == 3) {
    const int h0 = hi * kTB, wh = min(kTB, n - h0);
    const double* src = L + h0 + (size_t)me * lda;
#pragma unroll
    for (int r = 0; r < kTB; ++r) u[r] = src[min(r, wh - 1)];
  }
  __syncthreads();  // (1) dependency parts
  auto solve = [&](double z) {
    if (lane >= w) z = 0.0;
#pragma unroll
    for (int r = kTB - 1; r >= 0; --r) {
      const double xr = readlane_f64(z, r) * readlane_f64(dinv, r);
      const double zu = z - u[r] * xr;
      z = lane == r ? xr : (lane < r ? zu : z);
    }
    return z;
  };
  if (wv == 0) {
    double z = lane < w ? x[r0 + lane] : 0.0;
    z -= part[0][lane] + part[1][lane];
    z = solve(z);
    if (lane < w) x[r0 + lane] = z;
    xhi[lane] = lane < w ? z : 0.0;
    __threadfence();
  }
  __syncthreads();  // (2) x_hi
  if (wv == 3) {
    double a = 0.0;
#pragma unroll
    for (int c = 0; c < kTB; ++c) a += u[c] * xhi[c];
    part[3][lane] += a;
  }
  __syncthreads();  // (3) local fold
  if (wv == 2) {
    double z = lane < w ? x[r0 + lane] : 0.0;
    z -= part[2][lane] + part[3][lane];
    z = solve(z);
    if (lane < w) x[r0 + lane] = z;
    __threadfence();
  }
  __syncthreads();  // (4) both blocks stored
  if (threadIdx.x == 0) {
    __hip_atomic_store(flag + hi, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (lo >= 0) __hip_atomic_store(flag + lo, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}
#endif

// ---------------------------------------------------------------------------
// Panel factor in ONE launch (own_diag 6): the diagonal block's Cholesky AND
// the panel's triangular solve below it (replaces potrf_diag's 16 launches
// per 512-wide block plus rocBLAS dtrsm — together the look-ahead's critical
// path: 19.7 ms of side-stream work per nf = 12 000 factorisation against
// 15.4 ms of trailing dgemm, profiles/r2_chol_timeline.txt).
// Tiles are 64 x 64: column tile c (nc <= 8 of them, the last ragged), row
// tile r: r < nc the diagonal block's rows (tile height = that column tile's
// width), r >= nc 64-row blocks below it.  One 256-thread workgroup per row
// tile (atomic ticket = dispatch order), left-looking over its row:
//   T = A_rc - sum_{k<c} L_rk L_ck'         (MFMA f64 16x16x4 tile GEMMs)
//   c < r:  L_rc = T Linv_cc'                (Linv_cc from workgroup c)
//   c == r: L_rr = chol(T) in LDS, Linv_rr = L_rr^-1, published with L_rr
// A diagonal-block workgroup also keeps its diagonal tile's accumulator
// across its steps (A_rr -= L_rc L_rc' as soon as L_rc exists), so the step
// after a flag is one TRSM-GEMM + one SYRK-GEMM + the 64x64 factor.
// Workgroups only ever wait for lower-numbered ones (flag = epoch of this
// launch, release/acquire at agent scope, as the sweeps above).
typedef double pf_dvec4 __attribute__((ext_vector_type(4)));
constexpr int kPfMaxTiles = 16;  // column tiles per panel (panel <= 1024)
[[maybe_unused]] constexpr int kTinv = 512;  // own_diag 7: widest panel

__device__ __forceinline__ int pf_row0(int r, int kb, int nc) { return r < nc ? 64 * r : kb + 64 * (r - nc); }
__device__ __forceinline__ int pf_rows(int r, int kb, int nc, int mrows) {
  return r < nc ? min(64, kb - 64 * r) : min(64, mrows - kb - 64 * (r - nc));
}

// WM (wait mode): 0 every wave polls and takes the agent acquire; 1 one wave
// polls and takes the acquire for the workgroup (the acquire invalidates the
// CU's L1 for all its waves), its s_waitcnt holding the barrier until the
// invalidate has completed (MI355X_MICROARCH.md §visibility, consumer form);
// 2 one wave polls, no acquire: every load of the handed-off tiles is an sc1
// load (PfStage<true>) of bytes stored sc1 and drained before the flag, one
// workgroup per CU (the kernel's registers allow one) — the guide's table row
// 1; 3 as 2 with the next stage's tiles loaded during the current stage's
// GEMM when its flag is already set (pf_stages).  Called in
// workgroup-uniform control flow.
template <int WM>
__device__ __forceinline__ void pf_wait(const unsigned* f, unsigned epoch, unsigned* err, unsigned limit) {
  if constexpr (WM == 1) {
    if (threadIdx.x < 64) {
      flag_wait(f, epoch, err, limit);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  } else if constexpr (WM >= 2) {
    if (threadIdx.x < 64) {
      flag_poll(f, epoch, err, limit);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the poll
    }
    __syncthreads();
  } else {
    flag_wait(f, epoch, err, limit);
  }
}

// acc (wave w: rows 16w..16w+15 of the 64x64 tile, column tiles t = 0..3,
// v_mfma_f64_16x16x4f64 D layout D[4q + l/16][l%16]) += sign * X Y' over
// K = 64; ldx(i, k) / ldy(j, k) return X[i][k], Y[j][k] (zero-padded).
template <typename LX, typename LY>
__device__ __forceinline__ void pf_gemm_nt(pf_dvec4 (&acc)[4], double sign, LX ldx, LY ldy, int w, int lane) {
  const int m = lane & 15, k = lane >> 4;
#pragma unroll 4
  for (int s = 0; s < 16; ++s) {
    const double a = sign * ldx(16 * w + m, 4 * s + k);
    double b[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) b[t] = ldy(16 * t + m, 4 * s + k);
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[t], acc[t], 0, 0, 0);
  }
}

// pf_gemm_nt with Y lower triangular by 16x16 blocks (Y[j][k] read only for
// k-block <= j-block, the rest taken as zero: the published inverses'
// strict upper blocks are not stored): 40 of 64 MFMA steps.
template <typename LX, typename LY>
__device__ __forceinline__ void pf_gemm_nt_lt(pf_dvec4 (&acc)[4], double sign, LX ldx, LY ldy, int w, int lane) {
  const int m = lane & 15, k = lane >> 4;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const double a = sign * ldx(16 * w + m, 4 * s + k);
#pragma unroll
    for (int t = s / 4; t < 4; ++t)
      acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, ldy(16 * t + m, 4 * s + k), acc[t], 0, 0, 0);
  }
}

// LDS tiles are row-major with a padded stride (MFMA operand reads of 16
// consecutive rows then fall in distinct banks)
constexpr int kPfLd = 65;

// accumulator -> LDS tile T[i * kPfLd + j]
__device__ __forceinline__ void pf_acc_to_lds(const pf_dvec4 (&acc)[4], double* T, int w, int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) T[(16 * w + 4 * q + (lane >> 4)) * kPfLd + 16 * t + (lane & 15)] = acc[t][q];
}


// ---- 16x16 MFMA block helpers of the tile factor --------------------------
// acc (16x16, MFMA D layout) += sign * A(16x16) * op(B); A, B row-major with
// leading dimensions lda, ldb; op(B) = B' when TB.
template <bool TB>
__device__ __forceinline__ void blk16_mma(pf_dvec4& acc, double sign, const double* A, int lda, const double* B,
                                          int ldb, int lane) {
  const int m = lane & 15, k = lane >> 4;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const double a = sign * A[m * lda + 4 * s + k];
    const double b = TB ? B[m * ldb + 4 * s + k] : B[(4 * s + k) * ldb + m];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
}
__device__ __forceinline__ void blk16_load(pf_dvec4& acc, const double* C, int ldc, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = C[(4 * q + (lane >> 4)) * ldc + (lane & 15)];
}
__device__ __forceinline__ void blk16_store(const pf_dvec4& acc, double* C, int ldc, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) C[(4 * q + (lane >> 4)) * ldc + (lane & 15)] = acc[q];
}


// ---- 64x64 factor + inverse, block columns by register sweeps -------------
// M: row-major padded (ld kPfLd) 64x64, lower triangle valid; on return L in
// M's lower triangle, X = L^-1 (lower blocks), dinv[i] = 1 / L_ii, and the
// first non-positive pivot (1-based) or 0 (every thread).  Block column kb
// (16 wide) by wave 0 with lane = tile row: the 16 pivots of the diagonal
// block AND the solve of every row below it in one register sweep (x D' = a
// is the same elimination applied to the rows below the block), each pivot
// and multiplier broadcast by readlane — no LDS round trip or wave barrier
// per pivot (the previous per-pivot LDS exchange + lane-per-row substitution
// took 36 us per tile vs 15.6, profiles/r3_tile_probe.txt).  Trailing lower
// blocks by v_mfma_f64_16x16x4f64; X's off-diagonal blocks by block
// diagonals, X_ik = -X_ii sum_m L_im X_mk (MFMA).
// 1/sqrt(d) and sqrt(d) for a pivot: RSQ, v_rsq_f64 (~2^-23 relative) and
// two Goldschmidt steps (~1 ulp; six dependent ops on the pivot chain instead
// of the correctly rounded sqrt + divide expansions' ~25); else sqrt and 1/x.
template <bool RSQ>
__device__ __forceinline__ void pf_pivot(double d, double& sd, double& isd) {
  if (RSQ) {
    const double y = __builtin_amdgcn_rsq(d);
    double g = d * y, h = 0.5 * y;
    double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    sd = g;
    isd = h + h;
  } else {
    sd = sqrt(d);
    isd = 1.0 / sd;
  }
}

template <bool RSQ>
__device__ __forceinline__ int pf_col16(double* M, double* dinv, int o, int lane) {
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = M[lane * kPfLd + o + c];
  int bad = 0;
  double my_isd = 0.0;  // lane o + k keeps pivot k's reciprocal
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double d = readlane_f64(a[k], o + k);
    if (!(d > 0.0) && bad == 0) bad = o + k + 1;
    double sd, isd;
    pf_pivot<RSQ>(d, sd, isd);
    const bool piv = lane == o + k;
    const double l = piv ? sd : a[k] * isd;
    my_isd = piv ? isd : my_isd;
    a[k] = l;
#pragma unroll
    for (int c = k + 1; c < 16; ++c) a[c] -= l * readlane_f64(l, o + c);
  }
  // rows above the block computed garbage and are left alone; the block's
  // strict upper triangle is written as zero
  if (lane >= o) {
#pragma unroll
    for (int c = 0; c < 16; ++c) M[lane * kPfLd + o + c] = lane >= o + c ? a[c] : 0.0;
    if (lane < o + 16) dinv[lane] = my_isd;
  }
  return bad;
}

// pf_col16 with the next pivot formed from broadcast values: the
// multipliers of column k are (a[k] at lane o + c) * isd — taken by readlane
// of a[k] before the pivot is known — and the next pivot is (a[k + 1] at lane
// o + k + 1) - m * m, so the pivot chain runs rsq -> refinement -> one mul ->
// one fma without the per-lane select and the two readlanes of each column
// (the same operations on the same values: bitwise equal; tools build).
template <bool RSQ>
__device__ __forceinline__ int pf_col16_fp(double* M, double* dinv, int o, int lane) {
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = M[lane * kPfLd + o + c];
  int bad = 0;
  double my_isd = 0.0;  // lane o + k keeps pivot k's reciprocal
  double d = readlane_f64(a[0], o);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (!(d > 0.0) && bad == 0) bad = o + k + 1;
    double x[16];
#pragma unroll
    for (int c = k + 1; c < 16; ++c) x[c] = readlane_f64(a[k], o + c);
    const double y = k + 1 < 16 ? readlane_f64(a[k + 1], o + k + 1) : 0.0;
    double sd, isd;
    pf_pivot<RSQ>(d, sd, isd);
    const bool piv = lane == o + k;
    const double l = piv ? sd : a[k] * isd;
    my_isd = piv ? isd : my_isd;
    a[k] = l;
#pragma unroll
    for (int c = k + 1; c < 16; ++c) {
      const double m = x[c] * isd;
      a[c] -= l * m;
    }
    if (k + 1 < 16) {
      const double m1 = x[k + 1] * isd;
      d = y - m1 * m1;
    }
  }
  if (lane >= o) {
#pragma unroll
    for (int c = 0; c < 16; ++c) M[lane * kPfLd + o + c] = lane >= o + c ? a[c] : 0.0;
    if (lane < o + 16) dinv[lane] = my_isd;
  }
  return bad;
}

// Diagonal block b's inverse X_bb = L_bb^-1 by one wave: lane = column j
// (lanes 16.. repeat lanes 0..15 and store nothing), forward substitution
// over the block's rows with L broadcast from LDS.
__device__ __forceinline__ void pf_diag_inv16(const double* M, const double* dinv, double* X, int b, int lane) {
  const int j = lane & 15, o = 16 * b;
  double x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    double v = (i == j) ? 1.0 : 0.0;
#pragma unroll
    for (int m2 = 0; m2 < i; ++m2) v -= M[(o + i) * kPfLd + o + m2] * x[m2];
    x[i] = v * dinv[o + i];
  }
  if (lane < 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) X[(o + i) * kPfLd + o + j] = x[i];
  }
}

// pf_diag_inv16 with the operand loads ahead of the arithmetic: the 16
// reciprocal pivots up front and row i + 1's multipliers loaded while row i's
// substitution runs (the same operations in the same order: bitwise equal).
__device__ __forceinline__ void pf_diag_inv16_pipe(const double* M, const double* dinv, double* X, int b, int lane) {
  const int j = lane & 15, o = 16 * b;
  double x[16], di[16], cur[16], nxt[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) di[i] = dinv[o + i];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i + 1 < 16) {
#pragma unroll
      for (int m2 = 0; m2 < i + 1; ++m2) nxt[m2] = M[(o + i + 1) * kPfLd + o + m2];
    }
    double v = (i == j) ? 1.0 : 0.0;
#pragma unroll
    for (int m2 = 0; m2 < i; ++m2) v -= cur[m2] * x[m2];
    x[i] = v * di[i];
#pragma unroll
    for (int m2 = 0; m2 < 16; ++m2) cur[m2] = nxt[m2];
  }
  if (lane < 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) X[(o + i) * kPfLd + o + j] = x[i];
  }
}

// Factor + inverse of the 64x64 tile M (row-major padded, lower valid): the
// four block-column sweeps by wave 0 (pf_col16), the trailing lower blocks
// by all waves (MFMA); while wave 0 sweeps block column kb, wave
// 1 + (kb - 1) % 3 inverts diagonal block kb - 1 (final since sweep kb - 1).
// scr: [0, 1088) per-wave 16x16 scratch, [1088] the pivot status.
// X = L^-1 in its lower blocks only (the strict upper blocks are left as they
// are: every consumer reads X as lower triangular, pf_gemm_nt_lt).
// stamps (nullable, probes only): clock64() by thread 0 after each block
// column's sweep and trailing update (8), the last diagonal inverse, the end.
// OVL (tools build): the last diagonal inverse (wave 3) overlapped with the
// off-diagonal blocks that do not need it — only X_3k = -X_33 (sum) waits for
// it, every other block of X depends on its own wave's earlier blocks; PIPE:
// the diagonal inverses by pf_diag_inv16_pipe.  Bitwise equal to the default.
template <bool RSQ, bool OVL = false, bool PIPE = false, bool FP = false>
__device__ __forceinline__ int pf_chol_inv_fast(double* M, double* X, double* scr, double* dinv, int lane, int wv,
                                                long long* stamps = nullptr) {
  int bad = 0;
  auto stamp = [&](int k) {
    if (stamps && threadIdx.x == 0) stamps[k] = clock64();
  };
  for (int kb = 0; kb < 4; ++kb) {
    const int o = 16 * kb;
    if (wv == 0) {
      const int b = FP ? pf_col16_fp<RSQ>(M, dinv, o, lane) : pf_col16<RSQ>(M, dinv, o, lane);
      if (bad == 0) bad = b;
      // bad lives in wave 0; every thread returns it
      if (kb == 3 && lane == 0) reinterpret_cast<int*>(scr)[4 * 16 * 17 * 2] = bad;
    } else if (kb >= 1 && wv == 1 + (kb - 1) % 3) {
      if (PIPE)
        pf_diag_inv16_pipe(M, dinv, X, kb - 1, lane);
      else
        pf_diag_inv16(M, dinv, X, kb - 1, lane);
    }
    __syncthreads();
    stamp(2 * kb);
    // trailing lower blocks (ib >= jb > kb): A_ib,jb -= L_ib,kb L_jb,kb'
    int t = 0;
    for (int ib = kb + 1; ib < 4; ++ib)
      for (int jb = kb + 1; jb <= ib; ++jb, ++t) {
        if (t % 4 != wv) continue;
        pf_dvec4 acc;
        double* C = M + 16 * ib * kPfLd + 16 * jb;
        blk16_load(acc, C, kPfLd, lane);
        blk16_mma<true>(acc, -1.0, M + 16 * ib * kPfLd + o, kPfLd, M + 16 * jb * kPfLd + o, kPfLd, lane);
        blk16_store(acc, C, kPfLd, lane);
      }
    if (kb < 3) __syncthreads();
    stamp(2 * kb + 1);
  }
  double* T = scr + wv * 16 * 17;
  if constexpr (OVL) {
    // wave 3: X_33; wave k < 3: X_ik for i = k + 1 .. 2, then the sum of
    // X_3k (kept in its scratch) — the blocks it reads are its own or final
    if (wv == 3) {
      if (PIPE)
        pf_diag_inv16_pipe(M, dinv, X, 3, lane);
      else
        pf_diag_inv16(M, dinv, X, 3, lane);
    } else {
      const int k = wv;
      for (int i = k + 1; i < 4; ++i) {
        pf_dvec4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int m2 = k; m2 < i; ++m2)
          blk16_mma<false>(acc, 1.0, M + 16 * i * kPfLd + 16 * m2, kPfLd, X + 16 * m2 * kPfLd + 16 * k, kPfLd, lane);
        blk16_store(acc, T, 17, lane);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        if (i == 3) break;
        pf_dvec4 out = {0.0, 0.0, 0.0, 0.0};
        blk16_mma<false>(out, -1.0, X + 16 * i * kPfLd + 16 * i, kPfLd, T, 17, lane);
        blk16_store(out, X + 16 * i * kPfLd + 16 * k, kPfLd, lane);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      }
    }
    __syncthreads();
    stamp(8);
    bad = reinterpret_cast<const int*>(scr)[4 * 16 * 17 * 2];
    if (wv < 3) {
      pf_dvec4 out = {0.0, 0.0, 0.0, 0.0};
      blk16_mma<false>(out, -1.0, X + 48 * kPfLd + 48, kPfLd, T, 17, lane);
      blk16_store(out, X + 48 * kPfLd + 16 * wv, kPfLd, lane);
    }
    __syncthreads();
    stamp(9);
    return bad;
  }
  if (wv == 3) {
    if (PIPE)
      pf_diag_inv16_pipe(M, dinv, X, 3, lane);
    else
      pf_diag_inv16(M, dinv, X, 3, lane);
  }
  __syncthreads();
  stamp(8);
  bad = reinterpret_cast<const int*>(scr)[4 * 16 * 17 * 2];
  // off-diagonal blocks by block diagonals d: X_ik = -X_ii (sum_{m=k}^{i-1} L_im X_mk)
  for (int d = 1; d < 4; ++d) {
    const int k = wv;
    const int i = k + d;
    if (i < 4) {
      pf_dvec4 acc = {0.0, 0.0, 0.0, 0.0};
      for (int m2 = k; m2 < i; ++m2)
        blk16_mma<false>(acc, 1.0, M + 16 * i * kPfLd + 16 * m2, kPfLd, X + 16 * m2 * kPfLd + 16 * k, kPfLd, lane);
      blk16_store(acc, T, 17, lane);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      pf_dvec4 out = {0.0, 0.0, 0.0, 0.0};
      blk16_mma<false>(out, -1.0, X + 16 * i * kPfLd + 16 * i, kPfLd, T, 17, lane);
      blk16_store(out, X + 16 * i * kPfLd + 16 * k, kPfLd, lane);
    }
    __syncthreads();
  }
  stamp(9);
  return bad;
}

// dbg (nullable, probes only): wall_clock64() stamps [row tile][20]: 0 start,
// 1 + 2c after step c's waits (diagonal step: after the factor), 2 + 2c at
// step c's end; diagonal rows' last solve step (c = r - 1): 17 inverse staged,
// 18 solve GEMM done, 19 SYRK done and published.
constexpr int kPfDbgSlots = 36;

// Tile staging global -> LDS S[i * kPfLd + j] with every load of the tile
// in flight before the first LDS store (16 per thread, 256 threads): a
// load-then-store loop waits one memory round trip per element (32 KB: 3.9
// vs 0.4 us hot, profiles/r3_tile_probe.txt).  Column-major source: element
// (i, j) at src[j * ld + i], rows clamped to h and columns to w, zero outside.
struct PfStage {
  double v[16];
  // SC: sc1 loads (pf_wait mode 2)
  template <bool SC = false>
  __device__ __forceinline__ void load_cm(const double* __restrict__ src, size_t ld, int h, int w) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = threadIdx.x + 256 * q, i = e & 63, j = e >> 6;
      const double* a = src + (size_t)min(j, w - 1) * ld + min(i, h - 1);
      v[q] = SC ? ld_sc1(a) : *a;
    }
  }
  __device__ __forceinline__ void store_cm(double* S, int h, int w) const {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = threadIdx.x + 256 * q, i = e & 63, j = e >> 6;
      S[i * kPfLd + j] = (i < h && j < w) ? v[q] : 0.0;
    }
  }
  // row-major source with leading dimension 64 (the published inverses)
  template <bool SC = false>
  __device__ __forceinline__ void load_rm(const double* __restrict__ src) {
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = SC ? ld_sc1(src + threadIdx.x + 256 * q) : src[threadIdx.x + 256 * q];
  }
  __device__ __forceinline__ void store_rm(double* S) const {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = threadIdx.x + 256 * q;
      S[(e >> 6) * kPfLd + (e & 63)] = v[q];
    }
  }
};

// Hand-off store of the panel's published tiles: WT (write-through) = a
// relaxed agent-scope 8-byte atomic store (global_store sc1), drained by
// s_waitcnt vmcnt(0) before the flag, no release fence (the publish costs
// 0.84 vs 2.84 us per 32 KB, profiles/r3_tile_probe.txt); else a plain store
// behind __threadfence().
template <bool WT>
__device__ __forceinline__ void pf_st(double* p, double v) {
  if (WT)
    __hip_atomic_store((__attribute__((address_space(1))) unsigned long long*)p,
                       (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}
template <bool WT>
__device__ __forceinline__ void pf_drain() {
  if (WT)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else
    __threadfence();
}

// The left-looking updates of one tile: acc -= sum_{k < c} L_rk L_ck' (row
// tile r0 / hr, column tile c0 / wc; flags fc[k] = tile (c, k) final), L_rk
// staged in T and L_ck in Li.  WM 3: the tiles of stage k + 1 are loaded
// while stage k's GEMM runs if flag k + 1 is already set (one wave polls,
// the workgroup's barrier follows: sc1 loads, pf_wait mode 2), else after it;
// the same GEMMs in the same order (bitwise equal).
template <int WM>
__device__ __forceinline__ void pf_stages(pf_dvec4 (&acc)[4], const double* A, int lda, int r0, int hr, int c0, int wc,
                                          int c, const unsigned* fc, unsigned epoch, unsigned* err, unsigned limit,
                                          double* T, double* Li, int* s_ready, int wv, int lane,
                                          unsigned long long* st = nullptr) {
  // st (probes only): wall_clock64() after each phase of each stage, 3 per
  // stage (tiles loaded and staged, GEMM done) — slots 3k, 3k + 1, 3k + 2
  auto stamp = [&](int slot) {
    if (st && threadIdx.x == 0 && slot < 16) st[slot] = wall_clock64();
  };
  auto ltile = [&](const double* S) { return [=](int i, int j) { return S[i * kPfLd + j]; }; };
  if constexpr (WM == 3) {
    PfStage sr, sc;
    if (c > 0) {
      pf_wait<WM>(fc, epoch, err, limit);
      sr.template load_cm<true>(A + r0, lda, hr, 64);
      sc.template load_cm<true>(A + c0, lda, wc, 64);
    }
    for (int k = 0; k < c; ++k) {
      sr.store_cm(T, hr, 64);
      sc.store_cm(Li, wc, 64);
      if (threadIdx.x < 64)
        *s_ready = k + 1 < c && __hip_atomic_load(fc + k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
      __syncthreads();
      const bool ready = *s_ready != 0;
      if (ready) {
        sr.template load_cm<true>(A + (size_t)64 * (k + 1) * lda + r0, lda, hr, 64);
        sc.template load_cm<true>(A + (size_t)64 * (k + 1) * lda + c0, lda, wc, 64);
      }
      pf_gemm_nt(acc, -1.0, ltile(T), ltile(Li), wv, lane);
      __syncthreads();
      if (k + 1 < c && !ready) {
        pf_wait<WM>(fc + k + 1, epoch, err, limit);
        sr.template load_cm<true>(A + (size_t)64 * (k + 1) * lda + r0, lda, hr, 64);
        sc.template load_cm<true>(A + (size_t)64 * (k + 1) * lda + c0, lda, wc, 64);
      }
    }
  } else {
    for (int k = 0; k < c; ++k) {
      pf_wait<WM>(fc + k, epoch, err, limit);
      stamp(3 * k);
      {
        PfStage sr, sc;
        sr.template load_cm<WM == 2>(A + (size_t)64 * k * lda + r0, lda, hr, 64);
        sc.template load_cm<WM == 2>(A + (size_t)64 * k * lda + c0, lda, wc, 64);
        sr.store_cm(T, hr, 64);
        sc.store_cm(Li, wc, 64);
      }
      __syncthreads();
      stamp(3 * k + 1);
      pf_gemm_nt(acc, -1.0, ltile(T), ltile(Li), wv, lane);
      __syncthreads();
      stamp(3 * k + 2);
    }
  }
}

// FV: 64x64 tile factor pf_chol_inv_fast, 1 sqrt + divide pivots, 2 rsq
// pivots, 3 / 4 / 5 rsq with the overlapped last inverse and / or the
// pipelined diagonal inverses (tools build); WT: pf_st
template <int FV, bool WT, int WM>
__global__ __launch_bounds__(256) void panel_factor_kernel(double* __restrict__ A, int lda, int kb, int mrows,
                                                           int* __restrict__ info, double* __restrict__ linv,
                                                           unsigned* ctrl, unsigned base, unsigned epoch,
                                                           unsigned* err, unsigned limit, int below_groups = 0,
                                                           unsigned long long* dbg = nullptr, int r_off = 0,
                                                           unsigned* tick = nullptr) {
  __shared__ double T[64 * kPfLd];   // staging / factor tile (row-major padded)
  __shared__ double Li[64 * kPfLd];  // a diagonal tile's inverse (own, or workgroup c's)
  __shared__ double Lc[1152];        // pf_chol_inv_fast scratch: per-wave 16x16 tiles + the pivot status
  __shared__ double dinv[64];
  __shared__ int s_r, s_ready;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // row tile from the launch's ticket (tick: a second counter, r_off: the
  // first row tile of a below-rows launch of the split tail)
  if (threadIdx.x == 0) s_r = (int)(atomicAdd(tick ? tick : ctrl, 1u) - base) + r_off;
  __syncthreads();
  const int r = s_r;
  const int nc = (kb + 63) / 64;
  unsigned* flag = ctrl + 1;  // [16][16]: tile (r, c) of the diagonal block rows final in A
  auto stamp = [&](int slot) {
    if (dbg && threadIdx.x == 0) dbg[(size_t)r * kPfDbgSlots + slot] = wall_clock64();
  };
  stamp(0);
  // the panel's info starts at 0 (row tile 0 clears it before its first
  // publish; every other write follows one of its flags).  An agent-scope
  // store: with write-through publishes no release fence writes back a plain
  // store's dirty line, which could then land after another workgroup's CAS
  if (r == 0 && threadIdx.x == 0) __hip_atomic_store(info, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int r0 = pf_row0(r, kb, nc), hr = pf_rows(r, kb, nc, mrows);
  const int cmax = min(r, nc - 1);
  const bool diag_row = r < nc;
  const int m = lane & 15, kq = lane >> 4;
  // tile loaders (clamped addresses, zero padding)
  auto ltile = [&](const double* S) { return [=](int i, int j) { return S[i * kPfLd + j]; }; };
  // the diagonal tile's running accumulator (diagonal-block rows)
  pf_dvec4 dacc[4];
  if (diag_row) {
    const int w = hr;  // = the width of column tile r
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 16 * wv + 4 * q + kq, j = 16 * t + m;
        const double v = A[(size_t)(r0 + min(j, w - 1)) * lda + r0 + min(i, w - 1)];
        dacc[t][q] = (i < w && j < w) ? v : (i == j ? 1.0 : 0.0);
      }
  }
  if (!diag_row) {
    // below the diagonal block: left-looking over the panel's column tiles
    // (L_ck staged with L_rk per update), one 64-row tile at a time.  With
    // below_groups = G > 0 the launch has G below-diagonal workgroups, each
    // taking row tiles r, r + G, ...: its first tile follows the diagonal
    // chain, the later ones find every flag set.  Fewer resident workgroups
    // leave the CUs to the concurrent trailing dgemm while the panel has
    // slack (the look-ahead's dgemm-bound head).
    const int nbelow = (mrows - kb + 63) / 64;
    const int G = below_groups > 0 ? below_groups : nbelow;
    for (int rr = r; rr < nc + nbelow; rr += G) {
    const int r0 = pf_row0(rr, kb, nc), hr = pf_rows(rr, kb, nc, mrows);
    for (int c = 0; c < nc; ++c) {
      const int c0 = 64 * c, wc = min(64, kb - c0);
      pf_dvec4 acc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = 16 * wv + 4 * q + kq, jj = 16 * t + m;
          const double v = A[(size_t)(c0 + min(jj, wc - 1)) * lda + r0 + min(i, hr - 1)];
          acc[t][q] = (i < hr && jj < wc) ? v : 0.0;
        }
      pf_stages<WM>(acc, A, lda, r0, hr, c0, wc, c, flag + c * kPfMaxTiles, epoch, err, limit, T, Li, &s_ready, wv,
                    lane);
      pf_wait<WM>(flag + c * kPfMaxTiles + c, epoch, err, limit);
      stamp(1 + 2 * c);
      {
        PfStage sl;
        sl.template load_rm<WM >= 2>(linv + (size_t)c * 64 * 64);
        sl.store_rm(Li);
      }
      pf_acc_to_lds(acc, T, wv, lane);
      __syncthreads();
      pf_dvec4 out[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) out[t] = pf_dvec4{0.0, 0.0, 0.0, 0.0};
      pf_gemm_nt_lt(out, 1.0, ltile(T), ltile(Li), wv, lane);
      __syncthreads();
      // through T: each wave stores whole 512-byte column segments
      pf_acc_to_lds(out, T, wv, lane);
      __syncthreads();
      // L_rc is read back by this workgroup's next column steps (pf_stages
      // stages L_rk with sc1 loads under panel_wait 2): stored the hand-off
      // way — write-through, drained by every storing wave before the
      // barrier — so that no later load of another wave can overtake a store
      // still in flight (the invariant of the sc1 hand-off: every handed-off
      // byte stored sc1 and drained, then read by sc1 loads)
      for (int e = threadIdx.x; e < 64 * 64; e += 256) {
        const int i = e & 63, jj = e >> 6;
        if (i < hr && jj < wc) pf_st<WT>(A + (size_t)(c0 + jj) * lda + r0 + i, T[i * kPfLd + jj]);
      }
      pf_drain<WT>();
      stamp(2 + 2 * c);
      __syncthreads();  // T and Li are restaged next step
    }
    }
    return;
  }
  for (int c = 0; c <= cmax; ++c) {
    const int c0 = 64 * c, wc = min(64, kb - c0);
    if (c < r) {
      pf_dvec4 acc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = 16 * wv + 4 * q + kq, j = 16 * t + m;
          const double v = A[(size_t)(c0 + min(j, wc - 1)) * lda + r0 + min(i, hr - 1)];
          acc[t][q] = (i < hr && j < wc) ? v : 0.0;
        }
      pf_stages<WM>(acc, A, lda, r0, hr, c0, wc, c, flag + c * kPfMaxTiles, epoch, err, limit, T, Li, &s_ready, wv,
                    lane, dbg && c == r - 1 && r == nc - 1 ? dbg + (size_t)r * kPfDbgSlots + 20 : nullptr);
      pf_wait<WM>(flag + c * kPfMaxTiles + c, epoch, err, limit);
      stamp(1 + 2 * c);
      // L_rc = T Linv_cc' (Linv_cc row-major in linv, staged in LDS)
      pf_acc_to_lds(acc, T, wv, lane);
      {
        PfStage sl;
        sl.template load_rm<WM >= 2>(linv + (size_t)c * 64 * 64);
        sl.store_rm(Li);
      }
      __syncthreads();
      if (c == r - 1) stamp(17);
      pf_dvec4 out[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) out[t] = pf_dvec4{0.0, 0.0, 0.0, 0.0};
      pf_gemm_nt_lt(out, 1.0, ltile(T), ltile(Li), wv, lane);
      __syncthreads();  // every wave is done reading T
      // L_rc through T (whole column segments per store): its stores are
      // issued, folded into the diagonal tile (A_rr -= L_rc L_rc') while they
      // drain, then published (its consumers first need this row's factor)
      pf_acc_to_lds(out, T, wv, lane);
      __syncthreads();
      if (c == r - 1) stamp(18);
      for (int e = threadIdx.x; e < 64 * 64; e += 256) {
        const int i = e & 63, j = e >> 6;
        if (i < hr && j < wc) pf_st<WT>(A + (size_t)(c0 + j) * lda + r0 + i, T[i * kPfLd + j]);
      }
      pf_gemm_nt(dacc, -1.0, ltile(T), ltile(T), wv, lane);
      pf_drain<WT>();
      __syncthreads();
      if (threadIdx.x == 0)
        __hip_atomic_store(flag + r * kPfMaxTiles + c, epoch, WT ? __ATOMIC_RELAXED : __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_AGENT);
      if (c == r - 1) stamp(19);
      stamp(2 + 2 * c);
      continue;
    }
    // c == r: factor the diagonal tile, invert it, publish both
    pf_acc_to_lds(dacc, T, wv, lane);
    __syncthreads();
    // factor + inverse by 16x16 blocks (Lc: pivot columns + per-wave scratch)
    const int bad = FV == 6   ? pf_chol_inv_fast<true, true, true, true>(T, Li, Lc, dinv, lane, wv)
                    : FV == 3 ? pf_chol_inv_fast<true, true, true>(T, Li, Lc, dinv, lane, wv)
                    : FV == 4 ? pf_chol_inv_fast<true, true, false>(T, Li, Lc, dinv, lane, wv)
                    : FV == 5 ? pf_chol_inv_fast<true, false, true>(T, Li, Lc, dinv, lane, wv)
                    : FV == 2 ? pf_chol_inv_fast<true>(T, Li, Lc, dinv, lane, wv)
                              : pf_chol_inv_fast<false>(T, Li, Lc, dinv, lane, wv);
    stamp(1 + 2 * c);
    // publish the inverse's lower blocks (row-major, ld 64: the only part
    // its consumers read); the factor tile itself is read by no workgroup of
    // this launch and is stored after the flag
    double* lo = linv + (size_t)c * 64 * 64;
    for (int e = threadIdx.x; e < 64 * 64; e += 256)
      if (((e & 63) >> 4) <= (e >> 10)) pf_st<WT>(lo + e, Li[(e >> 6) * kPfLd + (e & 63)]);
    if (threadIdx.x == 0 && bad != 0 && bad <= wc) atomicCAS(info, 0, c0 + bad);
    pf_drain<WT>();
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(flag + r * kPfMaxTiles + r, epoch, WT ? __ATOMIC_RELAXED : __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
    for (int e = threadIdx.x; e < 64 * 64; e += 256) {
      const int i = e & 63, j = e >> 6;
      if (i < wc && j < wc && i >= j) A[(size_t)(c0 + j) * lda + c0 + i] = T[i * kPfLd + j];
    }
    stamp(2 + 2 * c);
  }
}

rocblas_status potrf_diag(rocblas_handle h, int n, double* A, int lda, int* info, double* scratch, int variant) {
  hipStream_t s;
  if (!scratch) return rocblas_status_invalid_pointer;
  if (rocblas_get_stream(h, &s) != rocblas_status_success) return rocblas_status_internal_error;
  if (hipMemsetAsync(info, 0, sizeof(int), s) != hipSuccess) return rocblas_status_internal_error;
  for (int k = 0; k < n; k += kSub) {
    const int w = std::min(kSub, n - k);
    const int m = n - k - w;  // rows (and columns) of the block after this sub-panel
    double* Akk = A + k + (size_t)k * lda;
    if (variant == 2)
      hipLaunchKernelGGL(diag_panel_blocked_kernel<4>, dim3(1 + (m + kSub - 1) / kSub), dim3(64 * kPanelWaves), 0, s,
                         Akk, lda, w, m, info, scratch, k);
    else if (variant == 3)
      hipLaunchKernelGGL(diag_panel_blocked_kernel<8>, dim3(1 + (m + kSub - 1) / kSub), dim3(64 * kPanelWaves), 0, s,
                         Akk, lda, w, m, info, scratch, k);
    else if (variant == 4)
      hipLaunchKernelGGL((diag_panel_blocked_kernel<4, 4>), dim3(1 + (m + kSub - 1) / kSub), dim3(64 * 4), 0, s, Akk,
                         lda, w, m, info, scratch, k);
    else if (variant == 5)
      hipLaunchKernelGGL((diag_panel_blocked_kernel<4, 2>), dim3(1 + (m + kSub - 1) / kSub), dim3(64 * 2), 0, s, Akk,
                         lda, w, m, info, scratch, k);
    else
      hipLaunchKernelGGL(diag_panel_kernel, dim3(1 + (m + kSub - 1) / kSub), dim3(64 * kPanelWaves), 0, s, Akk, lda,
                         w, m, info, scratch, k);
    // trailing tiles of the block + one workgroup writing the tile back
    const int T = (m + kSub - 1) / kSub;
    hipLaunchKernelGGL(diag_update_kernel, dim3(T * (T + 1) / 2 + 1), dim3(256), 0, s, Akk + w + (size_t)w * lda,
                       Akk + w, lda, m, w, scratch, Akk);
  }
  return hipGetLastError() == hipSuccess ? rocblas_status_success : rocblas_status_internal_error;
}

rocblas_status potrf_leaf(rocblas_handle h, int n, double* A, int lda, int* info, int own, double* scratch) {
  if (own) return potrf_diag(h, n, A, lda, info, scratch, own);
  return rocsolver_dpotrf(h, rocblas_fill_lower, n, A, lda, info);
}

constexpr int kLeaf = 768;  // diagonal leaves of the recursive factor
// dtrsv leaves of the solve (rocBLAS dtrsv, 135 us at 768); 384-wide leaves
// measured slower (5.9 -> 8.7 ms per solve at nf = 12 000: the extra dgemv
// calls cost more than the shorter column sweeps save)
constexpr int kSolveLeaf = 768;

int split(int n) {
  int n1 = n / 2;
  n1 = (n1 + 255) / 256 * 256;  // keep the big dtrsm/dsyrk operands 2 KB aligned
  return n1 < n ? n1 : n / 2;
}

rocblas_status factor(rocblas_handle h, int n, double* A, int lda, int*& info, int own, double* scratch) {
  if (n <= kLeaf) return potrf_leaf(h, n, A, lda, info++, own, scratch);
  const int n1 = split(n), n2 = n - n1;
  double* A11 = A;
  double* A21 = A + n1;
  double* A22 = A + n1 + (size_t)n1 * lda;
  rocblas_status st = factor(h, n1, A11, lda, info, own, scratch);
  if (st != rocblas_status_success) return st;
  const double one = 1.0, minus_one = -1.0;
  // A21 := A21 L11^-T
  st = rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                     rocblas_diagonal_non_unit, n2, n1, &one, A11, lda, A21, lda);
  if (st != rocblas_status_success) return st;
  // A22 := A22 - A21 A21'
  st = rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, n2, n1, &minus_one, A21, lda, &one, A22, lda);
  if (st != rocblas_status_success) return st;
  return factor(h, n2, A22, lda, info, own, scratch);
}

int leaves(int n) { return n <= kLeaf ? 1 : leaves(split(n)) + leaves(n - split(n)); }

// L y = b (forward) and L' x = y (backward), recursively.
rocblas_status forward(rocblas_handle h, int n, const double* A, int lda, double* x) {
  if (n <= kSolveLeaf)
    return rocblas_dtrsv(h, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit, n, A, lda, x, 1);
  const int n1 = split(n), n2 = n - n1;
  rocblas_status st = forward(h, n1, A, lda, x);
  if (st != rocblas_status_success) return st;
  const double one = 1.0, minus_one = -1.0;
  st = rocblas_dgemv(h, rocblas_operation_none, n2, n1, &minus_one, A + n1, lda, x, 1, &one, x + n1, 1);
  if (st != rocblas_status_success) return st;
  return forward(h, n2, A + n1 + (size_t)n1 * lda, lda, x + n1);
}

rocblas_status backward(rocblas_handle h, int n, const double* A, int lda, double* x) {
  if (n <= kSolveLeaf)
    return rocblas_dtrsv(h, rocblas_fill_lower, rocblas_operation_transpose, rocblas_diagonal_non_unit, n, A, lda, x,
                         1);
  const int n1 = split(n), n2 = n - n1;
  rocblas_status st = backward(h, n2, A + n1 + (size_t)n1 * lda, lda, x + n1);
  if (st != rocblas_status_success) return st;
  const double one = 1.0, minus_one = -1.0;
  // x1 -= L21' x2
  st = rocblas_dgemv(h, rocblas_operation_transpose, n2, n1, &minus_one, A + n1, lda, x + n1, 1, &one, x, 1);
  if (st != rocblas_status_success) return st;
  return backward(h, n1, A, lda, x);
}

// Right-looking blocked factorisation: per panel, dpotrf of the diagonal
// block, dtrsm of the panel below it, then the trailing lower triangle
// updated by dsyrk (or by dgemm per block column of width `panel`).
rocblas_status panel_factor(rocblas_handle h, int n, double* A, int lda, int k, int kb, int* info, int own,
                            double* scratch, CholWorkspace* ws, int ex);
rocblas_status panel_factor_fused(hipStream_t s, int n, double* A, int lda, int k, int kb, int* info,
                                  CholWorkspace* ws, int ex, int part);
rocblas_status gemm_nt(rocblas_handle h, int m, int n, int k, const double* P, int ldp, double* C, int ldc, int sol);
rocblas_status gemm_nt2(rocblas_handle h, int m, int n, int k, const double* Pa, const double* Pb, int ldp, double* C,
                        int ldc, int sol);
// split tail (CholConfig::split_tail_cols): does panel kk + 1 (start ps[kk + 1])
// get its block column in two dgemms?
// Tools build only: measured slower (Cholesky 16.2-16.6 vs 14.2 ms — the
// fourth stream shares a hardware queue, profiles/r5ag_ab_cholesky_split_tail.jsonl).
static bool split_tail(const CholConfig& cfg, const std::vector<int>& ps, int kk, int n, int ex) {
#ifndef MI_BA_AB_VARIANTS
  if (cfg.split_tail_cols >= 0) return false;
#endif
  if (cfg.split_tail_cols <= 0 || cfg.own_diag != 6 || kk + 2 >= (int)ps.size()) return false;
  const int k1 = ps[kk + 1], jb0 = ps[kk + 2] - k1;
  return n - k1 <= cfg.split_tail_cols && n - k1 + ex > jb0;
}

rocblas_status factor_blocked(rocblas_handle h, int n, double* A, int lda, int* info, const CholConfig& cfg,
                              double* scratch, CholWorkspace* ws, int ex) {
  const double one = 1.0, minus_one = -1.0;
  const int nb = cfg.panel;
  const std::vector<int> ps = chol_panel_starts(n, cfg);
  for (size_t pk = 0; pk + 1 < ps.size(); ++pk) {
    const int k = ps[pk], kb = ps[pk + 1] - k;
    double* Akk = A + k + (size_t)k * lda;
    rocblas_status st = panel_factor(h, n, A, lda, k, kb, info++, cfg.own_diag, scratch, ws, ex);
    if (st != rocblas_status_success) return st;
    const int m = n - k - kb;
    if (m == 0) break;
    double* Aik = Akk + kb;  // panel below the diagonal block
    double* T = Aik + (size_t)kb * lda;  // trailing matrix, lower triangle
    if (!cfg.gemm_update) {
      st = rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, m, kb, &minus_one, Aik, lda, &one, T, lda);
      if (st != rocblas_status_success) return st;
      if (ex > 0) {  // the extra rows below the trailing matrix
        st = rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, ex, m, kb, &minus_one, Aik + m, lda,
                           Aik, lda, &one, T + m, lda);
        if (st != rocblas_status_success) return st;
      }
    } else {
      // the look-ahead's partition and GEMM solution (block column k+1, then
      // columns of width nb or 2 nb): both orders run the same GEMMs on the
      // same shapes, so their factors are bitwise equal
      const int jb0 = ps[pk + 2] - ps[pk + 1];  // the next panel's width
      const int cw = cfg.rest_update == 3 ? 2 * nb : nb;
      for (int j = 0; j < m; j = j == 0 ? jb0 : j + cw) {
        const int jb = std::min(j == 0 ? jb0 : cw, m - j);
        if (j == 0 && split_tail(cfg, ps, (int)pk, n, ex)) {  // the look-ahead's two dgemms (split tail)
          st = gemm_nt(h, jb0, jb0, kb, Aik, lda, T, lda, cfg.gemm_solution);
          if (st == rocblas_status_success)
            st = gemm_nt2(h, m + ex - jb0, jb0, kb, Aik + jb0, Aik, lda, T + jb0, lda, cfg.gemm_solution);
        } else {
          st = gemm_nt(h, m - j + ex, jb, kb, Aik + j, lda, T + j + (size_t)j * lda, lda, cfg.gemm_solution);
        }
        if (st != rocblas_status_success) return st;
      }
    }
  }
  return rocblas_status_success;
}

// Look-ahead variant of factor_blocked (gemm update): as soon as panel k's
// dgemm has updated block column k+1, the diagonal factor and dtrsm of panel
// k+1 run on the workspace's side stream (own rocBLAS handle) while the rest
// of panel k's trailing dgemm runs on the caller's stream; the next
// iteration's dgemm waits on the side stream's event.  Hides the latency-bound
// diagonal factor behind the MFMA update.
// own_diag 6: diagonal factor + panel solve in one panel_factor_kernel launch
// part: 0 the whole panel, 1 its diagonal-block rows, 2 the rows below them
// (split tail: the same epoch as the part-1 launch before it, tickets from
// the second counter, row tiles from nc)
rocblas_status panel_factor_fused(hipStream_t s, int n, double* A, int lda, int k, int kb, int* info,
                                  CholWorkspace* ws, int ex, int part) {
  if (!ws || !ws->pf_ctrl || !ws->pf_linv || !ws->err || kb > 64 * kPfMaxTiles) return rocblas_status_invalid_pointer;
  const int mrows = n - k + ex;  // the extra rows below the matrix take the panel solve too
  const int nc = (kb + 63) / 64;
  const int nbelow = (mrows - kb + 63) / 64;
  // below-diagonal workgroups: one per row tile, or (while the trailing
  // update is long: rows below >= group_min_rows) one per rows_per_group
  // row tiles
  int groups = 0;
  if (ws->rows_per_group > 1 && mrows - kb >= ws->group_min_rows && nbelow > 0)
    groups = (nbelow + ws->rows_per_group - 1) / ws->rows_per_group;
  const int nbg = groups > 0 ? groups : nbelow;
  const int nr = part == 1 ? nc : part == 2 ? nbg : nc + nbg;  // workgroups (tickets) of the launch
  if (nr == 0) return rocblas_status_success;
  if (part != 2 && (ws->pf_base > 0x7fffffffu || ws->pf_base2 > 0x7fffffffu || ws->pf_epoch > 0xfffffff0u)) {
    if (hipMemsetAsync(ws->pf_ctrl, 0, sizeof(unsigned) * (2 + kPfMaxTiles * kPfMaxTiles), s) != hipSuccess)
      return rocblas_status_internal_error;
    ws->pf_base = 0;
    ws->pf_base2 = 0;
    ws->pf_epoch = 0;
  }
  const unsigned epoch = part == 2 ? ws->pf_epoch : ++ws->pf_epoch;
  unsigned* tick = part == 2 ? ws->pf_ctrl + 1 + kPfMaxTiles * kPfMaxTiles : nullptr;
  const unsigned base = part == 2 ? ws->pf_base2 : ws->pf_base;
#ifdef MI_BA_AB_VARIANTS
  auto pick = [&](auto wm) {
    constexpr int W = decltype(wm)::value;
    return ws->tile_factor == 6   ? panel_factor_kernel<6, true, W>
           : ws->tile_factor == 3 ? panel_factor_kernel<3, true, W>
           : ws->tile_factor == 4 ? panel_factor_kernel<4, true, W>
           : ws->tile_factor == 5 ? panel_factor_kernel<5, true, W>
           : ws->tile_factor == 2 ? (ws->write_through ? panel_factor_kernel<2, true, W> : panel_factor_kernel<2, false, W>)
                                  : (ws->write_through ? panel_factor_kernel<1, true, W> : panel_factor_kernel<1, false, W>);
  };
  auto kern = ws->panel_wait == 3   ? pick(std::integral_constant<int, 3>{})
              : ws->panel_wait == 2 ? pick(std::integral_constant<int, 2>{})
              : ws->panel_wait == 1 ? pick(std::integral_constant<int, 1>{})
                                    : pick(std::integral_constant<int, 0>{});
#else
  // the tools build keeps the other tile factors / plain stores / wait modes for A/B.
  // Wait mode 2 (sc1 loads, no acquire) is the hand-off form measured for one
  // workgroup per CU (MI355X_MICROARCH.md §visibility): the kernel's registers
  // give one; should a build ever admit more, the acquire form (mode 1) runs.
  constexpr CholConfig kDef{};
  static const bool one_per_cu = blocks_per_cu(reinterpret_cast<const void*>(
                                                   &panel_factor_kernel<kDef.tile_factor, true, kDef.panel_wait>),
                                               256) == 1;
  auto kern = one_per_cu ? panel_factor_kernel<kDef.tile_factor, true, kDef.panel_wait>
                         : panel_factor_kernel<kDef.tile_factor, true, 1>;
#endif
  hipLaunchKernelGGL(kern, dim3(nr), dim3(256), 0, s, A + k + (size_t)k * lda, lda, kb, mrows, info, ws->pf_linv,
                     ws->pf_ctrl, base, epoch, ws->err, ws->spin_limit, groups, nullptr, part == 2 ? nc : 0, tick);
  (part == 2 ? ws->pf_base2 : ws->pf_base) += (unsigned)nr;
  return hipGetLastError() == hipSuccess ? rocblas_status_success : rocblas_status_internal_error;
}

#ifdef MI_BA_AB_VARIANTS
// own_diag 7 (tools build only): the two-kernel diagonal factor, then the panel solve
// A_ik <- A_ik L_kk^-T as one dgemm against the explicit inverse of the
// diagonal block (rocBLAS dtrtri) instead of a dtrsm: the panel solve runs at
// dgemm rate off a copy of the panel.
rocblas_status panel_factor_inv(rocblas_handle h, int n, double* A, int lda, int k, int kb, int* info,
                                double* scratch, CholWorkspace* ws, int ex) {
  if (!ws || !ws->tinv || !ws->tbuf || kb > kTinv || n - k - kb + ex > ws->tbuf_rows) return rocblas_status_invalid_pointer;
  double* Akk = A + k + (size_t)k * lda;
  rocblas_status st = potrf_leaf(h, kb, Akk, lda, info, 2, scratch);
  if (st != rocblas_status_success) return st;
  const int m = n - k - kb + ex;
  if (m == 0) return st;
  hipStream_t s;
  if (rocblas_get_stream(h, &s) != rocblas_status_success) return rocblas_status_internal_error;
  if (hipMemsetAsync(ws->tinv, 0, sizeof(double) * kb * kb, s) != hipSuccess) return rocblas_status_internal_error;
  st = rocblas_dtrtri(h, rocblas_fill_lower, rocblas_diagonal_non_unit, kb, Akk, lda, ws->tinv, kb);
  if (st != rocblas_status_success) return st;
  if (hipMemcpy2DAsync(ws->tbuf, sizeof(double) * m, Akk + kb, sizeof(double) * lda, sizeof(double) * m, kb,
                       hipMemcpyDeviceToDevice, s) != hipSuccess)
    return rocblas_status_internal_error;
  const double one = 1.0, zero = 0.0;
  return rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, m, kb, kb, &one, ws->tbuf, m, ws->tinv,
                       kb, &zero, Akk + kb, lda);
}
#endif

rocblas_status panel_factor(rocblas_handle h, int n, double* A, int lda, int k, int kb, int* info, int own,
                            double* scratch, CholWorkspace* ws, int ex) {
  if (own == 6) {
    hipStream_t s;
    if (rocblas_get_stream(h, &s) != rocblas_status_success) return rocblas_status_internal_error;
    return panel_factor_fused(s, n, A, lda, k, kb, info, ws, ex, 0);
  }
#ifdef MI_BA_AB_VARIANTS
  if (own == 7) return panel_factor_inv(h, n, A, lda, k, kb, info, scratch, ws, ex);
#endif
  double* Akk = A + k + (size_t)k * lda;
  rocblas_status st = potrf_leaf(h, kb, Akk, lda, info, own, scratch);
  if (st != rocblas_status_success) return st;
  const int m = n - k - kb + ex;
  if (m == 0) return st;
  const double one = 1.0;
  return rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                       rocblas_diagonal_non_unit, m, kb, &one, Akk, lda, Akk + kb, lda);
}

// C -= P P' for the trailing update (P: m rows of the panel, its first n
// rows' block column of C): rocBLAS dgemm, or rocblas_gemm_ex with an
// explicit Tensile solution index (CholConfig::gemm_solution); an index the
// library does not accept for the shape falls back to the default solution.
// Whether this rocBLAS build offers Tensile solution `sol` for the update's
// problem (rocblas_gemm_ex_get_solutions), asked once per (device, solution,
// shape): Tensile's offer depends on the problem size, so an index offered for
// one trailing-update shape is not assumed for another, and an index from
// another rocBLAS build is never tried twice for a shape (no failing
// rocblas_gemm_ex call, or log line, per trailing update).
static bool gemm_solution_offered(rocblas_handle h, int m, int n, int k, const double* P, int ldp, double* C, int ldc,
                                  int sol) {
  static std::mutex mu;
  static std::map<std::array<long long, 6>, bool> cache;
  int dev = -1;
  (void)hipGetDevice(&dev);
  const std::array<long long, 6> key{dev, sol, m, n, k, (long long)ldp * 1000003LL + ldc};
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  const double minus_one = -1.0, one = 1.0;
  rocblas_int size = 0;
  bool offered = false;
  if (rocblas_gemm_ex_get_solutions(h, rocblas_operation_none, rocblas_operation_transpose, m, n, k, &minus_one, P,
                                    rocblas_datatype_f64_r, ldp, P, rocblas_datatype_f64_r, ldp, &one, C,
                                    rocblas_datatype_f64_r, ldc, C, rocblas_datatype_f64_r, ldc, rocblas_datatype_f64_r,
                                    rocblas_gemm_algo_solution_index, 0, nullptr, &size) == rocblas_status_success &&
      size > 0) {
    std::vector<rocblas_int> list(size);
    if (rocblas_gemm_ex_get_solutions(h, rocblas_operation_none, rocblas_operation_transpose, m, n, k, &minus_one, P,
                                      rocblas_datatype_f64_r, ldp, P, rocblas_datatype_f64_r, ldp, &one, C,
                                      rocblas_datatype_f64_r, ldc, C, rocblas_datatype_f64_r, ldc,
                                      rocblas_datatype_f64_r, rocblas_gemm_algo_solution_index, 0, list.data(),
                                      &size) == rocblas_status_success)
      offered = std::find(list.begin(), list.begin() + size, sol) != list.begin() + size;
  }
  std::lock_guard<std::mutex> g(mu);
  cache[key] = offered;
  return offered;
}

rocblas_status gemm_nt(rocblas_handle h, int m, int n, int k, const double* P, int ldp, double* C, int ldc, int sol) {
  return gemm_nt2(h, m, n, k, P, P, ldp, C, ldc, sol);
}

// C -= Pa Pb' (m x n, K = k): the rows below a block column's diagonal block
// (split tail), Pa those rows of the panel, Pb the block column's rows of it
rocblas_status gemm_nt2(rocblas_handle h, int m, int n, int k, const double* Pa, const double* Pb, int ldp, double* C,
                        int ldc, int sol) {
  const double minus_one = -1.0, one = 1.0;
  if (sol != 0 && gemm_solution_offered(h, m, n, k, Pa, ldp, C, ldc, sol)) {
    const rocblas_status st = rocblas_gemm_ex(h, rocblas_operation_none, rocblas_operation_transpose, m, n, k,
                                              &minus_one, Pa, rocblas_datatype_f64_r, ldp, Pb, rocblas_datatype_f64_r,
                                              ldp, &one, C, rocblas_datatype_f64_r, ldc, C, rocblas_datatype_f64_r, ldc,
                                              rocblas_datatype_f64_r, rocblas_gemm_algo_solution_index, sol, 0);
    if (st == rocblas_status_success) return st;
  }
  return rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, m, n, k, &minus_one, Pa, ldp, Pb, ldp,
                       &one, C, ldc);
}

#ifdef MI_BA_AB_VARIANTS
// rest_update 4 (tools build: measured slower, 16.5-18.2 vs 15.1 ms with two
// update streams at nf = 11 993, profiles/r5g_ab_cholesky_batched_tiles.jsonl):
// the tile pointer tables of every panel's trailing update
// after the next panel's block column (CholWorkspace::bgroups / bptr), made
// once per (A, n, lda, ex, tile, panel schedule) and kept for the context's
// later factorisations.
static bool batch_tables(CholWorkspace& ws, const std::vector<int>& ps, int n, double* A, int lda, int ex, int tile,
                         hipStream_t s) {
  std::vector<long long> key{(long long)(uintptr_t)A, n, lda, ex, tile};
  key.insert(key.end(), ps.begin(), ps.end());
  if (key == ws.bkey && ws.bptr) return true;
  std::vector<double*> host;
  std::vector<CholWorkspace::TileGroup> groups;
  const int np = (int)ps.size() - 1;
  for (int kk = 0; kk < np; ++kk) {
    const int k = ps[kk], kb = ps[kk + 1] - k, m = n - k - kb;
    const int jb0 = kk + 2 < (int)ps.size() ? ps[kk + 2] - ps[kk + 1] : 0;
    double* Aik = A + k + kb + (size_t)k * lda;
    double* T = Aik + (size_t)kb * lda;
    const int R = m - jb0;
    const int nt = R > 0 ? (R + tile - 1) / tile : 0;
    const int last = nt > 0 ? R - (nt - 1) * tile : 0;
    // full tiles: every (ti >= tj) when the last tile is full, else those above the last tile row
    const int nfull_rows = last == tile ? nt : nt - 1;
    auto add = [&](int m_, int n_, const std::vector<std::pair<int, int>>& tiles) {
      CholWorkspace::TileGroup g{(int)host.size(), (int)tiles.size(), m_, n_};
      for (auto& ij : tiles) host.push_back(Aik + jb0 + (size_t)ij.first * tile);
      for (auto& ij : tiles) host.push_back(Aik + jb0 + (size_t)ij.second * tile);
      for (auto& ij : tiles)
        host.push_back(T + jb0 + (size_t)ij.first * tile + (size_t)(jb0 + (size_t)ij.second * tile) * lda);
      groups.push_back(g);
    };
    std::vector<std::pair<int, int>> full, row, corner;
    for (int tj = 0; tj < nt; ++tj)
      for (int ti = tj; ti < nt; ++ti) {
        if (ti < nfull_rows) full.push_back({ti, tj});
        else if (tj < nt - 1) row.push_back({ti, tj});
        else corner.push_back({ti, tj});
      }
    add(tile, tile, full);
    add(last, tile, row);
    add(last, last, corner);
  }
  if (host.size() > ws.bptr_cap) {
    if (ws.bptr) (void)hipFree(ws.bptr);
    ws.bptr = nullptr;
    ws.bptr_cap = 0;
    if (hipMalloc(&ws.bptr, host.size() * sizeof(double*)) != hipSuccess) {
      ws.bptr = nullptr;
      return false;
    }
    ws.bptr_cap = host.size();
  }
  // (pageable source: wait for the copy before the vector goes)
  if (!host.empty() && (hipMemcpyAsync(ws.bptr, host.data(), host.size() * sizeof(double*), hipMemcpyHostToDevice, s) !=
                            hipSuccess ||
                        hipStreamSynchronize(s) != hipSuccess))
    return false;
  ws.bgroups = std::move(groups);
  ws.bkey = std::move(key);
  return true;
}
#endif

rocblas_status factor_lookahead(rocblas_handle h, int n, double* A, int lda, int* info, const CholConfig& cfg,
                                CholWorkspace& ws, int ex) {
  [[maybe_unused]] const double minus_one = -1.0, one = 1.0;  // rest_update 1 / 2 (tools build)
  const int nb = cfg.panel;
  hipStream_t s1;
  if (rocblas_get_stream(h, &s1) != rocblas_status_success) return rocblas_status_internal_error;
  const std::vector<int> ps = chol_panel_starts(n, cfg);
  if (ws.ev.size() < 2 * (ps.size() - 1)) return rocblas_status_invalid_size;
  double* scratch_main = ws.scratch;
  double* scratch_side = ws.scratch + kSub * kSub;
  auto own_for = [&](int k0) { return cfg.head_own > 0 && k0 < cfg.head_own_cols ? cfg.head_own : cfg.own_diag; };
#ifdef MI_BA_AB_VARIANTS
  const bool batched = cfg.rest_update == 4 && cfg.batch_tile > 0;
  if (batched && !batch_tables(ws, ps, n, A, lda, ex, cfg.batch_tile, s1)) return rocblas_status_internal_error;
#endif
  rocblas_status st = panel_factor(h, n, A, lda, 0, ps[1], info, own_for(0), scratch_main, &ws, ex);
  if (st != rocblas_status_success) return st;
  ws.col_rec = -1;
  // On a failure after the side stream got work, the caller's stream waits
  // for it (the caller may free A / info once its own stream is drained).
  // split head (CholConfig::split_cus): the panel factor and the trailing
  // dgemm on disjoint CU sets while the panel starts before split_cols
  const bool split_ok = cfg.split_cus > 0 && ws.split_n > 0 && ws.split_side_h && ws.split_main_h;
  rocblas_handle hm = h, hs = ws.side_h;
  hipStream_t sm = s1, ss = ws.side;
  // rest_streams k > 1 (not inside the split head): block columns dealt
  // round-robin over the dgemm stream and ws.rest_s[0 .. k-2], forked after
  // the next panel's block column and joined before the next iteration
  const int nrest = cfg.rest_streams > 1 && ws.rest_n == cfg.rest_streams &&
                            ws.ev_rest.size() >= (size_t)CholWorkspace::kMaxRest * (ws.ev.size() / 2)
                        ? cfg.rest_streams
                        : 1;
  auto fail = [&](rocblas_status e) {
    for (int r = 0; r + 1 < nrest; ++r) (void)hipStreamSynchronize(ws.rest_s[r]);
    if (ws.side2) (void)hipStreamSynchronize(ws.side2);
    if (split_ok) {
      (void)hipStreamSynchronize(ws.split_side);
      (void)hipStreamSynchronize(ws.split_main);
    }
    hipEvent_t last = ws.ev.back();
    if (hipEventRecord(last, ws.side) != hipSuccess || hipStreamWaitEvent(s1, last, 0) != hipSuccess)
      (void)hipStreamSynchronize(ws.side);
    return e;
  };
  for (int kk = 0; kk + 1 < (int)ps.size(); ++kk) {
    const int k = ps[kk], kb = ps[kk + 1] - k;
    const int m = n - k - kb;
    if (m == 0) break;
    const bool want = split_ok && k < cfg.split_cols;
    if (want && sm == s1) {  // into the split: the dgemm stream follows the caller's stream
      if (hipEventRecord(ws.ev_split[0], s1) != hipSuccess || hipStreamWaitEvent(ws.split_main, ws.ev_split[0], 0))
        return fail(rocblas_status_internal_error);
      hm = ws.split_main_h;
      hs = ws.split_side_h;
      sm = ws.split_main;
      ss = ws.split_side;
    } else if (!want && sm != s1) {  // out of it: the caller's stream follows the dgemm stream
      if (hipEventRecord(ws.ev_split[1], sm) != hipSuccess || hipStreamWaitEvent(s1, ws.ev_split[1], 0))
        return fail(rocblas_status_internal_error);
      hm = h;
      hs = ws.side_h;
      sm = s1;
      ss = ws.side;
    }
    double* Aik = A + k + kb + (size_t)k * lda;  // panel k below its diagonal block
    double* T = Aik + (size_t)kb * lda;          // trailing matrix, lower triangle
    // block column k+1 (the next panel) first
    const int jb0 = ps[kk + 2] - ps[kk + 1];
    hipEvent_t upd = ws.ev[2 * kk], pan = ws.ev[2 * kk + 1];
    // split tail: the diagonal block's rows of block column k+1, the panel's
    // diagonal-block rows on the side stream, then the rows below and the
    // panel's below-diagonal rows on side2 (factor_blocked: the same dgemms)
    hipStream_t s2 = cfg.split_tail_rest ? (nrest > 1 ? ws.rest_s[0] : nullptr) : ws.side2;
    const bool split = split_tail(cfg, ps, kk, n, ex) && sm == s1 && own_for(k + kb) == 6 && s2 &&
                       ws.ev2.size() >= 2 * (size_t)(kk + 1);
    if (split) {
      st = gemm_nt(hm, jb0, jb0, kb, Aik, lda, T, lda, cfg.gemm_solution);
      if (st != rocblas_status_success) return fail(st);
      if (hipEventRecord(upd, sm) != hipSuccess || hipStreamWaitEvent(ss, upd, 0) != hipSuccess)
        return fail(rocblas_status_internal_error);
      st = panel_factor_fused(ss, n, A, lda, k + kb, jb0, info + kk + 1, &ws, ex, 1);
      if (st != rocblas_status_success) return fail(st);
      st = gemm_nt2(hm, m + ex - jb0, jb0, kb, Aik + jb0, Aik, lda, T + jb0, lda, cfg.gemm_solution);
      if (st != rocblas_status_success) return fail(st);
      hipEvent_t upd2 = ws.ev2[2 * kk], pan2 = ws.ev2[2 * kk + 1];
      if (hipEventRecord(upd2, sm) != hipSuccess || hipStreamWaitEvent(s2, upd2, 0) != hipSuccess)
        return fail(rocblas_status_internal_error);
      st = panel_factor_fused(s2, n, A, lda, k + kb, jb0, info + kk + 1, &ws, ex, 2);
      if (st != rocblas_status_success) return fail(st);
      if (hipEventRecord(pan2, s2) != hipSuccess || hipStreamWaitEvent(ss, pan2, 0) != hipSuccess)
        return fail(rocblas_status_internal_error);
      if (hipEventRecord(pan, ss) != hipSuccess) return fail(rocblas_status_internal_error);
    }
#ifdef MI_BA_AB_VARIANTS
    const bool serial = !split && cfg.serial_head_cols > 0 && k + kb < cfg.serial_head_cols;
#else
    constexpr bool serial = false;
#endif
    // look-ahead dgemm on the side stream (CholConfig::la_side_from): after
    // panel k there (stream order) and the previous iteration's first
    // block-column dgemm (ev_col), which brought block column k+1 up to date
    const bool la_side = cfg.la_side_from >= 0 && kk >= 1 && k >= cfg.la_side_from && sm == s1 && !split &&
                         !serial && ws.ev_col.size() > (size_t)kk && ws.col_rec == kk - 1 &&
                         jb0 <= (cfg.rest_update == 3 ? 2 * nb : nb);
    if (!split) {
      if (la_side && hipStreamWaitEvent(ss, ws.ev_col[kk - 1], 0) != hipSuccess)
        return fail(rocblas_status_internal_error);
      st = gemm_nt(la_side ? hs : hm, m + ex, jb0, kb, Aik, lda, T, lda, cfg.gemm_solution);
      if (st != rocblas_status_success) return fail(st);
    }
    auto launch_panel = [&]() -> rocblas_status {
      if (!la_side && (hipEventRecord(upd, sm) != hipSuccess || hipStreamWaitEvent(ss, upd, 0) != hipSuccess))
        return rocblas_status_internal_error;
      rocblas_status ps_;
      if (cfg.split_panel_cols > 0 && k + kb < cfg.split_panel_cols && own_for(k + kb) == 6) {
        // split panel (CholConfig::split_panel_cols): the diagonal block's row
        // tiles, then the rows below them, one launch after the other on the
        // side stream (the same kernel and flags: bitwise the one-launch factor)
        ps_ = panel_factor_fused(ss, n, A, lda, k + kb, jb0, info + kk + 1, &ws, ex, 1);
        if (ps_ == rocblas_status_success) ps_ = panel_factor_fused(ss, n, A, lda, k + kb, jb0, info + kk + 1, &ws, ex, 2);
      } else {
        ps_ = panel_factor(hs, n, A, lda, k + kb, jb0, info + kk + 1, own_for(k + kb), scratch_side, &ws, ex);
      }
      if (ps_ != rocblas_status_success) return ps_;
      return hipEventRecord(pan, ss) == hipSuccess ? rocblas_status_success : rocblas_status_internal_error;
    };
    if (!split && !serial) {
      st = launch_panel();
      if (st != rocblas_status_success) return fail(st);
    }
    // the rest of the trailing lower triangle (columns jb0 .. m)
    [[maybe_unused]] const int mr = m - jb0;
#ifdef MI_BA_AB_VARIANTS
    if (mr > 0 && cfg.rest_update == 1 && ex == 0) {
      st = rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, mr, kb, &minus_one, Aik + jb0, lda, &one,
                         T + jb0 + (size_t)jb0 * lda, lda);
      if (st != rocblas_status_success) return fail(st);
    } else if (mr > 0 && cfg.rest_update == 2 && ex == 0) {
      st = rocblas_dgemmt(h, rocblas_fill_lower, rocblas_operation_none, rocblas_operation_transpose, mr, kb,
                          &minus_one, Aik + jb0, lda, Aik + jb0, lda, &one, T + jb0 + (size_t)jb0 * lda, lda);
      if (st != rocblas_status_success) return fail(st);
    } else if (batched && sm == s1) {
      for (int g = 0; g < 3; ++g) {
        const CholWorkspace::TileGroup& tg = ws.bgroups[3 * (size_t)kk + g];
        if (tg.count == 0) continue;
        double** pa = ws.bptr + tg.off;
        st = rocblas_dgemm_batched(hm, rocblas_operation_none, rocblas_operation_transpose, tg.m, tg.n, kb, &minus_one,
                                   pa, lda, pa + tg.count, lda, &one, pa + 2 * tg.count, lda, tg.count);
        if (st != rocblas_status_success) return fail(st);
      }
      // the carried rows below the matrix (the forward solve's row n)
      if (ex > 0 && mr > 0) {
        st = rocblas_dgemm(hm, rocblas_operation_none, rocblas_operation_transpose, ex, mr, kb, &minus_one, Aik + m, lda,
                           Aik + jb0, lda, &one, T + m + (size_t)jb0 * lda, lda);
        if (st != rocblas_status_success) return fail(st);
      }
    } else
#endif
    {
      // block columns of width nb (rest_update 0) or 2 nb (3)
      const int cw = cfg.rest_update == 3 ? 2 * nb : nb;
      // streams used this panel: no more than its block columns
      const int ns = sm == s1 && !(split && cfg.split_tail_rest) ? std::min(nrest, (mr + cw - 1) / cw) : 1;
      hipEvent_t* evr = ns > 1 ? ws.ev_rest.data() + (size_t)CholWorkspace::kMaxRest * kk : nullptr;
      if (ns > 1) {
        if (hipEventRecord(evr[0], sm) != hipSuccess) return fail(rocblas_status_internal_error);
        for (int r = 0; r + 1 < ns; ++r)
          if (hipStreamWaitEvent(ws.rest_s[r], evr[0], 0) != hipSuccess) return fail(rocblas_status_internal_error);
      }
      // the first block column as wide as the panel after next
      // (CholConfig::rest_first_panel): the one the next look-ahead waits for
      const int fw = cfg.rest_first_panel && kk + 3 < (int)ps.size() ? ps[kk + 3] - ps[kk + 2] : cw;
      int c = 0;
      for (int j = jb0; j < m; j += c == 0 ? fw : cw, ++c) {
        const int jb = std::min(c == 0 ? fw : cw, m - j);
        const int r = c % ns;
        st = gemm_nt(r ? ws.rest_h[r - 1] : hm, m - j + ex, jb, kb, Aik + j, lda, T + j + (size_t)j * lda, lda,
                     cfg.gemm_solution);
        if (st != rocblas_status_success) return fail(st);
        // the next panel's block column is this first dgemm's (la_side_from)
        if (c == 0 && cfg.la_side_from >= 0 && sm == s1 && ws.ev_col.size() > (size_t)kk) {
          if (hipEventRecord(ws.ev_col[kk], sm) != hipSuccess) return fail(rocblas_status_internal_error);
          ws.col_rec = kk;
        }
      }
      for (int r = 0; r + 1 < ns; ++r)
        if (hipEventRecord(evr[1 + r], ws.rest_s[r]) != hipSuccess || hipStreamWaitEvent(sm, evr[1 + r], 0) != hipSuccess)
          return fail(rocblas_status_internal_error);
    }
    if (serial) {  // after the whole trailing update (joined into sm above)
      st = launch_panel();
      if (st != rocblas_status_success) return fail(st);
    }
    // panel k+1 is read by the next iteration's updates (and by the solve)
    if (hipStreamWaitEvent(sm, pan, 0) != hipSuccess) return fail(rocblas_status_internal_error);
  }
  if (sm != s1 && (hipEventRecord(ws.ev_split[2], sm) != hipSuccess || hipStreamWaitEvent(s1, ws.ev_split[2], 0)))
    return fail(rocblas_status_internal_error);
  return rocblas_status_success;
}

}  // namespace

std::vector<int> chol_panel_starts(int n, const CholConfig& cfg) {
  std::vector<int> ps;
  for (int k = 0; k < n;) {
    ps.push_back(k);
    int w = cfg.panel;
    if (cfg.tail_panel > 0 && n - k <= cfg.tail_cols) w = cfg.tail_panel;
    else if (cfg.head_panel > 0 && k < cfg.head_cols) w = cfg.head_panel;
    k += std::min(std::max(w, 1), n - k);
  }
  ps.push_back(n);
  return ps;
}

int chol_leaf_count(int n, const CholConfig& cfg) {
  if (n <= 0) return 1;
  return cfg.panel > 0 ? (int)chol_panel_starts(n, cfg).size() - 1 : leaves(n);
}

bool CholWorkspace::create(int dev, int max_panels, int max_n) {
  destroy();
  device = dev;
  if (hipSetDevice(dev) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&clock_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) clock_khz = 0;
  spin_limit = wait_ticks(CholConfig{}.wait_ms);
  // The side stream carries the look-ahead's critical path (diagonal factor +
  // panel dtrsm).  A higher priority puts it on a hardware queue of its own:
  // with HIP's round-robin stream -> queue mapping (4 queues per process), a
  // normal-priority side stream can share the main stream's queue when other
  // streams exist in the process (torch, a second context), which serialises
  // the look-ahead (30.6 -> 34.6 ms at nf = 12 000).
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = least = 0;
  if (hipStreamCreateWithPriority(&side, hipStreamNonBlocking, greatest) != hipSuccess) {
    side = nullptr;
    return false;
  }
  side_cus = 0;
  if (rocblas_create_handle(&side_h) != rocblas_status_success) { side_h = nullptr; return false; }
  if (rocblas_set_stream(side_h, side) != rocblas_status_success) return false;
  for (int k = 0; k < 2 * std::max(1, max_panels); ++k) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return false;
    ev.push_back(e);
  }
  for (int k = 0; k < std::max(1, max_panels); ++k) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return false;
    ev_col.push_back(e);
  }
  if (hipMalloc(&scratch, 2 * sizeof(double) * kSub * kSub) != hipSuccess) { scratch = nullptr; return false; }
  const int nblk = (std::max(0, max_n) + kTB - 1) / kTB;
  if (nblk > 0) {
    if (hipMalloc(&linv, sizeof(double) * kTB * kTB * (size_t)nblk) != hipSuccess) { linv = nullptr; return false; }
    if (hipMalloc(&ybuf, sizeof(double) * kTB * (size_t)nblk) != hipSuccess) { ybuf = nullptr; return false; }
    // stream-ordered zero fills, complete before the workspace is used (a
    // null-stream memset is not ordered against the non-blocking streams)
    if (hipMemsetAsync(linv, 0, sizeof(double) * kTB * kTB * (size_t)nblk, side) != hipSuccess) return false;
    if (hipMalloc(&ctrl, sizeof(unsigned) * (2 + (size_t)nblk)) != hipSuccess) { ctrl = nullptr; return false; }
    if (hipMalloc(&pf_ctrl, sizeof(unsigned) * (2 + kPfMaxTiles * kPfMaxTiles)) != hipSuccess) {
      pf_ctrl = nullptr;
      return false;
    }
    if (hipMemsetAsync(pf_ctrl, 0, sizeof(unsigned) * (2 + kPfMaxTiles * kPfMaxTiles), side) != hipSuccess)
      return false;
    if (hipMalloc(&pf_linv, sizeof(double) * 64 * 64 * kPfMaxTiles) != hipSuccess) { pf_linv = nullptr; return false; }
    pf_base = 0;
    pf_base2 = 0;
    pf_epoch = 0;
    if (hipMemsetAsync(ctrl, 0, sizeof(unsigned) * (2 + (size_t)nblk), side) != hipSuccess) return false;
    if (hipMalloc(&err, 4 * sizeof(unsigned)) != hipSuccess) { err = nullptr; return false; }
    if (hipMemsetAsync(err, 0, 4 * sizeof(unsigned), side) != hipSuccess) return false;
#ifdef MI_BA_AB_VARIANTS
    if (hipMalloc(&tinv, sizeof(double) * kTinv * kTinv) != hipSuccess) { tinv = nullptr; return false; }
    if (hipMalloc(&tbuf, sizeof(double) * kTinv * (size_t)nblk * kTB) != hipSuccess) { tbuf = nullptr; return false; }
    tbuf_rows = nblk * kTB;
#endif
    if (hipStreamSynchronize(side) != hipSuccess) return false;
    epoch = 0;
    linv_rows = nblk * kTB;
  }
  return true;
}

bool CholWorkspace::set_side_cus(int ncu) {
  if (!side || !side_h) return false;
  if (hipStreamSynchronize(side) != hipSuccess) return false;
  hipStream_t ns = nullptr;
  if (ncu > 0) {
    int total = 0;
    if (hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || total <= 0)
      return false;
    ncu = std::min(ncu, total);
    std::vector<uint32_t> mask((total + 31) / 32, 0u);
    for (int k = 0; k < ncu; ++k) {
      const int cu = (int)((int64_t)k * total / ncu);
      mask[cu / 32] |= 1u << (cu % 32);
    }
    if (hipExtStreamCreateWithCUMask(&ns, (uint32_t)mask.size(), mask.data()) != hipSuccess) return false;
  } else {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = least = 0;
    if (hipStreamCreateWithPriority(&ns, hipStreamNonBlocking, greatest) != hipSuccess) return false;
  }
  if (rocblas_set_stream(side_h, ns) != rocblas_status_success) {
    (void)hipStreamDestroy(ns);
    return false;
  }
  (void)hipStreamDestroy(side);
  side = ns;
  side_cus = ncu;
  return true;
}

bool CholWorkspace::ensure(int dev, int max_panels, int max_n) {
  const int nblk = (std::max(0, max_n) + kTB - 1) / kTB;
  if (side && device == dev && (int)ev.size() >= 2 * std::max(1, max_panels) && linv_rows >= nblk * kTB) return true;
  return create(dev, max_panels, max_n);
}

bool CholWorkspace::set_split_cus(int ncu) {
  const int req = ncu;
  if (split_side) (void)hipStreamSynchronize(split_side);
  if (split_main) (void)hipStreamSynchronize(split_main);
  if (split_side_h) (void)rocblas_destroy_handle(split_side_h);
  if (split_main_h) (void)rocblas_destroy_handle(split_main_h);
  if (split_side) (void)hipStreamDestroy(split_side);
  if (split_main) (void)hipStreamDestroy(split_main);
  for (hipEvent_t& e : ev_split) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
  }
  split_side = split_main = nullptr;
  split_side_h = split_main_h = nullptr;
  split_n = 0;
  if (ncu <= 0) return true;
  if (hipSetDevice(device) != hipSuccess) return false;
  int total = 0;
  if (hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || total <= 1)
    return false;
  ncu = std::min(ncu, total - 1);
  std::vector<uint32_t> ms((total + 31) / 32, 0u), mm((total + 31) / 32, 0u);
  std::vector<char> in(total, 0);
  for (int k = 0; k < ncu; ++k) in[(int)((int64_t)k * total / ncu)] = 1;
  for (int cu = 0; cu < total; ++cu) (in[cu] ? ms : mm)[cu / 32] |= 1u << (cu % 32);
  if (hipExtStreamCreateWithCUMask(&split_side, (uint32_t)ms.size(), ms.data()) != hipSuccess) {
    split_side = nullptr;
    return false;
  }
  if (hipExtStreamCreateWithCUMask(&split_main, (uint32_t)mm.size(), mm.data()) != hipSuccess) {
    split_main = nullptr;
    return false;
  }
  if (rocblas_create_handle(&split_side_h) != rocblas_status_success) { split_side_h = nullptr; return false; }
  if (rocblas_create_handle(&split_main_h) != rocblas_status_success) { split_main_h = nullptr; return false; }
  if (rocblas_set_stream(split_side_h, split_side) != rocblas_status_success ||
      rocblas_set_stream(split_main_h, split_main) != rocblas_status_success)
    return false;
  for (hipEvent_t& e : ev_split)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      e = nullptr;
      return false;
    }
  split_n = req;
  return true;
}

bool CholWorkspace::set_rest_streams(int k, bool cumask, int priority) {
  for (int r = 0; r + 1 < kMaxRest; ++r) {
    if (rest_s[r]) (void)hipStreamSynchronize(rest_s[r]);
    if (rest_h[r]) (void)rocblas_destroy_handle(rest_h[r]);
    if (rest_s[r]) (void)hipStreamDestroy(rest_s[r]);
    rest_s[r] = nullptr;
    rest_h[r] = nullptr;
  }
  for (hipEvent_t e : ev_rest) (void)hipEventDestroy(e);
  ev_rest.clear();
  rest_n = 1;
  rest_cumask = false;
  rest_priority = 0;
  if (k <= 1) return true;
  if (k > kMaxRest || hipSetDevice(device) != hipSuccess) return false;
  std::vector<uint32_t> all;
  if (cumask) {
    int total = 0;
    if (hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || total <= 0)
      return false;
    all.assign((total + 31) / 32, 0u);
    for (int cu = 0; cu < total; ++cu) all[cu / 32] |= 1u << (cu % 32);
  }
  for (int r = 0; r + 1 < k; ++r) {
    int least = 0, greatest = 0;
    if (priority && hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = least = 0;
    const hipError_t e =
        cumask     ? hipExtStreamCreateWithCUMask(&rest_s[r], (uint32_t)all.size(), all.data())
        : priority ? hipStreamCreateWithPriority(&rest_s[r], hipStreamNonBlocking, priority == 1 ? greatest : least)
                   : hipStreamCreateWithFlags(&rest_s[r], hipStreamNonBlocking);
    if (e != hipSuccess) {
      rest_s[r] = nullptr;
      return false;
    }
    if (rocblas_create_handle(&rest_h[r]) != rocblas_status_success) {
      rest_h[r] = nullptr;
      return false;
    }
    if (rocblas_set_stream(rest_h[r], rest_s[r]) != rocblas_status_success) return false;
  }
  for (size_t i = 0; i < (size_t)kMaxRest * (ev.size() / 2); ++i) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return false;
    ev_rest.push_back(e);
  }
  rest_n = k;
  rest_cumask = cumask;
  rest_priority = priority;
  return true;
}

// split tail: the below-rows stream (the side stream's priority: a hardware
// queue of its own) and its events, made on first use
bool CholWorkspace::ensure_side2(int max_panels, bool stream) {
  if (stream && !side2) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = least = 0;
    if (hipStreamCreateWithPriority(&side2, hipStreamNonBlocking, greatest) != hipSuccess) {
      side2 = nullptr;
      return false;
    }
  }
  while (ev2.size() < 2 * (size_t)std::max(1, max_panels)) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return false;
    ev2.push_back(e);
  }
  return true;
}

void CholWorkspace::destroy() {
  if (device >= 0) (void)hipSetDevice(device);
  if (side) (void)hipStreamSynchronize(side);
  if (side2) (void)hipStreamSynchronize(side2);
  for (hipEvent_t e : ev2) (void)hipEventDestroy(e);
  ev2.clear();
  if (side2) (void)hipStreamDestroy(side2);
  side2 = nullptr;
  if (split_n > 0 || split_side || split_main) (void)set_split_cus(0);
  if (rest_s[0] || rest_n != 1) (void)set_rest_streams(1);
  for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  ev.clear();
  for (hipEvent_t e : ev_col) (void)hipEventDestroy(e);
  ev_col.clear();
  if (side_h) (void)rocblas_destroy_handle(side_h);
  side_h = nullptr;
  if (side) (void)hipStreamDestroy(side);
  side = nullptr;
  if (scratch) (void)hipFree(scratch);
  scratch = nullptr;
  if (linv) (void)hipFree(linv);
  linv = nullptr;
  if (ybuf) (void)hipFree(ybuf);
  ybuf = nullptr;
  if (ctrl) (void)hipFree(ctrl);
  ctrl = nullptr;
  if (pf_ctrl) (void)hipFree(pf_ctrl);
  pf_ctrl = nullptr;
  if (pf_linv) (void)hipFree(pf_linv);
  pf_linv = nullptr;
  if (tinv) (void)hipFree(tinv);
  tinv = nullptr;
  if (tbuf) (void)hipFree(tbuf);
  tbuf = nullptr;
  if (err) (void)hipFree(err);
  err = nullptr;
  if (bptr) (void)hipFree(bptr);
  bptr = nullptr;
  bptr_cap = 0;
  bkey.clear();
  bgroups.clear();
  tbuf_rows = 0;
  linv_rows = 0;
}

rocblas_status chol_factor(rocblas_handle h, int n, double* A, int lda, int* info, const CholConfig& cfg,
                           CholWorkspace* ws, int extra_rows) {
  if (n <= 0) return rocblas_status_success;
  if (extra_rows < 0 || lda < n + extra_rows || (extra_rows > 0 && cfg.panel <= 0)) return rocblas_status_invalid_size;
  if (cfg.own_diag && (!ws || !ws->scratch)) return rocblas_status_invalid_pointer;
  // the one-launch panel factor needs panels of at most 8 tiles: other panel
  // widths (and the recursive split) take the two-kernel diagonal factor
  CholConfig c = cfg;
  const int widest = std::max({c.panel, c.head_panel, c.tail_panel});
  if (c.own_diag == 6 && (c.panel <= 0 || widest > 64 * kPfMaxTiles)) c.own_diag = 2;
  if (c.head_own == 6 && (c.panel <= 0 || widest > 64 * kPfMaxTiles)) c.head_own = 2;
#ifdef MI_BA_AB_VARIANTS
  if (c.own_diag == 7 && (c.panel <= 0 || c.panel > kTinv)) c.own_diag = 2;
#else
  if (c.own_diag == 7) c.own_diag = 2;  // own_diag 7 is in the tools build only
#endif
  if (ws) {
#ifdef MI_BA_AB_VARIANTS
    if (c.split_tail_cols > 0 && c.own_diag == 6 && c.lookahead &&
        !ws->ensure_side2((int)chol_panel_starts(n, c).size(), !c.split_tail_rest))
      return rocblas_status_internal_error;
#endif
    ws->tile_factor = c.tile_factor;
    ws->write_through = c.write_through;
    ws->panel_wait = c.panel_wait;
    ws->solve_sc1 = c.solve_sc1;
    ws->spin_limit = c.spin_log2 <= 0 ? 0u : ws->wait_ticks(c.wait_ms);
    ws->rows_per_group = c.panel_rows_per_group;
    ws->bwd_pairs = c.bwd_pairs;
    ws->group_min_rows = c.panel_group_min_rows;
    if (ws->side && c.side_cus != ws->side_cus && !ws->set_side_cus(c.side_cus))
      return rocblas_status_internal_error;
    if (ws->side && c.split_cus != ws->split_n && !ws->set_split_cus(c.split_cus))
      return rocblas_status_internal_error;
    const int want_rest = std::min(std::max(c.rest_streams, 1), (int)CholWorkspace::kMaxRest);
    // (re)made when the count changes or the panel events outgrew them (create() re-makes ev)
    if (ws->side && (want_rest != ws->rest_n ||
                     (want_rest > 1 && (c.rest_cumask != ws->rest_cumask || c.rest_priority != ws->rest_priority)) ||
                     (want_rest > 1 && ws->ev_rest.size() < (size_t)CholWorkspace::kMaxRest * (ws->ev.size() / 2))) &&
        !ws->set_rest_streams(want_rest, c.rest_cumask, c.rest_priority))
      return rocblas_status_internal_error;
  }
  double* scratch = ws ? ws->scratch : nullptr;
  if (c.panel > 0 && c.gemm_update && c.lookahead && ws && ws->side)
    return factor_lookahead(h, n, A, lda, info, c, *ws, extra_rows);
  if (c.panel > 0) return factor_blocked(h, n, A, lda, info, c, scratch, ws, extra_rows);
  return factor(h, n, A, lda, info, c.own_diag, scratch);
}

hipError_t chol_error(CholWorkspace* ws, hipStream_t s, unsigned* word) {
  *word = 0;
  if (!ws || !ws->err) return hipSuccess;
  unsigned h = 0;
  hipError_t e = hipMemcpyAsync(&h, ws->err, sizeof(unsigned), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess && h != 0) e = hipMemsetAsync(ws->err, 0, sizeof(unsigned), s);
  if (e == hipSuccess) *word = h;
  return e;
}

rocblas_status chol_solve_backward(rocblas_handle h, int n, const double* A, int lda, double* x, CholWorkspace* ws) {
  if (n <= 0) return rocblas_status_success;
  if (!ws || !ws->ctrl || !ws->err || n > ws->linv_rows) return rocblas_status_invalid_pointer;
  hipStream_t s;
  if (rocblas_get_stream(h, &s) != rocblas_status_success) return rocblas_status_internal_error;
  if (ws->epoch > 0xfffffff0u) {
    if (hipMemsetAsync(ws->ctrl, 0, sizeof(unsigned) * (2 + (size_t)ws->linv_rows / kTB), s) != hipSuccess)
      return rocblas_status_internal_error;
    ws->epoch = 0;
  }
  if (hipMemsetAsync(ws->ctrl + 1, 0, sizeof(unsigned), s) != hipSuccess) return rocblas_status_internal_error;
  const unsigned e = ++ws->epoch;
  const int nblk = (n + kTB - 1) / kTB;
#ifdef MI_BA_AB_VARIANTS
  if (ws->bwd_pairs)
    hipLaunchKernelGGL(trsv_bwd_pair_kernel, dim3((nblk + 1) / 2), dim3(256), 0, s, A, lda, n, x, ws->ctrl, e, ws->err,
                       ws->spin_limit);
  else
#endif
    hipLaunchKernelGGL((ws->solve_sc1 && sweep_sc1_ok() ? trsv_sweep_kernel<false, true> : trsv_sweep_kernel<false, false>), dim3(nblk),
                       dim3(64 * kSweepWaves), 0, s, A, lda, n, x, ws->ctrl, e, ws->err, ws->spin_limit);
  return hipGetLastError() == hipSuccess ? rocblas_status_success : rocblas_status_internal_error;
}

rocblas_status chol_solve(rocblas_handle h, int n, const double* A, int lda, double* x, int variant,
                          CholWorkspace* ws) {
  if (n <= 0) return rocblas_status_success;
  if (variant == 0) {
    rocblas_status st = forward(h, n, A, lda, x);
    if (st != rocblas_status_success) return st;
    return backward(h, n, A, lda, x);
  }
  if (!ws || !ws->linv || !ws->ybuf || n > ws->linv_rows) return rocblas_status_invalid_pointer;
  hipStream_t s;
  if (rocblas_get_stream(h, &s) != rocblas_status_success) return rocblas_status_internal_error;
  if (variant == 2) {
    if (!ws->ctrl || !ws->err) return rocblas_status_invalid_pointer;
    // tickets reset; the flags carry the sweep's epoch (no reset needed)
    if (ws->epoch > 0xfffffff0u) {
      if (hipMemsetAsync(ws->ctrl, 0, sizeof(unsigned) * (2 + (size_t)ws->linv_rows / kTB), s) != hipSuccess)
        return rocblas_status_internal_error;
      ws->epoch = 0;
    }
    if (hipMemsetAsync(ws->ctrl, 0, 2 * sizeof(unsigned), s) != hipSuccess) return rocblas_status_internal_error;
    const unsigned e = ++ws->epoch;
    const unsigned e2 = ++ws->epoch;
    const int nblk = (n + kTB - 1) / kTB;
    hipLaunchKernelGGL((ws->solve_sc1 && sweep_sc1_ok() ? trsv_sweep_kernel<true, true> : trsv_sweep_kernel<true, false>), dim3(nblk),
                       dim3(64 * kSweepWaves), 0, s, A, lda, n, x, ws->ctrl, e, ws->err, ws->spin_limit);
    hipLaunchKernelGGL((ws->solve_sc1 && sweep_sc1_ok() ? trsv_sweep_kernel<false, true> : trsv_sweep_kernel<false, false>), dim3(nblk),
                       dim3(64 * kSweepWaves), 0, s, A, lda, n, x, ws->ctrl, e2, ws->err, ws->spin_limit);
    return hipGetLastError() == hipSuccess ? rocblas_status_success : rocblas_status_internal_error;
  }
  // inverses of the diagonal blocks (full blocks in one batched call, the
  // ragged last block on its own)
  const int nfull = n / kTB, tail = n - nfull * kTB;
  if (nfull > 0) {
    rocblas_status st = rocblas_dtrtri_strided_batched(h, rocblas_fill_lower, rocblas_diagonal_non_unit, kTB, A, lda,
                                                       (rocblas_stride)kTB * (lda + 1), ws->linv, kTB,
                                                       (rocblas_stride)kTB * kTB, nfull);
    if (st != rocblas_status_success) return st;
  }
  if (tail > 0) {
    rocblas_status st = rocblas_dtrtri(h, rocblas_fill_lower, rocblas_diagonal_non_unit, tail,
                                       A + (size_t)nfull * kTB * (lda + 1), lda, ws->linv + (size_t)nfull * kTB * kTB,
                                       kTB);
    if (st != rocblas_status_success) return st;
  }
  for (int k0 = 0; k0 < n; k0 += kTB) {
    const int w = std::min(kTB, n - k0);
    const int g = std::max(1, (n - k0 - w + kTB - 1) / kTB);
    hipLaunchKernelGGL(trsv_fwd_step_kernel, dim3(g), dim3(kTB), 0, s, A, lda, n, k0,
                       ws->linv + (size_t)(k0 / kTB) * kTB * kTB, x, ws->ybuf);
  }
  for (int k0 = ((n - 1) / kTB) * kTB; k0 >= 0; k0 -= kTB) {
    const int g = std::max(1, (k0 + kTB - 1) / kTB);
    hipLaunchKernelGGL(trsv_bwd_step_kernel, dim3(g), dim3(kTB), 0, s, A, lda, n, k0,
                       ws->linv + (size_t)(k0 / kTB) * kTB * kTB, ws->ybuf, x);
  }
  return hipGetLastError() == hipSuccess ? rocblas_status_success : rocblas_status_internal_error;
}

}  // namespace miba
