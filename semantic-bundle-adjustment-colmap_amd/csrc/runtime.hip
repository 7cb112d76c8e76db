// runtime.hip — device-resident problem, LM driver and C-ABI (product code).
//
// mi_ba_solve replaces BundleAdjuster::Solve (src/optim/bundle_adjustment.cc:
// 258-320) including its Ceres 2.1 call: a Levenberg-Marquardt trust-region
// loop (TrustRegionMinimizer + LevenbergMarquardtStrategy semantics restated:
// Jacobi scaling fixed at iteration 0, LM diagonal clamped to [1e-6, 1e32],
// radius update 1/max(1/3, 1-(2q-1)^3), decrease factor doubling, step
// acceptance at relative decrease > min_relative_decrease) whose linear
// system is solved by the implicit-Schur PCG of ITERATIVE_SCHUR with the
// SCHUR_JACOBI preconditioner and Ceres' Nash-Sofer q-termination (eta).
// No CPU fallback: without an MI355X the entry points return
// MI_BA_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <numeric>
#include <unordered_map>

#include "../../include/mi_ba.h"
#include "ba_math.h"
#include "cholesky.h"
#include "context.h"
#include "kernels.h"
#include "gsba.h"
#include "semantic.h"
#include "setup.h"
#include <rocsolver/rocsolver.h>

namespace miba {

namespace {

enum Scalar {
  kCost = 0, kCandCost = 1, kModelCost = 2, kRho = 3, kRhoPrev = 4, kPQ = 5, kXB = 6, kXR = 7,
  kStepNorm = 8, kSemCost = 9, kSemCand = 10, kSemModel = 11, kGsCost = 12, kGsCand = 13, kGsModel = 14,
  kNumScalars = 16
};

#define MI_HIP(expr)                                     \
  do {                                                   \
    hipError_t _e = (expr);                              \
    if (_e != hipSuccess) {                              \
      if (_e == hipErrorOutOfMemory) return MI_BA_ERR_OUT_OF_MEMORY; \
      return MI_BA_ERR_HIP;                              \
    }                                                    \
  } while (0)

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Host evaluation of one block's cost (fixed_cost of dropped blocks).
double host_block_cost(const mi_ba_options& o, const mi_ba_problem* p, const HostSetup& s, int64_t k) {
  const int img = p->obs_image[k];
  const int cam = p->image_camera[img];
  const int64_t pt = p->obs_point[k];
  const double* q = p->qvec + 4 * (size_t)img;
  const double* t = p->tvec + 3 * (size_t)img;
  const double* X = p->xyz + 3 * (size_t)pt;
  const double* prm = p->camera_params + s.cam_off[cam];
  double P[3];
  unit_quat_rotate(q, X, P);
  P[0] += t[0]; P[1] += t[1]; P[2] += t[2];
  const double u = P[0] / P[2], v = P[1] / P[2];
  double x = 0, y = 0;
  world_to_image_any(s.cam_model[cam], prm, u, v, &x, &y);
  const double r0 = x - p->obs_xy[2 * k], r1 = y - p->obs_xy[2 * k + 1];
  double rho[3];
  loss_eval(o.loss_function_type, o.loss_function_scale, r0 * r0 + r1 * r1, rho);
  return 0.5 * rho[0];
}

__global__ void identity_kernel(double* __restrict__ S, int64_t n, int64_t ld) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) S[k * ld + k] = 1.0;
}

// Row i of S (row-major view, leading dimension ld): zero columns
// [i rounded down to 512, ld).
__global__ __launch_bounds__(256) void zero_upper_kernel(double* __restrict__ S, int64_t n, int64_t ld) {
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const int64_t c0 = i / 512 * 512;
  double* row = S + i * ld;
  typedef double zvec2 __attribute__((ext_vector_type(2)));
  int64_t c = c0 + 2 * threadIdx.x;
  for (; c + 1 < ld; c += 512) *reinterpret_cast<zvec2*>(row + c) = zvec2{0.0, 0.0};
  if (c < ld) row[c] = 0.0;
}

// Spare column-major row n of S <-> a vector: to_row 1 writes v into it (the
// rhs the factorisation carries), 0 reads the forward solution back.
__global__ void rhs_row_kernel(double* __restrict__ S, int64_t n, int64_t ld, double* __restrict__ v, int to_row) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  if (to_row)
    S[j * ld + n] = v[j];
  else
    v[j] = S[j * ld + n];
}

// The forward solve rides in the factorisation (spare row) when the blocked
// factor and the sync-free backward sweep are in use ("cholesky_fused_rhs").
bool fused_rhs(const mi_ba_context* ctx) {
  const CholConfig& c = ctx->chol;
  return ctx->fused_rhs && c.panel > 0 && c.gemm_update && c.solve == 2 && ctx->dev.lds > ctx->dev.nf;
}

mi_ba_status comm_drain(mi_ba_context* ctx);

// A host wait on stream s of the context: pending collectives first
// (comm_drain, deadline-bounded), then the synchronisation.
#define MI_HIP_DRAIN(ctx_, s_)                          \
  do {                                                  \
    const mi_ba_status ds_ = comm_drain(ctx_);          \
    if (ds_ != MI_BA_OK) return ds_;                    \
    MI_HIP(hipStreamSynchronize(s_));                   \
  } while (0)

mi_ba_status read_scalars(mi_ba_context* ctx, int first, int count) {
  MI_HIP(hipMemcpyAsync(ctx->host_scalars + first, ctx->scalars.ptr + first, sizeof(double) * count,
                        hipMemcpyDeviceToHost, ctx->stream));
  mi_ba_status st = comm_drain(ctx);
  if (st != MI_BA_OK) return st;
  MI_HIP(hipStreamSynchronize(ctx->stream));
  return MI_BA_OK;
}

}  // namespace

namespace {

// A peer that died or diverged must not hang the LM: the communicator is
// aborted (its kernels leave their wait loops, the stream drains) and every
// later collective of this context fails at once.
mi_ba_status comm_fail(mi_ba_context* ctx) {
  if (ctx->comm && ctx->stall_flag && ctx->stall_flag[0] == 0) {
    // test hook: the stall was the only thing holding the stream; release it
    // and let the (1-rank) collective behind it finish before the abort
    __atomic_store_n(ctx->stall_flag, 1, __ATOMIC_RELEASE);
    const double until = now_s() + 10.0;
    while (hipStreamQuery(ctx->stream) == hipErrorNotReady && now_s() < until)
      std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  if (ctx->comm) (void)ncclCommAbort(ctx->comm);
  ctx->comm = nullptr;
  ctx->comm_failed = true;
  return MI_BA_ERR_HIP;
}

// Poll a non-blocking communicator until its pending call (set-up or the
// enqueue of a collective) is done, an asynchronous error shows, or the
// deadline passes.
mi_ba_status comm_settle(mi_ba_context* ctx, double deadline) {
  for (int spin = 0;; ++spin) {
    ncclResult_t e = ncclSuccess;
    if (ncclCommGetAsyncError(ctx->comm, &e) != ncclSuccess) return comm_fail(ctx);
    if (e == ncclSuccess) return MI_BA_OK;
    if (e != ncclInProgress || now_s() > deadline) return comm_fail(ctx);
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// Wait for the context stream (a collective just enqueued on it) with the
// same deadline, watching the communicator's asynchronous error state: a
// collective whose peer never arrives is aborted instead of waited on.
mi_ba_status comm_wait_stream(mi_ba_context* ctx, double deadline) {
  for (int spin = 0;; ++spin) {
    const hipError_t q = hipStreamQuery(ctx->stream);
    if (q == hipSuccess) return MI_BA_OK;
    if (q != hipErrorNotReady) return comm_fail(ctx);
    ncclResult_t e = ncclSuccess;
    if (ncclCommGetAsyncError(ctx->comm, &e) != ncclSuccess || (e != ncclSuccess && e != ncclInProgress) ||
        now_s() > deadline)
      return comm_fail(ctx);
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// Collectives are enqueued without a host wait (allreduce); the next host
// wait on the context stream goes through here first, bounded by their
// deadline and watching the communicator's error state, so a dead peer ends
// the wait instead of hanging it.  No pending collective: nothing to do.
mi_ba_status comm_drain(mi_ba_context* ctx) {
  if (!ctx->comm || ctx->comm_due <= 0.0) return MI_BA_OK;
  const double due = ctx->comm_due;
  ctx->comm_due = 0.0;
  return comm_wait_stream(ctx, due);
}

// Test hook ("comm_stall_ms"): hold the stream, as a collective whose peer
// never arrives would, until the host releases the flag or the stall time
// has passed.  One wave; it always ends (a bound on the constant-rate wall
// clock), so the grid drains by itself.
__global__ void stall_kernel(const int* flag, uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 && wall_clock64() - t0 < ticks)
    __builtin_amdgcn_s_sleep(64);
}

}  // namespace

// Sum n doubles of a device buffer over the ranks of a multi-rank solve (RCCL
// all-reduce on the context stream, or the host reducer); no-op without a
// reducer.  With RCCL the call returns once the collective is enqueued (the
// stream orders the kernels that read the sum behind it; back-to-back sums
// pipeline with no host round trip between them); the next host wait
// (comm_drain) bounds its completion by the context's deadline
// ("comm_timeout_ms").  A failed or timed-out collective aborts the
// communicator and returns MI_BA_ERR_HIP (on every rank that sees it; a rank
// whose peer failed sees its own collective time out).
mi_ba_status allreduce(mi_ba_context* ctx, double* d, int64_t n) {
  if (!ctx->distributed() || n <= 0) return MI_BA_OK;
  if (ctx->comm_failed) return MI_BA_ERR_HIP;
  if (ctx->comm) {
    const double deadline = now_s() + 1e-3 * ctx->comm_timeout_ms;
    if (ctx->comm_stall_ms > 0) {
      int khz = 0;
      if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device) != hipSuccess || khz <= 0)
        return MI_BA_ERR_HIP;
      if (!ctx->stall_flag && hipHostMalloc(&ctx->stall_flag, sizeof(int), hipHostMallocCoherent) != hipSuccess) {
        ctx->stall_flag = nullptr;
        return MI_BA_ERR_HIP;
      }
      __atomic_store_n(ctx->stall_flag, 0, __ATOMIC_RELEASE);
      hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, ctx->stream, ctx->stall_flag,
                         (uint64_t)khz * ctx->comm_stall_ms);
    }
    const ncclResult_t r = ncclAllReduce(d, d, (size_t)n, ncclDouble, ncclSum, ctx->comm, ctx->stream);
    if (r != ncclSuccess && r != ncclInProgress) return comm_fail(ctx);
    mi_ba_status st = comm_settle(ctx, deadline);
    if (st != MI_BA_OK) return st;
    ctx->comm_due = std::max(ctx->comm_due, deadline);
    return MI_BA_OK;
  }
  if (!ctx->host_reduce) return MI_BA_ERR_STATE;
  ctx->reduce_buf.resize(n);
  MI_HIP(hipMemcpyAsync(ctx->reduce_buf.data(), d, n * 8, hipMemcpyDeviceToHost, ctx->stream));
  MI_HIP_DRAIN(ctx, ctx->stream);
  if (ctx->host_reduce(ctx->reduce_buf.data(), n, ctx->host_reduce_user) != 0) return MI_BA_ERR_HIP;
  MI_HIP(hipMemcpyAsync(d, ctx->reduce_buf.data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
  MI_HIP_DRAIN(ctx, ctx->stream);
  return MI_BA_OK;
}

// Phase timer events: timing only (timer_collect synchronises the stream
// before reading them), so recorded without the system-scope fence — a
// default event's record writes back and invalidates the caches, which the
// next kernel then pays for (C4 step with timing on / off: 0.799-0.802 /
// 0.788-0.790 ms with default events, 0.790-0.792 / 0.787 ms with these,
// profiles/r6z_step_timing_events.txt)
static hipError_t timer_event(hipEvent_t* e) { return hipEventCreateWithFlags(e, hipEventDisableSystemFence); }

void timer_begin(mi_ba_context* ctx, const char* name, hipEvent_t* stop_out) {
  *stop_out = nullptr;
  if (!ctx->timing) return;
  hipEvent_t a, b;
  if (ctx->timer.pool.size() >= 2) {
    a = ctx->timer.pool.back(); ctx->timer.pool.pop_back();
    b = ctx->timer.pool.back(); ctx->timer.pool.pop_back();
  } else {
    (void)timer_event(&a);
    (void)timer_event(&b);
  }
  (void)hipEventRecord(a, ctx->stream);
  ctx->timer.pending.push_back({name, {a, b}});
  *stop_out = b;
}

void timer_end(mi_ba_context* ctx, hipEvent_t stop) {
  if (!ctx->timing || !stop) return;
  (void)hipEventRecord(stop, ctx->stream);
}

void timer_begin_after(mi_ba_context* ctx, const char* name, hipEvent_t start, hipEvent_t* stop_out) {
  if (!start) {
    timer_begin(ctx, name, stop_out);
    return;
  }
  *stop_out = nullptr;
  if (!ctx->timing) return;
  hipEvent_t b;
  if (!ctx->timer.pool.empty()) {
    b = ctx->timer.pool.back();
    ctx->timer.pool.pop_back();
  } else {
    (void)timer_event(&b);
  }
  ctx->timer.pending.push_back({name, {start, b}});
  ctx->timer.borrowed.push_back(start);
  *stop_out = b;
}

// Scoped phase timer (HIP events on the context stream; no-op unless timing).
struct Phase {
  mi_ba_context* ctx;
  hipEvent_t stop;
  Phase(mi_ba_context* c, const char* name) : ctx(c) { timer_begin(c, name, &stop); }
  ~Phase() { timer_end(ctx, stop); }
};

static void timer_collect(mi_ba_context* ctx) {
  if (ctx->timer.pending.empty()) return;
  (void)hipStreamSynchronize(ctx->stream);
  for (auto& e : ctx->timer.pending) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e.second.first, e.second.second);
    auto& t = ctx->timer.totals[e.first];
    t.first += ms;
    t.second += 1;
    if (std::find(ctx->timer.borrowed.begin(), ctx->timer.borrowed.end(), e.second.first) == ctx->timer.borrowed.end())
      ctx->timer.pool.push_back(e.second.first);
    ctx->timer.pool.push_back(e.second.second);
  }
  ctx->timer.pending.clear();
  ctx->timer.borrowed.clear();
}

// Pair list of the explicit Schur build: every unordered pair {a, b} of
// blocks of one variable point (a == b included), bucketed by image pair
// (ia <= ib) and cut into tiles of <= kPairTile pairs; self pairs (a == b)
// get tiles of their own.  Built once per problem (structure only).
// The pair tiles in image-block order (schur_pairs_variant 4): blocks of
// B x B image pairs, so the workgroups in flight at any time (dispatch order)
// gather the Z rows of ~2B images only — a working set the 256 MB MALL holds
// (2.9 MB of Z per image at C4), where the first-image order scatters the
// second image's rows over every image.
// The deterministic route with shared cameras (PairFlush::odest): every
// tile of the image-block order writes its accumulator to its own partial;
// the S blocks are summed per owner pair (pose / camera of the tile's two
// images) from those partials in tile order, long owner-pair lists (a
// camera shared by many images) in runs of 256 entries whose sums are then
// added in run order.
mi_ba_status order_owner_flush(mi_ba_context* ctx, const std::vector<DevPairTile>& tb) {
  const mi_ba_problem* p = &ctx->problem;
  std::map<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>> lists;
  for (uint32_t k = 0; k < (uint32_t)tb.size(); ++k) {
    const DevPairTile& tl = tb[k];
    const uint32_t ca = (uint32_t)p->image_camera[tl.ia], cb = (uint32_t)p->image_camera[tl.ib];
    for (uint32_t q = 0; q < 4; ++q) {
      if (tl.self && q == 2) continue;  // a self tile's (camera, pose) quadrant is the mirror of (pose, camera)
      uint32_t x = (q & 2) ? kOwnerCam | ca : tl.ia, y = (q & 1) ? kOwnerCam | cb : tl.ib;
      uint32_t sw = 0;
      if (x > y) {
        std::swap(x, y);
        sw = 1;
      }
      lists[{x, y}].push_back(k << 4 | q << 2 | sw << 1 | (tl.self ? 1u : 0u));
    }
  }
  if (tb.size() >= (1u << 27)) return MI_BA_ERR_INVALID_ARGUMENT;
  std::vector<uint4> dest, chunk;
  std::vector<uint32_t> ent;
  constexpr uint32_t kRun = 256;
  for (auto& kv : lists) {
    const std::vector<uint32_t>& l = kv.second;
    const uint32_t c0 = (uint32_t)chunk.size();
    for (uint32_t f = 0; f < l.size(); f += kRun)
      chunk.push_back(make_uint4((uint32_t)dest.size(), (uint32_t)ent.size() + f,
                                 std::min<uint32_t>(kRun, (uint32_t)l.size() - f), 0u));
    dest.push_back(make_uint4(kv.first.first, kv.first.second, c0, (uint32_t)chunk.size() - c0));
    ent.insert(ent.end(), l.begin(), l.end());
  }
  std::vector<int32_t> ps(tb.size());
  for (size_t k = 0; k < tb.size(); ++k) ps[k] = (int32_t)k;
  if (ctx->pslot.alloc(std::max<size_t>(1, ps.size())) || ctx->spart.alloc(std::max<size_t>(1, tb.size()) * 256) ||
      ctx->podest.alloc(std::max<size_t>(1, dest.size())) || ctx->pochunk.alloc(std::max<size_t>(1, chunk.size())) ||
      ctx->poent.alloc(std::max<size_t>(1, ent.size())) || ctx->popart.alloc(std::max<size_t>(1, chunk.size()) * 64))
    return MI_BA_ERR_OUT_OF_MEMORY;
  if ((!ps.empty() && hipMemcpy(ctx->pslot.ptr, ps.data(), ps.size() * 4, hipMemcpyHostToDevice) != hipSuccess) ||
      (!dest.empty() && hipMemcpy(ctx->podest.ptr, dest.data(), dest.size() * sizeof(uint4), hipMemcpyHostToDevice) !=
                            hipSuccess) ||
      (!chunk.empty() &&
       hipMemcpy(ctx->pochunk.ptr, chunk.data(), chunk.size() * sizeof(uint4), hipMemcpyHostToDevice) != hipSuccess) ||
      (!ent.empty() && hipMemcpy(ctx->poent.ptr, ent.data(), ent.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
    return MI_BA_ERR_HIP;
  ctx->npdest = 0;
  ctx->npodest = (int)dest.size();
  ctx->npochunk = (int)chunk.size();
  ctx->pflush_ok = true;
  return MI_BA_OK;
}

mi_ba_status order_block_tiles(mi_ba_context* ctx) {
#ifdef MI_BA_AB_VARIANTS
  // XCD-interleaved order (schur_pairs_variant 5, tools build: measured
  // slower, 3.39 vs 3.26 ms per schur_build call): rows of 8 first images;
  // within a row, image Ia + x's tiles in second-image order go to XCD x
  // (workgroup b runs on XCD b % 8, four tiles per workgroup), so each XCD
  // keeps ONE first image's Z rows (2.9 MB at C4) in its 4 MB L2 for the whole
  // sweep over second images, while the eight XCDs stream the same second
  // images through the MALL.  Empty tiles pad the shorter lists.
  {
    const std::vector<DevPairTile>& tl = ctx->ptiles_host;
    constexpr int kX = 8, kW = kBlock / 64;
    uint32_t nimg = 0;
    for (const DevPairTile& t : tl) nimg = std::max(nimg, t.ia + 1);
    std::vector<std::vector<uint32_t>> per(nimg);
    for (uint32_t k = 0; k < (uint32_t)tl.size(); ++k) per[tl[k].ia].push_back(k);
    std::vector<DevPairTile> tx;
    DevPairTile empty{};
    for (uint32_t i0 = 0; i0 < nimg; i0 += kX) {
      std::vector<std::vector<uint32_t>*> lists;
      size_t longest = 0;
      for (int x = 0; x < kX; ++x) {
        std::vector<uint32_t>* l = i0 + x < nimg ? &per[i0 + x] : nullptr;
        if (l) std::stable_sort(l->begin(), l->end(), [&](uint32_t a, uint32_t b) { return tl[a].ib < tl[b].ib; });
        lists.push_back(l);
        if (l) longest = std::max(longest, l->size());
      }
      for (size_t k = 0; k < longest; k += kW)
        for (int x = 0; x < kX; ++x)
          for (int w = 0; w < kW; ++w) {
            const std::vector<uint32_t>* l = lists[x];
            tx.push_back(l && k + w < l->size() ? tl[(*l)[k + w]] : empty);
          }
    }
    if (ctx->ptiles_xcd.alloc(std::max<size_t>(1, tx.size()))) return MI_BA_ERR_OUT_OF_MEMORY;
    ctx->nptiles_xcd = (int)tx.size();
    if (!tx.empty() && (hipStreamSynchronize(ctx->stream) != hipSuccess ||
                        hipMemcpy(ctx->ptiles_xcd.ptr, tx.data(), tx.size() * sizeof(DevPairTile),
                                  hipMemcpyHostToDevice) != hipSuccess))
      return MI_BA_ERR_HIP;
  }
#endif
  std::vector<DevPairTile> tb(ctx->ptiles_host);
  const uint32_t B = (uint32_t)std::max(1, ctx->schur_block);
  std::stable_sort(tb.begin(), tb.end(), [B](const DevPairTile& x, const DevPairTile& y) {
    const uint32_t xa = x.ia / B, xb = x.ib / B, ya = y.ia / B, yb = y.ib / B;
    return xa != ya ? xa < ya : xb < yb;
  });
  if (tb.empty()) return MI_BA_OK;
  // kernels of an earlier solve may still read the old order
  if (hipStreamSynchronize(ctx->stream) != hipSuccess ||
      hipMemcpy(ctx->ptiles_blk.ptr, tb.data(), tb.size() * sizeof(DevPairTile), hipMemcpyHostToDevice) != hipSuccess)
    return MI_BA_ERR_HIP;
  // The deterministic route (PairFlush): each S block written by one tile is
  // written directly, every other block (diagonal blocks, image pairs of
  // several tiles) summed from per-tile partials in tile order.  Needs every
  // camera on at most one image: a shared camera's columns gather many image
  // pairs' tiles, which stay on float atomics.
  ctx->pflush_ok = false;
  ctx->npodest = ctx->npochunk = 0;
  {
    const mi_ba_problem* p = &ctx->problem;
    std::vector<int> per_cam(p->num_cameras, 0);
    bool distinct = true;
    for (int i = 0; i < p->num_images && distinct; ++i) distinct = ++per_cam[p->image_camera[i]] <= 1;
    if (!distinct) return order_owner_flush(ctx, tb);
  }
  std::unordered_map<uint64_t, uint32_t> didx;
  std::vector<std::vector<uint32_t>> dtiles;
  std::vector<uint2> dkey;
  for (uint32_t k = 0; k < (uint32_t)tb.size(); ++k) {
    const uint64_t key = (uint64_t)tb[k].ia << 32 | tb[k].ib;
    auto it = didx.find(key);
    if (it == didx.end()) {
      it = didx.emplace(key, (uint32_t)dtiles.size()).first;
      dtiles.emplace_back();
      dkey.push_back(make_uint2(tb[k].ia, tb[k].ib));
    }
    dtiles[it->second].push_back(k);
  }
  std::vector<int32_t> ps(tb.size(), -1);
  std::vector<uint4> dest;
  std::vector<uint8_t> self;
  for (size_t d = 0; d < dtiles.size(); ++d) {
    if (dkey[d].x != dkey[d].y && dtiles[d].size() == 1) continue;  // direct
    dest.push_back(make_uint4(dkey[d].x, dkey[d].y, (uint32_t)self.size(), (uint32_t)dtiles[d].size()));
    for (uint32_t k : dtiles[d]) {
      ps[k] = (int32_t)self.size();
      self.push_back(tb[k].self ? 1 : 0);
    }
  }
  if (ctx->pslot.alloc(ps.size()) || ctx->spart.alloc(std::max<size_t>(1, self.size()) * 256) ||
      ctx->pdest.alloc(std::max<size_t>(1, dest.size())) || ctx->pself.alloc(std::max<size_t>(1, self.size())))
    return MI_BA_ERR_OUT_OF_MEMORY;
  if (hipMemcpy(ctx->pslot.ptr, ps.data(), ps.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      (!dest.empty() && hipMemcpy(ctx->pdest.ptr, dest.data(), dest.size() * sizeof(uint4), hipMemcpyHostToDevice) !=
                            hipSuccess) ||
      (!self.empty() && hipMemcpy(ctx->pself.ptr, self.data(), self.size(), hipMemcpyHostToDevice) != hipSuccess))
    return MI_BA_ERR_HIP;
  ctx->npdest = (int)dest.size();
  ctx->pflush_ok = true;
  return MI_BA_OK;
}

// The pair list in camera-major positions (zorder 1: Z row k is the block
// cm_perm[k]); pr: the block pairs (read back from the device when null).
mi_ba_status build_pairs_pos(mi_ba_context* ctx, const std::vector<uint2>* pr) {
  const int64_t nb = ctx->dev.nb;
  const size_t np = ctx->pairs.n;
  std::vector<uint2> host;
  if (!pr) {
    host.resize(np);
    if (np && hipMemcpy(host.data(), ctx->pairs.ptr, np * sizeof(uint2), hipMemcpyDeviceToHost) != hipSuccess)
      return MI_BA_ERR_HIP;
    pr = &host;
  }
  std::vector<uint32_t> perm(nb), inv(nb);
  if (nb && hipMemcpy(perm.data(), ctx->cm_perm.ptr, nb * 4, hipMemcpyDeviceToHost) != hipSuccess) return MI_BA_ERR_HIP;
  for (int64_t k = 0; k < nb; ++k) inv[perm[k]] = (uint32_t)k;
  std::vector<uint2> pos(np);
  for (size_t e = 0; e < np; ++e) pos[e] = make_uint2(inv[(*pr)[e].x], inv[(*pr)[e].y]);
  if (ctx->pairs_pos.alloc(std::max<size_t>(1, np))) return MI_BA_ERR_OUT_OF_MEMORY;
  // kernels of an earlier solve may still read the old list
  if (hipStreamSynchronize(ctx->stream) != hipSuccess ||
      (np && hipMemcpy(ctx->pairs_pos.ptr, pos.data(), np * sizeof(uint2), hipMemcpyHostToDevice) != hipSuccess))
    return MI_BA_ERR_HIP;
  return MI_BA_OK;
}

mi_ba_status build_pair_tiles(mi_ba_context* ctx) {
  const DevProblem& d = ctx->dev;
  const int I = d.num_images;
  const int64_t nb = d.nb;
  std::vector<DevPoint> vp(ctx->npv);
  std::vector<uint32_t> im(nb);
  if (ctx->npv && hipMemcpy(vp.data(), ctx->vpoints.ptr, ctx->npv * sizeof(DevPoint), hipMemcpyDeviceToHost))
    return MI_BA_ERR_HIP;
  if (nb && hipMemcpy(im.data(), ctx->obs_img.ptr, nb * 4, hipMemcpyDeviceToHost)) return MI_BA_ERR_HIP;
  // bucket key: first image ia (ia <= ib), self pairs in bucket I + ia
  std::vector<int64_t> cnt(2 * (size_t)I + 1, 0);
  auto visit = [&](auto&& f) {
    for (const DevPoint& q : vp)
      for (uint32_t x = 0; x < q.count; ++x)
        for (uint32_t y = x; y < q.count; ++y) {
          uint32_t a = q.start + x, b = q.start + y;
          if (im[a] > im[b]) std::swap(a, b);
          f(a, b, a == b ? (size_t)I + im[a] : (size_t)im[a]);
        }
  };
  visit([&](uint32_t, uint32_t, size_t key) { ++cnt[key + 1]; });
  for (size_t k = 1; k < cnt.size(); ++k) cnt[k] += cnt[k - 1];
  const int64_t npairs = cnt.back();
  std::vector<uint2> pr(npairs);
  {
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
    visit([&](uint32_t a, uint32_t b, size_t key) { pr[pos[key]++] = make_uint2(a, b); });
  }
  // within a first-image bucket, order by second image (counting sort, stable)
  {
    std::vector<int64_t> c2(I + 1);
    std::vector<uint2> tmp;
    for (int k = 0; k < 2 * I; ++k) {
      const int64_t b0 = cnt[k], b1 = cnt[k + 1];
      if (b1 - b0 < 2) continue;
      std::fill(c2.begin(), c2.end(), 0);
      for (int64_t e = b0; e < b1; ++e) ++c2[im[pr[e].y] + 1];
      for (int j = 1; j <= I; ++j) c2[j] += c2[j - 1];
      tmp.resize(b1 - b0);
      for (int64_t e = b0; e < b1; ++e) tmp[c2[im[pr[e].y]]++] = pr[e];
      std::copy(tmp.begin(), tmp.end(), pr.begin() + b0);
    }
  }
  std::vector<DevPairTile> tl;
  for (int k = 0; k < 2 * I; ++k) {
    int64_t a = cnt[k];
    while (a < cnt[k + 1]) {
      const uint32_t ib = im[pr[a].y];
      int64_t e = a;
      while (e < cnt[k + 1] && im[pr[e].y] == ib) ++e;
      for (int64_t t0 = a; t0 < e; t0 += kPairTile) {
        DevPairTile t;
        t.ia = im[pr[a].x];
        t.ib = ib;
        t.start = (uint32_t)t0;
        t.count = (uint32_t)std::min<int64_t>(kPairTile, e - t0);
        t.self = k >= I ? 1u : 0u;
        tl.push_back(t);
      }
      a = e;
    }
  }
  if (npairs >= (int64_t)UINT32_MAX || tl.size() >= (size_t)INT32_MAX) return MI_BA_ERR_UNSUPPORTED;
  ctx->nptiles = (int)tl.size();
  // the same tiles in image-block order (svariant 4): blocks of B x B image
  // pairs, so the workgroups in flight at any time (dispatch order) gather
  // the Z rows of ~2B images only — a working set the 256 MB MALL holds
  // (2.9 MB of Z per image at C4), where the first-image order scatters the
  // second image's rows over every image
  if (ctx->pairs.alloc(npairs) || ctx->ptiles.alloc(tl.size()) || ctx->ptiles_blk.alloc(tl.size()) ||
      ctx->Linv.alloc(6 * (size_t)d.num_points) || ctx->Z.alloc((size_t)nb * std::max<int64_t>(schur_record_width(d.ct, 4), schur_record_width(d.ct, 6))))
    return MI_BA_ERR_OUT_OF_MEMORY;
  if ((npairs && hipMemcpy(ctx->pairs.ptr, pr.data(), npairs * sizeof(uint2), hipMemcpyHostToDevice)) ||
      (!tl.empty() && hipMemcpy(ctx->ptiles.ptr, tl.data(), tl.size() * sizeof(DevPairTile), hipMemcpyHostToDevice)))
    return MI_BA_ERR_HIP;
  ctx->ptiles_host = std::move(tl);
  mi_ba_status st = order_block_tiles(ctx);
  if (st != MI_BA_OK) return st;
  if (d.zorder) {
    st = build_pairs_pos(ctx, &pr);
    if (st != MI_BA_OK) return st;
  } else {
    ctx->pairs_pos.release();
  }
  // stream-ordered: a null-stream memset is not ordered against the context's
  // non-blocking stream (the LM's kernels could overtake it)
  if (d.num_points && hipMemsetAsync(ctx->Linv.ptr, 0, 6 * (size_t)d.num_points * 8, ctx->stream)) return MI_BA_ERR_HIP;
  return MI_BA_OK;
}

mi_ba_status context_create(const mi_ba_options* o, const mi_ba_problem* pin, const mi_ba_semantic* sem,
                            mi_ba_context** out) {
  return context_recycle(nullptr, o, pin, sem, out);
}

namespace {
// Drops the problem state of a solved context, keeping its device resources.
void reset_problem_state(mi_ba_context* ctx) {
  semantic_destroy(ctx);
  gsba_destroy(ctx);
  ctx->timer.totals.clear();
  ctx->timing = false;
  ctx->solved = false;
  ctx->dense = false;
  ctx->nptiles = 0;
  ctx->chol = CholConfig{};
  ctx->fixed_cost = 0.0;
  ctx->block_obs.clear();
  ctx->setup = HostSetup{};
  ctx->dev = DevProblem{};
}
}  // namespace

mi_ba_status context_recycle(mi_ba_context* old, const mi_ba_options* o, const mi_ba_problem* pin,
                             const mi_ba_semantic* sem, mi_ba_context** out, const mi_ba_gsba* gsba) {
  if (!o || !pin || !out) {
    context_destroy(old);
    return MI_BA_ERR_INVALID_ARGUMENT;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    context_destroy(old);
    return MI_BA_ERR_NO_DEVICE;
  }
  if (o->device < 0 || o->device >= ndev) {
    context_destroy(old);
    return MI_BA_ERR_INVALID_ARGUMENT;
  }
  if (hipSetDevice(o->device) != hipSuccess) {
    context_destroy(old);
    return MI_BA_ERR_HIP;
  }
  mi_ba_context* ctx = nullptr;
  const bool recycled = old && old->device == o->device && !old->distributed() && old->timer.pending.empty();
  if (recycled) {
    ctx = old;
    reset_problem_state(ctx);
  } else {
    context_destroy(old);
    ctx = new mi_ba_context();
  }
  ctx->options = *o;
  ctx->problem = *pin;
  ctx->device = o->device;
  auto fail = [&](mi_ba_status e) { context_destroy(ctx); return e; };
  mi_ba_problem* p = &ctx->problem;
  mi_ba_status st = build_setup(*o, p, &ctx->setup);
  if (st != MI_BA_OK) return fail(st);
  const HostSetup& s = ctx->setup;
  if (!ctx->stream && hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    ctx->stream = nullptr;
    return fail(MI_BA_ERR_HIP);
  }

  const int I = p->num_images, C = p->num_cameras;
  const int64_t P = p->num_points;
  // Point-major order of reduced blocks (stable).
  std::vector<int64_t>& bo = ctx->block_obs;
  bo = s.reduced_obs;
  std::stable_sort(bo.begin(), bo.end(),
                   [&](int64_t a, int64_t b) { return p->obs_point[a] < p->obs_point[b]; });
  const int64_t nb = (int64_t)bo.size();
  {
    std::vector<double2> xy(nb);
    std::vector<uint32_t> im(nb), pt(nb);
    for (int64_t b = 0; b < nb; ++b) {
      const int64_t k = bo[b];
      xy[b] = make_double2(p->obs_xy[2 * k], p->obs_xy[2 * k + 1]);
      im[b] = (uint32_t)p->obs_image[k];
      pt[b] = (uint32_t)p->obs_point[k];
    }
    if (ctx->obs_xy.alloc(nb) || ctx->obs_img.alloc(nb) || ctx->obs_pt.alloc(nb)) return fail(MI_BA_ERR_OUT_OF_MEMORY);
    if (nb) {
      if (hipMemcpy(ctx->obs_xy.ptr, xy.data(), nb * sizeof(double2), hipMemcpyHostToDevice) ||
          hipMemcpy(ctx->obs_img.ptr, im.data(), nb * 4, hipMemcpyHostToDevice) ||
          hipMemcpy(ctx->obs_pt.ptr, pt.data(), nb * 4, hipMemcpyHostToDevice))
        return fail(MI_BA_ERR_HIP);
#ifdef MI_BA_AB_VARIANTS
      // packed ids of the reprojection kernel (device.h obs_ids; tools build,
      // jacobian_variant 43)
      const int64_t nw = (nb + 63) / 64;
      std::vector<uint32_t> ids(nb), w0(nw);
      bool packed = I <= 65536;
      for (int64_t b = 0; b < nb && packed; ++b) {
        if ((b & 63) == 0) w0[b >> 6] = pt[b];
        const uint32_t base = w0[b >> 6];
        packed = pt[b] >= base && pt[b] - base <= 65535u;
        ids[b] = im[b] | (pt[b] - base) << 16;
      }
      if (!packed) {
        ctx->obs_ids.release();
        ctx->wave_pt0.release();
      } else {
        if (ctx->obs_ids.alloc(nb) || ctx->wave_pt0.alloc(nw)) return fail(MI_BA_ERR_OUT_OF_MEMORY);
        if (hipMemcpy(ctx->obs_ids.ptr, ids.data(), nb * 4, hipMemcpyHostToDevice) ||
            hipMemcpy(ctx->wave_pt0.ptr, w0.data(), nw * 4, hipMemcpyHostToDevice))
          return fail(MI_BA_ERR_HIP);
      }
#endif
    }
    // camera-major permutation and image-aligned tiles
    std::vector<uint32_t> perm(nb);
    std::iota(perm.begin(), perm.end(), 0u);
    std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) { return im[a] < im[b]; });
    std::vector<DevTile> tl;
    int64_t a = 0;
    while (a < nb) {
      const uint32_t img = im[perm[a]];
      int64_t e = a;
      while (e < nb && im[perm[e]] == img) ++e;
      for (int64_t t0 = a; t0 < e; t0 += kTileObs) {
        DevTile t;
        t.image = img;
        t.start = (uint32_t)t0;
        t.count = (uint32_t)std::min<int64_t>(kTileObs, e - t0);
        t.pad = 0;
        tl.push_back(t);
      }
      a = e;
    }
    ctx->ntiles = (int)tl.size();
    if (ctx->cm_perm.alloc(nb) || ctx->tiles.alloc(tl.size())) return fail(MI_BA_ERR_OUT_OF_MEMORY);
    if (nb && (hipMemcpy(ctx->cm_perm.ptr, perm.data(), nb * 4, hipMemcpyHostToDevice) ||
               hipMemcpy(ctx->tiles.ptr, tl.data(), tl.size() * sizeof(DevTile), hipMemcpyHostToDevice)))
      return fail(MI_BA_ERR_HIP);
    // owners of the tile sums (deterministic flush): each image's tiles (a
    // contiguous, image-sorted range) and each camera's, image then tile order
    {
      std::vector<uint32_t> ito(I + 1, 0), cto(C + 1, 0), ct;
      for (const DevTile& x : tl) ++ito[x.image + 1];
      for (int i = 0; i < I; ++i) ito[i + 1] += ito[i];
      for (int i = 0; i < I; ++i) cto[p->image_camera[i] + 1] += ito[i + 1] - ito[i];
      for (int c = 0; c < C; ++c) cto[c + 1] += cto[c];
      ct.resize(tl.size());
      std::vector<uint32_t> pos(cto.begin(), cto.end() - 1);
      for (int i = 0; i < I; ++i)
        for (uint32_t k = ito[i]; k < ito[i + 1]; ++k) ct[pos[p->image_camera[i]]++] = k;
      if (ctx->img_tile_off.alloc(I + 1) || ctx->cam_tile_off.alloc(C + 1) ||
          ctx->cam_tiles.alloc(std::max<size_t>(1, ct.size())) ||
          ctx->tpart.alloc(std::max<size_t>(1, tl.size()) * kTilePartStride))
        return fail(MI_BA_ERR_OUT_OF_MEMORY);
      if (hipMemcpy(ctx->img_tile_off.ptr, ito.data(), ito.size() * 4, hipMemcpyHostToDevice) ||
          hipMemcpy(ctx->cam_tile_off.ptr, cto.data(), cto.size() * 4, hipMemcpyHostToDevice) ||
          (!ct.empty() && hipMemcpy(ctx->cam_tiles.ptr, ct.data(), ct.size() * 4, hipMemcpyHostToDevice)))
        return fail(MI_BA_ERR_HIP);
      ctx->owners_ = TileOwners{ctx->img_tile_off.ptr, ctx->cam_tile_off.ptr, ctx->cam_tiles.ptr, ctx->tpart.ptr,
                                kTilePartStride};
    }
    // camera-major point of each block, 0xffffffff for constant points: the
    // camera-block pass reads it coalesced instead of gathering obs_pt and
    // pt_var per block
    {
      std::vector<uint32_t> cp(nb);
      for (int64_t k = 0; k < nb; ++k) {
        const uint32_t q = pt[perm[k]];
        cp[k] = s.pt_var[q] ? q : 0xffffffffu;
      }
      if (ctx->cm_ptv.alloc(std::max<int64_t>(1, nb))) return fail(MI_BA_ERR_OUT_OF_MEMORY);
      if (nb && hipMemcpy(ctx->cm_ptv.ptr, cp.data(), nb * 4, hipMemcpyHostToDevice)) return fail(MI_BA_ERR_HIP);
    }
    // variable points with their contiguous block ranges
    std::vector<DevPoint> vp;
    int64_t b = 0, nb_var = 0;
    while (b < nb) {
      const uint32_t q = pt[b];
      int64_t e = b;
      while (e < nb && pt[e] == q) ++e;
      if (s.pt_var[q]) {
        DevPoint d;
        d.point = q;
        d.start = (uint32_t)b;
        d.count = (uint32_t)(e - b);
        d.pad = 0;
        vp.push_back(d);
        nb_var += e - b;
      }
      b = e;
    }
    ctx->npv = (int64_t)vp.size();
    ctx->nb_const = nb - nb_var;
    // point chunks of the back substitution: whole points, <= 64 blocks
    // (a point with more blocks is a chunk of its own)
    std::vector<uint32_t> ch;
    {
      int64_t c0 = 0, q = 0;
      while (q < nb) {
        int64_t e = q;
        while (e < nb && pt[e] == pt[q]) ++e;
        if (e - c0 > 64 && q > c0) {
          ch.push_back((uint32_t)c0);
          c0 = q;
        }
        q = e;
      }
      if (nb > 0) ch.push_back((uint32_t)c0);
      ch.push_back((uint32_t)nb);
    }
    ctx->npchunks = (int)ch.size() - 1;
    if (ctx->pchunks.alloc(ch.size())) return fail(MI_BA_ERR_OUT_OF_MEMORY);
    if (hipMemcpy(ctx->pchunks.ptr, ch.data(), ch.size() * 4, hipMemcpyHostToDevice)) return fail(MI_BA_ERR_HIP);
    if (ctx->vpoints.alloc(vp.size())) return fail(MI_BA_ERR_OUT_OF_MEMORY);
    if (!vp.empty() && hipMemcpy(ctx->vpoints.ptr, vp.data(), vp.size() * sizeof(DevPoint), hipMemcpyHostToDevice))
      return fail(MI_BA_ERR_HIP);
  }
  // parameters
  {
    std::vector<double> qt(8 * (size_t)I, 0.0), cm(8 * (size_t)C, 0.0);
    std::vector<uint8_t> cmod(C);
    std::vector<uint32_t> fl(I), ic(I);
    for (int i = 0; i < I; ++i) {
      for (int m = 0; m < 4; ++m) qt[8 * i + m] = p->qvec[4 * i + m];
      for (int m = 0; m < 3; ++m) qt[8 * i + 4 + m] = p->tvec[3 * i + m];
      fl[i] = (s.img_var[i] ? 1u : 0u) | ((uint32_t)s.img_tvec_mask[i] << 1);
      ic[i] = (uint32_t)p->image_camera[i];
    }
    for (int c = 0; c < C; ++c) {
      cmod[c] = (uint8_t)s.cam_model[c];
      for (int64_t m = s.cam_off[c]; m < s.cam_off[c + 1]; ++m) cm[8 * c + (m - s.cam_off[c])] = p->camera_params[m];
    }
    if (ctx->qt.alloc(8 * I) || ctx->qt_c.alloc(8 * I) || ctx->cam.alloc(8 * C) || ctx->cam_c.alloc(8 * C) ||
        ctx->X.alloc(3 * P) || ctx->X_c.alloc(3 * P) || ctx->img_flags.alloc(I) || ctx->img_cam.alloc(I) ||
        ctx->cam_var.alloc(C) || ctx->cam_model.alloc(C) || ctx->pt_var.alloc(P) || ctx->img_rec.alloc(kImgRec * (size_t)I))
      return fail(MI_BA_ERR_OUT_OF_MEMORY);
    if ((I && (hipMemcpy(ctx->qt.ptr, qt.data(), qt.size() * 8, hipMemcpyHostToDevice) ||
               hipMemcpy(ctx->img_flags.ptr, fl.data(), I * 4, hipMemcpyHostToDevice) ||
               hipMemcpy(ctx->img_cam.ptr, ic.data(), I * 4, hipMemcpyHostToDevice))) ||
        (C && (hipMemcpy(ctx->cam.ptr, cm.data(), cm.size() * 8, hipMemcpyHostToDevice) ||
               hipMemcpy(ctx->cam_var.ptr, s.cam_var.data(), C, hipMemcpyHostToDevice) ||
               hipMemcpy(ctx->cam_model.ptr, cmod.data(), C, hipMemcpyHostToDevice))) ||
        (P && (hipMemcpy(ctx->X.ptr, p->xyz, 3 * P * 8, hipMemcpyHostToDevice) ||
               hipMemcpy(ctx->pt_var.ptr, s.pt_var.data(), P, hipMemcpyHostToDevice))))
      return fail(MI_BA_ERR_HIP);
  }
  DevProblem& d = ctx->dev;
  d.model = s.model;
  d.np = s.np;
  d.ct = s.ct;
  d.W = 9 + s.ct;
  for (int k = 0; k < 8; ++k) d.cam_tan_idx[k] = s.cam_tan_idx[k];
  d.nb = nb;
  d.num_images = I;
  d.num_cameras = C;
  d.num_points = P;
  d.cyl0 = 6 * (int64_t)I + (int64_t)s.ct * C;
  {
    const int slots = gsba ? gsba_cylinder_slots(*o, p, gsba) : 0;
    d.nf = d.cyl0 + slots;
    d.lds = d.nf;  // the exact path widens it below
    d.cyl_var = slots > 0;
  }
  d.loss_type = o->loss_function_type;
  d.loss_scale = o->loss_function_scale;
  d.jvariant = 0;
  // image-block tile order, dispatch-order mapping: schur_build 4.9 -> 3.4 ms
  // at C4 (profiles/r3_ab_schur_order.jsonl)
  d.svariant = 4;
  d.fvariant = 0;
  d.zorder = 0;
  d.sself1 = 1;
  d.refine_mask = (o->refine_focal_length ? 1 : 0) | (o->refine_principal_point ? 2 : 0) |
                  (o->refine_extra_params ? 4 : 0);
  d.obs_xy = ctx->obs_xy.ptr;
  d.obs_img = ctx->obs_img.ptr;
  d.obs_pt = ctx->obs_pt.ptr;
  d.obs_ids = ctx->obs_ids.ptr;
  d.wave_pt0 = ctx->wave_pt0.ptr;
  d.img_flags = ctx->img_flags.ptr;
  d.img_cam = ctx->img_cam.ptr;
  d.cam_var = ctx->cam_var.ptr;
  d.cam_model = ctx->cam_model.ptr;
  d.pt_var = ctx->pt_var.ptr;
  d.qt = ctx->qt.ptr;
  d.cam = ctx->cam.ptr;
  d.X = ctx->X.ptr;
  d.img_rec = ctx->img_rec.ptr;
  // linearization + LM buffers
  ctx->npartial = std::max<int64_t>({1, reproj_grid(nb), (int64_t)ctx->npchunks});
  const int64_t nf = d.nf;
  const int ncs = s.ct * (s.ct + 1) / 2;
  if (ctx->r.alloc(nb) || ctx->J.alloc((size_t)nb * 2 * d.W) || ctx->Vg.alloc(9 * P) ||
      ctx->partial.alloc(ctx->npartial) || ctx->scale_p.alloc(3 * P) || ctx->diag_p.alloc(3 * P) ||
      ctx->Vinv.alloc(6 * P) || ctx->pose_blk.alloc(21 * (size_t)I) || ctx->cam_blk.alloc((size_t)ncs * C + 1) ||
      ctx->bvec.alloc(nf) || ctx->udiag.alloc(nf) || ctx->scale_f.alloc(nf) || ctx->diag_f.alloc(nf) ||
      ctx->lambda_f.alloc(nf) || ctx->prec_pose.alloc(36 * (size_t)I) ||
      ctx->prec_cam.alloc((size_t)s.ct * s.ct * C + 1) || ctx->cg_x.alloc(nf) || ctx->cg_r.alloc(nf) ||
      ctx->cg_z.alloc(nf) || ctx->cg_p.alloc(nf) || ctx->cg_q.alloc(nf) || ctx->cg_w.alloc(3 * P) ||
      ctx->dX.alloc(3 * P) || ctx->scalars.alloc(kNumScalars) || ctx->red.alloc(kReduceBlocks) ||
      ctx->sum_ws.alloc(kSumScratch))
    return fail(MI_BA_ERR_OUT_OF_MEMORY);
  if (!ctx->host_scalars &&
      hipHostMalloc(&ctx->host_scalars, sizeof(double) * kNumScalars, hipHostMallocDefault) != hipSuccess) {
    ctx->host_scalars = nullptr;
    return fail(MI_BA_ERR_OUT_OF_MEMORY);
  }
  // stream-ordered (see build_pair_tiles)
  if (hipMemsetAsync(ctx->scalars.ptr, 0, sizeof(double) * kNumScalars, ctx->stream) != hipSuccess ||
      hipMemsetAsync(ctx->sum_ws.ptr, 0, sizeof(double) * kSumScratch, ctx->stream) != hipSuccess)
    return fail(MI_BA_ERR_HIP);
  if (P && (hipMemsetAsync(ctx->dX.ptr, 0, 3 * P * 8, ctx->stream) ||
            hipMemsetAsync(ctx->Vinv.ptr, 0, 6 * P * 8, ctx->stream) ||
            hipMemsetAsync(ctx->cg_w.ptr, 0, 3 * P * 8, ctx->stream)))
    return fail(MI_BA_ERR_HIP);
  // Linear solver (bundle_adjustment.cc:276-286): Ceres factorises the
  // reduced camera system exactly up to 1000 images (DENSE_SCHUR <= 50,
  // SPARSE_SCHUR <= 1000 with SuiteSparse) and switches to ITERATIVE_SCHUR +
  // SCHUR_JACOBI above.  Random tracks make S dense, so the exact path builds
  // S explicitly in HBM and factorises it with rocSOLVER.
  {
    int64_t ncfg = 0;
    for (int i = 0; i < I; ++i) ncfg += p->image_in_config ? (p->image_in_config[i] != 0) : 1;
    const double s_bytes = 8.0 * (double)d.nf * (double)d.nf;
    const bool fits = s_bytes <= 24e9 && d.nf < (1 << 30) / 1;
    if (o->linear_solver_type == MI_BA_SOLVER_DENSE_SCHUR) {
      if (!fits) return fail(MI_BA_ERR_UNSUPPORTED);
      ctx->dense = true;
    } else if (o->linear_solver_type == MI_BA_SOLVER_AUTO) {
      ctx->dense = ncfg <= 1000 && fits;
    }
    if (ctx->dense) {
      // S's leading dimension: one spare column-major row (the rhs carried
      // through the factorisation), rounded to 16 doubles (128-B columns)
      d.lds = (d.nf + 1 + 15) / 16 * 16;
      if (ctx->S.alloc((size_t)d.nf * d.lds) ||
          ctx->info.alloc(std::max<int64_t>(chol_leaf_count((int)d.nf), d.nf / 64 + 1)))
        return fail(MI_BA_ERR_OUT_OF_MEMORY);
      st = build_pair_tiles(ctx);
      if (st != MI_BA_OK) return fail(st);
      if (!ctx->blas) {
        if (rocblas_create_handle(&ctx->blas) != rocblas_status_success) {
          ctx->blas = nullptr;
          return fail(MI_BA_ERR_HIP);
        }
        if (rocblas_set_stream(ctx->blas, ctx->stream) != rocblas_status_success) return fail(MI_BA_ERR_HIP);
      }
      // per-context look-ahead resources on this context's device (panel
      // widths down to 64 allowed by mi_ba_set_tuning)
      if (!ctx->cholws.ensure(ctx->device, (int)((d.nf + 63) / 64), (int)d.nf)) return fail(MI_BA_ERR_HIP);
      // (a recycled context has run factorisations already: no warm-up)
    }
    if (ctx->dense && !recycled) {
      // Warm the factorisation at this size once: rocBLAS / rocSOLVER load the
      // code objects of every (shape, kernel) pair on first use, hundreds of ms
      // that would otherwise land inside the first LM iterations.
      const int64_t nf = d.nf;
      if (hipMemsetAsync(ctx->S.ptr, 0, ctx->S.bytes(), ctx->stream) != hipSuccess ||
          hipMemsetAsync(ctx->cg_x.ptr, 0, nf * 8, ctx->stream) != hipSuccess)
        return fail(MI_BA_ERR_HIP);
      hipLaunchKernelGGL(identity_kernel, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, ctx->stream, ctx->S.ptr,
                         nf, d.lds);
      unsigned werr = 0;
      const int ex = fused_rhs(ctx) ? 1 : 0;
      if (chol_factor(ctx->blas, (int)nf, ctx->S.ptr, (int)d.lds, ctx->info.ptr, ctx->chol, &ctx->cholws, ex) !=
              rocblas_status_success ||
          (ex ? chol_solve_backward(ctx->blas, (int)nf, ctx->S.ptr, (int)d.lds, ctx->cg_x.ptr, &ctx->cholws)
              : chol_solve(ctx->blas, (int)nf, ctx->S.ptr, (int)d.lds, ctx->cg_x.ptr, ctx->chol.solve,
                           &ctx->cholws)) != rocblas_status_success ||
          chol_error(&ctx->cholws, ctx->stream, &werr) != hipSuccess || werr != 0)
        return fail(MI_BA_ERR_HIP);
    }
  }
  // fixed cost of dropped blocks
  double fixed = 0.0;
  for (int64_t k : s.fixed_obs) fixed += host_block_cost(*o, p, s, k);
  ctx->fixed_cost = fixed;
  if (sem) {
    st = semantic_create(ctx, sem);
    if (st != MI_BA_OK) return fail(st);
  }
  if (gsba) {
    st = gsba_create(ctx, gsba);
    if (st != MI_BA_OK) return fail(st);
  }
  *out = ctx;
  return MI_BA_OK;
}

void context_destroy(mi_ba_context* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  // collectives still pending (a solve that returned on another error after
  // enqueuing them): waited on against their deadline first, a dead peer
  // aborting the communicator, so that the stream sync below cannot hang
  if (ctx->comm && ctx->comm_due > 0.0) (void)comm_drain(ctx);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  semantic_destroy(ctx);
  gsba_destroy(ctx);
  for (auto& e : ctx->timer.pending) {
    (void)hipEventDestroy(e.second.first);
    (void)hipEventDestroy(e.second.second);
  }
  for (auto e : ctx->timer.pool) (void)hipEventDestroy(e);
  ctx->cholws.destroy();
  if (ctx->blas) (void)rocblas_destroy_handle(ctx->blas);
  if (ctx->comm) {
    // finalize (flushes the communicator's pending work; non-blocking, so
    // polled with a bound), then destroy; a communicator that does not
    // finalize cleanly is aborted
    const ncclResult_t f = ncclCommFinalize(ctx->comm);
    bool clean = f == ncclSuccess || f == ncclInProgress;
    const double deadline = now_s() + 10.0;
    while (clean) {
      ncclResult_t e = ncclSuccess;
      if (ncclCommGetAsyncError(ctx->comm, &e) != ncclSuccess) { clean = false; break; }
      if (e == ncclSuccess) break;
      if (e != ncclInProgress || now_s() > deadline) { clean = false; break; }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    (void)(clean ? ncclCommDestroy(ctx->comm) : ncclCommAbort(ctx->comm));
    ctx->comm = nullptr;
  }
  if (ctx->host_scalars) (void)hipHostFree(ctx->host_scalars);
  if (ctx->host_info) (void)hipHostFree(ctx->host_info);
  if (ctx->stall_flag) (void)hipHostFree(ctx->stall_flag);
  if (ctx->lin_side) {
    (void)hipStreamSynchronize(ctx->lin_side);
    (void)hipStreamDestroy(ctx->lin_side);
  }
  if (ctx->lm_side) {
    (void)hipStreamSynchronize(ctx->lm_side);
    (void)hipStreamDestroy(ctx->lm_side);
  }
  if (ctx->lm_ev[0]) (void)hipEventDestroy(ctx->lm_ev[0]);
  if (ctx->lm_ev[1]) (void)hipEventDestroy(ctx->lm_ev[1]);
  if (ctx->lin_ev[0]) (void)hipEventDestroy(ctx->lin_ev[0]);
  if (ctx->lin_ev[1]) (void)hipEventDestroy(ctx->lin_ev[1]);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

// Residuals + Jacobians + point blocks at the current parameters; cost into
// scalars[kCost] (geometric) + scalars[kSemCost] (semantic).
// The PCG path's camera-major copy of J, rebuilt after each linearization
// (one gather pass; the ~10-20 camera-side passes of an LM iteration then
// read their rows contiguously instead of gathering them).  Null when the
// key is off or the copy does not fit (the passes then gather from J).
static const double* pcg_jcm(mi_ba_context* ctx) {
  if (!ctx->pcg_jcm || ctx->dense || ctx->pcg_mf) return nullptr;
  const size_t nb = ctx->cm_perm.n;
  if (!ctx->Jcm.ptr || ctx->Jcm.n != ctx->J.n) {
    if (nb == 0 || ctx->Jcm.alloc(ctx->J.n) != hipSuccess) {
      (void)hipGetLastError();
      ctx->Jcm.release();
      return nullptr;
    }
    ctx->jcm_stale = true;
  }
  if (ctx->jcm_stale) {
    Phase ph_(ctx, "permute_rows");
    launch_permute_rows(ctx->dev, ctx->cm_perm.ptr, (int64_t)nb, ctx->J.ptr, ctx->Jcm.ptr, ctx->stream);
    ctx->jcm_stale = false;
  }
  return ctx->Jcm.ptr;
}

// point blocks on the point chunks unless the tools-build key says per point
static const uint32_t* pn_chunks(mi_ba_context* ctx) { return ctx->pn_chunks ? ctx->pchunks.ptr : nullptr; }

mi_ba_status context_linearize(mi_ba_context* ctx, double* cost_out) {
  hipStream_t s = ctx->stream;
  const DevProblem& d = ctx->dev;
  hipEvent_t stop;
  ctx->jcm_stale = true;
  ctx->xcm_stale = true;
  // image records + the scalar slots zeroed in one launch
  launch_pack_images(d, ctx->img_rec.ptr, s, ctx->scalars.ptr, kNumScalars);
#ifdef MI_BA_AB_VARIANTS
  // Step layouts measured slower than the default (tools build only):
  // linearize_overlap: 1 the semantic kernels on a second stream beside the
  // reprojection kernel; 2 the semantic flat pass first, then its
  // deferred-sample pass (latency-bound) on the second stream beside the
  // reprojection kernel (HBM-write-bound); joined below
  const bool overlap = ctx->sem && ctx->lin_overlap == 1;
  const bool split = ctx->sem && ctx->lin_overlap == 2;
  // warm_conc (tools build, linearize_warm_concurrent): the semantic pass
  // first; while its deferred pass runs, touch_kernel streams the reprojection
  // kernel's inputs on a side stream (measured: only the ids and points stay
  // cached that way, profiles/r4_ab_linearize_warm_ranges.jsonl)
  const bool warm = ctx->sem && !overlap && !split && ctx->lin_warm_conc && ctx->sem_variant == 6 && d.nb > 0;
  if ((overlap || split || warm) && !ctx->lin_side) {
    if (hipStreamCreateWithFlags(&ctx->lin_side, hipStreamNonBlocking) != hipSuccess) {
      ctx->lin_side = nullptr;
      return MI_BA_ERR_HIP;
    }
    MI_HIP(hipEventCreateWithFlags(&ctx->lin_ev[0], hipEventDisableTiming));
    MI_HIP(hipEventCreateWithFlags(&ctx->lin_ev[1], hipEventDisableTiming));
  }
  if (split) {
    mi_ba_status st = semantic_linearize(ctx, ctx->scalars.ptr + kSemCost, false, ctx->lin_side, ctx->lin_ev[0]);
    if (st != MI_BA_OK) return st;
    MI_HIP(hipEventRecord(ctx->lin_ev[1], ctx->lin_side));
  }
  if (overlap) {
    // with linearize_warm_inputs: the inputs streamed in first, then the two
    // passes side by side
    MI_HIP(hipEventRecord(ctx->lin_ev[0], s));
    MI_HIP(hipStreamWaitEvent(ctx->lin_side, ctx->lin_ev[0], 0));
    ctx->stream = ctx->lin_side;  // semantic_linearize launches (and times) on ctx->stream
    mi_ba_status st = semantic_linearize(ctx, ctx->scalars.ptr + kSemCost, false);
    ctx->stream = s;
    if (st != MI_BA_OK) return st;
    MI_HIP(hipEventRecord(ctx->lin_ev[1], ctx->lin_side));
  }
  if (warm) {
    auto after_flat = [&]() -> mi_ba_status {
      MI_HIP(hipEventRecord(ctx->lin_ev[0], s));
      MI_HIP(hipStreamWaitEvent(ctx->lin_side, ctx->lin_ev[0], 0));
      launch_touch_inputs(d, reinterpret_cast<unsigned*>(ctx->scalars.ptr + kNumScalars - 1), ctx->lin_side,
                          ctx->lin_warm_conc, ctx->warm_wgs);
      MI_HIP(hipEventRecord(ctx->lin_ev[1], ctx->lin_side));
      return MI_BA_OK;
    };
    mi_ba_status st = semantic_linearize(ctx, ctx->scalars.ptr + kSemCost, false, nullptr, nullptr, nullptr, nullptr, 0,
                                         nullptr, nullptr, after_flat);
    if (st != MI_BA_OK) return st;
    MI_HIP(hipStreamWaitEvent(s, ctx->lin_ev[1], 0));
  }
  // lin_order: 0 reprojection then semantic, 1 semantic first (A/B of the
  // reprojection kernel's in-step time after the semantic gathers)
  const bool sem_first = ctx->sem && !overlap && !split && !warm && ctx->lin_order == 1;
  if (sem_first) {
    mi_ba_status st = semantic_linearize(ctx, ctx->scalars.ptr + kSemCost, false);
    if (st != MI_BA_OK) return st;
  }
  // prep_early (semantic_prep_early; measured slower, off): the semantic pair
  // tables formed on the side stream beside the warm-up and the reprojection
  // kernel (they read the poses only), instead of on the critical path after
  // it — the warm-up beside it slows by more (profiles/r4q_ab_prep_early.jsonl)
  hipEvent_t prep_ev = nullptr;
  if (ctx->sem && ctx->sem_prep_early && !overlap && !split && !warm && !sem_first && ctx->sem_variant == 6) {
    if (!ctx->lin_side) {
      if (hipStreamCreateWithFlags(&ctx->lin_side, hipStreamNonBlocking) != hipSuccess) {
        ctx->lin_side = nullptr;
        return MI_BA_ERR_HIP;
      }
      MI_HIP(hipEventCreateWithFlags(&ctx->lin_ev[0], hipEventDisableTiming));
      MI_HIP(hipEventCreateWithFlags(&ctx->lin_ev[1], hipEventDisableTiming));
    }
    MI_HIP(hipEventRecord(ctx->lin_ev[0], s));
    MI_HIP(hipStreamWaitEvent(ctx->lin_side, ctx->lin_ev[0], 0));
    mi_ba_status st = semantic_pair_prep(ctx, ctx->lin_side);
    if (st != MI_BA_OK) return st;
    MI_HIP(hipEventRecord(ctx->lin_ev[1], ctx->lin_side));
    prep_ev = ctx->lin_ev[1];
  }
#else
  // the product's one layout: input warm-up, reprojection kernel, semantic pass
  constexpr bool overlap = false, split = false, warm = false, sem_first = false;
  hipEvent_t prep_ev = nullptr;
#endif
  // linearize_warm_inputs (default: every range): the reprojection kernel's
  // streamed inputs (264 MB at C4) read right before it, so the memory-side
  // cache serves its reads and HBM sees its J / r write stream alone (in-step
  // 0.576 -> 0.431 ms at C4 for a 0.055 ms read; the observations or ids alone
  // do not do it: profiles/r4_ab_linearize_warm_ranges.jsonl).  Only after the
  // semantic pass has used the cache; a geometric-only step finds them cached.
  hipEvent_t wstop = nullptr;
  if (ctx->sem && ctx->lin_warm && d.nb > 0) {
    timer_begin(ctx, "input_warm", &wstop);
    launch_touch_inputs(d, reinterpret_cast<unsigned*>(ctx->scalars.ptr + kNumScalars - 1), s, ctx->lin_warm,
                        ctx->warm_wgs, ctx->warm_unroll);
    timer_end(ctx, wstop);
  }
  timer_begin_after(ctx, "reproj_jacobian", wstop, &stop);  // starts at the warm-up's stop event
  launch_reproj_jacobian(d, ctx->r.ptr, ctx->J.ptr, ctx->partial.ptr, s);
  timer_end(ctx, stop);
  // default layout: the semantic pass right behind the reprojection kernel
  // (its timer starts at the reprojection kernel's stop event), then both
  // cost sums in one launch
  const bool sem_after = ctx->sem && !overlap && !split && !sem_first && !warm;
  if (sem_after) {
    mi_ba_status st = semantic_linearize(ctx, ctx->scalars.ptr + kSemCost, false, nullptr, nullptr, stop,
                                         d.nb ? ctx->partial.ptr : nullptr, reproj_grid(d.nb),
                                         ctx->scalars.ptr + kCost, ctx->sum_ws.ptr, nullptr, prep_ev);
    if (st != MI_BA_OK) return st;
  } else if (d.nb) {
    launch_sum(ctx->partial.ptr, reproj_grid(d.nb), ctx->scalars.ptr + kCost, s, ctx->sum_ws.ptr);
  }
  if (overlap || split) MI_HIP(hipStreamWaitEvent(s, ctx->lin_ev[1], 0));
  if (ctx->gsba) {
    mi_ba_status st = gsba_linearize(ctx, ctx->scalars.ptr + kGsCost);
    if (st != MI_BA_OK) return st;
  }
  MI_HIP(hipGetLastError());
  if (ctx->distributed() && cost_out) {
    mi_ba_status st = allreduce(ctx, ctx->scalars.ptr + kCost, 1);
    if (st == MI_BA_OK) st = allreduce(ctx, ctx->scalars.ptr + kSemCost, 1);
    if (st != MI_BA_OK) return st;
  }
  if (cost_out) {
    mi_ba_status st = read_scalars(ctx, 0, kNumScalars);
    if (st != MI_BA_OK) return st;
    *cost_out = ctx->host_scalars[kCost] + ctx->host_scalars[kSemCost] + ctx->host_scalars[kGsCost];
  }
  return MI_BA_OK;
}

namespace {

// One Schur product y = S x including the semantic pair term.  Multi-rank:
// every rank forms the product of its own points' observations and semantic
// pairs (the damping diagonal on rank 0 only) and the ranks sum y — one
// nf-vector all-reduce per product, the x / r / z / p vectors stay
// replicated (identical bits on every rank).
// The matrix-free product's camera-major copies (null when off or they do
// not fit: the product then reads J).
static const double* pcg_xcm(mi_ba_context* ctx) {
  if (!ctx->pcg_mf || ctx->dense || !ctx->pp_chunks) return nullptr;
  const size_t nb = ctx->cm_perm.n;
  const bool robust = ctx->dev.loss_type != MI_BA_LOSS_TRIVIAL;
  if (nb == 0) return nullptr;
  if (!ctx->Xcm.ptr || ctx->Xcm.n != 3 * nb || (robust && ctx->obs_cm.n != nb)) {
    if (ctx->Xcm.alloc(3 * nb) != hipSuccess || (robust && ctx->obs_cm.alloc(nb) != hipSuccess)) {
      (void)hipGetLastError();
      ctx->Xcm.release();
      ctx->obs_cm.release();
      return nullptr;
    }
    ctx->xcm_stale = true;
  }
  if (ctx->xcm_stale) {
    Phase ph_(ctx, "gather_cm");
    launch_gather_cm(ctx->dev, ctx->cm_perm.ptr, (int64_t)nb, ctx->Xcm.ptr, robust ? ctx->obs_cm.ptr : nullptr,
                     ctx->stream);
    ctx->xcm_stale = false;
  }
  return ctx->Xcm.ptr;
}

mi_ba_status schur_product(mi_ba_context* ctx, const double* x, double* y) {
  const DevProblem& d = ctx->dev;
  const double* xcm = pcg_xcm(ctx);
  launch_schur_product(d, ctx->vpoints.ptr, ctx->npv, ctx->tiles.ptr, ctx->ntiles, ctx->cm_perm.ptr, ctx->J.ptr,
                       ctx->Vinv.ptr, ctx->rank == 0 ? ctx->lambda_f.ptr : nullptr, x, ctx->cg_w.ptr, y, ctx->stream,
                       ctx->pp_chunks ? ctx->pchunks.ptr : nullptr, ctx->npchunks,
                       ctx->pp_chunks ? ctx->cm_ptv.ptr : nullptr, ctx->pcg_jcm && !ctx->jcm_stale ? ctx->Jcm.ptr : nullptr,
                       ctx->pcg_jcm == 2, xcm, xcm && ctx->obs_cm.ptr ? ctx->obs_cm.ptr : nullptr, ctx->owners());
  if (ctx->sem) semantic_schur_product(ctx, x, y);
  if (ctx->gsba) gsba_schur_product(ctx, x, y);
  return allreduce(ctx, y, d.nf);
}

// Preconditioned CG on the Schur complement, Ceres 2.1
// ConjugateGradientsSolver semantics (restated): x = 0, r = b; q-termination
// i (Q1 - Q0) / Q1 < eta with Q = -x'(b + r); r_tolerance off
// (LevenbergMarquardtStrategy passes -1); residual recomputed every 10
// iterations; FAILURE on rho or beta = rho / rho_prev 0 / inf or alpha inf
// (*failed: an invalid LM step, TrustRegionMinimizer::ComputeTrustRegionStep),
// NO_CONVERGENCE on pq <= 0 / inf or the iteration cap (the step is used).
// Where Ceres stops before x moves, the device step (launch_cg_step) leaves x
// and r as they are.  One host round trip per iteration (the scalars).
mi_ba_status pcg(mi_ba_context* ctx, int* iterations, bool* failed) {
  const DevProblem& d = ctx->dev;
  hipStream_t s = ctx->stream;
  const int64_t nf = d.nf;
  double* sc = ctx->scalars.ptr;
  double* hs = ctx->host_scalars;
  *failed = false;
  MI_HIP(hipMemsetAsync(ctx->cg_x.ptr, 0, nf * 8, s));
  MI_HIP(hipMemcpyAsync(ctx->cg_r.ptr, ctx->bvec.ptr, nf * 8, hipMemcpyDeviceToDevice, s));
  launch_dot(ctx->bvec.ptr, ctx->bvec.ptr, nf, sc + kXB, s);
  mi_ba_status st = read_scalars(ctx, kXB, 1);
  if (st != MI_BA_OK) return st;
  *iterations = 0;
  if (hs[kXB] == 0.0) return MI_BA_OK;  // "Convergence. |b| = 0."
  auto zero_or_inf = [](double v) { return v == 0.0 || std::isinf(v) || std::isnan(v); };
  double Q0 = 0.0;
  const int max_it = std::max(1, ctx->options.max_linear_solver_iterations);
  for (int it = 1; it <= max_it; ++it) {
    launch_precond(d, ctx->prec_pose.ptr, ctx->prec_cam.ptr, ctx->cg_r.ptr, ctx->cg_z.ptr, s);
    if (ctx->gsba) gsba_precond(ctx, ctx->cg_r.ptr, ctx->cg_z.ptr);
    if (it > 1) MI_HIP(hipMemcpyAsync(sc + kRhoPrev, sc + kRho, 8, hipMemcpyDeviceToDevice, s));
    launch_dot(ctx->cg_r.ptr, ctx->cg_z.ptr, nf, sc + kRho, s);
    if (it == 1) {
      MI_HIP(hipMemcpyAsync(ctx->cg_p.ptr, ctx->cg_z.ptr, nf * 8, hipMemcpyDeviceToDevice, s));
    } else {
      launch_xpby(ctx->cg_p.ptr, ctx->cg_z.ptr, sc + kRho, sc + kRhoPrev, nf, s);
    }
    st = schur_product(ctx, ctx->cg_p.ptr, ctx->cg_q.ptr);
    if (st != MI_BA_OK) return st;
    launch_dot(ctx->cg_p.ptr, ctx->cg_q.ptr, nf, sc + kPQ, s);
    const double* rho_prev = it > 1 ? sc + kRhoPrev : nullptr;
    if (it % 10 == 0) {
      // x += alpha p, then r = b - S x
      launch_cg_step(ctx->cg_x.ptr, ctx->cg_p.ptr, nullptr, nullptr, sc + kRho, rho_prev, sc + kPQ, false, nf, s);
      st = schur_product(ctx, ctx->cg_x.ptr, ctx->cg_q.ptr);
      if (st != MI_BA_OK) return st;
      MI_HIP(hipMemcpyAsync(ctx->cg_r.ptr, ctx->bvec.ptr, nf * 8, hipMemcpyDeviceToDevice, s));
      MI_HIP(hipMemcpyAsync(sc + kXR, sc + kPQ, 8, hipMemcpyDeviceToDevice, s));  // keep pq
      double one = 1.0;
      MI_HIP(hipMemcpyAsync(sc + kStepNorm, &one, 8, hipMemcpyHostToDevice, s));
      launch_axpy(ctx->cg_r.ptr, ctx->cg_q.ptr, sc + kStepNorm, sc + kStepNorm, -1.0, nf, s);
    } else {
      launch_cg_step(ctx->cg_x.ptr, ctx->cg_p.ptr, ctx->cg_r.ptr, ctx->cg_q.ptr, sc + kRho, rho_prev, sc + kPQ, true,
                     nf, s);
    }
    launch_dot(ctx->cg_x.ptr, ctx->bvec.ptr, nf, sc + kXB, s);
    launch_dot(ctx->cg_x.ptr, ctx->cg_r.ptr, nf, sc + kXR, s);
    st = read_scalars(ctx, kRho, 5);
    if (st != MI_BA_OK) return st;
    *iterations = it;
    const double rho = hs[kRho], pq = hs[kPQ];
    if (zero_or_inf(rho) || (it > 1 && zero_or_inf(rho / hs[kRhoPrev]))) {
      *failed = true;  // LINEAR_SOLVER_FAILURE: rho or beta 0 / inf
      break;
    }
    if (!(pq > 0.0) || std::isinf(pq)) break;  // NO_CONVERGENCE, x as it was
    if (std::isinf(rho / pq)) {
      *failed = true;  // alpha inf
      break;
    }
    const double Q1 = -1.0 * (hs[kXB] + hs[kXR]);
    const double zeta = it * (Q1 - Q0) / Q1;
    if (zeta < ctx->options.eta) break;
    Q0 = Q1;
  }
  return MI_BA_OK;
}

// Ceres' GradientToleranceReached at the current point (its Jacobian and the
// point blocks Vg current): |x - Plus(x, -g)|_inf <= gradient_tolerance with
// g = J'f, the raw tangent gradient (TrustRegionMinimizer::
// EvaluateGradientAndJacobian).  The variable points' part comes from Vg
// (one read of the point blocks); the image / camera / cylinder part needs a
// pass over the camera-side rows and is evaluated only when the point part
// alone does not already exceed the tolerance.  Multi-rank: each rank's
// point part goes into its own slot of a world-long vector (one sum), the
// camera-side gradient is summed like b.
mi_ba_status gradient_reached(mi_ba_context* ctx, bool* reached) {
  const DevProblem& d = ctx->dev;
  hipStream_t s = ctx->stream;
  const double tol = ctx->options.gradient_tolerance;
  const int nw = ctx->world;
  *reached = false;
  if (ctx->aux.n < (size_t)nw + 2 && ctx->aux.alloc(nw + 2) != hipSuccess) return MI_BA_ERR_OUT_OF_MEMORY;
  double* aux = ctx->aux.ptr;
  MI_HIP(hipMemsetAsync(aux, 0, (nw + 2) * 8, s));
  launch_grad_max_points(d, ctx->vpoints.ptr, ctx->npv, ctx->Vg.ptr, aux + ctx->rank, s);
  mi_ba_status st = allreduce(ctx, aux, nw);
  if (st != MI_BA_OK) return st;
  std::vector<double> h(nw + 2, 0.0);
  MI_HIP(hipMemcpyAsync(h.data(), aux, nw * 8, hipMemcpyDeviceToHost, s));
  MI_HIP_DRAIN(ctx, s);
  double gmax = 0.0;
  for (int k = 0; k < nw; ++k) gmax = std::max(gmax, h[k]);
  if (gmax > tol) return MI_BA_OK;
  // camera side: g_f = sum J_f' r (+ semantic pairs, GSBA blocks) into cg_z
  // (PCG scratch, free between solves)
  double* g = ctx->cg_z.ptr;
  MI_HIP(hipMemsetAsync(g, 0, d.nf * 8, s));
  launch_grad_f(d, ctx->tiles.ptr, ctx->ntiles, ctx->cm_perm.ptr, ctx->r.ptr, ctx->J.ptr, g, s, ctx->owners());
  if (ctx->sem) semantic_add_gradient(ctx, g);
  if (ctx->gsba) gsba_add_gradient(ctx, g);
  st = allreduce(ctx, g, d.nf);
  if (st != MI_BA_OK) return st;
  launch_grad_max_f(d, g, aux + nw, s);
  if (ctx->gsba) gsba_grad_max(ctx, g, aux + nw);
  MI_HIP(hipMemcpyAsync(h.data() + nw, aux + nw, 8, hipMemcpyDeviceToHost, s));
  MI_HIP_DRAIN(ctx, s);
  gmax = std::max(gmax, h[nw]);
  *reached = gmax <= tol;
  return MI_BA_OK;
}

// A device-side failure seen by this rank (a Cholesky flag wait that ran
// out) ends the solve with MI_BA_ERR_HIP on every rank: one 8-byte sum over
// the ranks, so no rank stays behind in a later collective.
mi_ba_status agree_on_error(mi_ba_context* ctx, bool failed) {
  if (!ctx->distributed()) return failed ? MI_BA_ERR_HIP : MI_BA_OK;
  double* slot = ctx->scalars.ptr + kXR;
  const double v = failed ? 1.0 : 0.0;
  MI_HIP(hipMemcpyAsync(slot, &v, 8, hipMemcpyHostToDevice, ctx->stream));
  mi_ba_status st = allreduce(ctx, slot, 1);
  if (st != MI_BA_OK) return st;
  st = read_scalars(ctx, kXR, 1);
  if (st != MI_BA_OK) return st;
  return ctx->host_scalars[kXR] != 0.0 ? MI_BA_ERR_HIP : MI_BA_OK;
}

// The Schur terms of S on ctx->stream: - sum_p W_p V_p^-1 W_p' (Z factors,
// then the image-pair tiles) and the semantic / GSBA blocks.
void launch_schur_terms(mi_ba_context* ctx) {
  const DevProblem& d = ctx->dev;
  hipEvent_t stop;
  timer_begin(ctx, "schur_build", &stop);
  const PairFlush pf{ctx->pslot.ptr,
                     ctx->spart.ptr,
                     ctx->pdest.ptr,
                     ctx->pself.ptr,
                     ctx->npdest,
                     ctx->npodest ? ctx->podest.ptr : nullptr,
                     ctx->pochunk.ptr,
                     ctx->poent.ptr,
                     ctx->popart.ptr,
                     ctx->npodest,
                     ctx->npochunk};
  // image-ordered Z rows (zorder 1) with the Z-row pair kernels only; the JG
  // record / pair-from-J variants index blocks
  DevProblem dz = d;
  dz.zorder = d.zorder && d.svariant <= 5 && ctx->pairs_pos.ptr ? 1 : 0;
  launch_dense_schur(dz, ctx->tiles.ptr, ctx->ntiles, ctx->cm_perm.ptr, ctx->cm_ptv.ptr, ctx->J.ptr, ctx->Linv.ptr,
                     ctx->Z.ptr,
                     d.svariant == 5 ? ctx->ptiles_xcd.ptr
                     : (d.svariant == 4 || d.svariant >= 6) ? ctx->ptiles_blk.ptr
                                                            : ctx->ptiles.ptr,
                     d.svariant == 5 ? ctx->nptiles_xcd : ctx->nptiles, dz.zorder ? ctx->pairs_pos.ptr : ctx->pairs.ptr,
                     ctx->S.ptr, false, ctx->stream, ctx->det_sums && ctx->pflush_ok ? &pf : nullptr);
  if (ctx->sem) semantic_add_dense(ctx, ctx->S.ptr);
  if (ctx->gsba) gsba_add_dense(ctx, ctx->S.ptr);
  timer_end(ctx, stop);
}

// Exact solve of S df = -b with the explicit reduced camera system.
// *ok = false when S is not positive definite (Ceres: invalid step).
// schur_launched: the Schur terms already run on lm_side (joined here).
// Single rank: the factor's info and the flag-wait word are only enqueued
// (ctx->chol_pending); the LM checks them at its next host wait, the model
// cost's, and treats a failed factorisation as the invalid step it is.
mi_ba_status chol_check_pending(mi_ba_context* ctx, bool* ok) {
  *ok = true;
  if (!ctx->chol_pending) return MI_BA_OK;
  ctx->chol_pending = false;
  const int leaves = ctx->chol_leaves;
  const unsigned werr = (unsigned)ctx->host_info[leaves];
  if (werr != 0) MI_HIP(hipMemsetAsync(ctx->cholws.err, 0, 4, ctx->stream));
  mi_ba_status st = agree_on_error(ctx, werr != 0);
  if (st != MI_BA_OK) return st;
  for (int k = 0; k < leaves; ++k)
    if (ctx->host_info[k] != 0) *ok = false;
  return MI_BA_OK;
}

mi_ba_status dense_solve(mi_ba_context* ctx, bool* ok, bool schur_launched) {
  const DevProblem& d = ctx->dev;
  hipStream_t s = ctx->stream;
  const int64_t nf = d.nf;
  *ok = true;
  hipEvent_t stop;
  // S was zeroed and took U from launch_fblock_dense (context_solve)
  if (schur_launched)
    MI_HIP(hipStreamWaitEvent(s, ctx->lm_ev[1], 0));
  else
    launch_schur_terms(ctx);
  if (ctx->distributed()) {
    // every rank holds the Schur contribution of its own points.  Only the
    // upper triangle (row <= col) is meaningful: one in-place all-reduce per
    // 512-row band over the band's contiguous range from its first diagonal
    // entry, [r0 nf + r0, r1 nf) — nf^2/2 + 256 nf doubles in all instead of
    // nf^2 (0.60 vs 1.15 GB over xGMI at nf = 12 000), and no pack kernels.
    Phase ph_(ctx, "s_allreduce");
    constexpr int64_t kBand = 512;
    const int64_t ld = d.lds;
    for (int64_t r0 = 0; r0 < nf; r0 += kBand) {
      const int64_t r1 = std::min<int64_t>(nf, r0 + kBand);
      mi_ba_status st = allreduce(ctx, ctx->S.ptr + r0 * ld + r0, r1 * ld - (r0 * ld + r0));
      if (st != MI_BA_OK) return st;
    }
  }
  timer_begin(ctx, "schur_build", &stop);
  launch_dense_finalize(d, ctx->lambda_f.ptr, ctx->S.ptr, s);
  timer_end(ctx, stop);
  // fused: the rhs rides in S's spare row and leaves it as the forward
  // solution y = L^-1 b (one backward sweep left); else the two sweeps on b
  const bool fused = fused_rhs(ctx);
  const unsigned gn = (unsigned)((nf + 255) / 256);
  if (fused)
    hipLaunchKernelGGL(rhs_row_kernel, dim3(gn), dim3(256), 0, s, ctx->S.ptr, nf, d.lds, ctx->bvec.ptr, 1);
  else
    MI_HIP(hipMemcpyAsync(ctx->cg_x.ptr, ctx->bvec.ptr, nf * 8, hipMemcpyDeviceToDevice, s));
  timer_begin(ctx, "cholesky", &stop);
  // S holds the upper triangle row-major == the lower triangle column-major.
  const int leaves = chol_leaf_count((int)nf, ctx->chol);
  if (chol_factor(ctx->blas, (int)nf, ctx->S.ptr, (int)d.lds, ctx->info.ptr, ctx->chol, &ctx->cholws,
                  fused ? 1 : 0) != rocblas_status_success)
    return MI_BA_ERR_HIP;
  timer_end(ctx, stop);
  // The backward sweep goes right behind the factorisation; its result is
  // used only when every diagonal block was positive definite and no flag
  // wait ran out, checked once after it (one host wait per solve instead of
  // two: the factor's info and the error word land in pinned memory).
  if (ctx->host_info_cap < leaves + 1) {
    if (ctx->host_info) (void)hipHostFree(ctx->host_info);
    ctx->host_info = nullptr;
    ctx->host_info_cap = 0;
    if (hipHostMalloc(&ctx->host_info, sizeof(int32_t) * (leaves + 1), hipHostMallocDefault) != hipSuccess) {
      ctx->host_info = nullptr;
      return MI_BA_ERR_OUT_OF_MEMORY;
    }
    ctx->host_info_cap = leaves + 1;
  }
  {
    Phase ph_(ctx, "cholesky_solve");
    if (fused) {
      hipLaunchKernelGGL(rhs_row_kernel, dim3(gn), dim3(256), 0, s, ctx->S.ptr, nf, d.lds, ctx->cg_x.ptr, 0);
      if (chol_solve_backward(ctx->blas, (int)nf, ctx->S.ptr, (int)d.lds, ctx->cg_x.ptr, &ctx->cholws) !=
          rocblas_status_success)
        return MI_BA_ERR_HIP;
    } else if (chol_solve(ctx->blas, (int)nf, ctx->S.ptr, (int)d.lds, ctx->cg_x.ptr, ctx->chol.solve, &ctx->cholws) !=
               rocblas_status_success) {
      return MI_BA_ERR_HIP;
    }
  }
  if (ctx->fail_factorizations > 0) {  // test hook
    --ctx->fail_factorizations;
    MI_HIP(hipMemsetAsync(ctx->info.ptr, 0x01, 4, s));
  }
  MI_HIP(hipMemcpyAsync(ctx->host_info, ctx->info.ptr, 4 * (size_t)leaves, hipMemcpyDeviceToHost, s));
  MI_HIP(hipMemcpyAsync(ctx->host_info + leaves, ctx->cholws.err, 4, hipMemcpyDeviceToHost, s));
  ctx->chol_pending = true;
  ctx->chol_leaves = leaves;
  if (!ctx->distributed()) return MI_BA_OK;  // checked at the LM's next host wait
  // multi-rank: checked here, agreed over the ranks (a flag wait of the
  // factorisation or the sweep that ran out makes the step invalid on every
  // rank, so no rank takes a step the others do not)
  MI_HIP_DRAIN(ctx, s);  // the S bands' sums, then the factorisation and the sweep
  return chol_check_pending(ctx, ok);
}

// Ceres RunCallbacks for one finished iteration: the stop flag, then the
// caller's IterationCallback (after writing the current point back into the
// problem arrays when update_state_every_iteration is set).  Multi-rank: the
// ranks' requests are summed so every rank takes the same decision (abort
// before terminate before continue).  Returns the MI_BA_SOLVER_* decision.
mi_ba_status run_callbacks(mi_ba_context* ctx, const mi_ba_iteration_summary& it, int32_t* decision) {
  const mi_ba_options& o = ctx->options;
  int32_t d = MI_BA_SOLVER_CONTINUE;
  if (o.stop_flag) {
    const int32_t v = __atomic_load_n(o.stop_flag, __ATOMIC_RELAXED);
    if (v == MI_BA_SOLVER_TERMINATE_SUCCESSFULLY || v == MI_BA_SOLVER_ABORT) d = v;
  }
  if (d == MI_BA_SOLVER_CONTINUE && o.iteration_callback) {
    if (o.update_state_every_iteration) {
      mi_ba_status st = context_writeback(ctx);
      if (st != MI_BA_OK) return st;
    }
    const int32_t v = o.iteration_callback(o.callback_user, &it);
    if (v == MI_BA_SOLVER_TERMINATE_SUCCESSFULLY || v == MI_BA_SOLVER_ABORT) d = v;
  }
  if (ctx->distributed()) {
    double* slot = ctx->scalars.ptr + kXB;  // kXB, kXR: PCG scratch, free between solves
    const double v[2] = {d == MI_BA_SOLVER_TERMINATE_SUCCESSFULLY ? 1.0 : 0.0, d == MI_BA_SOLVER_ABORT ? 1.0 : 0.0};
    MI_HIP(hipMemcpyAsync(slot, v, 16, hipMemcpyHostToDevice, ctx->stream));
    mi_ba_status st = allreduce(ctx, slot, 2);
    if (st != MI_BA_OK) return st;
    st = read_scalars(ctx, kXB, 2);
    if (st != MI_BA_OK) return st;
    d = ctx->host_scalars[kXR] != 0.0   ? MI_BA_SOLVER_ABORT
        : ctx->host_scalars[kXB] != 0.0 ? MI_BA_SOLVER_TERMINATE_SUCCESSFULLY
                                        : MI_BA_SOLVER_CONTINUE;
  }
  *decision = d;
  return MI_BA_OK;
}

}  // namespace

mi_ba_status context_solve(mi_ba_context* ctx, mi_ba_summary* sum) {
  if (ctx->solved) return MI_BA_ERR_STATE;
  ctx->solved = true;
  ctx->chol_pending = false;
  const double t_start = now_s();
  const mi_ba_options& o = ctx->options;
  const DevProblem& d = ctx->dev;
  hipStream_t s = ctx->stream;
  double* sc = ctx->scalars.ptr;
  double* hs = ctx->host_scalars;
  std::memset(sum, 0, sizeof(*sum));
  sum->num_residuals_reduced =
      ctx->setup.num_residuals_reduced + (ctx->sem ? ctx->sem->ns : 0) + (ctx->gsba ? ctx->gsba->nblocks : 0);
  sum->num_effective_parameters_reduced = ctx->setup.num_effective_parameters_reduced;
  sum->num_semantic_residuals = ctx->sem ? ctx->sem->ns : 0;
  sum->fixed_cost = ctx->fixed_cost;
  if (sum->num_residuals_reduced == 0 && ctx->world == 1) return MI_BA_ERR_NO_RESIDUALS;
  double tj = now_s();
  double x_cost = 0.0;
  mi_ba_status st = context_linearize(ctx, &x_cost);
  if (st != MI_BA_OK) return st;
  launch_point_normal(d, ctx->vpoints.ptr, ctx->npv, ctx->r.ptr, ctx->J.ptr, ctx->Vg.ptr, s, pn_chunks(ctx), ctx->npchunks);
  sum->jacobian_evaluation_time_in_seconds += now_s() - tj;
  sum->num_jacobian_evaluations = 1;
  sum->initial_cost = x_cost + ctx->fixed_cost;
  double radius = o.initial_trust_region_radius;
  double decrease_factor = 2.0;
  bool reuse_diag = false, first = true;
  int consecutive_invalid = 0, iteration = 0;
  sum->termination_type = MI_BA_NO_CONVERGENCE;
  // the finished iteration handed to the callbacks (iteration 0: the initial
  // evaluation, valid and successful as in Ceres' IterationZero)
  mi_ba_iteration_summary its{};
  its.step_is_valid = 1;
  its.step_is_successful = 1;
  double t_iter = t_start;
  const bool callbacks = o.iteration_callback || o.stop_flag || ctx->distributed();
  bool last_successful = true;  // iteration 0 counts as successful (IterationZero)
  while (true) {
    if (callbacks) {
      its.iteration = iteration;
      its.cost = x_cost + ctx->fixed_cost;
      its.trust_region_radius = radius;
      its.iteration_time_in_seconds = now_s() - t_iter;
      its.cumulative_time_in_seconds = now_s() - t_start;
      int32_t decision = MI_BA_SOLVER_CONTINUE;
      st = run_callbacks(ctx, its, &decision);
      if (st != MI_BA_OK) return st;
      if (decision == MI_BA_SOLVER_TERMINATE_SUCCESSFULLY) { sum->termination_type = MI_BA_USER_SUCCESS; break; }
      if (decision == MI_BA_SOLVER_ABORT) { sum->termination_type = MI_BA_USER_FAILURE; break; }
    }
    // FinalizeIterationAndCheckIfMinimizerCanContinue: the iteration cap,
    // the gradient tolerance (after a successful step or at iteration 0; with
    // the default tolerance 0 only an exactly zero gradient stops), the
    // minimum trust-region radius (1e-32)
    if (iteration >= o.max_num_iterations) { sum->termination_type = MI_BA_NO_CONVERGENCE; break; }
    if (last_successful) {
      bool reached = false;
      st = gradient_reached(ctx, &reached);
      if (st != MI_BA_OK) return st;
      if (reached) { sum->termination_type = MI_BA_CONVERGENCE; break; }
    }
    if (radius <= 1e-32) { sum->termination_type = MI_BA_CONVERGENCE; break; }
    ++iteration;
    t_iter = now_s();
    its = mi_ba_iteration_summary{};
    // Damped point inverses, Schur-Jacobi blocks, rhs.
    {
      Phase ph_(ctx, "point_prepare");
      launch_point_prepare(d, ctx->vpoints.ptr, ctx->npv, ctx->Vg.ptr, ctx->scale_p.ptr, ctx->diag_p.ptr,
                           ctx->Vinv.ptr, ctx->dense ? ctx->Linv.ptr : nullptr,
                           ctx->dense ? ctx->cg_w.ptr : nullptr,  // q_p: the PCG's point vector is free here
                           first, reuse_diag, radius, s);
    }
    MI_HIP(hipMemsetAsync(ctx->pose_blk.ptr, 0, ctx->pose_blk.bytes(), s));
    MI_HIP(hipMemsetAsync(ctx->cam_blk.ptr, 0, ctx->cam_blk.bytes(), s));
    MI_HIP(hipMemsetAsync(ctx->bvec.ptr, 0, ctx->bvec.bytes(), s));
    MI_HIP(hipMemsetAsync(ctx->udiag.ptr, 0, ctx->udiag.bytes(), s));
    if (ctx->dense) {
      Phase ph_(ctx, "s_zero");
      // the part of S the LM writes and the factorisation reads: row i of the
      // row-major upper triangle from the start of its 512-row diagonal block
      // (the trailing dgemms also rewrite the diagonal blocks' other half),
      // through the spare column — about half of S
      hipLaunchKernelGGL(zero_upper_kernel, dim3((unsigned)d.nf), dim3(256), 0, s, ctx->S.ptr, d.nf, d.lds);
    }
    // one rank: the Schur terms (fabric-bound pair gathers) on lm_side beside
    // the camera-block pass (HBM-bound row gathers); both only add into S
    // the side stream only with float-atomic flushes: the deterministic
    // flushes (det_sums) update S's diagonal blocks by plain read-modify-write
    // in FlushDense and in the Schur pair / owner flushes, which must not run
    // concurrently
    const bool schur_side = ctx->dense && !ctx->distributed() && ctx->schur_overlap && !ctx->det_sums;
    if (schur_side) {
      if (!ctx->lm_side) {
        if (hipStreamCreateWithFlags(&ctx->lm_side, hipStreamNonBlocking) != hipSuccess) {
          ctx->lm_side = nullptr;
          return MI_BA_ERR_HIP;
        }
        MI_HIP(hipEventCreateWithFlags(&ctx->lm_ev[0], hipEventDisableTiming));
        MI_HIP(hipEventCreateWithFlags(&ctx->lm_ev[1], hipEventDisableTiming));
      }
      MI_HIP(hipEventRecord(ctx->lm_ev[0], s));
      MI_HIP(hipStreamWaitEvent(ctx->lm_side, ctx->lm_ev[0], 0));
      ctx->stream = ctx->lm_side;  // launch_schur_terms launches (and times) on ctx->stream
      launch_schur_terms(ctx);
      ctx->stream = s;
      MI_HIP(hipEventRecord(ctx->lm_ev[1], ctx->lm_side));
    }
    {
      Phase ph_(ctx, "fblock");
      if (ctx->dense)
        launch_fblock_dense(d, ctx->tiles.ptr, ctx->ntiles, ctx->cm_perm.ptr, ctx->cm_ptv.ptr, ctx->r.ptr, ctx->J.ptr,
                            ctx->cg_w.ptr, ctx->bvec.ptr, ctx->udiag.ptr, ctx->S.ptr, s, ctx->owners());
      else
        launch_fblock(d, ctx->tiles.ptr, ctx->ntiles, ctx->cm_perm.ptr, ctx->r.ptr, ctx->J.ptr, pcg_jcm(ctx),
                      ctx->Vg.ptr, ctx->Vinv.ptr, ctx->pose_blk.ptr, ctx->cam_blk.ptr, ctx->bvec.ptr,
                      ctx->udiag.ptr, s, ctx->owners());
      if (ctx->sem) semantic_add_fblock(ctx);
      if (ctx->gsba) gsba_add_fblock(ctx);
    }
    if (ctx->distributed()) {
      Phase ph_(ctx, "f_allreduce");
      st = allreduce(ctx, ctx->pose_blk.ptr, (int64_t)ctx->pose_blk.n);
      if (st == MI_BA_OK) st = allreduce(ctx, ctx->cam_blk.ptr, (int64_t)ctx->cam_blk.n);
      if (st == MI_BA_OK) st = allreduce(ctx, ctx->bvec.ptr, (int64_t)ctx->bvec.n);
      if (st == MI_BA_OK) st = allreduce(ctx, ctx->udiag.ptr, (int64_t)ctx->udiag.n);
      if (st != MI_BA_OK) return st;
    }
    launch_fblock_finalize(d, ctx->pose_blk.ptr, ctx->cam_blk.ptr, ctx->udiag.ptr, ctx->scale_f.ptr,
                           ctx->diag_f.ptr, ctx->lambda_f.ptr, ctx->prec_pose.ptr, ctx->prec_cam.ptr,
                           ctx->bvec.ptr, first, reuse_diag, radius, s);
    if (ctx->gsba) gsba_finalize(ctx, first, reuse_diag, radius);
    first = false;
    reuse_diag = true;
    int cg_it = 0;
    bool solved_ok = true;
    if (ctx->dense) {
      st = dense_solve(ctx, &solved_ok, schur_side);
      cg_it = 1;
    } else {
      hipEvent_t pstop;
      timer_begin(ctx, "pcg", &pstop);
      bool failed = false;
      st = pcg(ctx, &cg_it, &failed);
      solved_ok = !failed;
      timer_end(ctx, pstop);
    }
    if (st != MI_BA_OK) return st;
    sum->num_linear_solver_iterations += cg_it;
    its.linear_solver_iterations = cg_it;
    if (!solved_ok) {
      last_successful = false;
      ++consecutive_invalid;
      ++sum->num_unsuccessful_steps;
      if (consecutive_invalid > o.max_num_consecutive_invalid_steps) {
        sum->termination_type = MI_BA_FAILURE;
        break;
      }
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      continue;
    }
    // back substitution and model cost change
    int64_t nmodel = 0;
    {
      Phase ph_(ctx, "backsub");
      nmodel = launch_backsub_chunks(d, ctx->pchunks.ptr, ctx->npchunks, ctx->J.ptr, ctx->r.ptr, ctx->Vg.ptr,
                                     ctx->Vinv.ptr, ctx->cg_x.ptr, ctx->dX.ptr, ctx->partial.ptr, s);
    }
    MI_HIP(hipMemsetAsync(sc + kModelCost, 0, 8, s));
    MI_HIP(hipMemsetAsync(sc + kSemModel, 0, 8, s));
    MI_HIP(hipMemsetAsync(sc + kGsModel, 0, 8, s));
    if (d.nb) launch_sum(ctx->partial.ptr, nmodel, sc + kModelCost, s, ctx->sum_ws.ptr);
    if (ctx->sem) semantic_model_cost(ctx, ctx->cg_x.ptr, sc + kSemModel);
    if (ctx->gsba) gsba_model_cost(ctx, ctx->cg_x.ptr, sc + kGsModel);
    if (ctx->distributed()) {
      st = allreduce(ctx, sc + kModelCost, 1);
      if (st == MI_BA_OK) st = allreduce(ctx, sc + kSemModel, 1);
      if (st != MI_BA_OK) return st;
    }
    st = read_scalars(ctx, 0, kNumScalars);
    if (st != MI_BA_OK) return st;
    // single rank: the factorisation's check, its copies landed with the scalars
    bool factored = true;
    st = chol_check_pending(ctx, &factored);
    if (st != MI_BA_OK) return st;
    const double model_cost_change = hs[kModelCost] + hs[kSemModel] + hs[kGsModel];
    const bool valid = factored && std::isfinite(model_cost_change) && model_cost_change > 0.0;
    if (!valid) {
      last_successful = false;
      ++consecutive_invalid;
      ++sum->num_unsuccessful_steps;
      if (consecutive_invalid > o.max_num_consecutive_invalid_steps) {
        sum->termination_type = MI_BA_FAILURE;
        break;
      }
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      continue;
    }
    consecutive_invalid = 0;
    its.step_is_valid = 1;
    // candidate
    launch_plus(d, ctx->cg_x.ptr, ctx->dX.ptr, ctx->qt.ptr, ctx->cam.ptr, ctx->X.ptr, ctx->qt_c.ptr,
                ctx->cam_c.ptr, ctx->X_c.ptr, s);
    if (ctx->gsba) gsba_plus(ctx, ctx->cg_x.ptr);
    MI_HIP(hipMemsetAsync(sc + kCandCost, 0, 8, s));
    MI_HIP(hipMemsetAsync(sc + kSemCand, 0, 8, s));
    MI_HIP(hipMemsetAsync(sc + kGsCand, 0, 8, s));
    {
      Phase ph_(ctx, "trial_cost");
      launch_reproj_cost(d, ctx->qt_c.ptr, ctx->cam_c.ptr, ctx->X_c.ptr, ctx->partial.ptr, s);
    }
    if (d.nb) launch_sum(ctx->partial.ptr, reproj_grid(d.nb), sc + kCandCost, s, ctx->sum_ws.ptr);
    if (ctx->sem) semantic_cost(ctx, ctx->qt_c.ptr, ctx->cam_c.ptr, sc + kSemCand);
    if (ctx->gsba) gsba_cost(ctx, ctx->qt_c.ptr, ctx->gsba->cyl_c.ptr, sc + kGsCand);
    // Ceres' |x|^2 and |x - candidate_x|^2 over the variable blocks, ambient
    // coordinates (kXB, kXR: PCG scratch, free here); images, cameras and
    // cylinders counted on rank 0, points on their own ranks
    launch_state_norms(d, ctx->qt_c.ptr, ctx->cam_c.ptr, ctx->X_c.ptr, ctx->rank == 0, sc + kXB, ctx->red.ptr, s);
    if (ctx->gsba && ctx->rank == 0) gsba_state_norms(ctx, sc + kXB);
    if (ctx->distributed()) {
      st = allreduce(ctx, sc + kCandCost, 1);
      if (st == MI_BA_OK) st = allreduce(ctx, sc + kSemCand, 1);
      if (st == MI_BA_OK) st = allreduce(ctx, sc + kXB, 2);
      if (st != MI_BA_OK) return st;
    }
    st = read_scalars(ctx, 0, kNumScalars);
    if (st != MI_BA_OK) return st;
    const double candidate_cost = hs[kCandCost] + hs[kSemCand] + hs[kGsCand];
    const double cost_change = x_cost - candidate_cost;
    const double relative_decrease = cost_change / model_cost_change;
    const bool success = std::isfinite(candidate_cost) && relative_decrease > o.min_relative_decrease;
    // ParameterToleranceReached (step_norm = |x - candidate_x| <= tol (|x| +
    // tol); with tol 0: the candidate equals x bitwise) /
    // FunctionToleranceReached: Ceres returns before accepting the candidate
    // (x stays at the current point).
    const double x_norm = std::sqrt(hs[kXB]);
    const double step_norm = std::sqrt(hs[kXR]);
    its.step_norm = step_norm;
    if (step_norm <= o.parameter_tolerance * (x_norm + o.parameter_tolerance) ||
        std::fabs(cost_change) <= o.function_tolerance * x_cost) {
      ++sum->num_unsuccessful_steps;
      sum->termination_type = MI_BA_CONVERGENCE;
      break;
    }
    its.relative_decrease = relative_decrease;
    its.cost_change = cost_change;  // every valid step, as Ceres (negative when rejected)
    last_successful = success;
    if (success) {
      ++sum->num_successful_steps;
      its.step_is_successful = 1;
      x_cost = candidate_cost;
      std::swap(ctx->qt.ptr, ctx->qt_c.ptr);
      std::swap(ctx->cam.ptr, ctx->cam_c.ptr);
      std::swap(ctx->X.ptr, ctx->X_c.ptr);
      ctx->dev.qt = ctx->qt.ptr;
      ctx->dev.cam = ctx->cam.ptr;
      ctx->dev.X = ctx->X.ptr;
      if (ctx->gsba) gsba_accept(ctx);
      radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * relative_decrease - 1.0, 3));
      radius = std::min(1e16, radius);
      decrease_factor = 2.0;
      reuse_diag = false;
      tj = now_s();
      st = context_linearize(ctx, nullptr);
      if (st != MI_BA_OK) return st;
      launch_point_normal(d, ctx->vpoints.ptr, ctx->npv, ctx->r.ptr, ctx->J.ptr, ctx->Vg.ptr, s, pn_chunks(ctx), ctx->npchunks);
      sum->num_jacobian_evaluations += 1;
      sum->jacobian_evaluation_time_in_seconds += now_s() - tj;
    } else {
      ++sum->num_unsuccessful_steps;
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
    }
  }
  sum->final_cost = x_cost + ctx->fixed_cost;
  MI_HIP_DRAIN(ctx, s);
  sum->total_time_in_seconds = now_s() - t_start;
  return MI_BA_OK;
}

mi_ba_status context_writeback(mi_ba_context* ctx) {
  mi_ba_problem* p = &ctx->problem;
  const HostSetup& s = ctx->setup;
  const int I = p->num_images, C = p->num_cameras;
  const int64_t P = p->num_points;
  std::vector<double> qt(8 * (size_t)I), cm(8 * (size_t)C), X(3 * (size_t)P);
  MI_HIP_DRAIN(ctx, ctx->stream);
  if (I) MI_HIP(hipMemcpy(qt.data(), ctx->qt.ptr, qt.size() * 8, hipMemcpyDeviceToHost));
  if (C) MI_HIP(hipMemcpy(cm.data(), ctx->cam.ptr, cm.size() * 8, hipMemcpyDeviceToHost));
  if (P) MI_HIP(hipMemcpy(X.data(), ctx->X.ptr, X.size() * 8, hipMemcpyDeviceToHost));
  for (int i = 0; i < I; ++i) {
    if (!s.img_var[i]) continue;
    for (int m = 0; m < 4; ++m) p->qvec[4 * i + m] = qt[8 * i + m];
    for (int m = 0; m < 3; ++m) p->tvec[3 * i + m] = qt[8 * i + 4 + m];
  }
  for (int c = 0; c < C; ++c) {
    if (!s.cam_var[c]) continue;
    for (int64_t m = s.cam_off[c]; m < s.cam_off[c + 1]; ++m) p->camera_params[m] = cm[8 * c + (m - s.cam_off[c])];
  }
  for (int64_t k = 0; k < P; ++k) {
    if (!s.pt_var[k]) continue;
    for (int m = 0; m < 3; ++m) p->xyz[3 * k + m] = X[3 * k + m];
  }
  if (ctx->gsba) return gsba_writeback(ctx);
  return MI_BA_OK;
}

}  // namespace miba

// ===========================================================================
// C ABI
// ===========================================================================
using namespace miba;

// Every entry point that works on a context makes the context's device current
// on the calling thread first (contexts on several devices may be driven from
// one host thread).
#define MI_BIND(ctx)                                               \
  do {                                                             \
    if (!(ctx)) return MI_BA_ERR_INVALID_ARGUMENT;                 \
    if (hipSetDevice((ctx)->device) != hipSuccess) return MI_BA_ERR_HIP; \
  } while (0)

extern "C" {

int32_t mi_ba_abi_version(void) { return MI_BA_ABI_VERSION; }

const char* mi_ba_status_string(int32_t status) {
  switch (status) {
    case MI_BA_OK: return "ok";
    case MI_BA_ERR_INVALID_ARGUMENT: return "invalid argument";
    case MI_BA_ERR_NO_DEVICE: return "no HIP device (MI355X required; no CPU fallback)";
    case MI_BA_ERR_UNSUPPORTED: return "unsupported";
    case MI_BA_ERR_HIP: return "HIP runtime error";
    case MI_BA_ERR_NO_RESIDUALS: return "problem has no residuals";
    case MI_BA_ERR_STATE: return "invalid state (single-use solver)";
    case MI_BA_ERR_OUT_OF_MEMORY: return "out of device memory";
  }
  return "unknown status";
}

int32_t mi_ba_num_params(int32_t camera_model) { return num_params(camera_model); }

mi_ba_status mi_ba_device_count(int32_t* count) {
  int n = 0;
  if (!count) return MI_BA_ERR_INVALID_ARGUMENT;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return MI_BA_OK;
}

// BundleAdjustmentOptions::BundleAdjustmentOptions (bundle_adjustment.h:49-92)
void mi_ba_default_options(mi_ba_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->loss_function_type = MI_BA_LOSS_TRIVIAL;
  o->loss_function_scale = 1.0;
  o->refine_focal_length = 1;
  o->refine_principal_point = 0;
  o->refine_extra_params = 1;
  o->refine_extrinsics = 1;
  o->print_summary = 0;
  o->max_num_iterations = 100;
  o->function_tolerance = 0.0;
  o->gradient_tolerance = 0.0;
  o->parameter_tolerance = 0.0;
  o->max_linear_solver_iterations = 200;
  o->max_num_consecutive_invalid_steps = 10;
  o->linear_solver_type = MI_BA_SOLVER_AUTO;
  o->eta = 1e-1;
  o->initial_trust_region_radius = 1e4;
  o->min_relative_decrease = 1e-3;
  o->device = 0;
  o->semantic_weight = 1.0;
  o->iteration_callback = nullptr;
  o->callback_user = nullptr;
  o->update_state_every_iteration = 0;
  o->stop_flag = nullptr;
}

mi_ba_status mi_ba_setup_stats(const mi_ba_options* o, const mi_ba_problem* p, mi_ba_setup_info* info) {
  if (!o || !p || !info) return MI_BA_ERR_INVALID_ARGUMENT;
  // SetUp normalises qvecs in place; work on a private copy of the qvecs.
  mi_ba_problem copy = *p;
  std::vector<double> q(p->qvec, p->qvec + 4 * (size_t)std::max(0, p->num_images));
  copy.qvec = q.data();
  HostSetup s;
  mi_ba_status st = build_setup(*o, &copy, &s);
  if (st != MI_BA_OK) return st;
  info->num_residual_blocks = s.num_residual_blocks;
  info->num_residuals_reduced = s.num_residuals_reduced;
  info->num_effective_parameters_reduced = s.num_effective_parameters_reduced;
  info->num_variable_images = std::accumulate(s.img_var.begin(), s.img_var.end(), (int64_t)0);
  info->num_variable_cameras = std::accumulate(s.cam_var.begin(), s.cam_var.end(), (int64_t)0);
  info->num_variable_points = std::accumulate(s.pt_var.begin(), s.pt_var.end(), (int64_t)0);
  info->camera_tangent_size = s.ct;
  return MI_BA_OK;
}

static void print_summary(const mi_ba_summary& s) {
  // PrintSolverSummary (bundle_adjustment.cc:1142-1196)
  const char* term = s.termination_type == MI_BA_CONVERGENCE ? "Convergence"
                     : s.termination_type == MI_BA_NO_CONVERGENCE ? "No convergence"
                     : s.termination_type == MI_BA_FAILURE ? "Failure"
                     : s.termination_type == MI_BA_USER_SUCCESS ? "User success"
                     : s.termination_type == MI_BA_USER_FAILURE ? "User failure" : "Unknown";
  std::printf("    Residuals : %lld\n   Parameters : %lld\n   Iterations : %d\n         Time : %g [s]\n"
              " Initial cost : %g [px]\n   Final cost : %g [px]\n  Termination : %s\n\n",
              (long long)s.num_residuals_reduced, (long long)s.num_effective_parameters_reduced,
              s.num_successful_steps + s.num_unsuccessful_steps, s.total_time_in_seconds,
              std::sqrt(s.initial_cost / s.num_residuals_reduced), std::sqrt(s.final_cost / s.num_residuals_reduced),
              term);
}

namespace {
// Ceres copies the solver state back into the user's parameter blocks only
// for a usable solution: not after FAILURE or USER_FAILURE (Solver::Solve).
bool solution_usable(const mi_ba_summary& s) {
  return s.termination_type != MI_BA_FAILURE && s.termination_type != MI_BA_USER_FAILURE;
}

// One BundleAdjuster::Solve on *arena (recycled, or created when null); the
// context is kept in *arena for the next solve, or destroyed on failure.
mi_ba_status solve_on(mi_ba_context** arena, const mi_ba_options* o, mi_ba_problem* p, const mi_ba_semantic* sem,
                      mi_ba_summary* sum) {
  if (!o || !p || !sum) return MI_BA_ERR_INVALID_ARGUMENT;
  const double t0 = now_s();
  mi_ba_context* ctx = nullptr;
  mi_ba_status st = context_recycle(*arena, o, p, sem, &ctx);
  *arena = ctx;
  if (st != MI_BA_OK) return st;
  // SetUp normalised the config qvecs of ctx->problem (== caller arrays).
  st = context_solve(ctx, sum);
  if (st == MI_BA_OK && solution_usable(*sum)) st = context_writeback(ctx);
  if (st != MI_BA_OK) {
    context_destroy(ctx);
    *arena = nullptr;
  }
  sum->total_time_in_seconds = now_s() - t0;
  if (st == MI_BA_OK && o->print_summary) print_summary(*sum);
  return st;
}
}  // namespace

void mi_ba_default_gsba(mi_ba_gsba* g) {
  if (!g) return;
  std::memset(g, 0, sizeof(*g));
  g->refine_geometry = 1;
  g->numeric_relative_step_size = 1e-3;
  g->include_landmark_error = 0;
  g->landmark_error_weight = 1.0;
  g->cylinder_parametrization = MI_BA_CYLINDER_DEFAULT;
}

// The GSBA problem (geometric_semantic_bundle_adjustment.cc:714-800): TRIVIAL
// loss required (Assert); the reprojection blocks only with
// include_landmark_error, under ScaledLoss(landmark_error_weight / #2D
// features of the config images).
static mi_ba_status gsba_problem(const mi_ba_options* o, const mi_ba_problem* p, const mi_ba_gsba* g,
                                 mi_ba_options* oo, mi_ba_problem* pp) {
  if (!o || !p || !g) return MI_BA_ERR_INVALID_ARGUMENT;
  if (o->loss_function_type != MI_BA_LOSS_TRIVIAL) return MI_BA_ERR_UNSUPPORTED;
  *oo = *o;
  *pp = *p;
  if (!g->include_landmark_error) {
    pp->num_obs = 0;
  } else {
    int64_t total = 0;
    for (int64_t k = 0; k < p->num_obs; ++k) {
      const int32_t i = p->obs_image[k];
      if (i < 0 || i >= p->num_images) return MI_BA_ERR_INVALID_ARGUMENT;
      total += p->image_in_config ? (p->image_in_config[i] != 0) : 1;
    }
    oo->loss_function_type = kLossScaled;
    oo->loss_function_scale = g->landmark_error_weight / (double)std::max<int64_t>(1, total);
  }
  return MI_BA_OK;
}

mi_ba_status mi_ba_gsba_solve(const mi_ba_options* o, mi_ba_problem* p, mi_ba_gsba* g, mi_ba_summary* sum) {
  if (!sum) return MI_BA_ERR_INVALID_ARGUMENT;
  mi_ba_options oo;
  mi_ba_problem pp;
  mi_ba_status st = gsba_problem(o, p, g, &oo, &pp);
  if (st != MI_BA_OK) return st;
  const double t0 = now_s();
  mi_ba_context* ctx = nullptr;
  st = context_recycle(nullptr, &oo, &pp, nullptr, &ctx, g);
  if (st != MI_BA_OK) return st;
  st = context_solve(ctx, sum);
  if (st == MI_BA_OK && solution_usable(*sum)) st = context_writeback(ctx);
  context_destroy(ctx);
  sum->total_time_in_seconds = now_s() - t0;
  if (st == MI_BA_OK && o->print_summary) print_summary(*sum);
  return st;
}

mi_ba_status mi_ba_gsba_evaluate(const mi_ba_options* o, mi_ba_problem* p, const mi_ba_gsba* g, int64_t capacity,
                                 int64_t* num_blocks, int32_t* ids, double* residuals, double* jacobians) {
  if (!num_blocks) return MI_BA_ERR_INVALID_ARGUMENT;
  mi_ba_options oo;
  mi_ba_problem pp;
  mi_ba_status st = gsba_problem(o, p, g, &oo, &pp);
  if (st != MI_BA_OK) return st;
  mi_ba_context* ctx = nullptr;
  st = context_recycle(nullptr, &oo, &pp, nullptr, &ctx, g);
  if (st != MI_BA_OK) return st;
  *num_blocks = ctx->gsba->nblocks;
  if (*num_blocks <= capacity && *num_blocks > 0) {
    if (!ids || !residuals || !jacobians) st = MI_BA_ERR_INVALID_ARGUMENT;
    else st = gsba_download(ctx, ids, residuals, jacobians);
  }
  context_destroy(ctx);
  return st;
}

mi_ba_status mi_ba_solve_in(mi_ba_context** arena, const mi_ba_options* o, mi_ba_problem* p,
                            const mi_ba_semantic* sem, mi_ba_summary* sum) {
  if (!arena) return MI_BA_ERR_INVALID_ARGUMENT;
  return solve_on(arena, o, p, sem, sum);
}

mi_ba_status mi_ba_solve(const mi_ba_options* o, mi_ba_problem* p, const mi_ba_semantic* sem, mi_ba_summary* sum) {
  mi_ba_context* ctx = nullptr;
  const mi_ba_status st = solve_on(&ctx, o, p, sem, sum);
  context_destroy(ctx);
  return st;
}

// Independent problems solved concurrently: up to max_concurrent host
// threads, each running whole solves on a context of its own (own HIP
// stream, rocBLAS handles, workspaces), so the small, latency-bound kernels
// and host round trips of one local problem overlap those of the others.
mi_ba_status mi_ba_solve_batch(const mi_ba_options* options, mi_ba_problem* problems,
                               const mi_ba_semantic* const* semantics, int32_t n, int32_t max_concurrent,
                               mi_ba_summary* summaries, int32_t* statuses) {
  if (n < 0 || (n > 0 && (!options || !problems || !summaries || !statuses))) return MI_BA_ERR_INVALID_ARGUMENT;
  if (n == 0) return MI_BA_OK;
  const int workers = std::max(1, std::min<int>(max_concurrent > 0 ? max_concurrent : 8, n));
  std::atomic<int> next{0};
  auto run = [&]() {
    // each worker recycles one context across its problems (device arrays,
    // stream, rocBLAS handles and workspaces are allocated once)
    mi_ba_context* arena = nullptr;
    for (int k = next.fetch_add(1); k < n; k = next.fetch_add(1)) {
      summaries[k] = mi_ba_summary{};
      statuses[k] = solve_on(&arena, &options[k], &problems[k], semantics ? semantics[k] : nullptr, &summaries[k]);
    }
    context_destroy(arena);
  };
  std::vector<std::thread> pool;
  for (int w = 1; w < workers; ++w) pool.emplace_back(run);
  run();
  for (auto& t : pool) t.join();
  return MI_BA_OK;
}

mi_ba_status mi_ba_context_create(const mi_ba_options* o, const mi_ba_problem* p, const mi_ba_semantic* sem,
                                  mi_ba_context** ctx) {
  return context_create(o, p, sem, ctx);
}

void mi_ba_context_destroy(mi_ba_context* ctx) { context_destroy(ctx); }

mi_ba_status mi_ba_linearize(mi_ba_context* ctx) {
  MI_BIND(ctx);
  return context_linearize(ctx, nullptr);
}

mi_ba_status mi_ba_evaluate_jacobian(mi_ba_context* ctx) {
  MI_BIND(ctx);
  const DevProblem& d = ctx->dev;
  hipEvent_t stop;
  launch_pack_images(d, ctx->img_rec.ptr, ctx->stream);
  timer_begin(ctx, "reproj_jacobian", &stop);
  launch_reproj_jacobian(d, ctx->r.ptr, ctx->J.ptr, ctx->partial.ptr, ctx->stream);
  timer_end(ctx, stop);
  MI_HIP(hipGetLastError());
  return MI_BA_OK;
}

mi_ba_status mi_ba_evaluate_semantic(mi_ba_context* ctx) {
  MI_BIND(ctx);
  if (!ctx->sem) return MI_BA_ERR_INVALID_ARGUMENT;
  return semantic_linearize(ctx, ctx->scalars.ptr + kSemCost, true);
}

mi_ba_status mi_ba_synchronize(mi_ba_context* ctx) {
  MI_BIND(ctx);
  MI_HIP_DRAIN(ctx, ctx->stream);
  return MI_BA_OK;
}

mi_ba_status mi_ba_context_dims(const mi_ba_context* ctx, int64_t* nb, int32_t* cols, int64_t* ns) {
  if (!ctx) return MI_BA_ERR_INVALID_ARGUMENT;
  if (nb) *nb = ctx->dev.nb;
  if (cols) *cols = ctx->dev.W;
  if (ns) *ns = ctx->sem ? ctx->sem->ns : 0;
  return MI_BA_OK;
}

mi_ba_status mi_ba_download_jacobian(mi_ba_context* ctx, int64_t* block_obs, double* residuals, double* jacobian) {
  MI_BIND(ctx);
  const int64_t nb = ctx->dev.nb;
  MI_HIP_DRAIN(ctx, ctx->stream);
  if (block_obs) std::memcpy(block_obs, ctx->block_obs.data(), nb * sizeof(int64_t));
  if (residuals && nb) MI_HIP(hipMemcpy(residuals, ctx->r.ptr, nb * sizeof(double2), hipMemcpyDeviceToHost));
  if (jacobian && nb)
    MI_HIP(hipMemcpy(jacobian, ctx->J.ptr, (size_t)nb * 2 * ctx->dev.W * sizeof(double), hipMemcpyDeviceToHost));
  return MI_BA_OK;
}

mi_ba_status mi_ba_download_semantic(mi_ba_context* ctx, int32_t* sample_pixel, int32_t* status, double* residuals,
                                     double* jacobian) {
  MI_BIND(ctx);
  if (!ctx->sem) return MI_BA_ERR_INVALID_ARGUMENT;
  SemanticState* S = ctx->sem;
  MI_HIP_DRAIN(ctx, ctx->stream);
  if (!S->samples_valid) return MI_BA_ERR_STATE;  // mi_ba_evaluate_semantic first
  const int64_t n = S->ns;
  if (sample_pixel) std::memcpy(sample_pixel, S->sample_pixel_host.data(), 3 * n * sizeof(int32_t));
  if (n == 0) return MI_BA_OK;
  if (status) MI_HIP(hipMemcpy(status, S->status.ptr, n * 4, hipMemcpyDeviceToHost));
  if (residuals) MI_HIP(hipMemcpy(residuals, S->r.ptr, n * 8, hipMemcpyDeviceToHost));
  if (jacobian) MI_HIP(hipMemcpy(jacobian, S->J.ptr, 12 * n * 8, hipMemcpyDeviceToHost));
  return MI_BA_OK;
}

mi_ba_status mi_ba_semantic_export(mi_ba_context* ctx, int32_t image1, int32_t image2, int64_t* count,
                                   int32_t* pixels, int32_t* status, double* error, double* world) {
  MI_BIND(ctx);
  return semantic_export(ctx, image1, image2, count, pixels, status, error, world);
}

mi_ba_status mi_ba_context_solve(mi_ba_context* ctx, mi_ba_summary* summary) {
  if (!summary) return MI_BA_ERR_INVALID_ARGUMENT;
  MI_BIND(ctx);
  return context_solve(ctx, summary);
}

mi_ba_status mi_ba_context_writeback(mi_ba_context* ctx) {
  MI_BIND(ctx);
  return context_writeback(ctx);
}

mi_ba_status mi_ba_context_cost(mi_ba_context* ctx, double* cost) {
  if (!cost) return MI_BA_ERR_INVALID_ARGUMENT;
  MI_BIND(ctx);
  hipStream_t s = ctx->stream;
  double* sc = ctx->scalars.ptr;
  MI_HIP(hipMemsetAsync(sc + kCandCost, 0, 8, s));
  MI_HIP(hipMemsetAsync(sc + kSemCand, 0, 8, s));
  launch_reproj_cost(ctx->dev, ctx->qt.ptr, ctx->cam.ptr, ctx->X.ptr, ctx->partial.ptr, s);
  if (ctx->dev.nb) launch_sum(ctx->partial.ptr, reproj_grid(ctx->dev.nb), sc + kCandCost, s, ctx->sum_ws.ptr);
  if (ctx->sem) semantic_cost(ctx, ctx->qt.ptr, ctx->cam.ptr, sc + kSemCand);
  MI_HIP(hipMemsetAsync(sc + kGsCand, 0, 8, s));
  if (ctx->gsba) gsba_cost(ctx, ctx->qt.ptr, ctx->gsba->cyl.ptr, sc + kGsCand);
  mi_ba_status st = allreduce(ctx, sc + kCandCost, 1);
  if (st == MI_BA_OK) st = allreduce(ctx, sc + kSemCand, 1);
  if (st != MI_BA_OK) return st;
  st = read_scalars(ctx, 0, kNumScalars);
  if (st != MI_BA_OK) return st;
  *cost = ctx->host_scalars[kCandCost] + ctx->host_scalars[kSemCand] + ctx->host_scalars[kGsCand] +
          ctx->fixed_cost;
  return MI_BA_OK;
}

// Fixed cost of the dropped all-constant blocks, summed over the ranks' shards.
static mi_ba_status reduce_fixed_cost(mi_ba_context* ctx) {
  double* slot = ctx->scalars.ptr + kXR;
  MI_HIP(hipMemcpyAsync(slot, &ctx->fixed_cost, 8, hipMemcpyHostToDevice, ctx->stream));
  mi_ba_status st = allreduce(ctx, slot, 1);
  if (st != MI_BA_OK) return st;
  MI_HIP(hipMemcpyAsync(&ctx->fixed_cost, slot, 8, hipMemcpyDeviceToHost, ctx->stream));
  MI_HIP_DRAIN(ctx, ctx->stream);
  return MI_BA_OK;
}

mi_ba_status mi_ba_comm_unique_id(char id[MI_BA_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) <= MI_BA_COMM_ID_BYTES, "RCCL unique id size");
  if (!id) return MI_BA_ERR_INVALID_ARGUMENT;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return MI_BA_ERR_HIP;
  std::memset(id, 0, MI_BA_COMM_ID_BYTES);
  std::memcpy(id, &u, sizeof(u));
  return MI_BA_OK;
}

// set_comm helper threads still running (mi_ba_comm_pending_setups)
static std::atomic<int32_t> g_setup_helpers{0};

int32_t mi_ba_comm_pending_setups(void) { return g_setup_helpers.load(); }

mi_ba_status mi_ba_context_set_comm(mi_ba_context* ctx, int32_t rank, int32_t world,
                                    const char id[MI_BA_COMM_ID_BYTES]) {
  if (!ctx || !id || world < 1 || rank < 0 || rank >= world) return MI_BA_ERR_INVALID_ARGUMENT;
  if (ctx->comm || ctx->host_reduce || ctx->solved) return MI_BA_ERR_STATE;
  MI_HIP(hipSetDevice(ctx->device));
  if (ctx->comm_failed) return MI_BA_ERR_STATE;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  // The set-up runs on a helper thread that the caller waits for only until
  // the deadline; it then returns MI_BA_ERR_HIP with the context still
  // single-rank.  Once the init call returns, the helper polls the
  // non-blocking set-up against the same deadline and aborts the half-built
  // communicator, so it never outlives the set-up by polling.  The
  // communicator's collectives are polled against the deadline as well
  // (comm_settle, comm_wait_stream).
  struct InitJob {
    std::mutex m;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclResult_t res = ncclInternalError;
    ncclComm_t comm = nullptr;
  };
  auto job = std::make_shared<InitJob>();
  const int dev = ctx->device;
  const double deadline = now_s() + 1e-3 * std::max(1, ctx->comm_timeout_ms);
  g_setup_helpers.fetch_add(1);
  std::thread([job, u, world, rank, dev, deadline]() {
    ncclComm_t c = nullptr;
    ncclResult_t r = hipSetDevice(dev) == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
    if (r == ncclSuccess) {
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      cfg.blocking = 0;
      ncclUniqueId uu = u;
      // RCCL 2.27 runs the bootstrap inside this call even for a non-blocking
      // communicator (and inside ncclGroupEnd when wrapped in a group, with
      // NCCL_COMM_BLOCKING=0 too, measured): while a peer is missing it does
      // not return, and has no timeout.  The helper then stays blocked here
      // until the peer joins or the process ends (counted by
      // mi_ba_comm_pending_setups); it holds nothing of the context.
      r = ncclCommInitRankConfig(&c, world, uu, rank, &cfg);
      // poll the non-blocking set-up until it completes, fails, the caller
      // gave up on it (abandoned) or the deadline passes: the last two end
      // the helper too (the communicator is aborted below), so a peer that
      // never joins leaves no polling thread behind
      while (r == ncclInProgress || r == ncclSuccess) {
        ncclResult_t e = ncclSuccess;
        if (!c || ncclCommGetAsyncError(c, &e) != ncclSuccess) { r = ncclInternalError; break; }
        if (e != ncclInProgress) { r = e; break; }
        bool gave_up;
        {
          std::lock_guard<std::mutex> g(job->m);
          gave_up = job->abandoned;
        }
        if (gave_up || now_s() > deadline) { r = ncclInternalError; break; }
        std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
    }
    bool abandoned;
    {
      std::lock_guard<std::mutex> g(job->m);
      job->done = true;
      job->res = r;
      job->comm = c;
      abandoned = job->abandoned;
    }
    job->cv.notify_all();
    if ((abandoned || r != ncclSuccess) && c) (void)ncclCommAbort(c);
    g_setup_helpers.fetch_sub(1);
  }).detach();
  bool ok;
  {
    std::unique_lock<std::mutex> g(job->m);
    job->cv.wait_for(g, std::chrono::milliseconds(std::max(1, ctx->comm_timeout_ms)), [&] { return job->done; });
    ok = job->done && job->res == ncclSuccess && job->comm;
    if (!job->done) job->abandoned = true;
    if (ok) ctx->comm = job->comm;
  }
  if (!ok) return MI_BA_ERR_HIP;  // the context stays usable as a single-rank context
  ctx->rank = rank;
  ctx->world = world;
  return reduce_fixed_cost(ctx);
}

mi_ba_status mi_ba_context_set_host_reducer(mi_ba_context* ctx, int32_t rank, int32_t world,
                                            mi_ba_host_allreduce_fn fn, void* user) {
  if (!ctx || !fn || world < 1 || rank < 0 || rank >= world) return MI_BA_ERR_INVALID_ARGUMENT;
  if (ctx->comm || ctx->host_reduce || ctx->solved) return MI_BA_ERR_STATE;
  ctx->host_reduce = fn;
  ctx->host_reduce_user = user;
  ctx->rank = rank;
  ctx->world = world;
  return reduce_fixed_cost(ctx);
}

// A/B variants measured slower than the defaults are compiled into the tools
// build only (make ab -> libmi_ba_ab.so, MI_BA_AB_VARIANTS); the product
// library accepts their keys with the default value alone.
#ifdef MI_BA_AB_VARIANTS
static bool ab_value(int, int) { return true; }
#else
static bool ab_value(int value, int product) { return value == product; }
#endif

mi_ba_status mi_ba_set_tuning(mi_ba_context* ctx, const char* key, int32_t value) {
  if (!ctx || !key) return MI_BA_ERR_INVALID_ARGUMENT;
  if (std::strcmp(key, "jacobian_variant") == 0 && value >= 0 && value <= 63 && ab_value(value, 0)) {
    ctx->dev.jvariant = value;
    return MI_BA_OK;
  }
  // multi-rank: deadline of one collective or of the communicator set-up
  // (a timed-out collective aborts the communicator, MI_BA_ERR_HIP)
  if (std::strcmp(key, "comm_timeout_ms") == 0 && value >= 1) {
    ctx->comm_timeout_ms = value;
    return MI_BA_OK;
  }
  // test hook: the next `value` factorisations of the exact solve report a
  // non-positive pivot in their first diagonal block
  if (std::strcmp(key, "test_fail_factorizations") == 0 && value >= 0 && value <= 1000) {
    ctx->fail_factorizations = value;
    return MI_BA_OK;
  }
  // test hook: hold the stream ahead of every RCCL collective for `value` ms
  if (std::strcmp(key, "comm_stall_ms") == 0 && value >= 0 && value <= 60000) {
    ctx->comm_stall_ms = value;
    return MI_BA_OK;
  }
  // range mask of the inputs read right before the reprojection kernel (1
  // observations, 2 image ids, 4 point ids, 8 points; default 15; 0 off)
  if (std::strcmp(key, "linearize_warm_inputs") == 0 && value >= 0 && value <= 15) {
    ctx->lin_warm = value;
    return MI_BA_OK;
  }
  // tools build: the same read beside the semantic deferred pass instead
  if (std::strcmp(key, "linearize_warm_concurrent") == 0 && value >= 0 && value <= 15 && ab_value(value, 0)) {
    ctx->lin_warm_conc = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "warm_unroll") == 0 && (value == 4 || value == 8) && ab_value(value, 4)) {
    ctx->warm_unroll = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "warm_workgroups") == 0 && value >= 0 && value <= 65536) {
    ctx->warm_wgs = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "linearize_order") == 0 && (value == 0 || value == 1) && ab_value(value, 0)) {
    ctx->lin_order = value;
    return MI_BA_OK;
  }
  // stream layouts 1 / 2 measured slower (step 1.04 / 1.06-1.07 vs 1.01-1.03 ms
  // at C4, profiles/r3_ab_linearize_overlap.jsonl)
  if (std::strcmp(key, "linearize_overlap") == 0 && value >= 0 && value <= 2 && ab_value(value, 0)) {
    ctx->lin_overlap = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "semantic_prep_early") == 0 && (value == 0 || value == 1) && ab_value(value, 0)) {
    ctx->sem_prep_early = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "semantic_deferred_variant") == 0 && value >= 0 && value <= 4 && ab_value(value, 0)) {
    ctx->sem_dvar = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "semantic_deferred_grid") == 0 && value >= 1 && value <= 64) {
    ctx->sem_dgrid = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "semantic_deferred_compact") == 0 && (value == 0 || value == 1)) {
    ctx->sem_compact = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "semantic_flat_coarse") == 0 && value >= 0 && value <= 3) {
    ctx->sem_coarse = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "semantic_diag") == 0 && value >= 0 && value <= 2) {
    ctx->sem_diag = value;
    return MI_BA_OK;
  }
  // the flat pass decides samples from 3x3 window summaries of the rasters
  // (16 B per raster pixel more HBM) before reading the raster
  if (std::strcmp(key, "semantic_window_summary") == 0 && (value == 0 || value == 1)) {
    if (!ctx->sem) return value ? MI_BA_ERR_STATE : MI_BA_OK;
    return semantic_set_window_summary(ctx, value != 0);
  }
  // 1: the flat pass reads the label planes first (8-bit label indices + 8 x 8
  // tile depth ranges; ~1.1 GB at C4), 0: not
  if (std::strcmp(key, "semantic_label_planes") == 0 && (value == 0 || value == 1)) {
    if (!ctx->sem) return value ? MI_BA_ERR_STATE : MI_BA_OK;
    return semantic_set_label_planes(ctx, value != 0);
  }
  if (std::strcmp(key, "semantic_deferred_box") == 0 && (value == 0 || value == 1)) {
    ctx->sem_deferred_box = value != 0;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "semantic_variant") == 0 && value >= 0 && value <= 6 && ab_value(value, 6)) {
    ctx->sem_variant = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "schur_pairs_variant") == 0 && value >= 0 && value <= 9 &&
      (value == 0 || value == 4 || value == 6 || ab_value(value, 0))) {
    ctx->dev.svariant = value;
    return MI_BA_OK;
  }
  // 1: the pair kernel's self tiles load each Z row once (a == b), 0: twice
  if (std::strcmp(key, "schur_self_one_load") == 0 && (value == 0 || value == 1) && ab_value(value, 1)) {
    ctx->dev.sself1 = value;
    return MI_BA_OK;
  }
  // 1: the Schur factors Z in image order (camera-major positions), the pair
  // list in positions; 0: Z in block order
  // (tools build: slower, kernels.hip launch_dense_schur)
  if (std::strcmp(key, "schur_z_image_order") == 0 && (value == 0 || value == 1) && ab_value(value, 0)) {
    ctx->dev.zorder = value;
    if (!value) {
      ctx->pairs_pos.release();
      return MI_BA_OK;
    }
    return ctx->pairs.n ? build_pairs_pos(ctx, nullptr) : MI_BA_OK;
  }
  if (std::strcmp(key, "fblock_variant") == 0 && value >= 0 && value <= 2 && ab_value(value, 0)) {
    ctx->dev.fvariant = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "schur_block_images") == 0 && value >= 1) {
    ctx->schur_block = value;
    return ctx->ptiles_host.empty() ? MI_BA_OK : order_block_tiles(ctx);
  }
  if (std::strcmp(key, "cholesky_panel") == 0 && (value == 0 || (value >= 64 && value <= 4096))) {
    ctx->chol.panel = value;
    return MI_BA_OK;
  }
  // non-uniform panel schedule (CholConfig::head_panel / tail_panel)
  if (std::strcmp(key, "cholesky_head_panel") == 0 && (value == 0 || (value >= 64 && value <= 1024))) {
    ctx->chol.head_panel = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_head_cols") == 0 && value >= 0) {
    ctx->chol.head_cols = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_tail_panel") == 0 && (value == 0 || (value >= 64 && value <= 1024))) {
    ctx->chol.tail_panel = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_tail_cols") == 0 && value >= 0) {
    ctx->chol.tail_cols = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_lookahead") == 0 && (value == 0 || value == 1)) {
    ctx->chol.lookahead = value != 0;
    return MI_BA_OK;
  }
  // tools build: measured 18.7-22.2 vs 15.7 ms (profiles/r4_ab_cholesky_head_own_diag.jsonl)
  if (std::strcmp(key, "cholesky_head_own_diag") == 0 && (value == 0 || value == 2 || value == 6) &&
      ab_value(value, 0)) {
    ctx->chol.head_own = (int)value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_head_own_cols") == 0 && value >= 0) {
    ctx->chol.head_own_cols = (int)value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_own_diag") == 0 && value >= 0 && value <= 7 && (value != 7 || ab_value(value, 6))) {
    ctx->chol.own_diag = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_solve") == 0 && value >= 0 && value <= 2) {
    ctx->chol.solve = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_gemm_solution") == 0) {
    ctx->chol.gemm_solution = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_rest_update") == 0 && value >= 0 && value <= 4 &&
      (value == 0 || value == 3 || ab_value(value, 3))) {
    ctx->chol.rest_update = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_batch_tile") == 0 && value >= 64 && value % 64 == 0) {
    ctx->chol.batch_tile = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_tile_factor") == 0 && value >= 1 && value <= 6 && ab_value(value, CholConfig{}.tile_factor)) {
    ctx->chol.tile_factor = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_split_tail_cols") == 0 && value >= 0 && ab_value(value, CholConfig{}.split_tail_cols)) {
    ctx->chol.split_tail_cols = value;
    return MI_BA_OK;
  }
  // tools build: measured slower at every width (profiles/r6c_ab_cholesky_split_panel.jsonl)
  if (std::strcmp(key, "cholesky_rest_first_panel") == 0 && (value == 0 || value == 1) && ab_value(value, 0)) {
    ctx->chol.rest_first_panel = value != 0;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_la_side_from") == 0 && value >= -1) {
    ctx->chol.la_side_from = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_split_panel_cols") == 0 && value >= 0 && ab_value(value, 0)) {
    ctx->chol.split_panel_cols = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_serial_head_cols") == 0 && value >= 0 && ab_value(value, 0)) {
    ctx->chol.serial_head_cols = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_split_tail_rest") == 0 && (value == 0 || value == 1) && ab_value(value, 0)) {
    ctx->chol.split_tail_rest = value != 0;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_panel_wait") == 0 && value >= 0 && value <= 3 &&
      ab_value(value, CholConfig{}.panel_wait)) {
    ctx->chol.panel_wait = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_solve_sc1") == 0 && (value == 0 || value == 1) &&
      ab_value(value, CholConfig{}.solve_sc1 ? 1 : 0)) {
    ctx->chol.solve_sc1 = value != 0;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_write_through") == 0 && (value == 0 || value == 1) && ab_value(value, 1)) {
    ctx->chol.write_through = value != 0;
    return MI_BA_OK;
  }
  // grouped below-diagonal panel rows: measured slower (Cholesky 15.6 -> 15.7 / 16.9 ms
  // with 2 rows per group, 18-22 ms with 4; profiles/r3_ab_panel_groups.jsonl)
  if (std::strcmp(key, "cholesky_panel_rows_per_group") == 0 && value >= 1 && value <= 64 && ab_value(value, 1)) {
    ctx->chol.panel_rows_per_group = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_rest_priority") == 0 && value >= 0 && value <= 2) {
    ctx->chol.rest_priority = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_rest_cumask") == 0 && (value == 0 || value == 1)) {
    ctx->chol.rest_cumask = value != 0;
    return MI_BA_OK;
  }
  // trailing-update block columns over this many streams (1..4)
  if (std::strcmp(key, "cholesky_rest_streams") == 0 && value >= 1 && value <= 4) {
    ctx->chol.rest_streams = (int)value;
    return MI_BA_OK;
  }
  // split head: panel factor on this many CUs, trailing dgemm on the rest,
  // while the panel starts before column cholesky_split_cols (tools build:
  // measured 22.5-27.5 vs 15.6 ms, profiles/r4_ab_cholesky_split_cus.jsonl)
  if (std::strcmp(key, "cholesky_split_cus") == 0 && value >= 0 && value <= 4096 && ab_value(value, 0)) {
    ctx->chol.split_cus = (int)value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_split_cols") == 0 && value >= 0) {
    ctx->chol.split_cols = (int)value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_panel_cus") == 0 && value >= 0 && value <= 4096 && ab_value(value, 0)) {
    ctx->chol.side_cus = (int)value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_panel_group_min_rows") == 0 && value >= 0) {
    ctx->chol.panel_group_min_rows = value;
    return MI_BA_OK;
  }
  // PCG product without J reads (the passes recompute the Jacobian rows)
  if (std::strcmp(key, "pcg_matrix_free") == 0 && (value == 0 || value == 1)) {
    ctx->pcg_mf = value != 0;
    if (ctx->pcg_mf) ctx->Jcm.release();
    else {
      ctx->Xcm.release();
      ctx->obs_cm.release();
    }
    return MI_BA_OK;
  }
  if (std::strcmp(key, "pcg_jcm") == 0 && value >= 0 && value <= 2 && ab_value(value, 2)) {
    ctx->pcg_jcm = (int)value;
    if (!ctx->pcg_jcm) ctx->Jcm.release();
    return MI_BA_OK;
  }
  if (std::strcmp(key, "point_normal_chunks") == 0 && (value == 0 || value == 1) && ab_value(value, 1)) {
    ctx->pn_chunks = value != 0;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "pcg_point_chunks") == 0 && (value == 0 || value == 1) && ab_value(value, 1)) {
    ctx->pp_chunks = value != 0;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_bwd_pairs") == 0 && (value == 0 || value == 1) && ab_value(value, 0)) {
    ctx->chol.bwd_pairs = value != 0;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "schur_overlap") == 0 && (value == 0 || value == 1) && ab_value(value, 0)) {
    ctx->schur_overlap = value != 0;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_fused_rhs") == 0 && (value == 0 || value == 1)) {
    ctx->fused_rhs = value != 0;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_wait_ms") == 0 && value >= 1 && value <= 40000) {
    ctx->chol.wait_ms = value;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_spin_log2") == 0 && value >= 0 && value <= 30) {
    ctx->chol.spin_log2 = value;
    return MI_BA_OK;
  }
  // 1 (default): camera-side sums flushed per image / camera in a fixed order
  // (bitwise reproducible LM); 0: float-atomic flushes
  if (std::strcmp(key, "deterministic_sums") == 0 && (value == 0 || value == 1)) {
    ctx->det_sums = value != 0;
    return MI_BA_OK;
  }
  if (std::strcmp(key, "cholesky_gemm_update") == 0 && (value == 0 || value == 1)) {
    ctx->chol.gemm_update = value != 0;
    return MI_BA_OK;
  }
  return MI_BA_ERR_INVALID_ARGUMENT;
}

mi_ba_status mi_ba_dense_cholesky(int32_t device, int32_t n, double* A, double* b, int32_t panel, int32_t lookahead,
                                  int32_t own_diag, int32_t* info) {
  return mi_ba_dense_cholesky_ex(device, n, A, b, panel, lookahead, own_diag, CholConfig{}.solve, info);
}

mi_ba_status mi_ba_dense_cholesky_ex(int32_t device, int32_t n, double* A, double* b, int32_t panel,
                                     int32_t lookahead, int32_t own_diag, int32_t solve, int32_t* info) {
  if (n < 0 || !A || !info || (panel != 0 && (panel < 64 || panel > 4096)) || (lookahead != 0 && lookahead != 1) ||
      (own_diag < 0 || own_diag > 6) || solve < 0 || solve > 2)
    return MI_BA_ERR_INVALID_ARGUMENT;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return MI_BA_ERR_NO_DEVICE;
  if (device < 0 || device >= ndev) return MI_BA_ERR_INVALID_ARGUMENT;
  MI_HIP(hipSetDevice(device));
  *info = 0;
  if (n == 0) return MI_BA_OK;
  CholConfig cfg;
  cfg.panel = panel;
  cfg.lookahead = lookahead != 0;
  cfg.own_diag = own_diag;
  cfg.solve = solve;
  // all resources are owned by this call: concurrent calls share nothing
  hipStream_t s = nullptr;
  rocblas_handle h = nullptr;
  CholWorkspace ws;
  DevArray<double> dA, dx;
  DevArray<int32_t> dinfo;
  const int nleaf = chol_leaf_count(n, cfg);
  mi_ba_status st = MI_BA_OK;
  std::vector<int32_t> hinfo(nleaf, 0);
  do {
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) { s = nullptr; st = MI_BA_ERR_HIP; break; }
    if (rocblas_create_handle(&h) != rocblas_status_success) { h = nullptr; st = MI_BA_ERR_HIP; break; }
    if (rocblas_set_stream(h, s) != rocblas_status_success || !ws.create(device, (n + 63) / 64, n)) {
      st = MI_BA_ERR_HIP;
      break;
    }
    if (dA.alloc((size_t)n * n) || dx.alloc(n) || dinfo.alloc(nleaf)) { st = MI_BA_ERR_OUT_OF_MEMORY; break; }
    if (hipMemcpyAsync(dA.ptr, A, dA.bytes(), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(dinfo.ptr, 0, dinfo.bytes(), s) != hipSuccess ||
        (b && hipMemcpyAsync(dx.ptr, b, dx.bytes(), hipMemcpyHostToDevice, s) != hipSuccess)) {
      st = MI_BA_ERR_HIP;
      break;
    }
    if (chol_factor(h, n, dA.ptr, n, dinfo.ptr, cfg, &ws) != rocblas_status_success) { st = MI_BA_ERR_HIP; break; }
    unsigned werr = 0;
    if (hipMemcpyAsync(hinfo.data(), dinfo.ptr, dinfo.bytes(), hipMemcpyDeviceToHost, s) != hipSuccess ||
        chol_error(&ws, s, &werr) != hipSuccess || werr != 0) {
      st = MI_BA_ERR_HIP;
      break;
    }
    // first failing block: report its first column (1-based) like potrf
    int64_t col0 = 0;
    for (int k = 0; k < nleaf && *info == 0; ++k) {
      const int width = cfg.panel > 0 ? std::min(cfg.panel, n - (int)col0) : 0;
      if (hinfo[k] != 0) *info = (int32_t)(col0 + hinfo[k]);
      col0 += width;
    }
    if (b && *info == 0 &&
        (chol_solve(h, n, dA.ptr, n, dx.ptr, cfg.solve, &ws) != rocblas_status_success ||
         chol_error(&ws, s, &werr) != hipSuccess || werr != 0)) {
      st = MI_BA_ERR_HIP;
      break;
    }
    if (hipMemcpyAsync(A, dA.ptr, dA.bytes(), hipMemcpyDeviceToHost, s) != hipSuccess ||
        (b && hipMemcpyAsync(b, dx.ptr, dx.bytes(), hipMemcpyDeviceToHost, s) != hipSuccess) ||
        hipStreamSynchronize(s) != hipSuccess) {
      st = MI_BA_ERR_HIP;
      break;
    }
  } while (false);
  if (s) (void)hipStreamSynchronize(s);
  ws.destroy();
  if (h) (void)rocblas_destroy_handle(h);
  dA.release();
  dx.release();
  dinfo.release();
  if (s) (void)hipStreamDestroy(s);
  return st;
}

mi_ba_status mi_ba_set_timing(mi_ba_context* ctx, int32_t enabled) {
  if (!ctx) return MI_BA_ERR_INVALID_ARGUMENT;
  timer_collect(ctx);
  ctx->timing = enabled != 0;
  return MI_BA_OK;
}

mi_ba_status mi_ba_kernel_time(mi_ba_context* ctx, const char* name, double* total_ms, int64_t* launches) {
  if (!ctx || !name) return MI_BA_ERR_INVALID_ARGUMENT;
  timer_collect(ctx);
  auto it = ctx->timer.totals.find(name);
  if (total_ms) *total_ms = it == ctx->timer.totals.end() ? 0.0 : it->second.first;
  if (launches) *launches = it == ctx->timer.totals.end() ? 0 : it->second.second;
  return MI_BA_OK;
}

mi_ba_status mi_ba_reset_kernel_times(mi_ba_context* ctx) {
  if (!ctx) return MI_BA_ERR_INVALID_ARGUMENT;
  timer_collect(ctx);
  ctx->timer.totals.clear();
  return MI_BA_OK;
}

}  // extern "C"
