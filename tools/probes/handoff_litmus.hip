// Litmus probe of the Cholesky panel's hand-off (csrc/cholesky.cpp
// panel_factor_kernel, panel_wait 2): a 64x64 f64 tile stored with 8-byte
// relaxed agent-scope atomic stores (global_store sc1) by every thread, each
// storing wave drained by s_waitcnt vmcnt(0), a workgroup barrier, then one
// relaxed agent-scope flag store; the consumer's first wave polls the flag
// with relaxed agent-scope loads, the workgroup joins at a barrier, and every
// thread reads the tile with 8-byte relaxed agent-scope loads (global_load
// sc1) — no acquire fence anywhere.  Producer and consumer are consecutive
// workgroups (different XCDs under the round-robin dispatch).
//   mode 0  the pattern above (must see 0 stale elements)
//   mode 1  the same workgroup re-reading tiles its other waves stored that
//           way after a barrier (the below-diagonal rows' own L tiles)
//   mode 2  control: plain stores, no drain, plain loads, no acquire
//           (stale reads expected; shows the probe can see them)
// Every wait is bounded by wall-clock time; a timed-out wait is counted and
// ends that workgroup's loop, so the grid always drains.
//   hipcc --offload-arch=gfx950 -O3 -o handoff_litmus tools/probes/handoff_litmus.hip
//   ./handoff_litmus [iterations] [pairs]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace {

constexpr int kTile = 64 * 64;

__device__ __forceinline__ double ld_ag(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(
      (const __attribute__((address_space(1))) unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_ag(double* p, double v) {
  __hip_atomic_store((__attribute__((address_space(1))) unsigned long long*)p,
                     (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bounded wait for *f >= v (relaxed agent-scope polls); false on timeout
__device__ bool wait_ge(const unsigned* f, unsigned v, uint64_t limit) {
  const uint64_t t0 = wall_clock64();
  for (unsigned spin = 0;; ++spin) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= v) return true;
    if ((spin & 15u) == 15u && wall_clock64() - t0 >= limit) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ double value(unsigned e, int pair, int i) {
  return (double)e * 1048576.0 + (double)pair * 8192.0 + (double)i + 0.25;
}

// mode 0 / 2: workgroup 2p produces, 2p + 1 consumes; mode 1: every
// workgroup re-reads its own tiles
__global__ __launch_bounds__(256) void litmus_kernel(int mode, unsigned iters, double* tiles, unsigned* flags,
                                                     unsigned* acks, unsigned long long* stale,
                                                     unsigned long long* timeouts, uint64_t limit) {
  __shared__ int s_ok;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (mode == 1) {
    double* t = tiles + (size_t)b * kTile;
    unsigned long long bad = 0;
    for (unsigned e = 1; e <= iters; ++e) {
      // wave w stores rows 16w..16w+15, then reads rows of wave (w + 1) % 4
      for (int q = 0; q < 16; ++q) {
        const int i = tid + 256 * q;
        st_ag(t + i, value(e, b, i));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int q = 0; q < 16; ++q) {
        const int i = (tid + 64 + 256 * q) % kTile;
        bad += ld_ag(t + i) != value(e, b, i);
      }
      __syncthreads();
    }
    if (bad) atomicAdd(stale, bad);
    return;
  }
  const int pair = b >> 1;
  double* t = tiles + (size_t)pair * kTile;
  unsigned* flag = flags + pair;
  unsigned* ack = acks + pair;
  const bool producer = (b & 1) == 0;
  unsigned long long bad = 0;
  for (unsigned e = 1; e <= iters; ++e) {
    if (producer) {
      // the consumer has read iteration e - 1
      if (tid == 0) s_ok = wait_ge(ack, e - 1, limit);
      __syncthreads();
      if (!s_ok) {
        if (tid == 0) atomicAdd(timeouts, 1ull);
        break;
      }
      for (int q = 0; q < 16; ++q) {
        const int i = tid + 256 * q;
        if (mode == 0)
          st_ag(t + i, value(e, pair, i));
        else
          t[i] = value(e, pair, i);
      }
      if (mode == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(flag, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (tid < 64) {
        const bool ok = wait_ge(flag, e, limit);
        if (tid == 0) s_ok = ok;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: the loads stay below the poll
      }
      __syncthreads();
      if (!s_ok) {
        if (tid == 0) atomicAdd(timeouts, 1ull);
        break;
      }
      for (int q = 0; q < 16; ++q) {
        const int i = tid + 256 * q;
        const double v = mode == 0 ? ld_ag(t + i) : *(volatile const double*)(t + i);
        bad += v != value(e, pair, i);
      }
      __syncthreads();  // every read done before the ack
      if (tid == 0) __hip_atomic_store(ack, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (bad) atomicAdd(stale, bad);
}

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

}  // namespace

int main(int argc, char** argv) {
  const unsigned iters = argc > 1 ? (unsigned)std::atoi(argv[1]) : 20000u;
  const int pairs = argc > 2 ? std::atoi(argv[2]) : 64;
  int khz = 0;
  CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const uint64_t limit = (uint64_t)(khz > 0 ? khz : 100000) * 2000;  // 2 s per wait
  double* tiles;
  unsigned *flags, *acks;
  unsigned long long *stale, *timeouts;
  CHECK(hipMalloc(&tiles, sizeof(double) * kTile * 2 * pairs));
  CHECK(hipMalloc(&flags, sizeof(unsigned) * pairs));
  CHECK(hipMalloc(&acks, sizeof(unsigned) * pairs));
  CHECK(hipMalloc(&stale, 8));
  CHECK(hipMalloc(&timeouts, 8));
  const char* names[3] = {"sc1 stores + vmcnt drain + relaxed flag / relaxed poll + sc1 loads (panel hand-off)",
                          "same workgroup: sc1 stores + vmcnt drain + barrier / sc1 loads of other waves' rows",
                          "control: plain stores, no drain / plain loads, no acquire"};
  for (int mode = 0; mode < 3; ++mode) {
    CHECK(hipMemset(tiles, 0, sizeof(double) * kTile * 2 * pairs));
    CHECK(hipMemset(flags, 0, sizeof(unsigned) * pairs));
    CHECK(hipMemset(acks, 0, sizeof(unsigned) * pairs));
    CHECK(hipMemset(stale, 0, 8));
    CHECK(hipMemset(timeouts, 0, 8));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(litmus_kernel, dim3(2 * pairs), dim3(256), 0, 0, mode, iters, tiles, flags, acks, stale,
                       timeouts, limit);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long hs = 0, ht = 0;
    CHECK(hipMemcpy(&hs, stale, 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&ht, timeouts, 8, hipMemcpyDeviceToHost));
    const double checked = (double)iters * kTile * (mode == 1 ? 2 * pairs : pairs);
    std::printf("mode %d: %s\n  %u iterations x %d %s, %.3g elements checked: stale %llu, timed-out waits %llu, "
                "%.2f us per iteration\n",
                mode, names[mode], iters, mode == 1 ? 2 * pairs : pairs, mode == 1 ? "workgroups" : "pairs", checked,
                hs, ht, 1e3 * ms / iters);
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
  }
  return 0;
}
