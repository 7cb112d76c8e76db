// Phase costs inside one 256-thread workgroup for the panel factor's
// building blocks (csrc/cholesky.cpp): 64x64 tile load global -> LDS, the
// in-LDS factor + inverse (pf_chol_inv_blocked), a 64x64x64 MFMA GEMM with
// LDS operands and with global operands (gtile-style loads), and the publish
// of a 32 KB tile by plain stores + __threadfence() vs sc1 (write-through)
// stores + vmcnt(0).  Stamps: wall_clock64 (100 MHz) and clock64 (cycles).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/tile_probe.cpp -lrocsolver -lrocblas -o tools/probes/tile_probe.bin
#include "../../semantic-bundle-adjustment-colmap_amd/csrc/cholesky.cpp"

#include <cstdio>
#include <vector>

using namespace miba;

constexpr int kReps = 8;
constexpr int kPhases = 7;

__global__ __launch_bounds__(256) void tile_probe_kernel(double* __restrict__ A, int lda, double* __restrict__ out,
                                                         unsigned long long* __restrict__ st) {
  __shared__ double T[64 * kPfLd];
  __shared__ double Li[64 * kPfLd];
  __shared__ double Lc[64 * 64];
  __shared__ double dinv[64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int m = lane & 15, kq = lane >> 4;
  auto gtile = [&](int row0, int col0) {
    return [=](int i, int j) { return A[(size_t)(col0 + j) * lda + row0 + i]; };
  };
  auto ltile = [&](const double* S) { return [=](int i, int j) { return S[i * kPfLd + j]; }; };
  double sink = 0.0;
  for (int rep = 0; rep < kReps; ++rep) {
    unsigned long long w[kPhases + 1], c[kPhases + 1];
    __syncthreads();
    w[0] = wall_clock64(); c[0] = clock64();
    // 0: load the SPD tile (rows/cols 0..63) into registers (MFMA D layout) -> LDS
    pf_dvec4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 16 * wv + 4 * q + kq, j = 16 * t + m;
        acc[t][q] = A[(size_t)j * lda + i];
      }
    pf_acc_to_lds(acc, T, wv, lane);
    __syncthreads();
    w[1] = wall_clock64(); c[1] = clock64();
    // 1: factor + inverse in LDS
    const int bad = pf_chol_inv_blocked(T, Li, Lc, dinv, lane, wv);
    __syncthreads();
    w[2] = wall_clock64(); c[2] = clock64();
    // 2: GEMM with LDS operands: out = T Li'
    pf_dvec4 o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = pf_dvec4{0.0, 0.0, 0.0, 0.0};
    pf_gemm_nt(o, 1.0, ltile(T), ltile(Li), wv, lane);
    __syncthreads();
    w[3] = wall_clock64(); c[3] = clock64();
    // 3: GEMM with both operands read from global inside the loop
    pf_gemm_nt(o, -1.0, gtile(64, 0), gtile(128, 0), wv, lane);
    __syncthreads();
    w[4] = wall_clock64(); c[4] = clock64();
    // 4: publish 32 KB with plain stores + __threadfence()
    double* dst = out + (size_t)blockIdx.x * 2 * 4096;
    for (int e = threadIdx.x; e < 4096; e += 256) dst[e] = Li[(e >> 6) * kPfLd + (e & 63)] + o[e & 3][0];
    __threadfence();
    __syncthreads();
    w[5] = wall_clock64(); c[5] = clock64();
    // 5: publish 32 KB with sc1 stores (relaxed agent atomics) + vmcnt(0)
    for (int e = threadIdx.x; e < 4096; e += 256) {
      const double v = Li[(e >> 6) * kPfLd + (e & 63)];
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst + 4096 + e), (unsigned long long)__double_as_longlong(v),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    w[6] = wall_clock64(); c[6] = clock64();
    // 6: stage a 32 KB row-major tile global -> LDS (the Linv staging loop)
    const double* src = out + (size_t)blockIdx.x * 2 * 4096 + 4096;
    for (int e = threadIdx.x; e < 4096; e += 256) Li[(e >> 6) * kPfLd + (e & 63)] = src[e];
    __syncthreads();
    w[7] = wall_clock64(); c[7] = clock64();
    sink += (double)bad + o[0][0] + Li[lane];
    if (threadIdx.x == 0 && blockIdx.x == 0)
      for (int k = 0; k < kPhases; ++k) {
        st[(size_t)rep * kPhases * 2 + 2 * k] = w[k + 1] - w[k];
        st[(size_t)rep * kPhases * 2 + 2 * k + 1] = c[k + 1] - c[k];
      }
  }
  if (sink == 12345.678) out[0] = sink;
}

int main() {
  const int n = 512;
  std::vector<double> h((size_t)n * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) h[(size_t)j * n + i] = (i == j) ? 64.0 : 0.01 * sin(0.37 * (i + j));
  double *A, *out;
  unsigned long long* st;
  hipMalloc(&A, 8ull * n * n);
  hipMalloc(&out, 8ull * 2 * 4096 * 64);
  hipMalloc(&st, 8ull * kReps * kPhases * 2);
  hipMemcpy(A, h.data(), 8ull * n * n, hipMemcpyHostToDevice);
  const char* names[kPhases] = {"load tile -> LDS", "chol+inv (pf_chol_inv_blocked)", "gemm LDS operands",
                                "gemm global operands", "publish 32KB plain + threadfence",
                                "publish 32KB sc1 + vmcnt", "stage 32KB global -> LDS"};
  for (int grid : {1, 8}) {
    hipLaunchKernelGGL(tile_probe_kernel, dim3(grid), dim3(256), 0, 0, A, n, out, st);
    hipDeviceSynchronize();
    std::vector<unsigned long long> s((size_t)kReps * kPhases * 2);
    hipMemcpy(s.data(), st, 8 * s.size(), hipMemcpyDeviceToHost);
    printf("grid %d (workgroup 0), per phase: min / median over %d reps  [us, cycles]\n", grid, kReps);
    for (int k = 0; k < kPhases; ++k) {
      std::vector<double> us, cy;
      for (int r = 1; r < kReps; ++r) {
        us.push_back(s[(size_t)r * kPhases * 2 + 2 * k] / 100.0);
        cy.push_back((double)s[(size_t)r * kPhases * 2 + 2 * k + 1]);
      }
      std::sort(us.begin(), us.end());
      std::sort(cy.begin(), cy.end());
      printf("  %-36s %8.2f / %8.2f us   %9.0f / %9.0f cyc\n", names[k], us[0], us[us.size() / 2], cy[0],
             cy[cy.size() / 2]);
    }
  }
  return 0;
}
