// Phase costs inside one 256-thread workgroup for the panel factor's
// building blocks (csrc/cholesky.cpp): 64x64 tile load global -> LDS, the
// in-LDS factor + inverse (pf_chol_inv_fast, sqrt / rsq pivots, with phase
// stamps), a 64x64x64 MFMA GEMM with
// LDS operands and with global operands (gtile-style loads), and the publish
// of a 32 KB tile by plain stores + __threadfence() vs sc1 (write-through)
// stores + vmcnt(0).  Stamps: wall_clock64 (100 MHz) and clock64 (cycles).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/tile_probe.cpp -lrocsolver -lrocblas -o tools/probes/tile_probe.bin
#include "../../semantic-bundle-adjustment-colmap_amd/csrc/cholesky.cpp"

#include <cstdio>
#include <vector>

using namespace miba;

constexpr int kReps = 8;
constexpr int kPhases = 10;

template <int V>
__global__ __launch_bounds__(256) void tile_probe_kernel(double* __restrict__ A, int lda, double* __restrict__ out,
                                                         unsigned long long* __restrict__ st, double* __restrict__ res) {
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
    long long* sub = (long long*)(st + (size_t)kReps * kPhases * 2) + rep * 10;
    long long* sp = blockIdx.x == 0 ? sub : nullptr;
    const int bad = V == 1   ? pf_chol_inv_fast<false>(T, Li, Lc, dinv, lane, wv, sp)
                    : V == 3 ? pf_chol_inv_fast<true, true, true>(T, Li, Lc, dinv, lane, wv, sp)
                    : V == 4 ? pf_chol_inv_fast<true, true, false>(T, Li, Lc, dinv, lane, wv, sp)
                    : V == 5 ? pf_chol_inv_fast<true, false, true>(T, Li, Lc, dinv, lane, wv, sp)
                    : V == 6 ? pf_chol_inv_fast<true, true, true, true>(T, Li, Lc, dinv, lane, wv, sp)
                             : pf_chol_inv_fast<true>(T, Li, Lc, dinv, lane, wv, sp);
    __syncthreads();
    if (rep == kReps - 1 && blockIdx.x == 0)
      for (int e = threadIdx.x; e < 4096; e += 256) {
        res[e] = T[(e >> 6) * kPfLd + (e & 63)];
        res[4096 + e] = Li[(e >> 6) * kPfLd + (e & 63)];
      }
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
    // 7: the same staging with 16-byte loads, all eight per thread in flight
    {
      const sweep_dvec2* src2 = reinterpret_cast<const sweep_dvec2*>(src);
      sweep_dvec2 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = src2[threadIdx.x + 256 * j];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = 2 * (threadIdx.x + 256 * j);
        Li[(e >> 6) * kPfLd + (e & 63)] = v[j].x;
        Li[(e >> 6) * kPfLd + (e & 63) + 1] = v[j].y;
      }
    }
    __syncthreads();
    w[8] = wall_clock64(); c[8] = clock64();
    // 8: GEMM with global operands on cold tiles (a different pair per rep, per workgroup)
    {
      const int cc = 64 * (1 + rep + kReps * blockIdx.x);
      pf_gemm_nt(o, -1.0, gtile(cc, 0), gtile(cc + 64 * kReps * 8, 0), wv, lane);
    }
    __syncthreads();
    w[9] = wall_clock64(); c[9] = clock64();
    // 9: stage two cold 64x64 column-major tiles (16-byte loads in flight) + LDS GEMM
    {
      const int cc = 64 * (1 + rep + kReps * blockIdx.x) + 64 * kReps * 16;
      sweep_dvec2 v[16];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = 2 * (threadIdx.x + 256 * j);  // column e >> 6, rows e & 63, e & 63 + 1
        v[j] = *reinterpret_cast<const sweep_dvec2*>(A + (size_t)(e >> 6) * lda + cc + (e & 63));
        v[8 + j] = *reinterpret_cast<const sweep_dvec2*>(A + (size_t)(e >> 6) * lda + cc + 64 * kReps * 8 + (e & 63));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = 2 * (threadIdx.x + 256 * j);
        T[(e & 63) * kPfLd + (e >> 6)] = v[j].x;
        T[((e & 63) + 1) * kPfLd + (e >> 6)] = v[j].y;
        Li[(e & 63) * kPfLd + (e >> 6)] = v[8 + j].x;
        Li[((e & 63) + 1) * kPfLd + (e >> 6)] = v[8 + j].y;
      }
      __syncthreads();
      pf_gemm_nt(o, -1.0, ltile(T), ltile(Li), wv, lane);
    }
    __syncthreads();
    w[10] = wall_clock64(); c[10] = clock64();
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
  const int n = 64 * (1 + kReps * 8) + 64 * kReps * 24;
  std::vector<double> h((size_t)n * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) h[(size_t)j * n + i] = (i == j) ? 64.0 : 0.01 * sin(0.37 * (i + j));
  double *A, *out;
  unsigned long long* st;
  hipMalloc(&A, 8ull * n * n);
  hipMalloc(&out, 8ull * 2 * 4096 * 64);
  hipMalloc(&st, 8ull * kReps * kPhases * 2 + 8ull * kReps * 10);
  double* res;
  hipMalloc(&res, 8ull * 7 * 2 * 4096);
  hipMemcpy(A, h.data(), 8ull * n * n, hipMemcpyHostToDevice);
  const char* names[kPhases] = {"load tile -> LDS", "chol+inv", "gemm LDS operands",
                                "gemm global operands", "publish 32KB plain + threadfence",
                                "publish 32KB sc1 + vmcnt", "stage 32KB global -> LDS",
                                "stage 32KB 16B loads in flight", "gemm global operands, cold tiles",
                                "stage 2 cold tiles (16B) + LDS gemm"};
  const char* vname[7] = {"", "pf_chol_inv_fast<sqrt>", "pf_chol_inv_fast<rsq>", "pf_chol_inv_fast<rsq, ovl, pipe>",
                          "pf_chol_inv_fast<rsq, ovl>", "pf_chol_inv_fast<rsq, pipe>", "pf_chol_inv_fast<rsq, ovl, pipe, fast pivots>"};
  for (int cfg = 2; cfg < 14; ++cfg) {
    const int grid = cfg & 1 ? 8 : 1, V = cfg >> 1;
    double* rv = res + (size_t)V * 8192;
    if (V == 1)
      hipLaunchKernelGGL(tile_probe_kernel<1>, dim3(grid), dim3(256), 0, 0, A, n, out, st, rv);
    else if (V == 2)
      hipLaunchKernelGGL(tile_probe_kernel<2>, dim3(grid), dim3(256), 0, 0, A, n, out, st, rv);
    else if (V == 3)
      hipLaunchKernelGGL(tile_probe_kernel<3>, dim3(grid), dim3(256), 0, 0, A, n, out, st, rv);
    else if (V == 4)
      hipLaunchKernelGGL(tile_probe_kernel<4>, dim3(grid), dim3(256), 0, 0, A, n, out, st, rv);
    else if (V == 5)
      hipLaunchKernelGGL(tile_probe_kernel<5>, dim3(grid), dim3(256), 0, 0, A, n, out, st, rv);
    else
      hipLaunchKernelGGL(tile_probe_kernel<6>, dim3(grid), dim3(256), 0, 0, A, n, out, st, rv);
    hipDeviceSynchronize();
    std::vector<unsigned long long> s((size_t)kReps * kPhases * 2);
    hipMemcpy(s.data(), st, 8 * s.size(), hipMemcpyDeviceToHost);
    printf("%s, grid %d (workgroup 0), per phase: min / median over %d reps  [us, cycles]\n", vname[V], grid, kReps);
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
    {
      std::vector<long long> sub(kReps * 10);
      hipMemcpy(sub.data(), st + (size_t)kReps * kPhases * 2, 8 * sub.size(), hipMemcpyDeviceToHost);
      const long long* q = sub.data() + (kReps - 1) * 10;
      printf("  factor sub-phases (last rep, cycles from the first stamp): ");
      for (int k = 1; k < 10; ++k) printf(" %lld", q[k] - q[0]);
      printf("\n    (sweep kb0 | upd0 sweep1 upd1 sweep2 upd2 sweep3 upd3 last diag-inv, inverse)\n");
    }
  }
  // L and X of both variants vs a host Cholesky of the same tile
  std::vector<double> r(14 * 4096);
  hipMemcpy(r.data(), res, 8ull * r.size(), hipMemcpyDeviceToHost);
  std::vector<double> L(4096, 0.0);
  for (int j = 0; j < 64; ++j) {
    double s = h[(size_t)j * n + j];
    for (int k = 0; k < j; ++k) s -= L[j * 64 + k] * L[j * 64 + k];
    L[j * 64 + j] = sqrt(s);
    for (int i = j + 1; i < 64; ++i) {
      double v = h[(size_t)j * n + i];
      for (int k = 0; k < j; ++k) v -= L[i * 64 + k] * L[j * 64 + k];
      L[i * 64 + j] = v / L[j * 64 + j];
    }
  }
  for (int V = 3; V < 7; ++V) {  // the tools-build variants against rsq (same operations: bitwise)
    bool same = true;
    for (int i = 0; i < 64; ++i)
      for (int j = 0; j < 64; ++j) {
        if (j <= i && r[V * 8192 + i * 64 + j] != r[2 * 8192 + i * 64 + j]) same = false;
        if ((j >> 4) <= (i >> 4) && r[V * 8192 + 4096 + i * 64 + j] != r[2 * 8192 + 4096 + i * 64 + j]) same = false;
      }
    printf("variant %d: L and X bitwise equal to variant 2: %s\n", V, same ? "yes" : "NO");
  }
  for (int V = 1; V < 7; ++V) {
    double el = 0.0, ex = 0.0;
    for (int i = 0; i < 64; ++i)
      for (int j = 0; j < 64; ++j) {
        if (j <= i) el = std::max(el, fabs(r[V * 8192 + i * 64 + j] - L[i * 64 + j]));
        double lx = 0.0;  // (L X)_ij - I
        for (int k = 0; k < 64; ++k)  // X's strict upper blocks are not stored
          if ((j >> 4) <= (k >> 4)) lx += L[i * 64 + k] * r[V * 8192 + 4096 + k * 64 + j];
        ex = std::max(ex, fabs(lx - (i == j ? 1.0 : 0.0)));
      }
    printf("variant %d: max |L - L_host| %.3e, max |L X - I| %.3e\n", V, el, ex);
  }
  return 0;
}
