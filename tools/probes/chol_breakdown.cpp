// Per-operation time of the right-looking blocked Cholesky (csrc/cholesky.cpp
// factor_blocked) at the C4 reduced-camera-system size: dpotrf of the
// diagonal blocks vs dtrsm of the panels vs the trailing dgemm updates, plus
// the hand-written diagonal-block factor (chol_potrf_diag) on the same blocks.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/chol_breakdown.cpp \
//     semantic-bundle-adjustment-colmap_amd/csrc/cholesky.cpp -lrocsolver -lrocblas -o tools/chol_breakdown.bin
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../semantic-bundle-adjustment-colmap_amd/csrc/cholesky.h"

__global__ void fill_spd(double* A, int n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)n * n) return;
  int r = i % n, c = i / n;
  A[i] = (r == c) ? n * 0.02 + 1.0 : 0.01 * sin(0.37 * (r + c)) + 0.005 * cos(0.011 * (double)r * c);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 12000;
  const int nb = argc > 2 ? atoi(argv[2]) : 512;
  rocblas_handle h;
  rocblas_create_handle(&h);
  hipStream_t st;
  hipStreamCreate(&st);
  rocblas_set_stream(h, st);
  double *S, *S2;
  int* info;
  hipMalloc(&S, 8ull * n * n);
  hipMalloc(&S2, 8ull * n * n);
  hipMalloc(&info, 4 * 4096);
  const int nk = (n + nb - 1) / nb;
  std::vector<hipEvent_t> ev(4 * nk + 1);
  for (auto& e : ev) hipEventCreate(&e);
  const double one = 1.0, minus_one = -1.0;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(fill_spd, dim3((unsigned)(((size_t)n * n + 255) / 256)), dim3(256), 0, st, S, n);
    hipMemcpyAsync(S2, S, 8ull * n * n, hipMemcpyDeviceToDevice, st);
    int e = 0;
    hipEventRecord(ev[e++], st);
    for (int k = 0, kk = 0; k < n; k += nb, ++kk) {
      const int kb = std::min(nb, n - k);
      double* Akk = S + k + (size_t)k * n;
      rocsolver_dpotrf(h, rocblas_fill_lower, kb, Akk, n, info + kk);
      hipEventRecord(ev[e++], st);
      const int m = n - k - kb;
      if (m > 0) {
        rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose, rocblas_diagonal_non_unit,
                      m, kb, &one, Akk, n, Akk + kb, n);
      }
      hipEventRecord(ev[e++], st);
      for (int j = 0; j < m; j += nb) {
        const int jb = std::min(nb, m - j);
        rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, m - j, jb, kb, &minus_one, Akk + kb + j,
                      n, Akk + kb + j, n, &one, Akk + kb + (size_t)kb * n + j + (size_t)j * n, n);
      }
      hipEventRecord(ev[e++], st);
    }
    hipEventSynchronize(ev[e - 1]);
    double tp = 0, tt = 0, tg = 0;
    for (int k = 0; k < nk; ++k) {
      float a, b, c;
      hipEventElapsedTime(&a, ev[3 * k], ev[3 * k + 1]);
      hipEventElapsedTime(&b, ev[3 * k + 1], ev[3 * k + 2]);
      hipEventElapsedTime(&c, ev[3 * k + 2], ev[3 * k + 3]);
      tp += a;
      tt += b;
      tg += c;
    }
    printf("{\"n\": %d, \"panel\": %d, \"potrf_ms\": %.3f, \"trsm_ms\": %.3f, \"gemm_ms\": %.3f, \"total_ms\": %.3f}\n",
           n, nb, tp, tt, tg, tp + tt + tg);
    // the library's factor with its current configuration, and the diagonal factor alone
    hipLaunchKernelGGL(fill_spd, dim3((unsigned)(((size_t)n * n + 255) / 256)), dim3(256), 0, st, S, n);
    miba::CholConfig cfg;
    hipEventRecord(ev[0], st);
    { static miba::CholWorkspace ws; if (ws.device < 0) ws.create(0, (n + 63) / 64, n); miba::chol_factor(h, n, S, n, info, cfg, &ws); }
    hipEventRecord(ev[1], st);
    hipEventSynchronize(ev[1]);
    float ms;
    hipEventElapsedTime(&ms, ev[0], ev[1]);
    hipLaunchKernelGGL(fill_spd, dim3((unsigned)(((size_t)n * n + 255) / 256)), dim3(256), 0, st, S, n);
    hipEventRecord(ev[0], st);
    for (int k = 0; k < n; k += nb) rocsolver_dpotrf(h, rocblas_fill_lower, std::min(nb, n - k), S + k + (size_t)k * n, n, info);
    hipEventRecord(ev[1], st);
    hipEventSynchronize(ev[1]);
    float ms2;
    hipEventElapsedTime(&ms2, ev[0], ev[1]);
    printf("{\"library_factor_ms\": %.3f, \"rocsolver_diag_blocks_only_ms\": %.3f}\n", ms, ms2);
  }
  return 0;
}
