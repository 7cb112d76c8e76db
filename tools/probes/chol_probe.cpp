#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
#include <vector>
#include "../semantic-bundle-adjustment-colmap_amd/csrc/cholesky.h"
__global__ void fill_spd(double* A, int n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)n * n) return;
  int r = i / n, c = i % n;
  A[i] = (r == c) ? n * 0.02 + 1.0 : 0.01 * sin(0.37 * (r + c)) ;
}
int main() {
  rocblas_handle h; rocblas_create_handle(&h);
  hipStream_t st; hipStreamCreate(&st); rocblas_set_stream(h, st);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms;
  int n = 12000;
  double *S, *x; int* info; hipMalloc(&S, 8ull*n*n); hipMalloc(&x, 8ull*n); hipMalloc(&info, 4 * miba::chol_leaf_count(n));
  std::vector<double> hx(n, 1.0);
  for (int rep = 0; rep < 4; ++rep) {
    hipLaunchKernelGGL(fill_spd, dim3((n*(size_t)n+255)/256), dim3(256), 0, st, S, n);
    hipMemcpyAsync(x, hx.data(), 8*n, hipMemcpyHostToDevice, st);
    hipEventRecord(e0, st);
    { static miba::CholWorkspace ws; if (ws.device < 0) ws.create(0, (n + 63) / 64, n); miba::chol_factor(h, n, S, n, info, {}, &ws); }
    hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("chol_factor n=%d: %.3f ms (%.1f TF)\n", n, ms, (double)n*n*n/3.0/(ms*1e-3)/1e12);
    hipEventRecord(e0, st);
    miba::chol_solve(h, n, S, n, x);
    hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("chol_solve: %.3f ms\n", ms);
  }
  // per-op timing of the pieces at the top level
  int n1 = 6144, n2 = n - n1; double one = 1, m1 = -1;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0, st);
    rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose, rocblas_diagonal_non_unit, n2, n1, &one, S, n, S + n1, n);
    hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("trsm %dx%d: %.3f ms (%.1f TF)\n", n2, n1, ms, (double)n2*n1*n1/(ms*1e-3)/1e12);
    hipEventRecord(e0, st);
    rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, n2, n1, &m1, S + n1, n, &one, S + n1 + (size_t)n1*n, n);
    hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("syrk %dx%d: %.3f ms (%.1f TF)\n", n2, n1, ms, (double)n2*n2*n1/(ms*1e-3)/1e12);
    hipEventRecord(e0, st);
    rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, n2, n2, n1, &m1, S + n1, n, S + n1, n, &one, S + n1 + (size_t)n1*n, n);
    hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("gemm-as-syrk %dx%d: %.3f ms (%.1f TF)\n", n2, n1, ms, 2.0*n2*n2*n1/(ms*1e-3)/1e12);
    hipEventRecord(e0, st);
    rocblas_dtrsv(h, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit, 768, S, n, x, 1);
    hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("trsv 768: %.3f ms\n", ms);
    hipEventRecord(e0, st);
    rocblas_dgemv(h, rocblas_operation_none, n2, n1, &m1, S + n1, n, x, 1, &one, x + n1, 1);
    hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("gemv %dx%d: %.3f ms\n", n2, n1, ms);
    hipEventRecord(e0, st);
    rocblas_dgemv(h, rocblas_operation_transpose, n2, n1, &m1, S + n1, n, x + n1, 1, &one, x, 1);
    hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("gemv-T %dx%d: %.3f ms\n", n2, n1, ms);
  }
  return 0;
}
