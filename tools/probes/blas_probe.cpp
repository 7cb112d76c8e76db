#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <cstdio>
#include <vector>
#include <cmath>
__global__ void fill_spd(double* A, int n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)n * n) return;
  int r = i / n, c = i % n;
  double v = sin(0.37 * r + 0.11 * c) * sin(0.13 * c + 0.29 * r) * 0.01;  // symmetric-ish small
  if (r == c) v = n * 0.01 + 1.0;
  A[i] = (r < c) ? 0.0 : v;  // only lower in column-major sense used
  if (r == c) A[i] = n * 0.02 + 1.0;
}
int main() {
  rocblas_handle h; rocblas_create_handle(&h);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms;
  // dgemm
  for (int n : {4096, 8192}) {
    double *A, *B, *C; hipMalloc(&A, 8ull*n*n); hipMalloc(&B, 8ull*n*n); hipMalloc(&C, 8ull*n*n);
    hipMemset(A, 0, 8ull*n*n); hipMemset(B, 0, 8ull*n*n); hipMemset(C, 0, 8ull*n*n);
    double al = 1, be = 0;
    rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, n, n, n, &al, A, n, B, n, &be, C, n);
    hipEventRecord(e0);
    for (int k = 0; k < 3; ++k) rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, n, n, n, &al, A, n, B, n, &be, C, n);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("dgemm n=%d: %.3f ms, %.1f TF\n", n, ms / 3, 2.0 * n * n * (double)n / (ms / 3 * 1e-3) / 1e12);
    hipEventRecord(e0);
    for (int k = 0; k < 3; ++k) rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, n, n, &al, A, n, &be, C, n);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("dsyrk n=%d: %.3f ms, %.1f TF\n", n, ms / 3, 1.0 * n * n * (double)n / (ms / 3 * 1e-3) / 1e12);
    hipFree(A); hipFree(B); hipFree(C);
  }
  int n = 12000;
  double *S, *x; int* info; hipMalloc(&S, 8ull*n*n); hipMalloc(&x, 8ull*n); hipMalloc(&info, 4);
  std::vector<double> hx(n, 1.0); hipMemcpy(x, hx.data(), 8*n, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(fill_spd, dim3((n*(size_t)n+255)/256), dim3(256), 0, 0, S, n);
    hipEventRecord(e0);
    rocsolver_dpotrf(h, rocblas_fill_lower, n, S, n, info);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    int hi; hipMemcpy(&hi, info, 4, hipMemcpyDeviceToHost);
    printf("dpotrf n=%d: %.3f ms (%.1f TF) info=%d\n", n, ms, (double)n*n*n/3.0/(ms*1e-3)/1e12, hi);
  }
  hipEventRecord(e0);
  rocsolver_dpotrs(h, rocblas_fill_lower, n, 1, S, n, x, n);
  hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("dpotrs: %.3f ms\n", ms);
  hipEventRecord(e0);
  rocblas_dtrsv(h, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit, n, S, n, x, 1);
  rocblas_dtrsv(h, rocblas_fill_lower, rocblas_operation_transpose, rocblas_diagonal_non_unit, n, S, n, x, 1);
  hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("2x dtrsv: %.3f ms\n", ms);
  hipEventRecord(e0);
  rocblas_dtrsm(h, rocblas_side_left, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit, n, 1, &hx[0], S, n, x, n);
  rocblas_dtrsm(h, rocblas_side_left, rocblas_fill_lower, rocblas_operation_transpose, rocblas_diagonal_non_unit, n, 1, &hx[0], S, n, x, n);
  hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("2x dtrsm: %.3f ms\n", ms);
  return 0;
}
