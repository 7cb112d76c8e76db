#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <cstdio>
__global__ void fill_spd(double* A, int n, int lda) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)n * n) return;
  int r = i / n, c = i % n;
  A[(size_t)c * lda + r] = (r == c) ? n * 0.02 + 1.0 : 0.01 * sin(0.37 * (r + c));
}
int main() {
  rocblas_handle h; rocblas_create_handle(&h);
  hipStream_t st; hipStreamCreate(&st); rocblas_set_stream(h, st);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms; int lda = 12000;
  double *A, *B; int* info; hipMalloc(&A, 8ull*lda*2048); hipMalloc(&B, 8ull*lda*2048); hipMalloc(&info, 64);
  for (int n : {128, 256, 384, 512, 768, 1024}) {
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(fill_spd, dim3((n*(size_t)n+255)/256), dim3(256), 0, st, A, n, lda);
      hipEventRecord(e0, st);
      rocsolver_dpotrf(h, rocblas_fill_lower, n, A, lda, info);
      hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
      float m2;
      hipEventRecord(e0, st);
      rocsolver_dtrtri(h, rocblas_fill_lower, rocblas_diagonal_non_unit, n, A, lda, info);
      hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&m2, e0, e1);
      if (rep == 2) printf("n=%d potrf %.3f ms trtri %.3f ms\n", n, ms, m2);
    }
  }
  double one = 1, m1 = -1;
  for (int nb : {256, 512, 1024}) {
    int m = 11000;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0, st);
      rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, m, nb, nb, &one, A, lda, A, lda, &m1, B, lda);
      hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
      float m2;
      hipEventRecord(e0, st);
      rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose, rocblas_diagonal_non_unit, m, nb, &one, A, lda, B, lda);
      hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&m2, e0, e1);
      if (rep) printf("panel m=%d nb=%d: gemm %.3f ms (%.1f TF), trsm %.3f ms\n", m, nb, ms, 2.0*m*nb*nb/(ms*1e-3)/1e12, m2);
    }
  }
  for (int k : {256, 512, 1024}) {
    int n = 11000;
    double *C; hipMalloc(&C, 8ull * n * n);
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0, st);
      rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, n, k, &m1, A, lda, &one, C, n);
      hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
      float m2;
      hipEventRecord(e0, st);
      rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, n, n, k, &m1, A, lda, A, lda, &one, C, n);
      hipEventRecord(e1, st); hipEventSynchronize(e1); hipEventElapsedTime(&m2, e0, e1);
      if (rep) printf("syrk n=%d k=%d: %.3f ms (%.1f TF) | gemm %.3f ms (%.1f TF eff-syrk)\n", n, k, ms, 1.0*n*n*k/(ms*1e-3)/1e12, m2, 1.0*n*n*k/(m2*1e-3)/1e12);
    }
    hipFree(C);
  }
  return 0;
}
