// Hand-written f64 MFMA GEMM C -= A B' (column-major, the Cholesky trailing
// update's shape: M x N block columns, K = 512 panel) against rocBLAS dgemm:
// time and max |difference| per shape.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/dgemm_probe.cpp -lrocblas -o tools/probes/dgemm_probe.bin
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../semantic-bundle-adjustment-colmap_amd/csrc/dgemm_nt.h"

__global__ void fill(double* x, size_t n, unsigned seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    x[i] = (double)(h & 0xffffff) / 16777216.0 - 0.5;
  }
}

int main() {
  const int ld = 12001;  // odd, like nf = 11 993
  const size_t cols = 3072;
  double *A, *C0, *C1;
  hipMalloc(&A, 8ull * ld * cols);
  hipMalloc(&C0, 8ull * ld * 1024);
  hipMalloc(&C1, 8ull * ld * 1024);
  hipLaunchKernelGGL(fill, dim3((unsigned)((8ull * ld * cols / 8 + 255) / 256)), dim3(256), 0, 0, A, (size_t)ld * cols, 7u);
  rocblas_handle h;
  rocblas_create_handle(&h);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct Shape { int m, n, k; };
  const Shape shapes[] = {{11488, 512, 512}, {10976, 1024, 512}, {8000, 1024, 512}, {4000, 1024, 512},
                          {1500, 1024, 512}, {333, 217, 512}, {10976, 1024, 1024}};
  for (const Shape& s : shapes) {
    const double* Ap = A + 5;             // rows 5.. (unaligned start)
    const double* Bp = A + 2048ull * ld;  // another column range
    const double flops = 2.0 * s.m * s.n * s.k;
    const double minus_one = -1.0, one = 1.0;
    hipLaunchKernelGGL(fill, dim3((unsigned)((ld * 1024ull + 255) / 256)), dim3(256), 0, 0, C0, (size_t)ld * 1024, 3u);
    hipMemcpy(C1, C0, 8ull * ld * 1024, hipMemcpyDeviceToDevice);
    rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, s.m, s.n, s.k, &minus_one, Ap, ld, Bp, ld,
                  &one, C0, ld);
    miba::dgemm_nt_sub(s.m, s.n, s.k, Ap, ld, Bp, ld, C1, ld, false, 0);
    hipDeviceSynchronize();
    std::vector<double> h0((size_t)ld * s.n), h1((size_t)ld * s.n);
    hipMemcpy(h0.data(), C0, 8ull * ld * s.n, hipMemcpyDeviceToHost);
    hipMemcpy(h1.data(), C1, 8ull * ld * s.n, hipMemcpyDeviceToHost);
    double err = 0.0, mx = 0.0;
    for (int j = 0; j < s.n; ++j)
      for (int i = 0; i < ld; ++i) {
        err = std::max(err, std::fabs(h0[(size_t)j * ld + i] - h1[(size_t)j * ld + i]));
        mx = std::max(mx, std::fabs(h0[(size_t)j * ld + i]));
      }
    float t_rb = 0, t_own = 0;
    const int reps = 10;
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r)
      rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, s.m, s.n, s.k, &minus_one, Ap, ld, Bp, ld,
                    &one, C0, ld);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&t_rb, e0, e1);
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) miba::dgemm_nt_sub(s.m, s.n, s.k, Ap, ld, Bp, ld, C1, ld, false, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&t_own, e0, e1);
    t_rb /= reps;
    t_own /= reps;
    printf("M %5d N %4d K %4d: rocBLAS %7.1f us %5.1f TF | own %7.1f us %5.1f TF | max|diff| %.2e (max|C| %.2e)\n",
           s.m, s.n, s.k, t_rb * 1e3, flops / (t_rb * 1e-3) / 1e12, t_own * 1e3, flops / (t_own * 1e-3) / 1e12, err,
           mx);
    fflush(stdout);
  }
  rocblas_destroy_handle(h);
  return 0;
}
