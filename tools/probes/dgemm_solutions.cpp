// rocBLAS dgemm solution sweep for the Cholesky trailing-update shapes
// (C -= A B', column-major, lda = 12 000, K = panel width): every solution
// rocblas_gemm_ex_get_solutions lists for the shape, timed with HIP events,
// against the default (algo standard, index 0).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/dgemm_solutions.cpp -lrocblas -o tools/probes/dgemm_solutions.bin
#define ROCBLAS_BETA_FEATURES_API
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <algorithm>
#include <cstdio>
#include <vector>

static float time_gemm(rocblas_handle h, int m, int n, int k, const double* A, const double* B, double* C, int ld,
                       rocblas_gemm_algo algo, int sol, int reps) {
  const double alpha = -1.0, beta = 1.0;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto call = [&]() {
    return rocblas_gemm_ex(h, rocblas_operation_none, rocblas_operation_transpose, m, n, k, &alpha, A,
                           rocblas_datatype_f64_r, ld, B, rocblas_datatype_f64_r, ld, &beta, C, rocblas_datatype_f64_r,
                           ld, C, rocblas_datatype_f64_r, ld, rocblas_datatype_f64_r, algo, sol, 0);
  };
  if (call() != rocblas_status_success) return -1.0f;
  hipDeviceSynchronize();
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r) call();
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.0f;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms / reps;
}

int main() {
  const int ld = 12000;
  double *A, *C;
  hipMalloc(&A, 8ull * ld * 2048);
  hipMalloc(&C, 8ull * ld * 2048);
  hipMemset(A, 0, 8ull * ld * 2048);
  hipMemset(C, 0, 8ull * ld * 2048);
  rocblas_handle h;
  rocblas_create_handle(&h);
  struct Shape { int m, n, k; };
  const Shape shapes[] = {{11488, 512, 512}, {10976, 1024, 512}, {8000, 1024, 512}, {4000, 1024, 512},
                          {1500, 1024, 512}, {10976, 1024, 1024}, {8192, 2048, 512}};
  for (const Shape& s : shapes) {
    const double flops = 2.0 * s.m * s.n * s.k;
    const float t0 = time_gemm(h, s.m, s.n, s.k, A, A + 1024, C, ld, rocblas_gemm_algo_standard, 0, 10);
    rocblas_int nsol = 0;
    const double alpha = -1.0, beta = 1.0;
    rocblas_gemm_ex_get_solutions(h, rocblas_operation_none, rocblas_operation_transpose, s.m, s.n, s.k, &alpha, A,
                                  rocblas_datatype_f64_r, ld, A + 1024, rocblas_datatype_f64_r, ld, &beta, C,
                                  rocblas_datatype_f64_r, ld, C, rocblas_datatype_f64_r, ld, rocblas_datatype_f64_r,
                                  rocblas_gemm_algo_solution_index, 0, nullptr, &nsol);
    std::vector<rocblas_int> sols(std::max(1, (int)nsol));
    rocblas_gemm_ex_get_solutions(h, rocblas_operation_none, rocblas_operation_transpose, s.m, s.n, s.k, &alpha, A,
                                  rocblas_datatype_f64_r, ld, A + 1024, rocblas_datatype_f64_r, ld, &beta, C,
                                  rocblas_datatype_f64_r, ld, C, rocblas_datatype_f64_r, ld, rocblas_datatype_f64_r,
                                  rocblas_gemm_algo_solution_index, 0, sols.data(), &nsol);
    float best = 1e30f;
    int best_sol = -1;
    for (int i = 0; i < nsol; ++i) {
      const float t = time_gemm(h, s.m, s.n, s.k, A, A + 1024, C, ld, rocblas_gemm_algo_solution_index, sols[i], 5);
      if (t > 0 && t < best) {
        best = t;
        best_sol = sols[i];
      }
    }
    printf("M %5d N %4d K %4d: default %.1f us = %.1f TF; %d solutions, best %d: %.1f us = %.1f TF\n", s.m, s.n, s.k,
           t0 * 1e3, flops / (t0 * 1e-3) / 1e12, (int)nsol, best_sol, best * 1e3, flops / (best * 1e-3) / 1e12);
    fflush(stdout);
  }
  rocblas_destroy_handle(h);
  return 0;
}
