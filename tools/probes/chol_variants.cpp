// Times and cross-checks the Cholesky variants of csrc/cholesky.cpp on an
// SPD matrix of the C4 reduced-camera-system size.
//   hipcc --offload-arch=gfx950 -O2 -I. tools/probes/chol_variants.cpp \
//     semantic-bundle-adjustment-colmap_amd/csrc/cholesky.cpp -lrocsolver -lrocblas -o tools/chol_variants.bin
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

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
  rocblas_handle h;
  rocblas_create_handle(&h);
  hipStream_t st;
  hipStreamCreate(&st);
  rocblas_set_stream(h, st);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double *S, *x;
  int* info;
  hipMalloc(&S, 8ull * n * n);
  hipMalloc(&x, 8ull * n);
  hipMalloc(&info, 4 * 4096);
  std::vector<double> hx(n), ref(n);
  for (int i = 0; i < n; ++i) hx[i] = sin(0.1 * i);
  struct V { int panel; bool gemm; } vs[] = {{0, false}, {256, false}, {384, false}, {512, false}, {768, false},
                                              {1024, false}, {512, true}, {768, true}, {1024, true}};
  for (const V& v : vs) {
    miba::CholConfig cfg;
    cfg.panel = v.panel;
    cfg.gemm_update = v.gemm;
    float best = 1e30f, fs = 0.f;
    std::vector<double> out(n);
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(fill_spd, dim3((unsigned)(((size_t)n * n + 255) / 256)), dim3(256), 0, st, S, n);
      hipMemcpyAsync(x, hx.data(), 8 * n, hipMemcpyHostToDevice, st);
      hipEventRecord(e0, st);
      { static miba::CholWorkspace ws; if (ws.device < 0) ws.create(0, (n + 63) / 64, n); miba::chol_factor(h, n, S, n, info, cfg, &ws); }
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
      hipEventRecord(e0, st);
      miba::chol_solve(h, n, S, n, x);
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&fs, e0, e1);
    }
    hipMemcpy(out.data(), x, 8 * n, hipMemcpyDeviceToHost);
    std::vector<int> hi(miba::chol_leaf_count(n, cfg));
    hipMemcpy(hi.data(), info, 4 * hi.size(), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int k : hi) bad += k != 0;
    if (v.panel == 0) ref = out;
    double md = 0, mx = 0;
    for (int i = 0; i < n; ++i) {
      md = std::fmax(md, std::fabs(out[i] - ref[i]));
      mx = std::fmax(mx, std::fabs(ref[i]));
    }
    printf("{\"panel\": %d, \"gemm_update\": %d, \"factor_ms\": %.3f, \"TF\": %.1f, \"solve_ms\": %.3f, "
           "\"max_rel_diff_vs_recursive\": %.3e, \"bad_info\": %d}\n",
           v.panel, (int)v.gemm, best, (double)n * n * n / 3.0 / (best * 1e-3) / 1e12, fs, md / mx, bad);
  }
  return 0;
}
