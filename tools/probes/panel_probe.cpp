// Phase timeline of one panel_factor_kernel launch (csrc/cholesky.cpp,
// own_diag 6) on the first 512-wide panel of an nf = 12 000 SPD matrix:
// wall_clock64() stamps per row tile (kernel's dbg buffer).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/panel_probe.cpp -lrocsolver -lrocblas -o tools/probes/panel_probe.bin
//   tools/probes/panel_probe.bin [n] [tile_factor] [write_through] [concurrent dgemms] [panel wait mode]
#include "../../semantic-bundle-adjustment-colmap_amd/csrc/cholesky.cpp"

#include <cstdio>

__global__ void fill_spd(double* A, int n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)n * n) return;
  int r = i % n, c = i / n;
  A[i] = (r == c) ? n * 0.02 + 1.0 : 0.01 * sin(0.37 * (r + c)) + 0.005 * cos(0.011 * (double)r * c);
}

int main(int argc, char** argv) {
  using namespace miba;
  const int n = argc > 1 ? atoi(argv[1]) : 12000;
  const int kb = 512;
  double* A;
  int* info;
  unsigned long long* dbg;
  hipMalloc(&A, 8ull * n * n);
  hipMalloc(&info, 64);
  const int fv = argc > 2 ? atoi(argv[2]) : 2;  // tile factor: 2 rsq, 1 sqrt pivots, 3-5 tools-build variants
  const int wt = argc > 3 ? atoi(argv[3]) : 1;  // write-through publish
  const int busy = argc > 4 ? atoi(argv[4]) : 0;  // 1: trailing-update dgemms on a second stream meanwhile
  const int ow = argc > 5 ? atoi(argv[5]) : 0;  // panel wait mode (CholConfig::panel_wait)
  printf("n %d, tile_factor %d, write_through %d, concurrent dgemms %d, panel wait %d\n", n, fv, wt, busy, ow);
  const int nr = 8 + (n - kb + 63) / 64;
  hipMalloc(&dbg, 8ull * nr * kPfDbgSlots);
  CholWorkspace ws;
  ws.create(0, (n + 511) / 512, n);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(fill_spd, dim3((unsigned)(((size_t)n * n + 255) / 256)), dim3(256), 0, 0, A, n);
    hipMemset(dbg, 0, 8ull * nr * kPfDbgSlots);
    hipMemset(info, 0, 4);
    hipDeviceSynchronize();
    const unsigned epoch = ++ws.pf_epoch;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipStream_t bs = nullptr;
    rocblas_handle bh = nullptr;
    if (busy) {
      // the look-ahead's rest update beside the panel: 1024-wide block columns
      // of the trailing matrix, C -= P P' with K = 512 (default solution index)
      hipStreamCreateWithFlags(&bs, hipStreamNonBlocking);
      rocblas_create_handle(&bh);
      rocblas_set_stream(bh, bs);
      const double m1 = -1.0, p1 = 1.0;
      for (int j = 2 * kb; j + 1024 <= n; j += 1024)
        rocblas_gemm_ex(bh, rocblas_operation_none, rocblas_operation_transpose, n - j, 1024, kb, &m1, A + j, rocblas_datatype_f64_r,
                        n, A + j, rocblas_datatype_f64_r, n, &p1, A + j + (size_t)j * n, rocblas_datatype_f64_r, n,
                        A + j + (size_t)j * n, rocblas_datatype_f64_r, n, rocblas_datatype_f64_r,
                        rocblas_gemm_algo_solution_index, CholConfig{}.gemm_solution, 0);
    }
    hipEventRecord(e0, ws.side);
    auto pick = [&](auto wm) {
      constexpr int W = decltype(wm)::value;
      return fv == 6   ? panel_factor_kernel<6, true, W>
             : fv == 3 ? panel_factor_kernel<3, true, W>
             : fv == 4 ? panel_factor_kernel<4, true, W>
             : fv == 5 ? panel_factor_kernel<5, true, W>
             : fv == 2 ? (wt ? panel_factor_kernel<2, true, W> : panel_factor_kernel<2, false, W>)
                       : (wt ? panel_factor_kernel<1, true, W> : panel_factor_kernel<1, false, W>);
    };
    auto kern = ow == 3 ? pick(std::integral_constant<int, 3>{})
                : ow == 2 ? pick(std::integral_constant<int, 2>{})
                : ow == 1 ? pick(std::integral_constant<int, 1>{}) : pick(std::integral_constant<int, 0>{});
    hipLaunchKernelGGL(kern, dim3(nr), dim3(256), 0, ws.side, A, n, kb, n, info, ws.pf_linv, ws.pf_ctrl, ws.pf_base, epoch,
                       ws.err, ws.spin_limit, 0, dbg, 0, nullptr);
    hipEventRecord(e1, ws.side);
    hipEventSynchronize(e1);
    if (busy) {
      hipStreamSynchronize(bs);
      rocblas_destroy_handle(bh);
      hipStreamDestroy(bs);
    }
    ws.pf_base += nr;
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h((size_t)nr * kPfDbgSlots);
    hipMemcpy(h.data(), dbg, 8ull * h.size(), hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull;
    for (int r = 0; r < nr; ++r) t0 = std::min(t0, h[(size_t)r * kPfDbgSlots]);
    int hinfo = 0;
    hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost);
    printf("rep %d: kernel %.1f us, info %d (stamps in us from the first start, 100 MHz clock)\n", rep, ms * 1e3, hinfo);
    for (int r = 0; r < nr; ++r) {
      if (r > 9 && r != nr - 1) continue;
      printf("  row %3d:", r);
      for (int k = 0; k < kPfDbgSlots; ++k) {
        const unsigned long long v = h[(size_t)r * kPfDbgSlots + k];
        if (v) printf(" %d:%.1f", k, (v - t0) / 100.0);
      }
      printf("\n");
    }
  }
  return 0;
}
