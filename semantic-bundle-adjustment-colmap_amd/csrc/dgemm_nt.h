// dgemm_nt.h — C -= A B' in f64 on the MFMA f64 pipe (v_mfma_f64_16x16x4f64),
// the Cholesky trailing update's shape (cholesky.cpp): A is M x K, B is N x K,
// C is M x N, all column-major with arbitrary (odd) leading dimensions, K a
// multiple of 16.  Product code: included by cholesky.cpp (and by the probe
// tools/probes/dgemm_probe.cpp).
//
// One 256-thread workgroup per 128 x 128 tile of C (four waves, 64 x 64 each:
// 4 x 4 MFMA blocks, 64 f64 accumulators per lane); K in chunks of 16 staged
// through LDS k-major (a chunk column is 128 contiguous doubles of A or B, so
// the copy is a straight coalesced one), double-buffered: chunk c+1's 16
// loads per thread are in flight while chunk c's 64 MFMAs per wave run.
// lower: tiles entirely above the diagonal of C (row < column everywhere,
// with C's row r and column c at global index row0 + r, col0 + c and
// row0 == col0 for the diagonal block) are skipped — the trailing update
// only needs the lower triangle.  Tiles are mapped XCD-major so the tiles of
// one M-stripe (sharing their A rows) run on one XCD's L2.
#pragma once

#include <hip/hip_runtime.h>

namespace miba {

namespace dgemm_detail {
constexpr int kBM = 128, kBN = 128, kKC = 16;
typedef double dvec4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256, 2) void dgemm_nt_sub_kernel(int M, int N, int K, const double* __restrict__ A,
                                                              int lda, const double* __restrict__ B, int ldb,
                                                              double* __restrict__ C, int ldc, int lower, int tiles_m,
                                                              int tiles_n) {
  __shared__ double As[2][kKC][kBM];
  __shared__ double Bs[2][kKC][kBN];
  // XCD-major tile order: workgroup b runs on XCD b % 8; XCD x takes the
  // contiguous linear range [x * per, (x + 1) * per) of M-major tiles
  const int ntiles = tiles_m * tiles_n;
  const int per = (ntiles + 7) / 8;
  const int b = blockIdx.x;
  const int lin = (b % 8) * per + b / 8;
  if (lin >= ntiles) return;
  const int tm = lin / tiles_n, tn = lin % tiles_n;
  const int m0 = tm * kBM, n0 = tn * kBN;
  if (lower && m0 + kBM <= n0) return;  // every row < every column: strictly upper
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv & 1, wn = wv >> 1;
  const int mr = lane & 15, kq = lane >> 4;
  // global -> register staging: each thread copies 8 doubles of A's chunk and
  // 8 of B's (q = tid + 256 j: chunk column q / 128, row q % 128)
  double ra[8], rb[8];
  auto load_chunk = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int q = tid + 256 * j, kk = q >> 7, r = q & 127;
      const int am = min(m0 + r, M - 1), bn = min(n0 + r, N - 1);
      ra[j] = A[(size_t)(k0 + kk) * lda + am];
      rb[j] = B[(size_t)(k0 + kk) * ldb + bn];
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int q = tid + 256 * j, kk = q >> 7, r = q & 127;
      As[buf][kk][r] = ra[j];
      Bs[buf][kk][r] = rb[j];
    }
  };
  dvec4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = dvec4{0.0, 0.0, 0.0, 0.0};
  const int nk = K / kKC;
  load_chunk(0);
  store_chunk(0);
  __syncthreads();
  for (int c = 0; c < nk; ++c) {
    const int buf = c & 1;
    if (c + 1 < nk) load_chunk((c + 1) * kKC);
#pragma unroll
    for (int s = 0; s < kKC / 4; ++s) {
      double a[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[buf][4 * s + kq][wm * 64 + 16 * i + mr];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[buf][4 * s + kq][wn * 64 + 16 * j + mr];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (c + 1 < nk) store_chunk(buf ^ 1);
    __syncthreads();
  }
  // C -= acc (D layout: acc[r] at lane l is D[4r + l/16][l%16])
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + 16 * i + 4 * r + (lane >> 4);
        const int col = n0 + wn * 64 + 16 * j + (lane & 15);
        if (row < M && col < N && (!lower || row >= col)) {
          double* p = C + (size_t)col * ldc + row;
          *p -= acc[i][j][r];
        }
      }
}
}  // namespace dgemm_detail

// C -= A B' on `stream`; K % 16 == 0.  lower: only C's lower triangle (row >=
// column, C's top-left element on the diagonal) is updated.
inline hipError_t dgemm_nt_sub(int M, int N, int K, const double* A, int lda, const double* B, int ldb, double* C,
                               int ldc, bool lower, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return hipSuccess;
  if (K % dgemm_detail::kKC != 0) return hipErrorInvalidValue;
  const int tm = (M + dgemm_detail::kBM - 1) / dgemm_detail::kBM, tn = (N + dgemm_detail::kBN - 1) / dgemm_detail::kBN;
  const int ntiles = tm * tn;
  const int grid = ((ntiles + 7) / 8) * 8;
  hipLaunchKernelGGL(dgemm_detail::dgemm_nt_sub_kernel, dim3(grid), dim3(256), 0, stream, M, N, K, A, lda, B, ldb, C,
                     ldc, lower ? 1 : 0, tm, tn);
  return hipGetLastError();
}

}  // namespace miba
