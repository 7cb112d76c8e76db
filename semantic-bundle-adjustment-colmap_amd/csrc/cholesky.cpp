// cholesky.cpp — recursive blocked Cholesky over rocBLAS/rocSOLVER (see cholesky.h).
#include "cholesky.h"

#include <rocsolver/rocsolver.h>

#include <algorithm>

namespace miba {

namespace {

constexpr int kLeaf = 768;  // diagonal leaves factored by rocSOLVER

int split(int n) {
  int n1 = n / 2;
  n1 = (n1 + 255) / 256 * 256;  // keep the big dtrsm/dsyrk operands 2 KB aligned
  return n1 < n ? n1 : n / 2;
}

rocblas_status factor(rocblas_handle h, int n, double* A, int lda, int*& info) {
  if (n <= kLeaf) return rocsolver_dpotrf(h, rocblas_fill_lower, n, A, lda, info++);
  const int n1 = split(n), n2 = n - n1;
  double* A11 = A;
  double* A21 = A + n1;
  double* A22 = A + n1 + (size_t)n1 * lda;
  rocblas_status st = factor(h, n1, A11, lda, info);
  if (st != rocblas_status_success) return st;
  const double one = 1.0, minus_one = -1.0;
  // A21 := A21 L11^-T
  st = rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                     rocblas_diagonal_non_unit, n2, n1, &one, A11, lda, A21, lda);
  if (st != rocblas_status_success) return st;
  // A22 := A22 - A21 A21'
  st = rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, n2, n1, &minus_one, A21, lda, &one, A22, lda);
  if (st != rocblas_status_success) return st;
  return factor(h, n2, A22, lda, info);
}

int leaves(int n) { return n <= kLeaf ? 1 : leaves(split(n)) + leaves(n - split(n)); }

// L y = b (forward) and L' x = y (backward), recursively.
rocblas_status forward(rocblas_handle h, int n, const double* A, int lda, double* x) {
  if (n <= kLeaf)
    return rocblas_dtrsv(h, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit, n, A, lda, x, 1);
  const int n1 = split(n), n2 = n - n1;
  rocblas_status st = forward(h, n1, A, lda, x);
  if (st != rocblas_status_success) return st;
  const double one = 1.0, minus_one = -1.0;
  st = rocblas_dgemv(h, rocblas_operation_none, n2, n1, &minus_one, A + n1, lda, x, 1, &one, x + n1, 1);
  if (st != rocblas_status_success) return st;
  return forward(h, n2, A + n1 + (size_t)n1 * lda, lda, x + n1);
}

rocblas_status backward(rocblas_handle h, int n, const double* A, int lda, double* x) {
  if (n <= kLeaf)
    return rocblas_dtrsv(h, rocblas_fill_lower, rocblas_operation_transpose, rocblas_diagonal_non_unit, n, A, lda, x,
                         1);
  const int n1 = split(n), n2 = n - n1;
  rocblas_status st = backward(h, n2, A + n1 + (size_t)n1 * lda, lda, x + n1);
  if (st != rocblas_status_success) return st;
  const double one = 1.0, minus_one = -1.0;
  // x1 -= L21' x2
  st = rocblas_dgemv(h, rocblas_operation_transpose, n2, n1, &minus_one, A + n1, lda, x + n1, 1, &one, x, 1);
  if (st != rocblas_status_success) return st;
  return backward(h, n1, A, lda, x);
}

// Right-looking blocked factorisation: per panel, dpotrf of the diagonal
// block, dtrsm of the panel below it, then the trailing lower triangle
// updated by dsyrk (or by dgemm per block column of width `panel`).
rocblas_status factor_blocked(rocblas_handle h, int n, double* A, int lda, int* info, const CholConfig& cfg) {
  const double one = 1.0, minus_one = -1.0;
  const int nb = cfg.panel;
  for (int k = 0; k < n; k += nb) {
    const int kb = std::min(nb, n - k);
    double* Akk = A + k + (size_t)k * lda;
    rocblas_status st = rocsolver_dpotrf(h, rocblas_fill_lower, kb, Akk, lda, info++);
    if (st != rocblas_status_success) return st;
    const int m = n - k - kb;
    if (m == 0) break;
    double* Aik = Akk + kb;  // panel below the diagonal block
    st = rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                       rocblas_diagonal_non_unit, m, kb, &one, Akk, lda, Aik, lda);
    if (st != rocblas_status_success) return st;
    double* T = Aik + (size_t)kb * lda;  // trailing matrix, lower triangle
    if (!cfg.gemm_update) {
      st = rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, m, kb, &minus_one, Aik, lda, &one, T, lda);
      if (st != rocblas_status_success) return st;
    } else {
      for (int j = 0; j < m; j += nb) {
        const int jb = std::min(nb, m - j);
        st = rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, m - j, jb, kb, &minus_one, Aik + j,
                           lda, Aik + j, lda, &one, T + j + (size_t)j * lda, lda);
        if (st != rocblas_status_success) return st;
      }
    }
  }
  return rocblas_status_success;
}

}  // namespace

int chol_leaf_count(int n, const CholConfig& cfg) {
  if (n <= 0) return 1;
  return cfg.panel > 0 ? (n + cfg.panel - 1) / cfg.panel : leaves(n);
}

rocblas_status chol_factor(rocblas_handle h, int n, double* A, int lda, int* info, const CholConfig& cfg) {
  if (n <= 0) return rocblas_status_success;
  if (cfg.panel > 0) return factor_blocked(h, n, A, lda, info, cfg);
  return factor(h, n, A, lda, info);
}

rocblas_status chol_solve(rocblas_handle h, int n, const double* A, int lda, double* x) {
  if (n <= 0) return rocblas_status_success;
  rocblas_status st = forward(h, n, A, lda, x);
  if (st != rocblas_status_success) return st;
  return backward(h, n, A, lda, x);
}

}  // namespace miba
