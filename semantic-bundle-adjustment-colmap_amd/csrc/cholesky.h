// cholesky.h — dense Cholesky of the reduced camera system (product code).
//
// The exact Schur path factors S (nf x nf f64, column-major lower) every LM
// iteration.  rocSOLVER's dpotrf runs ~10 TF/s and dpotrs ~0.1 s at
// nf = 12 000 (measured on MI355X), while rocBLAS' MFMA dgemm/dsyrk run
// 60-75 TF/s, so the factorisation is a recursive (left/right split)
// blocked Cholesky whose work is all in dtrsm + dsyrk, with dpotrf only on
// diagonal leaves; the solve recurses the same way (dtrsv leaves + dgemv).
#pragma once

#include <rocblas/rocblas.h>

#include <vector>

namespace miba {

// In-place lower Cholesky of the n x n column-major matrix A (leading
// dimension lda).  info[k] (device, one int per leaf, `leaves` from
// chol_leaf_count) is 0 for every leaf of a positive-definite A.
rocblas_status chol_factor(rocblas_handle h, int n, double* A, int lda, int* info);
int chol_leaf_count(int n);
// x := (L L')^-1 x with the factor chol_factor left in A.
rocblas_status chol_solve(rocblas_handle h, int n, const double* A, int lda, double* x);

}  // namespace miba
