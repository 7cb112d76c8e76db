// cholesky.h — dense Cholesky of the reduced camera system (product code).
//
// The exact Schur path factors S (nf x nf f64, column-major lower) every LM
// iteration.  rocSOLVER's dpotrf runs ~10 TF/s and dpotrs ~0.1 s at
// nf = 12 000 (measured on MI355X), while rocBLAS' MFMA dgemm/dsyrk run
// 40-65 TF/s.  Two factorisations are provided, both with all their work in
// rocBLAS level-3 calls and dpotrf only on small diagonal blocks:
//   panel == 0: recursive left/right split (half the flops in dtrsm);
//   panel  > 0: right-looking blocked with panel width `panel` (dtrsm on the
//               panel only, the trailing update as dsyrk, or as dgemm on
//               block columns of the lower triangle when `gemm_update`).
// The solve recurses the same way (dtrsv leaves + dgemv).
#pragma once

#include <rocblas/rocblas.h>

namespace miba {

// Default: right-looking, 512-wide panels, dgemm trailing update (48 ms vs
// 62 ms for the recursive split at nf = 12 000 on MI355X; profiles/r1/
// chol_variants.txt).
struct CholConfig {
  int panel = 512;        // 0: recursive split; > 0: right-looking panel width
  bool gemm_update = true;
  // panel k+1's diagonal factor + dtrsm on a side stream under panel k's dgemm
  // (34.6 -> 30.4 ms at nf = 12 000); one event pair per panel — re-recording one
  // event per iteration let a wait slip past its producer (a diverged C4 run)
  bool lookahead = true;
  bool own_diag = true;   // diagonal blocks by the hand-written 64-wide factor, else rocsolver_dpotrf
};

// In-place lower Cholesky of the n x n column-major matrix A (leading
// dimension lda).  info[k] (device, one int per diagonal block, count from
// chol_leaf_count) is 0 for every block of a positive-definite A.
rocblas_status chol_factor(rocblas_handle h, int n, double* A, int lda, int* info, const CholConfig& cfg = {});
int chol_leaf_count(int n, const CholConfig& cfg = {});
// x := (L L')^-1 x with the factor chol_factor left in A.
rocblas_status chol_solve(rocblas_handle h, int n, const double* A, int lda, double* x);

}  // namespace miba
