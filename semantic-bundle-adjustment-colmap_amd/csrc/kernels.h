// kernels.h — launch wrappers of the gfx950 kernels (product code).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device.h"

namespace miba {

struct SemDevice;  // defined in semantic.h

// Residual + tangent Jacobian of every reduced block (J-materialising), with
// the loss Corrector applied and the cost folded into per-workgroup partials.
// p.jvariant selects A/B builds of the C4 shape (0 = production).
// Rebuild p.img_rec from qt / cam / flags (before every Jacobian launch).
// also zeroes zero[0..nzero) when zero is given
void launch_pack_images(const DevProblem& p, double* rec, hipStream_t s, double* zero = nullptr, int nzero = 0);
void launch_reproj_jacobian(const DevProblem& p, double2* r, double* J, double* cost_partial, hipStream_t s);
// mask: bit 0 observations, 1 image ids, 2 point ids, 3 points; wgs <= 0: one workgroup per CU
void launch_touch_inputs(const DevProblem& p, unsigned* sink, hipStream_t s, int mask = 15, int wgs = 0,
                         int unroll = 4);
int reproj_grid(int64_t nb);

// Cost 0.5*sum(rho) of every reduced block at parameters (qt, cam, X).
void launch_reproj_cost(const DevProblem& p, const double* qt, const double* cam, const double* X,
                        double* cost_partial, hipStream_t s);

// Sum n partials into out[0] (single workgroup).
// out[0] = sum of partial[0..n) in a fixed order.  scratch (kSumScratch
// doubles, last slot a zeroed ticket) enables the many-workgroup pass for long
// lists; launches sharing a scratch must be stream-ordered.
constexpr int kSumScratch = 65 + 17;  // launch_sum: [64] stage + ticket; launch_sum2 adds [16] + ticket
void launch_sum(const double* partial, int64_t n, double* out, hipStream_t s, double* scratch = nullptr);
// Both sums in one launch, each by a many-workgroup pass (64 and 16
// workgroups; scratch1: kSumScratch doubles, zeroed tickets).
void launch_sum2(const double* p1, int64_t n1, double* out1, double* scratch1, const double* p2, int64_t n2,
                 double* out2, hipStream_t s);

// Point side: Jacobi scale (first), LM diagonal (when !reuse_diag) and the
// damped inverse Vinv[P][6] of V_p + Lambda_p.
// Point blocks Vg[P][9] = (V_p packed upper 6, g_p 3) of the variable points
// from J and r (the solver's point-side normal equations).
// chunks: the point chunks (one lane per block; else one lane per point)
void launch_point_normal(const DevProblem& p, const DevPoint* vp, int64_t npv, const double2* r, const double* J,
                         double* Vg, hipStream_t s, const uint32_t* chunks = nullptr, int nchunks = 0);
void launch_point_prepare(const DevProblem& p, const DevPoint* vp, int64_t npv, const double* Vg,
                          double* scale_p, double* diag_p, double* Vinv, double* Linv, double* q, int first,
                          int reuse_diag, double radius, hipStream_t s);
// (q, nullable: q_p = V_p^-1 g_p [P][3] for launch_fblock_dense)

// Camera-side tile pass: per image/camera tangent block S_ii = U_ii - sum W V^-1 W',
// b = g - sum W V^-1 g_p and diag(U) (undamped column norms).
// Jcm (nullable): J's rows in camera-major order (launch_permute_rows).
// own (nullable): the deterministic flush (per-tile partials summed per image /
// camera in a fixed order, owner_flush_kernel) instead of float atomics; the
// same for every camera-side tile pass below.
void launch_fblock(const DevProblem& p, const DevTile* tiles, int ntiles, const uint32_t* cm_perm,
                   const double2* r, const double* J, const double* Jcm, const double* Vg, const double* Vinv,
                   double* pose_blk, double* cam_blk, double* b, double* udiag, hipStream_t s,
                   const TileOwners* own = nullptr);
// Jcm[k] = J[cm_perm[k]] for k < n (2 (9 + ct) doubles per block).
// Doubles per block of the Schur build's per-block records (Z rows, or the
// JG records of schur_pairs_variant 6).
inline int64_t schur_record_width(int ct, int svariant) {
  const int F = 6 + ct;
  return svariant == 6 ? ((2 * F + 6 + 15) / 16) * 16 : 3 * F;
}
void launch_permute_rows(const DevProblem& p, const uint32_t* cm_perm, int64_t n, const double* J, double* Jcm,
                         hipStream_t s);

// Exact-solver variant of launch_fblock: U = sum J_f'J_f added into S's image
// blocks, b = g - sum W V^-1 g_p and diag(U), in one pass (no Schur-Jacobi
// blocks, which only the PCG preconditioner uses).
void launch_fblock_dense(const DevProblem& p, const DevTile* tiles, int ntiles, const uint32_t* cm_perm,
                         const uint32_t* cm_ptv, const double2* r, const double* J, const double* q, double* b,
                         double* udiag, double* S, hipStream_t s, const TileOwners* own = nullptr);

// Finalise: Jacobi scale (first), LM diagonal, damping Lambda_f, block-Jacobi
// preconditioner (inverse of the damped diagonal blocks), rhs = -b.
void launch_fblock_finalize(const DevProblem& p, const double* pose_blk, const double* cam_blk,
                            const double* udiag, double* scale_f, double* diag_f, double* lambda_f,
                            double* prec_pose, double* prec_cam, double* b, int first, int reuse_diag,
                            double radius, hipStream_t s);

// Implicit Schur product y = S x (without the semantic pair term); lambda_f
// null leaves out the damping diagonal (multi-rank: added by rank 0 only).
// chunks: the back substitution's point chunks (the point pass runs on them).
// Jcm: J's rows in camera-major order (the f pass reads them contiguously;
// staged: through LDS by coalesced loads, one residual row per lane).
void launch_schur_product(const DevProblem& p, const DevPoint* vp, int64_t npv, const DevTile* tiles,
                          int ntiles, const uint32_t* cm_perm, const double* J, const double* Vinv,
                          const double* lambda_f, const double* x, double* w, double* y, hipStream_t s,
                          const uint32_t* chunks = nullptr, int nchunks = 0, const uint32_t* cm_ptv = nullptr,
                          const double* Jcm = nullptr, bool staged = false, const double* Xcm = nullptr,
                          const double2* obs_cm = nullptr, const TileOwners* own = nullptr);
// Matrix-free product (Xcm non-null, with chunks and cm_ptv): both passes
// recompute the blocks' Jacobian rows instead of reading J; Xcm / obs_cm are
// the camera-major copies of the blocks' points / observations (obs_cm only
// with a robust loss) built by launch_gather_cm.
void launch_gather_cm(const DevProblem& p, const uint32_t* cm_perm, int64_t n, double* Xcm, double2* obs_cm,
                      hipStream_t s);

// Block-Jacobi preconditioner apply z = M^-1 r.
void launch_precond(const DevProblem& p, const double* prec_pose, const double* prec_cam,
                    const double* r, double* z, hipStream_t s);

// Vector ops on the f-vector.
// n 8xNxN parameter blocks (GSBA cylinders): Jacobi scaling, LM damping,
// Schur-Jacobi preconditioner blocks, rhs sign (as the pose / camera blocks);
// pointers offset to the first block's f-vector slots.
// width 8 (Cylinder: q 3, t 3, radius, height) or 7 (CylinderBy2Points).
void launch_finalize_n(int width, int n, const double* blk, const double* udiag, double* scale_f, double* diag_f,
                       double* lambda_f, double* prec, double* b, int var, int first, int reuse_diag, double radius,
                       hipStream_t s);
void launch_precond_n(int width, int n, const double* prec, const double* r, double* z, hipStream_t s);
void launch_dot(const double* a, const double* b, int64_t n, double* out, hipStream_t s);
void launch_axpy(double* y, const double* x, const double* alpha_num, const double* alpha_den,
                 double sign, int64_t n, hipStream_t s);
void launch_xpby(double* p, const double* z, const double* beta_num, const double* beta_den,
                 int64_t n, hipStream_t s);

// Back substitution dX_p = -Vinv (g_p + sum Jp' Jf df) for variable points.
void launch_backsub(const DevProblem& p, const DevPoint* vp, int64_t npv, const double* J,
                    const double* Vg, const double* Vinv, const double* df, double* dX, hipStream_t s);

// Back substitution + model cost change in one pass over the variable
// points' blocks (per-wave partials into partial, count returned; the
// blocks of constant points, const_blocks, atomically into partial[0]).
// Back substitution + model cost change over point chunks (blocks
// [chunk[c], chunk[c+1]) of whole points, <= 64 unless one point has more):
// one partial per chunk into partial[0..nchunks), returns nchunks.
int64_t launch_backsub_chunks(const DevProblem& p, const uint32_t* chunk, int nchunks, const double* J,
                              const double2* r, const double* Vg, const double* Vinv, const double* df, double* dX,
                              double* partial, hipStream_t s);
int64_t launch_backsub_cost(const DevProblem& p, const DevPoint* vp, int64_t npv, const double* J, const double2* r,
                            const double* Vg, const double* Vinv, const double* df, double* dX, double* partial,
                            bool const_blocks, hipStream_t s);

// Model cost change partials: -(J d).(r + J d / 2) per block.
void launch_model_cost(const DevProblem& p, const double2* r, const double* J, const double* df,
                       const double* dX, double* partial, hipStream_t s);

// Candidate parameters: manifold Plus of the tangent step (scaled back).
void launch_plus(const DevProblem& p, const double* df, const double* dX, const double* qt,
                 const double* cam, const double* X, double* qt_out, double* cam_out, double* X_out,
                 hipStream_t s);

// Explicit reduced camera system (nf x nf, row-major, upper triangle row <= col,
// i.e. rocSOLVER's column-major lower): S += U (image tile pass, with_u; else
// launch_fblock_dense added it) - sum_p W_p V_p^-1 W_p' (Z factors, then MFMA
// image-pair tiles).
void launch_dense_schur(const DevProblem& p, const DevTile* tiles, int ntiles, const uint32_t* cm_perm,
                        const uint32_t* cm_ptv, const double* J, const double* Linv, double* Z, const DevPairTile* ptiles, int nptiles,
                        const uint2* pairs, double* S, bool with_u, hipStream_t s, const PairFlush* pflush = nullptr);
// S_kk += Lambda_k on parameter slots, S_kk = 1 on non-parameter slots.
void launch_dense_finalize(const DevProblem& p, const double* lambda_f, double* S, hipStream_t s);

// Squared norms of df and dX (for the parameter tolerance test).
// |a|^2 + |b|^2 into out[0]; scratch (kReduceBlocks doubles, or null for a
// one-workgroup reduction) holds per-workgroup partials
constexpr int kReduceBlocks = 256;
void launch_sqnorm2(const double* a, int64_t na, const double* b, int64_t nb, double* out, double* scratch,
                    hipStream_t s);

// One CG step x += alpha p (and r -= alpha q when update_r), alpha = rho /
// pq, skipped where Ceres' ConjugateGradientsSolver stops before moving x
// (rho or beta = rho / rho_prev 0 / inf, pq <= 0 / inf, alpha inf; rho_prev
// nullable on the first iteration).
void launch_cg_step(double* x, const double* p, double* r, const double* q, const double* rho,
                    const double* rho_prev, const double* pq, bool update_r, int64_t n, hipStream_t s);

// Gradient tolerance (TrustRegionMinimizer::EvaluateGradientAndJacobian):
// g += sum J_f' r over the camera-major tiles (raw tangent gradient of the
// image / camera slots); |x - Plus(x, -g)|_inf of the image and camera
// blocks, and of the variable points (g_p from Vg), atomically max-ed into
// out[0] (non-negative doubles, as bit patterns).
void launch_grad_f(const DevProblem& p, const DevTile* tiles, int ntiles, const uint32_t* cm_perm, const double2* r,
                   const double* J, double* g, hipStream_t s, const TileOwners* own = nullptr);
void launch_grad_max_f(const DevProblem& p, const double* g, double* out, hipStream_t s);
void launch_grad_max_points(const DevProblem& p, const DevPoint* vp, int64_t npv, const double* Vg, double* out,
                            hipStream_t s);
// Ceres' ambient state norms for ParameterToleranceReached: out[0] = |x|^2,
// out[1] = |x - x_c|^2 over the variable image / camera blocks (when with_f)
// and variable points; scratch: kReduceBlocks doubles.
void launch_state_norms(const DevProblem& p, const double* qt_c, const double* cam_c, const double* X_c, bool with_f,
                        double* out, double* scratch, hipStream_t s);

}  // namespace miba
