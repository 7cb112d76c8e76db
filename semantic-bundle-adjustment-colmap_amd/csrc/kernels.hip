// kernels.hip — gfx950 kernels of the geometric BA hot path (product code).
//
// Replaces, on MI355X, the Ceres 2.1 evaluation of every
// BundleAdjustmentCostFunction / BundleAdjustmentConstantPoseCostFunction
// residual block (src/base/cost_functions.h:44-152, AutoDiff) and the Ceres
// ITERATIVE_SCHUR + SCHUR_JACOBI linear algebra that BundleAdjuster::Solve
// selects (src/optim/bundle_adjustment.cc:276-286).
//
// One lane per residual block; blocks are point-major so the point-side
// normal-equation blocks reduce inside a wavefront (segmented Hillis-Steele
// scan over 64 lanes, atomics only for the two segments that may straddle a
// wave boundary).  Camera-side reductions run over image-aligned tiles of a
// camera-major permutation (one atomic flush per tile and value).
#include <hip/hip_runtime.h>

#include "ba_math.h"
#include "device.h"
#include "kernels.h"

namespace miba {

namespace {

typedef double dvec2 __attribute__((ext_vector_type(2)));  // native 16-B vector (nontemporal builtins)

constexpr int kSymPose = 21;  // packed upper triangle of 6x6

__host__ __device__ constexpr int sym_size(int n) { return n * (n + 1) / 2; }

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Reduce NV per-thread values over the workgroup; result in sred[0..NV).
template <int NV>
__device__ inline void block_reduce(double (&v)[NV], double* sred) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double s = wave_sum(v[k]);
    if (lane == 0) sred[wid * NV + k] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    const int k = threadIdx.x;
    sred[k] = sred[k] + sred[NV + k] + sred[2 * NV + k] + sred[3 * NV + k];
  }
  __syncthreads();
}


// Segmented sum over runs of equal key in the wavefront; the run's tail lane
// stores (interior run) or atomically adds (run touching a wave boundary).
template <int NV>
__device__ inline void wave_segmented_store(uint32_t key, bool store, double (&v)[NV], double* dst_base) {
  const int lane = threadIdx.x & 63;
  const uint32_t prev = __shfl_up(key, 1, 64);
  const bool head = (lane == 0) || prev != key;
  const uint64_t heads = __ballot(head);
  const uint64_t upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
  const int head_lane = 63 - __clzll(heads & upto);
  const int idx = lane - head_lane;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const double o = __shfl_up(v[k], off, 64);
      if (idx >= off) v[k] += o;
    }
  }
  const uint32_t next = __shfl_down(key, 1, 64);
  const bool tail = (lane == 63) || next != key;
  if (tail && store) {
    double* dst = dst_base + (size_t)key * NV;
    if (head_lane > 0 && lane < 63) {
#pragma unroll
      for (int k = 0; k < NV; ++k) dst[k] = v[k];
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) atomicAdd(dst + k, v[k]);
    }
  }
}

// ---------------------------------------------------------------------------
// Cost of one block at trial parameters (the LM's candidate evaluation).
// ---------------------------------------------------------------------------
template <int M>
__device__ inline double block_cost(const DevProblem& p, const double* __restrict__ qt_all,
                                    const double* __restrict__ cam_all, const double* __restrict__ X_all,
                                    int64_t i) {
  constexpr int np = Model<M>::kNumParams;
  const double2 o = p.obs_xy[i];
  const uint32_t img = p.obs_img[i];
  const uint32_t pt = p.obs_pt[i];
  const double* qt = qt_all + 8 * (size_t)img;
  const double q[4] = {qt[0], qt[1], qt[2], qt[3]};
  const double t[3] = {qt[4], qt[5], qt[6]};
  const uint32_t cam_idx = p.img_cam[img];
  const double* pc = cam_all + 8 * (size_t)cam_idx;
  double prm[np];
#pragma unroll
  for (int k = 0; k < np; ++k) prm[k] = pc[k];
  const double X[3] = {X_all[3 * (size_t)pt], X_all[3 * (size_t)pt + 1], X_all[3 * (size_t)pt + 2]};
  double P[3];
  unit_quat_rotate(q, X, P);
  P[0] += t[0];
  P[1] += t[1];
  P[2] += t[2];
  const double iz = 1.0 / P[2];
  const double u = P[0] * iz, v = P[1] * iz;
  double x, y;
  if constexpr (M == kMixedModels)
    world_to_image_any(p.cam_model[cam_idx], prm, u, v, &x, &y);
  else
    world_to_image<M>(prm, u, v, &x, &y);
  const double r0 = x - o.x, r1 = y - o.y;
  double rho[3];
  loss_eval(p.loss_type, p.loss_scale, r0 * r0 + r1 * r1, rho);
  return 0.5 * rho[0];
}

// Refined-intrinsics mask per model and refine flags (bit 0 focal, bit 1
// principal point, bit 2 extra params): camera_models.h *Idxs, and
// BundleAdjuster::ParameterizeCameras (bundle_adjustment.cc:480-516).
__host__ __device__ constexpr unsigned cam_tangent_mask(int M, int RF) {
  unsigned f = 0, pp = 0, ex = 0;
  if (M == kSimplePinhole) { f = 0x1; pp = 0x6; ex = 0x0; }
  if (M == kPinhole) { f = 0x3; pp = 0xC; ex = 0x0; }
  if (M == kSimpleRadial) { f = 0x1; pp = 0x6; ex = 0x8; }
  if (M == kRadial) { f = 0x1; pp = 0x6; ex = 0x18; }
  if (M == kOpenCV) { f = 0x3; pp = 0xC; ex = 0xF0; }
  return ((RF & 1) ? f : 0u) | ((RF & 2) ? pp : 0u) | ((RF & 4) ? ex : 0u);
}
__host__ __device__ constexpr int popcount8(unsigned m) {
  return (int)((m & 1) + ((m >> 1) & 1) + ((m >> 2) & 1) + ((m >> 3) & 1) + ((m >> 4) & 1) + ((m >> 5) & 1) +
               ((m >> 6) & 1) + ((m >> 7) & 1));
}

// Jacobian entries of one block row (rw = 0: x, 1: y) into dst[0..W).
// Columns: rotation tangent (3), translation (3), point (3), refined
// intrinsics (CT, SubsetManifold PlusJacobian = column selection).
__device__ inline void emit_row_pose_point(int rw, double* dst, const double (&B)[6], const double (&Mq)[9],
                                           bool pose_var, uint32_t flags, const double (&jx)[2][3]) {
#pragma unroll
  for (int b = 0; b < 3; ++b)
    dst[b] = pose_var ? B[rw * 3 + 0] * Mq[b] + B[rw * 3 + 1] * Mq[3 + b] + B[rw * 3 + 2] * Mq[6 + b] : 0.0;
#pragma unroll
  for (int b = 0; b < 3; ++b) dst[3 + b] = (pose_var && !((flags >> (1 + b)) & 1u)) ? B[rw * 3 + b] : 0.0;
#pragma unroll
  for (int b = 0; b < 3; ++b) dst[6 + b] = jx[rw][b];
}

template <int M, unsigned CM>
__device__ inline void emit_row(int rw, double* dst, const double (&B)[6], const double (&Mq)[9], bool pose_var,
                                uint32_t flags, const double (&jx)[2][3], const double* Jp, double sc, bool cv) {
  constexpr int np = Model<M>::kNumParams;
  emit_row_pose_point(rw, dst, B, Mq, pose_var, flags, jx);
  int c = 0;
#pragma unroll
  for (int m = 0; m < np; ++m) {
    if ((CM >> m) & 1u) {
      dst[9 + c] = cv ? Jp[rw * np + m] * sc : 0.0;
      ++c;
    }
  }
}

// Mixed camera models: the camera's refined intrinsics (run-time mask cmask,
// parameter order) fill the first of CT slots, the rest are zero.  Jp8 holds
// d(x,y)/dparams in 8-wide rows.
template <int CT>
__device__ inline void emit_row_mixed(int rw, double* dst, const double (&B)[6], const double (&Mq)[9],
                                      bool pose_var, uint32_t flags, const double (&jx)[2][3], const double* Jp8,
                                      double sc, bool cv, unsigned cmask) {
  emit_row_pose_point(rw, dst, B, Mq, pose_var, flags, jx);
  int c = 0;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    if ((cmask >> m) & 1u) {
      if (c < CT) dst[9 + c] = cv ? Jp8[rw * 8 + m] * sc : 0.0;
      ++c;
    }
  }
  for (; c < CT; ++c) dst[9 + c] = 0.0;
}

// Copy NR rows of R doubles (LDS stride LS) into a global range whose rows
// are G doubles apart, one wavefront, 8 B per lane per step.
template <int R, int LS, int G, bool NT = false>
__device__ inline void wave_readout(const double* __restrict__ src, double* __restrict__ dst, int nrows) {
  const int lane = threadIdx.x & 63;
  const int total = nrows * R;
  int row = lane / R, col = lane - (lane / R) * R;
  constexpr int dr = 64 / R, dc = 64 % R;
#pragma unroll 4
  for (int e = lane; e < total; e += 64) {
    if constexpr (NT)
      __builtin_nontemporal_store(src[row * LS + col], dst + row * G + col);
    else
      dst[row * G + col] = src[row * LS + col];
    row += dr;
    col += dc;
    if (col >= R) { col -= R; ++row; }
  }
}

// As wave_readout, 16 B per lane: R (even) doubles per row, LDS row stride
// LS (even), so no pair straddles a row.
template <int R, int LS, int G, bool NT = false>
__device__ inline void wave_readout16(const double* __restrict__ src, double* __restrict__ dst, int nrows) {
  constexpr int R2 = R / 2;
  const int lane = threadIdx.x & 63;
  const int total = nrows * R2;
  int row = lane / R2, col = lane - (lane / R2) * R2;
  constexpr int dr = 64 / R2, dc = 64 % R2;
#pragma unroll 4
  for (int e = lane; e < total; e += 64) {
    const dvec2 v = *reinterpret_cast<const dvec2*>(src + row * LS + 2 * col);
    dvec2* d = reinterpret_cast<dvec2*>(dst + row * G + 2 * col);
    if constexpr (NT)
      __builtin_nontemporal_store(v, d);
    else
      *d = v;
    row += dr;
    col += dc;
    if (col >= R2) { col -= R2; ++row; }
  }
}

// Coalesced copy of nrows contiguous rows of R doubles from global memory
// into a wave-private LDS slab with row stride LS (mirror of wave_readout).
template <int R, int LS>
__device__ inline void wave_load_rows(const double* __restrict__ src, double* __restrict__ dst, int nrows) {
  const int lane = threadIdx.x & 63;
  const int total = nrows * R;
  int row = lane / R, col = lane - (lane / R) * R;
  constexpr int dr = 64 / R, dc = 64 % R;
#pragma unroll 4
  for (int e = lane; e < total; e += 64) {
    dst[row * LS + col] = __builtin_nontemporal_load(src + e);
    row += dr;
    col += dc;
    if (col >= R) { col -= R; ++row; }
  }
}

// As wave_load_rows for at most NR rows, fully unrolled: every load of the
// wave is issued before the first LDS write waits on one (the looped form
// kept ~4 loads in flight per wave, too few to cover HBM latency at the
// occupancy the slabs allow).
template <int R, int LS, int NR>
__device__ inline void wave_load_rows_u(const double* __restrict__ src, double* __restrict__ dst, int nrows) {
  constexpr int T = (NR * R + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int total = nrows * R;
  double v[T];
#pragma unroll
  for (int i = 0; i < T; ++i) {
    const int e = lane + 64 * i;
    v[i] = e < total ? __builtin_nontemporal_load(src + e) : 0.0;
  }
#pragma unroll
  for (int i = 0; i < T; ++i) {
    const int e = lane + 64 * i;
    if (e < total) {
      const int row = e / R;
      dst[row * LS + (e - row * R)] = v[i];
    }
  }
}

// As wave_load_rows_u for the rows idx[0..nrows) of src (idx: the wave's 64
// row indices, one per lane; a lane's element finds its row's index by
// ds_bpermute).
template <int R, int LS, int NR>
__device__ inline void wave_gather_rows_u(const double* __restrict__ src, uint32_t idx, double* __restrict__ dst,
                                          int nrows) {
  constexpr int T = (NR * R + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int total = nrows * R;
  double v[T];
#pragma unroll
  for (int i = 0; i < T; ++i) {
    const int e = lane + 64 * i;
    const int row = e / R;
    const uint32_t r = (uint32_t)__builtin_amdgcn_ds_bpermute((row & 63) << 2, (int)idx);
    v[i] = e < total ? __builtin_nontemporal_load(src + (size_t)r * R + (e - row * R)) : 0.0;
  }
#pragma unroll
  for (int i = 0; i < T; ++i) {
    const int e = lane + 64 * i;
    if (e < total) {
      const int row = e / R;
      dst[row * LS + (e - row * R)] = v[i];
    }
  }
}

// One lane per reduced block, one wavefront per 64 consecutive blocks; the
// kernel writes residuals, tangent Jacobian rows and a per-workgroup cost
// partial, nothing else (the point/camera normal-equation blocks are reduced
// by the solver's own passes over J, as Ceres' SchurEliminator does after
// its Jacobian evaluation).
//
// Jacobian rows are 2W doubles per block.  A lane's row is not a coalesced
// store shape, so rows go through a wave-private LDS slab and leave as
// 8-B-per-lane stores over contiguous memory (512 B per wave-instruction).
// The slab holds 64/NP rows and is filled in NP passes: NP = 2 keeps the
// LDS at 7.9 KB per wave so 5 workgroups (20 waves) share a CU, enough for
// one wave's f64 arithmetic to hide another's store issue (the kernel sits
// on the HBM write roof: DESIGN.md §4).  LOSS = 0 compiles the TrivialLoss
// path without the Corrector.  D: diagnostic builds for the roofline
// decomposition (1 = no J store, 2 = no arithmetic); never used by the LM.
// Build options (bits of D): 8 nontemporal J stores, 16 nontemporal obs
// loads and r stores, 32 16-B J stores, 128 per-block loads issued up front;
// 1 and 2 are the diagnostic builds; 512 closed-form rotation columns, 1024
// R X through the rotation matrix.
// (8192, the packed ids, is a tools-build variant: 0.496 vs 0.460 ms in the
// bench step on one box, profiles/r5ae_bench_packed_ids_vs_r4.jsonl)
constexpr int kJacProduction = 8 | 16 | 32 | 128 | 512 | 1024;  // 0.583 -> 0.543 ms at C4 with 512 | 1024
// J rows staged in one slab pass (64 rows, 17 KB of LDS per wave at OPENCV: 2
// waves per SIMD, each store burst 15 KB): 0.554 (2 passes) -> 0.454 ms at C4
// once the arithmetic was cut by the closed-form rotation columns
constexpr int kJacPasses = 1;
[[maybe_unused]] constexpr int kJacR1 = 8 | 16 | 32;  // round-1 production (three serial round trips), A/B variant 23
// TB: threads per workgroup.  The cost partial is per wave (no workgroup
// barrier), cost_partial[i / 64].
// CTX: the camera-slot width of a mixed-model build (M == kMixedModels, RF
// then unused: the refine flags are applied per camera at run time).
template <int M, int RF, int LOSS, int NP, int D = kJacProduction, int WPE = 4, int TB = kBlock, int CTX = 0>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(WPE))) void reproj_jacobian_kernel(DevProblem p, double2* __restrict__ r_out,
                                                                 double* __restrict__ J_out,
                                                                 double* __restrict__ cost_partial) {
  constexpr int np = Model<M>::kNumParams;
  constexpr unsigned CM = cam_tangent_mask(M, RF);
  constexpr int CT = M == kMixedModels ? CTX : popcount8(CM);
  constexpr int W = 9 + CT;
  constexpr int W2 = 2 * W;
  unsigned cmask = 0;  // mixed models: the lane's camera's refined-intrinsics mask
  // odd row stride: conflict-free row writes; D & 32 (16-B readout) needs an
  // even stride: W2 + 4 gives 2-way conflicts on the row writes
  constexpr int LS = (D & 32) ? W2 + 4 : (W2 | 1);
  constexpr int RP = 64 / NP;
  // LDS stride of an image record: 144 B (the first 128 B: conflict-free
  // ds_read_b128), 272 B with the per-image rotation matrix (D & 2048)
  constexpr int RS = (D & 2048) ? 34 : 18;
  // D & 64: image records fetched per lane (no LDS staging), slab = J rows only
  constexpr int SLAB = ((D & 64) || RP * LS > 64 * RS) ? RP * LS : 64 * RS;
  __shared__ double sJ[(TB / 64) * SLAB];
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * TB + threadIdx.x;
  const int64_t wb0 = i - lane;  // first block of this wavefront
  double* slab = sJ + (threadIdx.x >> 6) * SLAB;
  double cost = 0.0;
  double B[6] = {0, 0, 0, 0, 0, 0}, Mq[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, jx[2][3] = {{0, 0, 0}, {0, 0, 0}};
  double Jp[2 * np];
#pragma unroll
  for (int k = 0; k < 2 * np; ++k) Jp[k] = 0.0;
  double sc = 1.0;
  bool cv = false, pose_var = false;
  uint32_t flags = 0;
  if ((D & 2) && i < p.nb) {
    const double2 o = p.obs_xy[i];
    B[0] = o.x; B[1] = o.y; B[2] = o.x + o.y; B[3] = o.x - o.y; B[4] = o.x * 2.0; B[5] = o.y * 2.0;
    pose_var = true;
    cv = true;
    r_out[i] = o;
  } else if constexpr (!(D & 2)) {
    // Image records (pose, camera, flags; 128 B each) of the wave's 64 blocks:
    // consecutive blocks belong to different images (point-major order), so a
    // per-lane fetch would touch 64 lines per instruction.  Instead 8 lanes
    // fetch one record with 16-B loads (8 whole lines per instruction) and the
    // records are handed out through the wave's LDS slab.
    const bool live = i < p.nb;
    uint32_t img = 0u;
    // D & 128: every per-block input is requested up front (image, point,
    // observation), the point gathers as soon as the point index lands, so
    // they overlap the image-record fetch: two dependent memory round trips
    // before the arithmetic instead of three.
    uint32_t pt_e = 0u;
    double2 o_e = make_double2(0.0, 0.0);
    double X_e[3] = {0.0, 0.0, 0.0};
    bool ptv_e = false;
    bool packed = false;
    if constexpr ((D & 8192) != 0) {
      // packed ids (device.h obs_ids): image and the point's offset from the
      // wave's first point in one 4-B read
      packed = p.obs_ids != nullptr;
      if (packed) {
        const uint32_t w0 = wb0 < p.nb ? p.wave_pt0[__builtin_amdgcn_readfirstlane((int)(wb0 >> 6))] : 0u;
        if (live) {
          const uint32_t v = __builtin_nontemporal_load(p.obs_ids + i);
          img = v & 0xffffu;
          pt_e = w0 + (v >> 16);
        }
      }
    }
    if (!packed && live) img = (D & 16) ? __builtin_nontemporal_load(p.obs_img + i) : p.obs_img[i];
    if constexpr ((D & 128) != 0) {
      if (live) {
        if (!packed) pt_e = __builtin_nontemporal_load(p.obs_pt + i);
        const dvec2 ov = __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(p.obs_xy) + i);
        o_e = make_double2(ov.x, ov.y);
        X_e[0] = p.X[3 * (size_t)pt_e];
        X_e[1] = p.X[3 * (size_t)pt_e + 1];
        X_e[2] = p.X[3 * (size_t)pt_e + 2];
        ptv_e = p.pt_var[pt_e] != 0;
      }
    }
    if constexpr ((D & 4) != 0) img &= 127u;  // diagnostic: L1-resident record working set
    double q[4], t[3], prm[np];
    double Rrec[9];  // D & 2048: the image record's rotation matrix
    bool unit_rec = false;
    uint32_t meta;
    if constexpr ((D & 64) != 0) {
      // per-lane record fetch: 16-B loads of the lane's own 128-B line (L1/L2
      // resident, 1000 images = 128 KB), no LDS and no wave barrier
      const double2* rv = reinterpret_cast<const double2*>(p.img_rec + kImgRec * (size_t)img);
      const double2 a0 = rv[0], a1 = rv[1], a2 = rv[2], a3 = rv[3];
      q[0] = a0.x; q[1] = a0.y; q[2] = a1.x; q[3] = a1.y;
      t[0] = a2.x; t[1] = a2.y; t[2] = a3.x;
      meta = (uint32_t)__double_as_longlong(a3.y);
#pragma unroll
      for (int k = 0; k < (np + 1) / 2; ++k) {
        const double2 c = rv[4 + k];
        prm[2 * k] = c.x;
        if (2 * k + 1 < np) prm[2 * k + 1] = c.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int src = 8 * j + (lane >> 3);
        const uint32_t is = __shfl(img, src, 64);
        const double2* rv = reinterpret_cast<const double2*>(p.img_rec + kImgRec * (size_t)is);
        const double2 v = rv[lane & 7];
        reinterpret_cast<double2*>(slab + src * RS)[lane & 7] = v;
        if constexpr ((D & 2048) != 0) {
          if ((lane & 7) < 5) reinterpret_cast<double2*>(slab + src * RS)[8 + (lane & 7)] = rv[8 + (lane & 7)];
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      const double* rec = slab + lane * RS;
      q[0] = rec[0]; q[1] = rec[1]; q[2] = rec[2]; q[3] = rec[3];
      t[0] = rec[4]; t[1] = rec[5]; t[2] = rec[6];
      meta = (uint32_t)__double_as_longlong(rec[7]);
#pragma unroll
      for (int k = 0; k < np; ++k) prm[k] = rec[8 + k];
      if constexpr ((D & 2048) != 0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) Rrec[k] = rec[16 + k];
        unit_rec = rec[25] != 0.0;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    if (live) {
      double2 o;
      uint32_t pt;
      bool ptv;
      double X[3];
      if constexpr ((D & 128) != 0) {
        o = o_e;
        pt = pt_e;
        ptv = ptv_e;
        X[0] = X_e[0]; X[1] = X_e[1]; X[2] = X_e[2];
      } else {
        if constexpr ((D & 16) != 0) {
          const dvec2 ov = __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(p.obs_xy) + i);
          o = make_double2(ov.x, ov.y);
        } else {
          o = p.obs_xy[i];
        }
        pt = (D & 16) ? __builtin_nontemporal_load(p.obs_pt + i) : p.obs_pt[i];
        ptv = p.pt_var[pt] != 0;
        X[0] = p.X[3 * (size_t)pt]; X[1] = p.X[3 * (size_t)pt + 1]; X[2] = p.X[3 * (size_t)pt + 2];
      }
      (void)pt;
      flags = meta & 0xffu;
      pose_var = flags & 1u;
      cv = (meta >> 8) & 1u;
      double P[3];
      double Rm[9];
      if constexpr ((D & 2048) != 0) {
        // R X from the record's rotation matrix (computed once per image)
#pragma unroll
        for (int c = 0; c < 9; ++c) Rm[c] = Rrec[c];
#pragma unroll
        for (int c = 0; c < 3; ++c) P[c] = Rm[3 * c] * X[0] + Rm[3 * c + 1] * X[1] + Rm[3 * c + 2] * X[2];
      } else if constexpr ((D & 1024) != 0) {
        // R X from the rotation matrix the point columns need anyway
        unit_quat_matrix(q, Rm);
#pragma unroll
        for (int c = 0; c < 3; ++c) P[c] = Rm[3 * c] * X[0] + Rm[3 * c + 1] * X[1] + Rm[3 * c + 2] * X[2];
      } else {
        unit_quat_rotate(q, X, P);
      }
      const double a0 = P[0], a1 = P[1], a2 = P[2];  // R X
      P[0] += t[0];
      P[1] += t[1];
      P[2] += t[2];
      const double iz = 1.0 / P[2];
      const double u = P[0] * iz, v = P[1] * iz;
      double x, y, A[4];
      if constexpr (M == kMixedModels) {
        const int model = (int)((meta >> 16) & 0xffu);
        world_to_image_jac_any(model, prm, u, v, &x, &y, A, Jp);
        cmask = cam_tangent_mask(model, p.refine_mask);
      } else {
        world_to_image_jac<M>(prm, u, v, &x, &y, A, Jp);
      }
      const double r0 = x - o.x, r1 = y - o.y;
      if constexpr (LOSS == 0) {
        cost = 0.5 * (r0 * r0 + r1 * r1);
      } else {
        double rho[3];
        loss_eval(p.loss_type, p.loss_scale, r0 * r0 + r1 * r1, rho);
        cost = 0.5 * rho[0];
        // Ceres Corrector, rho'' <= 0 branch (Trivial/SoftL1/Cauchy): r, J *= sqrt(rho')
        sc = sqrt(rho[1]);
      }
      // B = d(x,y)/dP (2x3) = A * d(u,v)/dP, loss-scaled
      B[0] = A[0] * iz; B[1] = A[1] * iz; B[2] = -(A[0] * u + A[1] * v) * iz;
      B[3] = A[2] * iz; B[4] = A[3] * iz; B[5] = -(A[2] * u + A[3] * v) * iz;
      if constexpr (LOSS != 0) {
  #pragma unroll
        for (int k = 0; k < 6; ++k) B[k] *= sc;
      }
      // d(R X)/d(tangent) of QuaternionManifold (plus = q_delta * q, rotation
      // angle 2|delta|) = -2 [R X]x: the product Dq * PlusJacobian below in
      // closed form, equal up to rounding for a unit q (the general product
      // serves a quaternion that is not normalised, as AutoDiff would)
      const bool unit_q =
          (D & 512) && ((D & 4096) || ((D & 2048) ? unit_rec
                                                  : fabs(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3] - 1.0) <= 1e-12));
      if (pose_var && unit_q) {
        Mq[0] = 0.0;       Mq[1] = 2.0 * a2;  Mq[2] = -2.0 * a1;
        Mq[3] = -2.0 * a2; Mq[4] = 0.0;       Mq[5] = 2.0 * a0;
        Mq[6] = 2.0 * a1;  Mq[7] = -2.0 * a0; Mq[8] = 0.0;
      } else if (pose_var) {
        double Dq[12], PJ[12];
        unit_quat_rotate_dq(q, X, Dq);
        quat_plus_jacobian(q, PJ);
  #pragma unroll
        for (int a = 0; a < 3; ++a)
  #pragma unroll
          for (int b = 0; b < 3; ++b)
            Mq[a * 3 + b] = Dq[a * 4 + 0] * PJ[0 * 3 + b] + Dq[a * 4 + 1] * PJ[1 * 3 + b] +
                            Dq[a * 4 + 2] * PJ[2 * 3 + b] + Dq[a * 4 + 3] * PJ[3 * 3 + b];
      }
      if (ptv) {
        double R[9];
        if constexpr ((D & (1024 | 2048)) != 0) {
#pragma unroll
          for (int c = 0; c < 9; ++c) R[c] = Rm[c];
        } else {
          unit_quat_matrix(q, R);
        }
  #pragma unroll
        for (int rw = 0; rw < 2; ++rw)
  #pragma unroll
          for (int b = 0; b < 3; ++b)
            jx[rw][b] = B[rw * 3 + 0] * R[b] + B[rw * 3 + 1] * R[3 + b] + B[rw * 3 + 2] * R[6 + b];
      }
      if constexpr ((D & 16) != 0)
        __builtin_nontemporal_store(dvec2{r0 * sc, r1 * sc}, reinterpret_cast<dvec2*>(r_out) + i);
      else
        r_out[i] = make_double2(r0 * sc, r1 * sc);
    }
  }
  if constexpr (!(D & 1)) {
    const int live = wb0 >= p.nb ? 0 : (p.nb - wb0 < 64 ? (int)(p.nb - wb0) : 64);
#pragma unroll
    for (int h = 0; h < NP; ++h) {
      if (lane / RP == h && i < p.nb) {
        double* row = slab + (lane % RP) * LS;
        if constexpr (M == kMixedModels) {
          emit_row_mixed<CT>(0, row, B, Mq, pose_var, flags, jx, Jp, sc, cv, cmask);
          emit_row_mixed<CT>(1, row + W, B, Mq, pose_var, flags, jx, Jp, sc, cv, cmask);
        } else {
          emit_row<M, CM>(0, row, B, Mq, pose_var, flags, jx, Jp, sc, cv);
          emit_row<M, CM>(1, row + W, B, Mq, pose_var, flags, jx, Jp, sc, cv);
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      const int rows = live - h * RP < 0 ? 0 : (live - h * RP > RP ? RP : live - h * RP);
      // D & 256: the store bursts issue at raised priority (the arithmetic of
      // the SIMD's other waves fills around them)
      if constexpr ((D & 256) != 0) __builtin_amdgcn_s_setprio(2);
      if constexpr ((D & 32) != 0)
        wave_readout16<W2, LS, W2, (D & 8) != 0>(slab, J_out + (wb0 + h * RP) * W2, rows);
      else
        wave_readout<W2, LS, W2, (D & 8) != 0>(slab, J_out + (wb0 + h * RP) * W2, rows);
      if constexpr ((D & 256) != 0) __builtin_amdgcn_s_setprio(0);
      if (h + 1 < NP) {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      }
    }
  }
  const double s = wave_sum(cost);
  if (lane == 0 && wb0 < p.nb) cost_partial[wb0 >> 6] = s;
}

// Image records img_rec[I][kImgRec] = q(4) t(3) meta camera-params(8)
// R(9) unit-q(1) pad, meta = img_flags | cam_var << 8 | model << 16 (bit
// pattern in a double slot), R = the rotation matrix of q and unit-q = 1.0
// when |q|^2 is 1 within 1e-12 (the Jacobian kernels' closed-form test) —
// both per image instead of per block: two 128-B lines per image, rebuilt
// whenever poses or intrinsics change.
// zero[0..nzero) is cleared too (the step's scalar slots: one launch fewer
// than a separate memset ahead of it).
__global__ void pack_images_kernel(DevProblem p, double* __restrict__ rec, double* __restrict__ zero, int nzero) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nzero) zero[k] = 0.0;
  if (k >= p.num_images) return;
  const uint32_t cam = p.img_cam[k];
  double* o = rec + kImgRec * (size_t)k;
#pragma unroll
  for (int m = 0; m < 7; ++m) o[m] = p.qt[8 * (size_t)k + m];
  o[7] = __longlong_as_double(
      (long long)(p.img_flags[k] | ((p.cam_var[cam] != 0 ? 1u : 0u) << 8) | ((uint32_t)p.cam_model[cam] << 16)));
#pragma unroll
  for (int m = 0; m < 8; ++m) o[8 + m] = p.cam[8 * (size_t)cam + m];
  const double q[4] = {o[0], o[1], o[2], o[3]};
  double R[9];
  unit_quat_matrix(q, R);
#pragma unroll
  for (int m = 0; m < 9; ++m) o[16 + m] = R[m];
  o[25] = fabs(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3] - 1.0) <= 1e-12 ? 1.0 : 0.0;
#pragma unroll
  for (int m = 26; m < kImgRec; ++m) o[m] = 0.0;
}

template <int M>
__global__ __launch_bounds__(kBlock) void reproj_cost_kernel(DevProblem p, const double* __restrict__ qt,
                                                              const double* __restrict__ cam,
                                                              const double* __restrict__ X,
                                                              double* __restrict__ cost_partial) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double cost = 0.0;
  if (i < p.nb) cost = block_cost<M>(p, qt, cam, X, i);
  const double s = wave_sum(cost);  // per-wave partial (reproj_grid)
  if ((threadIdx.x & 63) == 0 && i < p.nb) cost_partial[i >> 6] = s;
}

// One workgroup; each thread sums its strided share with kSumIlp loads in
// flight (a serial load-add chain ran 40 us over the 156k partials of C4's
// reprojection pass).  The order is fixed: results are deterministic.
constexpr int kSumIlp = 16;
__global__ __launch_bounds__(1024) void sum_kernel(const double* __restrict__ partial, int64_t n,
                                                   double* __restrict__ out) {
  __shared__ double sred[16];
  double v = 0.0;
  int64_t k = threadIdx.x;
  for (; k + (kSumIlp - 1) * 1024 < n; k += kSumIlp * 1024) {
    double x[kSumIlp];
#pragma unroll
    for (int u = 0; u < kSumIlp; ++u) x[u] = partial[k + u * 1024];
#pragma unroll
    for (int u = 0; u < kSumIlp; ++u) v += x[u];
  }
  for (; k < n; k += 1024) v += partial[k];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int k = 0; k < 16; ++k) s += sred[k];
    out[0] = s;
  }
}

// Many-workgroup variant for long partial lists (one workgroup is bound by
// one CU's load bandwidth: 21 us over C4's 156k partials): workgroup g sums
// the contiguous range g of the list, thread 0 parks the workgroup's sum in
// stage[g] and takes a ticket; the last workgroup sums stage[0..G) in order
// and resets the ticket.  Deterministic (fixed ranges, fixed orders).
constexpr int kSumGroups = 64;
__global__ __launch_bounds__(256) void sum_multi_kernel(const double* __restrict__ partial, int64_t n,
                                                        double* __restrict__ out, double* __restrict__ stage,
                                                        unsigned* __restrict__ ticket) {
  __shared__ double sred[4];
  __shared__ bool last;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(n, b0 + per);
  double v = 0.0;
  int64_t k = b0 + threadIdx.x;
  for (; k + 3 * 256 < b1; k += 4 * 256) {
    const double x0 = partial[k], x1 = partial[k + 256], x2 = partial[k + 512], x3 = partial[k + 768];
    v += x0;
    v += x1;
    v += x2;
    v += x3;
  }
  for (; k < b1; k += 256) v += partial[k];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    stage[blockIdx.x] = ((sred[0] + sred[1]) + sred[2]) + sred[3];
    __threadfence();
    last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  double w = threadIdx.x < gridDim.x ? __hip_atomic_load(stage + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : 0.0;
  w = wave_sum(w);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = ((sred[0] + sred[1]) + sred[2]) + sred[3];
    *ticket = 0u;
  }
}

// Two partial lists in one launch: workgroups 0..kSumGroups-1 sum list 1,
// the next kSumGroups2 list 2, each set as sum_multi_kernel does (its own
// stage slots and ticket in the scratch).  Deterministic.
constexpr int kSumGroups2 = 16;
__device__ inline void group_sum(const double* __restrict__ p, int64_t n, double* __restrict__ out,
                                 double* __restrict__ stage, unsigned* __restrict__ ticket, int G, int g,
                                 double* sred, bool* last) {
  const int64_t per = (n + G - 1) / G;
  const int64_t b0 = (int64_t)g * per, b1 = min(n, b0 + per);
  double v = 0.0;
  int64_t k = b0 + threadIdx.x;
  for (; k + 3 * 256 < b1; k += 4 * 256) {
    const double x0 = p[k], x1 = p[k + 256], x2 = p[k + 512], x3 = p[k + 768];
    v += x0;
    v += x1;
    v += x2;
    v += x3;
  }
  for (; k < b1; k += 256) v += p[k];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    stage[g] = ((sred[0] + sred[1]) + sred[2]) + sred[3];
    __threadfence();
    *last = atomicAdd(ticket, 1u) == (unsigned)G - 1;
  }
  __syncthreads();
  if (!*last) return;
  __threadfence();
  double w = (int)threadIdx.x < G ? __hip_atomic_load(stage + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : 0.0;
  w = wave_sum(w);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = ((sred[0] + sred[1]) + sred[2]) + sred[3];
    *ticket = 0u;
  }
}

__global__ __launch_bounds__(256) void sum2_kernel(const double* __restrict__ p1, int64_t n1, double* __restrict__ out1,
                                                   double* __restrict__ scratch, const double* __restrict__ p2,
                                                   int64_t n2, double* __restrict__ out2) {
  __shared__ double sred[4];
  __shared__ bool last;
  if (blockIdx.x < kSumGroups)
    group_sum(p1, n1, out1, scratch, reinterpret_cast<unsigned*>(scratch + kSumGroups), kSumGroups, blockIdx.x, sred,
              &last);
  else
    group_sum(p2, n2, out2, scratch + kSumGroups + 1,
              reinterpret_cast<unsigned*>(scratch + kSumGroups + 1 + kSumGroups2), kSumGroups2,
              blockIdx.x - kSumGroups, sred, &last);
}

// ---------------------------------------------------------------------------
// Point side
// ---------------------------------------------------------------------------
__device__ inline void sym3_inverse(const double a[6], double inv[6]) {
  // a = [xx xy xz yy yz zz]
  const double c00 = a[3] * a[5] - a[4] * a[4];
  const double c01 = a[2] * a[4] - a[1] * a[5];
  const double c02 = a[1] * a[4] - a[2] * a[3];
  const double det = a[0] * c00 + a[1] * c01 + a[2] * c02;
  const double id = 1.0 / det;
  inv[0] = c00 * id;
  inv[1] = c01 * id;
  inv[2] = c02 * id;
  inv[3] = (a[0] * a[5] - a[2] * a[2]) * id;
  inv[4] = (a[1] * a[2] - a[0] * a[4]) * id;
  inv[5] = (a[0] * a[3] - a[1] * a[1]) * id;
}

__device__ inline void sym3_mul(const double s[6], const double x[3], double y[3]) {
  y[0] = s[0] * x[0] + s[1] * x[1] + s[2] * x[2];
  y[1] = s[1] * x[0] + s[3] * x[1] + s[4] * x[2];
  y[2] = s[2] * x[0] + s[4] * x[1] + s[5] * x[2];
}

// Point blocks V_p = sum J_p'J_p (6, packed upper) and g_p = sum J_p'r (3)
// of every variable point from its contiguous (point-major) blocks.
template <int CT>
__global__ __launch_bounds__(kBlock) void point_normal_kernel(const DevPoint* __restrict__ vp, int64_t npv,
                                                               const double2* __restrict__ rr,
                                                               const double* __restrict__ J,
                                                               double* __restrict__ Vg) {
  constexpr int W = 9 + CT;
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= npv) return;
  const DevPoint d = vp[k];
  double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t n = 0; n < d.count; ++n) {
    const size_t b = d.start + n;
    const double* Jb = J + b * 2 * W;
    const double2 r = rr[b];
    const double a0 = Jb[6], a1 = Jb[7], a2 = Jb[8];
    const double c0 = Jb[W + 6], c1 = Jb[W + 7], c2 = Jb[W + 8];
    v[0] += a0 * a0 + c0 * c0;
    v[1] += a0 * a1 + c0 * c1;
    v[2] += a0 * a2 + c0 * c2;
    v[3] += a1 * a1 + c1 * c1;
    v[4] += a1 * a2 + c1 * c2;
    v[5] += a2 * a2 + c2 * c2;
    v[6] += a0 * r.x + c0 * r.y;
    v[7] += a1 * r.x + c1 * r.y;
    v[8] += a2 * r.x + c2 * r.y;
  }
  double* out = Vg + 9 * (size_t)d.point;
#pragma unroll
  for (int m = 0; m < 9; ++m) out[m] = v[m];
}

// point_normal_kernel on the point chunks: one lane per block (its J_p
// rows and r, no serial walk per lane), then the first lane of each
// variable point sums its blocks' terms in lane order (the per-point loop's
// order; a point of more than 64 blocks sums per 64-block pass).
template <int CT>
__global__ __launch_bounds__(kBlock) void point_normal_chunk_kernel(DevProblem p, const uint32_t* __restrict__ chunk,
                                                                     int nchunks, const double2* __restrict__ rr,
                                                                     const double* __restrict__ J,
                                                                     double* __restrict__ Vg) {
  constexpr int W = 9 + CT;
  __shared__ double sv[kBlock / 64][64 * 9];
  __shared__ uint32_t spt[kBlock / 64][64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* tvs = sv[wv];
  uint32_t* wpt = spt[wv];
  const int c = blockIdx.x * (kBlock / 64) + wv;
  if (c >= nchunks) return;  // wave-uniform
  const uint32_t b0 = chunk[c], b1 = chunk[c + 1];
  const bool multi = b1 - b0 > 64u;  // one point with more than 64 blocks
  double carry[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t carry_pt = 0;
  bool carry_var = false;
  for (uint32_t s0 = b0; s0 < b1; s0 += 64) {
    const int live = (int)min(64u, b1 - s0);
    const bool on = lane < live;
    const uint32_t b = s0 + (on ? lane : 0);
    const uint32_t pt = p.obs_pt[b];
    const bool var = on && p.pt_var[pt] != 0;
    double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (var) {
      const double* Jb = J + (size_t)b * 2 * W;
      const double2 r = rr[b];
      const double a0 = Jb[6], a1 = Jb[7], a2 = Jb[8];
      const double c0 = Jb[W + 6], c1 = Jb[W + 7], c2 = Jb[W + 8];
      v[0] = a0 * a0 + c0 * c0;
      v[1] = a0 * a1 + c0 * c1;
      v[2] = a0 * a2 + c0 * c2;
      v[3] = a1 * a1 + c1 * c1;
      v[4] = a1 * a2 + c1 * c2;
      v[5] = a2 * a2 + c2 * c2;
      v[6] = a0 * r.x + c0 * r.y;
      v[7] = a1 * r.x + c1 * r.y;
      v[8] = a2 * r.x + c2 * r.y;
    }
#pragma unroll
    for (int m = 0; m < 9; ++m) tvs[lane * 9 + m] = v[m];
    wpt[lane] = on ? pt : 0xffffffffu;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const bool head = var && (lane == 0 || wpt[lane - 1] != pt);
    if (head) {
      for (int l = lane + 1; l < live && wpt[l] == pt; ++l)
#pragma unroll
        for (int m = 0; m < 9; ++m) v[m] += tvs[l * 9 + m];
      if (multi) {
#pragma unroll
        for (int m = 0; m < 9; ++m) carry[m] += v[m];
        carry_pt = pt;
        carry_var = true;
      } else {
        double* out = Vg + 9 * (size_t)pt;
#pragma unroll
        for (int m = 0; m < 9; ++m) out[m] = v[m];
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  if (multi && carry_var) {  // lane 0
    double* out = Vg + 9 * (size_t)carry_pt;
#pragma unroll
    for (int m = 0; m < 9; ++m) out[m] = carry[m];
  }
}

__global__ __launch_bounds__(kBlock) void point_prepare_kernel(const DevPoint* __restrict__ vp, int64_t npv,
                                                                const double* __restrict__ Vg,
                                                                double* __restrict__ scale_p,
                                                                double* __restrict__ diag_p,
                                                                double* __restrict__ Vinv,
                                                                double* __restrict__ Linv,
                                                                double* __restrict__ q, int first,
                                                                int reuse_diag, double radius) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= npv) return;
  const uint32_t pt = vp[k].point;
  const double* g = Vg + 9 * (size_t)pt;
  double V[6] = {g[0], g[1], g[2], g[3], g[4], g[5]};
  const double dg[3] = {V[0], V[3], V[5]};
  const int di[3] = {0, 3, 5};
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    double s;
    if (first) {
      s = 1.0 / (1.0 + sqrt(dg[m]));
      scale_p[3 * (size_t)pt + m] = s;
    } else {
      s = scale_p[3 * (size_t)pt + m];
    }
    double d;
    if (!reuse_diag) {
      d = fmin(fmax(s * s * dg[m], 1e-6), 1e32);
      diag_p[3 * (size_t)pt + m] = d;
    } else {
      d = diag_p[3 * (size_t)pt + m];
    }
    V[di[m]] += d / (radius * s * s);
  }
  double inv[6];
  sym3_inverse(V, inv);
#pragma unroll
  for (int m = 0; m < 6; ++m) Vinv[6 * (size_t)pt + m] = inv[m];
  if (q) {
    // q_p = V_p^-1 g_p: the point term of the reduced rhs (fblock_dense_kernel)
    double o[3];
    sym3_mul(inv, g + 6, o);
#pragma unroll
    for (int m = 0; m < 3; ++m) q[3 * (size_t)pt + m] = o[m];
  }
  if (Linv) {
    // inverse Cholesky factor of the damped block: V^-1 = Linv' Linv, so the
    // Schur term W V^-1 W' = Z Z' with Z = W Linv' (schur_z_kernel)
    const double l00 = sqrt(V[0]);
    const double l10 = V[1] / l00, l20 = V[2] / l00;
    const double l11 = sqrt(V[3] - l10 * l10);
    const double l21 = (V[4] - l20 * l10) / l11;
    const double l22 = sqrt(V[5] - l20 * l20 - l21 * l21);
    const double i00 = 1.0 / l00, i11 = 1.0 / l11, i22 = 1.0 / l22;
    const double i10 = -l10 * i00 * i11;
    const double i21 = -l21 * i11 * i22;
    const double i20 = -(l20 * i00 + l21 * i10) * i22;
    double* o = Linv + 6 * (size_t)pt;  // packed lower, row-major
    o[0] = i00; o[1] = i10; o[2] = i11; o[3] = i20; o[4] = i21; o[5] = i22;
  }
}

// ---------------------------------------------------------------------------
// Camera side: tile pass building the Schur-Jacobi diagonal blocks and rhs.
// ---------------------------------------------------------------------------
#ifdef MI_BA_AB_VARIANTS  // one lane per block: fblock_variant 2 (tools build)
template <int CT>
__global__ __launch_bounds__(kBlock) void fblock_kernel(DevProblem p, const DevTile* __restrict__ tiles,
                                                         const uint32_t* __restrict__ cm_perm,
                                                         const double2* __restrict__ rr,
                                                         const double* __restrict__ J,
                                                         const double* __restrict__ Jcm,
                                                         const double* __restrict__ Vg,
                                                         const double* __restrict__ Vinv,
                                                         double* __restrict__ pose_blk,
                                                         double* __restrict__ cam_blk,
                                                         double* __restrict__ bvec,
                                                         double* __restrict__ udiag) {
  constexpr int NC = sym_size(CT);
  constexpr int NV = kSymPose + 6 + 6 + NC + 2 * CT;
  __shared__ double sred[4 * NV];
  const DevTile tile = tiles[blockIdx.x];
  const int W = 9 + CT;
  double acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.0;
  for (uint32_t k = threadIdx.x; k < tile.count; k += kBlock) {
    const uint32_t b = cm_perm[tile.start + k];
    const double* Jb = Jcm ? Jcm + (size_t)(tile.start + k) * 2 * W : J + (size_t)b * 2 * W;
    const double2 r = rr[b];
    double jf[2][6 + CT], jx[2][3];
#pragma unroll
    for (int row = 0; row < 2; ++row) {
#pragma unroll
      for (int m = 0; m < 6; ++m) jf[row][m] = Jb[row * W + m];
#pragma unroll
      for (int m = 0; m < 3; ++m) jx[row][m] = Jb[row * W + 6 + m];
#pragma unroll
      for (int m = 0; m < CT; ++m) jf[row][6 + m] = Jb[row * W + 9 + m];
    }
    const double rv[2] = {r.x, r.y};
    // g, U (diag blocks) contributions
    double g[6 + CT];
#pragma unroll
    for (int m = 0; m < 6 + CT; ++m) g[m] = jf[0][m] * rv[0] + jf[1][m] * rv[1];
    const uint32_t pt = p.obs_pt[b];
    double Y[6 + CT][3];
    double Yg[6 + CT];
    const bool ptv = p.pt_var[pt] != 0;
    if (ptv) {
      double Wm[6 + CT][3];
#pragma unroll
      for (int m = 0; m < 6 + CT; ++m)
#pragma unroll
        for (int n = 0; n < 3; ++n) Wm[m][n] = jf[0][m] * jx[0][n] + jf[1][m] * jx[1][n];
      const double* vi = Vinv + 6 * (size_t)pt;
      const double Vi[6] = {vi[0], vi[1], vi[2], vi[3], vi[4], vi[5]};
      const double* gp = Vg + 9 * (size_t)pt + 6;
      const double gpv[3] = {gp[0], gp[1], gp[2]};
#pragma unroll
      for (int m = 0; m < 6 + CT; ++m) {
        sym3_mul(Vi, Wm[m], Y[m]);
        Yg[m] = Y[m][0] * gpv[0] + Y[m][1] * gpv[1] + Y[m][2] * gpv[2];
      }
      // Schur diagonal blocks: U - Y W'
      int o = 0;
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int c = a; c < 6; ++c, ++o)
          acc[o] += jf[0][a] * jf[0][c] + jf[1][a] * jf[1][c] -
                    (Y[a][0] * Wm[c][0] + Y[a][1] * Wm[c][1] + Y[a][2] * Wm[c][2]);
      o = kSymPose + 12;
#pragma unroll
      for (int a = 0; a < CT; ++a)
#pragma unroll
        for (int c = a; c < CT; ++c, ++o)
          acc[o] += jf[0][6 + a] * jf[0][6 + c] + jf[1][6 + a] * jf[1][6 + c] -
                    (Y[6 + a][0] * Wm[6 + c][0] + Y[6 + a][1] * Wm[6 + c][1] + Y[6 + a][2] * Wm[6 + c][2]);
    } else {
#pragma unroll
      for (int m = 0; m < 6 + CT; ++m) Yg[m] = 0.0;
      int o = 0;
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int c = a; c < 6; ++c, ++o) acc[o] += jf[0][a] * jf[0][c] + jf[1][a] * jf[1][c];
      o = kSymPose + 12;
#pragma unroll
      for (int a = 0; a < CT; ++a)
#pragma unroll
        for (int c = a; c < CT; ++c, ++o) acc[o] += jf[0][6 + a] * jf[0][6 + c] + jf[1][6 + a] * jf[1][6 + c];
    }
#pragma unroll
    for (int m = 0; m < 6; ++m) {
      acc[kSymPose + m] += g[m] - Yg[m];
      acc[kSymPose + 6 + m] += jf[0][m] * jf[0][m] + jf[1][m] * jf[1][m];
    }
#pragma unroll
    for (int m = 0; m < CT; ++m) {
      acc[kSymPose + 12 + NC + m] += g[6 + m] - Yg[6 + m];
      acc[kSymPose + 12 + NC + CT + m] += jf[0][6 + m] * jf[0][6 + m] + jf[1][6 + m] * jf[1][6 + m];
    }
  }
  block_reduce<NV>(acc, sred);
  const int k = threadIdx.x;
  if (k < NV) {
    const uint32_t img = tile.image;
    const uint32_t cam = p.img_cam[img];
    const bool pose_var = p.img_flags[img] & 1u;
    const bool cam_var = p.cam_var[cam] != 0;
    const double v = sred[k];
    if (k < kSymPose) {
      if (pose_var) atomicAdd(pose_blk + (size_t)img * kSymPose + k, v);
    } else if (k < kSymPose + 6) {
      if (pose_var) atomicAdd(bvec + 6 * (size_t)img + (k - kSymPose), v);
    } else if (k < kSymPose + 12) {
      if (pose_var) atomicAdd(udiag + 6 * (size_t)img + (k - kSymPose - 6), v);
    } else if (k < kSymPose + 12 + NC) {
      if (cam_var) atomicAdd(cam_blk + (size_t)cam * NC + (k - kSymPose - 12), v);
    } else if (k < kSymPose + 12 + NC + CT) {
      if (cam_var) atomicAdd(bvec + 6 * (size_t)p.num_images + (size_t)CT * cam + (k - kSymPose - 12 - NC), v);
    } else {
      if (cam_var)
        atomicAdd(udiag + 6 * (size_t)p.num_images + (size_t)CT * cam + (k - kSymPose - 12 - NC - CT), v);
    }
  }
}
#endif  // MI_BA_AB_VARIANTS

// packed upper-triangle index of (a, c), a <= c < n
__device__ inline int sym_index(int a, int c, int n) { return a * n - a * (a - 1) / 2 + (c - a); }

// fblock_kernel with two lanes per block: the even lane takes the pose
// columns, the odd lane the camera columns (their Schur-Jacobi diagonal
// blocks, rhs and diag(U) are disjoint), so each lane holds half the
// accumulators — 256 -> ~130 VGPRs, 1 -> 3 waves per SIMD for the row
// gathers to overlap.  Same terms, summed per half in lane order by a
// butterfly that skips the parity bit, then over the waves in order.
template <int CT>
__global__ __launch_bounds__(kBlock) void fblock_pair_kernel(DevProblem p, const DevTile* __restrict__ tiles,
                                                              const uint32_t* __restrict__ cm_perm,
                                                              const double2* __restrict__ rr,
                                                              const double* __restrict__ J,
                                                              const double* __restrict__ Jcm,
                                                              const double* __restrict__ Vg,
                                                              const double* __restrict__ Vinv,
                                                              double* __restrict__ pose_blk,
                                                              double* __restrict__ cam_blk,
                                                              double* __restrict__ bvec,
                                                              double* __restrict__ udiag,
                                                              double* __restrict__ part) {
  constexpr int NH = CT > 6 ? CT : 6;  // columns per half
  constexpr int NS = sym_size(NH), NA = NS + 2 * NH;
  __shared__ double sred[kBlock / 64][2][NA];
  const DevTile tile = tiles[blockIdx.x];
  const int W = 9 + CT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, hf = lane & 1;
  const int base = hf ? 9 : 0, nh = hf ? CT : 6;
  double acc[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) acc[k] = 0.0;
  for (uint32_t k = threadIdx.x >> 1; k < tile.count; k += kBlock / 2) {
    const uint32_t b = cm_perm[tile.start + k];
    const double* Jb = Jcm ? Jcm + (size_t)(tile.start + k) * 2 * W : J + (size_t)b * 2 * W;
    const double2 r = rr[b];
    double jf[2][NH], jx[2][3];
#pragma unroll
    for (int row = 0; row < 2; ++row) {
#pragma unroll
      for (int m = 0; m < NH; ++m) jf[row][m] = m < nh ? Jb[row * W + base + m] : 0.0;
#pragma unroll
      for (int m = 0; m < 3; ++m) jx[row][m] = Jb[row * W + 6 + m];
    }
    double gm[NH];
#pragma unroll
    for (int m = 0; m < NH; ++m) gm[m] = jf[0][m] * r.x + jf[1][m] * r.y;
    const uint32_t pt = p.obs_pt[b];
    if (p.pt_var[pt] != 0) {
      // W_m = J_f,m' J_p (3 values) recomputed where used rather than held
      // for all m: the registers go to the accumulators
      const double* vi = Vinv + 6 * (size_t)pt;
      const double Vi[6] = {vi[0], vi[1], vi[2], vi[3], vi[4], vi[5]};
      const double* gp = Vg + 9 * (size_t)pt + 6;
      const double gpv[3] = {gp[0], gp[1], gp[2]};
      int o = 0;
#pragma unroll
      for (int a = 0; a < NH; ++a) {
        double Wa[3], Ya[3];
#pragma unroll
        for (int n = 0; n < 3; ++n) Wa[n] = jf[0][a] * jx[0][n] + jf[1][a] * jx[1][n];
        sym3_mul(Vi, Wa, Ya);
        gm[a] -= Ya[0] * gpv[0] + Ya[1] * gpv[1] + Ya[2] * gpv[2];
#pragma unroll
        for (int c = a; c < NH; ++c, ++o) {
          double Wc[3];
#pragma unroll
          for (int n = 0; n < 3; ++n) Wc[n] = jf[0][c] * jx[0][n] + jf[1][c] * jx[1][n];
          acc[o] += jf[0][a] * jf[0][c] + jf[1][a] * jf[1][c] - (Ya[0] * Wc[0] + Ya[1] * Wc[1] + Ya[2] * Wc[2]);
        }
      }
    } else {
      int o = 0;
#pragma unroll
      for (int a = 0; a < NH; ++a)
#pragma unroll
        for (int c = a; c < NH; ++c, ++o) acc[o] += jf[0][a] * jf[0][c] + jf[1][a] * jf[1][c];
    }
#pragma unroll
    for (int m = 0; m < NH; ++m) {
      acc[NS + m] += gm[m];
      acc[NS + NH + m] += jf[0][m] * jf[0][m] + jf[1][m] * jf[1][m];
    }
  }
  // per half: butterfly over the lanes of one parity, then the waves in order
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    double v = acc[k];
#pragma unroll
    for (int off = 2; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
    acc[k] = v;
  }
  if (lane < 2) {
#pragma unroll
    for (int k = 0; k < NA; ++k) sred[wv][lane][k] = acc[k];
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= 2 * NA) return;
  const int h = t / NA, k = t - h * NA;
  double v = sred[0][h][k];
#pragma unroll
  for (int w = 1; w < kBlock / 64; ++w) v += sred[w][h][k];
  if (part) {  // deterministic flush (owner_flush_kernel, FlushPair)
    part[(size_t)blockIdx.x * kTilePartStride + t] = v;
    return;
  }
  const uint32_t img = tile.image, cam = p.img_cam[img];
  const int n = h ? CT : 6;
  if (h == 0 ? !(p.img_flags[img] & 1u) : !p.cam_var[cam]) return;
  if (k < NS) {
    int a = 0, rem = k;
    while (rem >= NH - a) { rem -= NH - a; ++a; }
    const int c = a + rem;
    if (c >= n) return;
    if (h == 0)
      atomicAdd(pose_blk + (size_t)img * kSymPose + sym_index(a, c, 6), v);
    else
      atomicAdd(cam_blk + (size_t)cam * sym_size(CT) + sym_index(a, c, CT), v);
    return;
  }
  const int m = (k - NS) % NH;
  if (m >= n) return;
  double* dst = k < NS + NH ? bvec : udiag;
  atomicAdd(dst + (h == 0 ? 6 * (size_t)img + m : 6 * (size_t)p.num_images + (size_t)CT * cam + m), v);
}

// f-vector slot of tangent column m (pose 0..5, camera 6..) of an image's block
__device__ inline int64_t fslot(const DevProblem& p, uint32_t img, uint32_t cam, int m) {
  return m < 6 ? 6 * (int64_t)img + m : 6 * (int64_t)p.num_images + (int64_t)p.ct * cam + (m - 6);
}

// ---------------------------------------------------------------------------
// Deterministic camera-side flush.  The tile kernels (one workgroup per
// image-aligned tile of camera-major blocks) write their block-reduced sums
// to TileOwners::part[tile][k] instead of adding them atomically into the
// shared image / camera slots; owner_flush_kernel then sums each value over
// its owner's tiles — an image's tiles, or the tiles of every image of a
// camera — in one fixed order (lane-strided partial sums, then the wave's
// butterfly) and adds the total to its destination, which no other workgroup
// writes.  The LM's camera-side sums (S's image blocks, b, diag(U), the
// Schur-Jacobi blocks, every Schur product) are then bitwise reproducible
// run to run.  D: has(cam, k) whether value k belongs to an image (cam =
// false) or a camera owner; put(cam, owner, k, v) its destination.
// ---------------------------------------------------------------------------
template <class D>
__global__ __launch_bounds__(64) void owner_flush_kernel(D d, TileOwners o, int stride, int nimg) {
  const int ow = blockIdx.x, lane = threadIdx.x;
  const bool cam = ow >= nimg;
  const uint32_t id = cam ? (uint32_t)(ow - nimg) : (uint32_t)ow;
  const uint32_t t0 = cam ? o.cam_tile_off[id] : o.img_tile_off[id];
  const uint32_t t1 = cam ? o.cam_tile_off[id + 1] : o.img_tile_off[id + 1];
  if (t0 == t1) return;
  for (int k = 0; k < stride; ++k) {
    if (!d.has(cam, k)) continue;
    double v = 0.0;
    for (uint32_t t = t0 + lane; t < t1; t += 64) {
      const uint32_t tile = cam ? o.cam_tiles[t] : t;
      v += o.part[(size_t)tile * o.stride + k];
    }
    v = wave_sum(v);
    if (lane == 0) d.put(cam, id, k, v);
  }
}

template <class D>
void launch_owner_flush(const D& d, const TileOwners& o, int stride, const DevProblem& p, hipStream_t s) {
  const int n = p.num_images + p.num_cameras;
  if (n > 0) hipLaunchKernelGGL(owner_flush_kernel<D>, dim3(n), dim3(64), 0, s, d, o, stride, p.num_images);
}

// y[f-slot] += v: F = 6 + CT values per tile (pose 0..5, camera 6..)
struct FlushFVec {
  DevProblem p;
  double* y;
  __device__ bool has(bool cam, int k) const { return cam ? k >= 6 : k < 6; }
  __device__ void put(bool cam, uint32_t id, int k, double v) const {
    if (!cam) {
      if (p.img_flags[id] & 1u) y[6 * (size_t)id + k] += v;
    } else if (p.cam_var[id]) {
      y[6 * (size_t)p.num_images + (size_t)p.ct * id + (k - 6)] += v;
    }
  }
};

// fblock_dense_kernel's NU + F values: U's packed upper triangle over the
// image's tangent columns (pose 0..5, camera 6..), then b.  Pose-pose and
// pose-camera entries belong to the image, camera-camera ones to the camera.
struct FlushDense {
  DevProblem p;
  double* S;
  double* bvec;
  double* udiag;
  int F, NU;
  __device__ void pair(int k, int* a, int* c) const {
    int aa = 0, rem = k;
    while (rem >= F - aa) { rem -= F - aa; ++aa; }
    *a = aa;
    *c = aa + rem;
  }
  __device__ bool has(bool cam, int k) const {
    if (k >= NU + F) return false;
    if (k >= NU) return cam ? k - NU >= 6 : k - NU < 6;
    int a, c;
    pair(k, &a, &c);
    return cam ? a >= 6 : a < 6;
  }
  __device__ void put(bool cam, uint32_t id, int k, double v) const {
    // camera owner: the camera's own slots only (a, c >= 6)
    const uint32_t img = cam ? 0u : id, cm = cam ? id : p.img_cam[id];
    const bool pv = !cam && (p.img_flags[img] & 1u), cv = p.cam_var[cm] != 0;
    if (k >= NU) {
      const int m = k - NU;
      if (m < 6 ? pv : cv) bvec[fslot(p, img, cm, m)] += v;
      return;
    }
    int a, c;
    pair(k, &a, &c);
    if (!((a < 6 ? pv : cv) && (c < 6 ? pv : cv))) return;
    const int64_t ra = fslot(p, img, cm, a), rc = fslot(p, img, cm, c);
    S[(ra <= rc ? ra * p.lds + rc : rc * p.lds + ra)] += v;
    if (a == c) udiag[ra] += v;
  }
};

// fblock_pair_kernel's 2 NA values: per half h (0 pose, 1 camera) the packed
// upper Schur-Jacobi block over NH columns, then NH of b and NH of diag(U).
struct FlushPair {
  DevProblem p;
  double* pose_blk;
  double* cam_blk;
  double* bvec;
  double* udiag;
  int NH, NS, NA;
  __device__ bool has(bool cam, int t) const { return t < 2 * NA && (cam ? t >= NA : t < NA); }
  __device__ void put(bool cam, uint32_t id, int t, double v) const {
    const int h = cam ? 1 : 0, k = t - h * NA, n = h ? p.ct : 6;
    if (h == 0 ? !(p.img_flags[id] & 1u) : !p.cam_var[id]) return;
    if (k < NS) {
      int a = 0, rem = k;
      while (rem >= NH - a) { rem -= NH - a; ++a; }
      const int c = a + rem;
      if (c >= n) return;
      if (h == 0)
        pose_blk[(size_t)id * kSymPose + sym_index(a, c, 6)] += v;
      else
        cam_blk[(size_t)id * sym_size(p.ct) + sym_index(a, c, p.ct)] += v;
      return;
    }
    const int m = (k - NS) % NH;
    if (m >= n) return;
    double* dst = k < NS + NH ? bvec : udiag;
    dst[h == 0 ? 6 * (size_t)id + m : 6 * (size_t)p.num_images + (size_t)p.ct * id + m] += v;
  }
};

// Exact (explicit S) path: one pass over an image tile's J rows giving
//   U = sum J_f'J_f into S's image block (upper triangle, as dense_u_kernel),
//   b = g - sum W V^-1 g_p = sum J_f'(r - J_p q_p), q_p = V_p^-1 g_p (point_prepare),
//   diag(U) (the LM damping's column norms).
// Replaces fblock_kernel + dense_u_kernel there: the Schur-Jacobi blocks
// fblock_kernel also forms are only the PCG preconditioner's.
template <int CT>
__global__ __launch_bounds__(kBlock) void fblock_dense_kernel(DevProblem p, const DevTile* __restrict__ tiles,
                                                               const uint32_t* __restrict__ cm_perm,
                                                               const uint32_t* __restrict__ cm_ptv,
                                                               const double2* __restrict__ rr,
                                                               const double* __restrict__ J,
                                                               const double* __restrict__ q,
                                                               double* __restrict__ bvec,
                                                               double* __restrict__ udiag, double* __restrict__ S,
                                                               double* __restrict__ part) {
  constexpr int F = 6 + CT, W = 9 + CT;
  constexpr int NU = F * (F + 1) / 2, NV = NU + F;
  __shared__ double sred[4 * NV];
  const DevTile tile = tiles[blockIdx.x];
  double acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.0;
  for (uint32_t k = threadIdx.x; k < tile.count; k += kBlock) {
    const uint32_t b = cm_perm[tile.start + k];
    const double* Jb = J + (size_t)b * 2 * W;
    const uint32_t pt = cm_ptv[tile.start + k];
    const double2 r = rr[b];
    const bool ptv = pt != 0xffffffffu;
    double qp[3] = {0.0, 0.0, 0.0};
    if (ptv) {
      qp[0] = q[3 * (size_t)pt];
      qp[1] = q[3 * (size_t)pt + 1];
      qp[2] = q[3 * (size_t)pt + 2];
    }
    double jf[2][F];
    double e[2];
#pragma unroll
    for (int row = 0; row < 2; ++row) {
#pragma unroll
      for (int m = 0; m < 6; ++m) jf[row][m] = Jb[row * W + m];
#pragma unroll
      for (int m = 0; m < CT; ++m) jf[row][6 + m] = Jb[row * W + 9 + m];
      e[row] = (row == 0 ? r.x : r.y) -
               (Jb[row * W + 6] * qp[0] + Jb[row * W + 7] * qp[1] + Jb[row * W + 8] * qp[2]);
    }
    int o = 0;
#pragma unroll
    for (int a = 0; a < F; ++a)
#pragma unroll
      for (int c = a; c < F; ++c, ++o) acc[o] += jf[0][a] * jf[0][c] + jf[1][a] * jf[1][c];
#pragma unroll
    for (int m = 0; m < F; ++m) acc[NU + m] += jf[0][m] * e[0] + jf[1][m] * e[1];
  }
  block_reduce<NV>(acc, sred);
  const int k = threadIdx.x;
  if (k >= NV) return;
  if (part) {  // deterministic flush (owner_flush_kernel, FlushDense)
    part[(size_t)blockIdx.x * kTilePartStride + k] = sred[k];
    return;
  }
  const uint32_t img = tile.image, cam = p.img_cam[img];
  const bool pv = p.img_flags[img] & 1u, cv = p.cam_var[cam] != 0;
  const double v = sred[k];
  if (k < NU) {
    int a = 0, rem = k;
    while (rem >= F - a) { rem -= F - a; ++a; }
    const int c = a + rem;
    const bool va = a < 6 ? pv : cv, vc = c < 6 ? pv : cv;
    if (!(va && vc)) return;
    const int64_t ra = fslot(p, img, cam, a), rc = fslot(p, img, cam, c);
    if (ra <= rc)
      atomicAdd(S + ra * p.lds + rc, v);
    else
      atomicAdd(S + rc * p.lds + ra, v);
    if (a == c) atomicAdd(udiag + ra, v);
  } else {
    const int m = k - NU;
    if (m < 6 ? pv : cv) atomicAdd(bvec + fslot(p, img, cam, m), v);
  }
}

// As fblock_dense_kernel, on the matrix cores (tools build, fblock_variant
// 1: measured slower — the row gathers bind, and the 70 KB LDS slab halves
// the waves in flight): with
// X = [J_f | e] (two rows per block, F + 1 <= 16 columns, e = r - J_p q_p),
// U and b are blocks of X'X, one v_mfma_f64_16x16x4f64 per two blocks: lane
// (m, k) supplies X[4s + k][m] as both the A (X') and the B (X) operand.
// Each wave gathers its 64 camera-major rows into an LDS slab with 16-B
// loads spread over the rows (about 4 rows per wave-instruction, where a
// lane walking its own row touches 64 lines per instruction), forms e there,
// then runs the MFMA steps; the four waves' accumulators are summed in fixed
// order and scattered as fblock_dense_kernel does.
#ifdef MI_BA_AB_VARIANTS
template <int CT>
__global__ __launch_bounds__(kBlock) void fblock_mfma_kernel(DevProblem p, const DevTile* __restrict__ tiles,
                                                              const uint32_t* __restrict__ cm_perm,
                                                              const double2* __restrict__ rr,
                                                              const double* __restrict__ J,
                                                              const double* __restrict__ q,
                                                              double* __restrict__ bvec,
                                                              double* __restrict__ udiag, double* __restrict__ S) {
  constexpr int F = 6 + CT, W = 9 + CT, W2 = 2 * W, H = W;  // H: 16-B pieces per J row
  constexpr int LS = W2 + 4;                                // J row, e (2), pad: 16-B rows
  static_assert(F + 1 <= 16, "X = [J_f | e] must fit the 16-wide MFMA tile");
  typedef double dvec4 __attribute__((ext_vector_type(4)));
  __shared__ double sl[kBlock / 64][64 * LS];
  const DevTile tile = tiles[blockIdx.x];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* slab = sl[wv];
  const int m = lane & 15, kq = lane >> 4;
  const int cm = m < 6 ? m : (m < F ? 3 + m : (m == F ? W2 : -1));  // X column m within a slab row (+ rw W)
  dvec4 acc = {0.0, 0.0, 0.0, 0.0};
  for (uint32_t c0 = 64u * wv; c0 < tile.count; c0 += kBlock) {
    const int live = (int)min(64u, tile.count - c0);
    const uint32_t bl = lane < live ? cm_perm[tile.start + c0 + lane] : 0u;
#pragma unroll
    for (int it = 0; it < H; ++it) {
      const int e = lane + 64 * it;
      const int row = e / H, col = e - row * H;
      const uint32_t b = (uint32_t)__shfl((int)bl, row < 64 ? row : 0);
      if (row < live) {
        const dvec2 v = __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(J + (size_t)b * W2) + col);
        *reinterpret_cast<dvec2*>(slab + row * LS + 2 * col) = v;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (lane < live) {
      const uint32_t pt = p.obs_pt[bl];
      const double2 r = rr[bl];
      double qp[3] = {0.0, 0.0, 0.0};
      if (p.pt_var[pt]) {
        qp[0] = q[3 * (size_t)pt];
        qp[1] = q[3 * (size_t)pt + 1];
        qp[2] = q[3 * (size_t)pt + 2];
      }
      double* row = slab + lane * LS;
      row[W2] = r.x - (row[6] * qp[0] + row[7] * qp[1] + row[8] * qp[2]);
      row[W2 + 1] = r.y - (row[W + 6] * qp[0] + row[W + 7] * qp[1] + row[W + 8] * qp[2]);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int nsteps = (2 * live + 3) >> 2;
    for (int st = 0; st < nsteps; ++st) {
      const int R = 4 * st + kq, j = R >> 1, rw = R & 1;
      double x = 0.0;
      if (j < live && cm >= 0) x = slab[j * LS + (cm == W2 ? W2 + rw : rw * W + cm)];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, acc, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  // the four waves' tiles summed in wave order
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) slab[r * 64 + lane] = acc[r];
  __syncthreads();
  if (wv != 0) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = sl[0][r * 64 + lane] + sl[1][r * 64 + lane] + sl[2][r * 64 + lane] + sl[3][r * 64 + lane];
  const uint32_t img = tile.image, cam = p.img_cam[img];
  const bool pv = p.img_flags[img] & 1u, cv = p.cam_var[cam] != 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int a = 4 * r + kq, c = m;  // D[4r + l/16][l%16]
    if (a >= F || c > F || (c < F && c < a)) continue;
    const double v = acc[r];
    const bool va = a < 6 ? pv : cv;
    if (!va) continue;
    const int64_t ra = fslot(p, img, cam, a);
    if (c == F) {
      atomicAdd(bvec + ra, v);
      continue;
    }
    if (!(c < 6 ? pv : cv)) continue;
    const int64_t rc = fslot(p, img, cam, c);
    if (ra <= rc)
      atomicAdd(S + ra * p.lds + rc, v);
    else
      atomicAdd(S + rc * p.lds + ra, v);
    if (a == c) atomicAdd(udiag + ra, v);
  }
}

#endif  // MI_BA_AB_VARIANTS

// Damp, Jacobi-scale and invert the diagonal blocks (one thread per block).
template <int N>
__device__ inline void chol_inverse(double (&A)[N][N], double (&Ainv)[N][N]) {
  // in-place Cholesky (lower), then inverse via L^-1
  double L[N][N];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) L[i][j] = 0.0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double d = A[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k];
    d = sqrt(fmax(d, 1e-300));
    L[j][j] = d;
    const double id = 1.0 / d;
#pragma unroll
    for (int i = j + 1; i < N; ++i) {
      double v = A[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k];
      L[i][j] = v * id;
    }
  }
  // Linv (lower)
  double Li[N][N];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) Li[i][j] = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    Li[i][i] = 1.0 / L[i][i];
#pragma unroll
    for (int j = 0; j < i; ++j) {
      double v = 0.0;
#pragma unroll
      for (int k = j; k < i; ++k) v -= L[i][k] * Li[k][j];
      Li[i][j] = v * Li[i][i];
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) {
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < N; ++k) v += Li[k][i] * Li[k][j];
      Ainv[i][j] = v;
    }
}

// Parameter block of tangent slot a within an N-wide finalize block (the
// SCHUR_JACOBI preconditioner has one diagonal block per Ceres parameter
// block, SchurJacobiPreconditioner): KIND 0 one block (camera intrinsics),
// 1 an image's qvec (3) | tvec (3), 2 a cylinder's qvec (3) | tvec (3) |
// radius | height (by two points: tvec_1 (3) | tvec_2 (3) | radius).
template <int KIND>
__device__ constexpr int param_group(int a) {
  return KIND == 0 ? 0 : KIND == 1 ? (a < 3 ? 0 : 1) : (a < 3 ? 0 : a < 6 ? 1 : a);
}

template <int N, int KIND = 0>
__device__ void finalize_block(const double* __restrict__ blk, const double* __restrict__ udiag,
                               double* __restrict__ scale_f, double* __restrict__ diag_f,
                               double* __restrict__ lambda_f, double* __restrict__ prec, double* __restrict__ b,
                               bool var, int first, int reuse_diag, double radius) {
  double A[N][N], Ai[N][N];
  int o = 0;
#pragma unroll
  for (int a = 0; a < N; ++a)
#pragma unroll
    for (int c = a; c < N; ++c, ++o) {
      // the preconditioner keeps the diagonal blocks of the parameter blocks
      A[a][c] = var && param_group<KIND>(a) == param_group<KIND>(c) ? blk[o] : 0.0;
      A[c][a] = A[a][c];
    }
#pragma unroll
  for (int m = 0; m < N; ++m) {
    if (!var) {
      scale_f[m] = 1.0;
      diag_f[m] = 0.0;
      lambda_f[m] = 0.0;
      A[m][m] = 1.0;
      b[m] = 0.0;
      continue;
    }
    double s;
    if (first) {
      s = 1.0 / (1.0 + sqrt(udiag[m]));
      scale_f[m] = s;
    } else {
      s = scale_f[m];
    }
    double d;
    if (!reuse_diag) {
      d = fmin(fmax(s * s * udiag[m], 1e-6), 1e32);
      diag_f[m] = d;
    } else {
      d = diag_f[m];
    }
    const double lam = d / (radius * s * s);
    lambda_f[m] = lam;
    A[m][m] += lam;
    b[m] = -b[m];
  }
  chol_inverse<N>(A, Ai);
#pragma unroll
  for (int a = 0; a < N; ++a)
#pragma unroll
    for (int c = 0; c < N; ++c) prec[a * N + c] = var ? Ai[a][c] : (a == c ? 1.0 : 0.0);
}

template <int CT>
__global__ __launch_bounds__(64) void fblock_finalize_kernel(DevProblem p, const double* __restrict__ pose_blk,
                                                              const double* __restrict__ cam_blk,
                                                              const double* __restrict__ udiag,
                                                              double* __restrict__ scale_f,
                                                              double* __restrict__ diag_f,
                                                              double* __restrict__ lambda_f,
                                                              double* __restrict__ prec_pose,
                                                              double* __restrict__ prec_cam,
                                                              double* __restrict__ b, int first,
                                                              int reuse_diag, double radius) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  const int I = p.num_images, C = p.num_cameras;
  if (k < I) {
    const bool var = p.img_flags[k] & 1u;
    const size_t o = 6 * (size_t)k;
    finalize_block<6, 1>(pose_blk + (size_t)k * kSymPose, udiag + o, scale_f + o, diag_f + o, lambda_f + o,
                         prec_pose + 36 * (size_t)k, b + o, var, first, reuse_diag, radius);
  } else if (CT > 0 && k < I + C) {
    const int c = k - I;
    const bool var = p.cam_var[c] != 0;
    const size_t o = 6 * (size_t)I + (size_t)CT * c;
    finalize_block<(CT > 0 ? CT : 1)>(cam_blk + (size_t)c * sym_size(CT), udiag + o, scale_f + o, diag_f + o,
                                      lambda_f + o, prec_cam + (size_t)CT * CT * c, b + o, var, first,
                                      reuse_diag, radius);
  }
}

// n generic NxN blocks (GSBA cylinders, N = 8 or 7): blk [n][N (N + 1) / 2]
// packed upper, f-vector arrays already offset to the first block's slots.
template <int N>
__global__ __launch_bounds__(64) void finalize_n_kernel(int n, const double* __restrict__ blk,
                                                        const double* __restrict__ udiag, double* __restrict__ scale_f,
                                                        double* __restrict__ diag_f, double* __restrict__ lambda_f,
                                                        double* __restrict__ prec, double* __restrict__ b, int var,
                                                        int first, int reuse_diag, double radius) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= n) return;
  const size_t o = N * (size_t)k;
  finalize_block<N, 2>(blk + (N * (N + 1) / 2) * (size_t)k, udiag + o, scale_f + o, diag_f + o, lambda_f + o,
                       prec + N * N * (size_t)k, b + o, var != 0, first, reuse_diag, radius);
}

template <int N>
__global__ __launch_bounds__(64) void precond_n_kernel(int n, const double* __restrict__ prec,
                                                       const double* __restrict__ r, double* __restrict__ z) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= n) return;
  const double* M = prec + N * N * (size_t)k;
  double rr[N];
#pragma unroll
  for (int m = 0; m < N; ++m) rr[m] = r[N * (size_t)k + m];
#pragma unroll
  for (int a = 0; a < N; ++a) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < N; ++c) s += M[a * N + c] * rr[c];
    z[N * (size_t)k + a] = s;
  }
}

// ---------------------------------------------------------------------------
// Implicit Schur product y = (U + Lambda_f) x - W V^-1 W' x
// ---------------------------------------------------------------------------
template <int CT>
__device__ inline void load_jf_x(const DevProblem& p, const double* __restrict__ Jb, uint32_t img,
                                 const double* __restrict__ x, double e[2]) {
  const int W = 9 + CT;
  const double* xi = x + 6 * (size_t)img;
  const uint32_t cam = p.img_cam[img];
  const double* xc = x + 6 * (size_t)p.num_images + (size_t)CT * cam;
  double xv[6 + CT];
#pragma unroll
  for (int m = 0; m < 6; ++m) xv[m] = xi[m];
#pragma unroll
  for (int m = 0; m < CT; ++m) xv[6 + m] = xc[m];
#pragma unroll
  for (int row = 0; row < 2; ++row) {
    double s = 0.0;
#pragma unroll
    for (int m = 0; m < 6; ++m) s += Jb[row * W + m] * xv[m];
#pragma unroll
    for (int m = 0; m < CT; ++m) s += Jb[row * W + 9 + m] * xv[6 + m];
    e[row] = s;
  }
}

template <int CT>
__global__ __launch_bounds__(kBlock) void schur_point_pass(DevProblem p, const DevPoint* __restrict__ vp,
                                                            int64_t npv, const double* __restrict__ J,
                                                            const double* __restrict__ Vinv,
                                                            const double* __restrict__ x,
                                                            double* __restrict__ w) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= npv) return;
  const DevPoint d = vp[k];
  const int W = 9 + CT;
  double t[3] = {0.0, 0.0, 0.0};
  for (uint32_t m = 0; m < d.count; ++m) {
    const uint32_t b = d.start + m;
    const double* Jb = J + (size_t)b * 2 * W;
    double e[2];
    load_jf_x<CT>(p, Jb, p.obs_img[b], x, e);
#pragma unroll
    for (int n = 0; n < 3; ++n) t[n] += Jb[6 + n] * e[0] + Jb[W + 6 + n] * e[1];
  }
  const double* vi = Vinv + 6 * (size_t)d.point;
  const double Vi[6] = {vi[0], vi[1], vi[2], vi[3], vi[4], vi[5]};
  double wv[3];
  sym3_mul(Vi, t, wv);
#pragma unroll
  for (int n = 0; n < 3; ++n) w[3 * (size_t)d.point + n] = wv[n];
}

template <int CT>
__global__ __launch_bounds__(kBlock) void schur_f_pass(DevProblem p, const DevTile* __restrict__ tiles,
                                                        const uint32_t* __restrict__ cm_perm,
                                                        const uint32_t* __restrict__ cm_ptv,
                                                        const double* __restrict__ J,
                                                        const double* __restrict__ Jcm,
                                                        const double* __restrict__ x,
                                                        const double* __restrict__ w,
                                                        double* __restrict__ y, double* __restrict__ part) {
  constexpr int NV = 6 + CT;
  __shared__ double sred[4 * NV];
  const DevTile tile = tiles[blockIdx.x];
  const int W = 9 + CT;
  double acc[NV];
#pragma unroll
  for (int m = 0; m < NV; ++m) acc[m] = 0.0;
  for (uint32_t k = threadIdx.x; k < tile.count; k += kBlock) {
    // Jcm: the rows in camera-major order (contiguous over the tile)
    const double* Jb = Jcm ? Jcm + (size_t)(tile.start + k) * 2 * W : J + (size_t)cm_perm[tile.start + k] * 2 * W;
    double e[2];
    load_jf_x<CT>(p, Jb, tile.image, x, e);
    uint32_t pt;
    if (cm_ptv) {
      pt = cm_ptv[tile.start + k];  // coalesced; 0xffffffff: constant point
    } else {
      pt = p.obs_pt[cm_perm[tile.start + k]];
      if (!p.pt_var[pt]) pt = 0xffffffffu;
    }
    if (pt != 0xffffffffu) {
      const double wv[3] = {w[3 * (size_t)pt], w[3 * (size_t)pt + 1], w[3 * (size_t)pt + 2]};
#pragma unroll
      for (int row = 0; row < 2; ++row)
        e[row] -= Jb[row * W + 6] * wv[0] + Jb[row * W + 7] * wv[1] + Jb[row * W + 8] * wv[2];
    }
#pragma unroll
    for (int m = 0; m < 6; ++m) acc[m] += Jb[m] * e[0] + Jb[W + m] * e[1];
#pragma unroll
    for (int m = 0; m < CT; ++m) acc[6 + m] += Jb[9 + m] * e[0] + Jb[W + 9 + m] * e[1];
  }
  block_reduce<NV>(acc, sred);
  const int k = threadIdx.x;
  if (k < NV && part) {
    part[(size_t)blockIdx.x * kTilePartStride + k] = sred[k];
  } else if (k < NV) {
    const uint32_t img = tile.image;
    if (k < 6) {
      if (p.img_flags[img] & 1u) atomicAdd(y + 6 * (size_t)img + k, sred[k]);
    } else {
      const uint32_t cam = p.img_cam[img];
      if (p.cam_var[cam]) atomicAdd(y + 6 * (size_t)p.num_images + (size_t)CT * cam + (k - 6), sred[k]);
    }
  }
}

// schur_f_pass on the camera-major copy, rows staged through the wave's LDS
// slab by coalesced loads, 32 blocks per pass: lane l takes residual row
// l / 32 of block l % 32 (y_f = sum over residual rows of J_f,row' e_row).
template <int CT>
__global__ __launch_bounds__(kBlock) void schur_f_rows_kernel(DevProblem p, const DevTile* __restrict__ tiles,
                                                               const uint32_t* __restrict__ cm_ptv,
                                                               const double* __restrict__ Jcm,
                                                               const double* __restrict__ x,
                                                               const double* __restrict__ w,
                                                               double* __restrict__ y, double* __restrict__ part) {
  constexpr int NV = 6 + CT, W = 9 + CT, W2 = 2 * W, LS = W2 | 1;
  __shared__ double sl[(kBlock / 64) * 32 * LS];
  __shared__ double sred[4 * NV];
  const DevTile tile = tiles[blockIdx.x];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* slab = sl + wv * 32 * LS;
  const uint32_t img = tile.image, cam = p.img_cam[img];
  double xv[NV];
#pragma unroll
  for (int m = 0; m < 6; ++m) xv[m] = x[6 * (size_t)img + m];
#pragma unroll
  for (int m = 0; m < CT; ++m) xv[6 + m] = x[6 * (size_t)p.num_images + (size_t)CT * cam + m];
  double acc[NV];
#pragma unroll
  for (int m = 0; m < NV; ++m) acc[m] = 0.0;
  const int bi = lane & 31, rw = lane >> 5;
  for (uint32_t k0 = 32u * wv; k0 < tile.count; k0 += 32u * (kBlock / 64)) {
    const int live = (int)min(32u, tile.count - k0);
    wave_load_rows_u<W2, LS, 32>(Jcm + (size_t)(tile.start + k0) * W2, slab, live);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (bi < live) {
      const double* jr = slab + bi * LS + rw * W;
      double e = 0.0;
#pragma unroll
      for (int m = 0; m < 6; ++m) e += jr[m] * xv[m];
#pragma unroll
      for (int m = 0; m < CT; ++m) e += jr[9 + m] * xv[6 + m];
      const uint32_t pt = cm_ptv[tile.start + k0 + bi];
      if (pt != 0xffffffffu)
        e -= jr[6] * w[3 * (size_t)pt] + jr[7] * w[3 * (size_t)pt + 1] + jr[8] * w[3 * (size_t)pt + 2];
#pragma unroll
      for (int m = 0; m < 6; ++m) acc[m] += jr[m] * e;
#pragma unroll
      for (int m = 0; m < CT; ++m) acc[6 + m] += jr[9 + m] * e;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  block_reduce<NV>(acc, sred);
  const int k = threadIdx.x;
  if (k < NV && part) {
    part[(size_t)blockIdx.x * kTilePartStride + k] = sred[k];
  } else if (k < NV) {
    if (k < 6) {
      if (p.img_flags[img] & 1u) atomicAdd(y + 6 * (size_t)img + k, sred[k]);
    } else if (p.cam_var[cam]) {
      atomicAdd(y + 6 * (size_t)p.num_images + (size_t)CT * cam + (k - 6), sred[k]);
    }
  }
}

// ---------------------------------------------------------------------------
// Matrix-free implicit Schur product (PCG path, "pcg_matrix_free").  The two
// passes of y = S x recompute each block's tangent Jacobian rows from the
// block's inputs — the point (24 B, point-major / camera-major copy), the
// image record (L2-resident), the CG vector — instead of reading the 2 (9+c)
// stored doubles (240 B at OPENCV) twice per product: the rows are the
// production reproj_jacobian_kernel arithmetic (R X through the rotation
// matrix, closed-form rotation columns for a unit q, Dq * PlusJacobian
// otherwise, the Corrector's sqrt(rho') with a robust loss; the model and
// its refined-intrinsics mask from the image record at run time).
// ---------------------------------------------------------------------------
template <int CT, int LOSS>
__device__ inline void block_rows_mf(const DevProblem& p, const double* q, const double* t, const double* prm,
                                     uint32_t meta, const double* X, bool ptv, double2 o, double (&Jr)[2][9 + CT]) {
  const uint32_t flags = meta & 0xffu;
  const bool pose_var = flags & 1u;
  const bool cv = (meta >> 8) & 1u;
  const int model = (int)((meta >> 16) & 0xffu);
  double Rm[9];
  unit_quat_matrix(q, Rm);
  double P[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) P[c] = Rm[3 * c] * X[0] + Rm[3 * c + 1] * X[1] + Rm[3 * c + 2] * X[2];
  const double a0 = P[0], a1 = P[1], a2 = P[2];  // R X
  P[0] += t[0];
  P[1] += t[1];
  P[2] += t[2];
  const double iz = 1.0 / P[2];
  const double u = P[0] * iz, v = P[1] * iz;
  double x, y, A[4], Jp[16];
  world_to_image_jac_any(model, prm, u, v, &x, &y, A, Jp);
  const unsigned cmask = cam_tangent_mask(model, p.refine_mask);
  double sc = 1.0;
  if constexpr (LOSS != 0) {
    const double r0 = x - o.x, r1 = y - o.y;
    double rho[3];
    loss_eval(p.loss_type, p.loss_scale, r0 * r0 + r1 * r1, rho);
    sc = sqrt(rho[1]);
  }
  double B[6] = {A[0] * iz, A[1] * iz, -(A[0] * u + A[1] * v) * iz,
                 A[2] * iz, A[3] * iz, -(A[2] * u + A[3] * v) * iz};
  if constexpr (LOSS != 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) B[k] *= sc;
  }
  double Mq[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const bool unit_q = fabs(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3] - 1.0) <= 1e-12;
  if (pose_var && unit_q) {
    Mq[1] = 2.0 * a2;  Mq[2] = -2.0 * a1;
    Mq[3] = -2.0 * a2; Mq[5] = 2.0 * a0;
    Mq[6] = 2.0 * a1;  Mq[7] = -2.0 * a0;
  } else if (pose_var) {
    double Dq[12], PJ[12];
    unit_quat_rotate_dq(q, X, Dq);
    quat_plus_jacobian(q, PJ);
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b)
        Mq[a * 3 + b] = Dq[a * 4 + 0] * PJ[0 * 3 + b] + Dq[a * 4 + 1] * PJ[1 * 3 + b] + Dq[a * 4 + 2] * PJ[2 * 3 + b] +
                        Dq[a * 4 + 3] * PJ[3 * 3 + b];
  }
  double jx[2][3] = {{0, 0, 0}, {0, 0, 0}};
  if (ptv) {
#pragma unroll
    for (int rw = 0; rw < 2; ++rw)
#pragma unroll
      for (int b = 0; b < 3; ++b)
        jx[rw][b] = B[rw * 3 + 0] * Rm[b] + B[rw * 3 + 1] * Rm[3 + b] + B[rw * 3 + 2] * Rm[6 + b];
  }
#pragma unroll
  for (int rw = 0; rw < 2; ++rw) emit_row_mixed<CT>(rw, Jr[rw], B, Mq, pose_var, flags, jx, Jp, sc, cv, cmask);
}

// The image record of img (q, t, meta, camera parameters) from img_rec.
__device__ inline uint32_t load_image_record(const DevProblem& p, uint32_t img, double q[4], double t[3],
                                             double prm[8]) {
  const double2* rv = reinterpret_cast<const double2*>(p.img_rec + kImgRec * (size_t)img);
  const double2 a0 = rv[0], a1 = rv[1], a2 = rv[2], a3 = rv[3];
  q[0] = a0.x; q[1] = a0.y; q[2] = a1.x; q[3] = a1.y;
  t[0] = a2.x; t[1] = a2.y; t[2] = a3.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double2 c = rv[4 + k];
    prm[2 * k] = c.x;
    prm[2 * k + 1] = c.y;
  }
  return (uint32_t)__double_as_longlong(a3.y);
}

// Point pass, matrix-free: w_p = V_p^-1 sum_a J_p,a' (J_f,a x) over the
// point chunks (one wave per chunk, one lane per block, the points' sums
// segmented in lane order as backsub_chunk_kernel's).
template <int CT, int LOSS>
__global__ __launch_bounds__(kBlock) void pcg_point_pass_mf(DevProblem p, const uint32_t* __restrict__ chunk,
                                                             int nchunks, const double* __restrict__ Vinv,
                                                             const double* __restrict__ x, double* __restrict__ w) {
  __shared__ double stv[kBlock / 64][64 * 3];
  __shared__ uint32_t spt[kBlock / 64][64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* tvs = stv[wv];
  uint32_t* wpt = spt[wv];
  const int c = blockIdx.x * (kBlock / 64) + wv;
  if (c >= nchunks) return;  // wave-uniform
  const uint32_t b0 = chunk[c], b1 = chunk[c + 1];
  const bool multi = b1 - b0 > 64u;
  double carry[3] = {0.0, 0.0, 0.0};
  uint32_t carry_pt = 0;
  bool carry_var = false;
  auto finalize = [&](uint32_t pt, const double tt[3]) {
    const double* vi = Vinv + 6 * (size_t)pt;
    const double Vi[6] = {vi[0], vi[1], vi[2], vi[3], vi[4], vi[5]};
    double o[3];
    sym3_mul(Vi, tt, o);
#pragma unroll
    for (int n = 0; n < 3; ++n) w[3 * (size_t)pt + n] = o[n];
  };
  for (uint32_t s0 = b0; s0 < b1; s0 += 64) {
    const int live = (int)min(64u, b1 - s0);
    const bool on = lane < live;
    const uint32_t b = s0 + (on ? lane : 0);
    const uint32_t pt = p.obs_pt[b];
    const bool var = on && p.pt_var[pt] != 0;
    double te[3] = {0.0, 0.0, 0.0};
    if (var) {
      const uint32_t img = p.obs_img[b];
      double q[4], t[3], prm[8];
      const uint32_t meta = load_image_record(p, img, q, t, prm);
      const double X[3] = {p.X[3 * (size_t)pt], p.X[3 * (size_t)pt + 1], p.X[3 * (size_t)pt + 2]};
      const double2 o = LOSS != 0 ? p.obs_xy[b] : make_double2(0.0, 0.0);
      double Jr[2][9 + CT];
      block_rows_mf<CT, LOSS>(p, q, t, prm, meta, X, true, o, Jr);
      const double* xi = x + 6 * (size_t)img;
      const double* xc = x + 6 * (size_t)p.num_images + (size_t)CT * p.img_cam[img];
      double xv[6 + CT];
#pragma unroll
      for (int m = 0; m < 6; ++m) xv[m] = xi[m];
#pragma unroll
      for (int m = 0; m < CT; ++m) xv[6 + m] = xc[m];
#pragma unroll
      for (int rw = 0; rw < 2; ++rw) {
        double e = 0.0;
#pragma unroll
        for (int m = 0; m < 6; ++m) e += Jr[rw][m] * xv[m];
#pragma unroll
        for (int m = 0; m < CT; ++m) e += Jr[rw][9 + m] * xv[6 + m];
#pragma unroll
        for (int n = 0; n < 3; ++n) te[n] += Jr[rw][6 + n] * e;
      }
    }
    double* tv = tvs + lane * 3;
    tv[0] = te[0];
    tv[1] = te[1];
    tv[2] = te[2];
    wpt[lane] = on ? pt : 0xffffffffu;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const bool head = var && (lane == 0 || wpt[lane - 1] != pt);
    if (head) {
      double tt[3] = {te[0], te[1], te[2]};
      for (int l = lane + 1; l < live && wpt[l] == pt; ++l) {
        tt[0] += tvs[l * 3];
        tt[1] += tvs[l * 3 + 1];
        tt[2] += tvs[l * 3 + 2];
      }
      if (multi) {
        carry[0] += tt[0];
        carry[1] += tt[1];
        carry[2] += tt[2];
        carry_pt = pt;
        carry_var = true;
      } else {
        finalize(pt, tt);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  if (multi && carry_var) finalize(carry_pt, carry);
}

// Camera pass, matrix-free: y_f = sum over the tile's blocks of J_f'
// (J_f x - J_p w_p), the image record tile-uniform, the blocks' points from
// the camera-major copy Xcm (and the observations from obs_cm with a robust
// loss), w_p gathered for variable points (cm_ptv).
template <int CT, int LOSS>
__global__ __launch_bounds__(kBlock) void pcg_camera_pass_mf(DevProblem p, const DevTile* __restrict__ tiles,
                                                              const uint32_t* __restrict__ cm_ptv,
                                                              const double* __restrict__ Xcm,
                                                              const double2* __restrict__ obs_cm,
                                                              const double* __restrict__ x,
                                                              const double* __restrict__ w, double* __restrict__ y,
                                                              double* __restrict__ part) {
  constexpr int NV = 6 + CT;
  __shared__ double sred[4 * NV];
  const DevTile tile = tiles[blockIdx.x];
  const uint32_t img = tile.image, cam = p.img_cam[img];
  double q[4], t[3], prm[8];
  const uint32_t meta = load_image_record(p, img, q, t, prm);
  double xv[NV];
#pragma unroll
  for (int m = 0; m < 6; ++m) xv[m] = x[6 * (size_t)img + m];
#pragma unroll
  for (int m = 0; m < CT; ++m) xv[6 + m] = x[6 * (size_t)p.num_images + (size_t)CT * cam + m];
  double acc[NV];
#pragma unroll
  for (int m = 0; m < NV; ++m) acc[m] = 0.0;
  for (uint32_t k = threadIdx.x; k < tile.count; k += kBlock) {
    const size_t kk = (size_t)tile.start + k;
    const double X[3] = {Xcm[3 * kk], Xcm[3 * kk + 1], Xcm[3 * kk + 2]};
    const uint32_t pt = cm_ptv[kk];
    const bool ptv = pt != 0xffffffffu;
    const double2 o = LOSS != 0 ? obs_cm[kk] : make_double2(0.0, 0.0);
    double Jr[2][9 + CT];
    block_rows_mf<CT, LOSS>(p, q, t, prm, meta, X, ptv, o, Jr);
    double wv3[3] = {0.0, 0.0, 0.0};
    if (ptv) {
      wv3[0] = w[3 * (size_t)pt];
      wv3[1] = w[3 * (size_t)pt + 1];
      wv3[2] = w[3 * (size_t)pt + 2];
    }
#pragma unroll
    for (int rw = 0; rw < 2; ++rw) {
      double e = 0.0;
#pragma unroll
      for (int m = 0; m < 6; ++m) e += Jr[rw][m] * xv[m];
#pragma unroll
      for (int m = 0; m < CT; ++m) e += Jr[rw][9 + m] * xv[6 + m];
      if (ptv) e -= Jr[rw][6] * wv3[0] + Jr[rw][7] * wv3[1] + Jr[rw][8] * wv3[2];
#pragma unroll
      for (int m = 0; m < 6; ++m) acc[m] += Jr[rw][m] * e;
#pragma unroll
      for (int m = 0; m < CT; ++m) acc[6 + m] += Jr[rw][9 + m] * e;
    }
  }
  block_reduce<NV>(acc, sred);
  const int k = threadIdx.x;
  if (k < NV && part) {
    part[(size_t)blockIdx.x * kTilePartStride + k] = sred[k];
  } else if (k < NV) {
    if (k < 6) {
      if (p.img_flags[img] & 1u) atomicAdd(y + 6 * (size_t)img + k, sred[k]);
    } else if (p.cam_var[cam]) {
      atomicAdd(y + 6 * (size_t)p.num_images + (size_t)CT * cam + (k - 6), sred[k]);
    }
  }
}

// The camera-major copies the matrix-free camera pass reads: Xcm[k] =
// X[obs_pt[cm_perm[k]]] (rebuilt whenever X changes) and, with a robust loss,
// obs_cm[k] = obs_xy[cm_perm[k]] (static).
__global__ __launch_bounds__(kBlock) void gather_cm_kernel(DevProblem p, const uint32_t* __restrict__ cm_perm,
                                                           int64_t n, double* __restrict__ Xcm,
                                                           double2* __restrict__ obs_cm) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const uint32_t b = cm_perm[k];
  const uint32_t pt = p.obs_pt[b];
  Xcm[3 * k] = p.X[3 * (size_t)pt];
  Xcm[3 * k + 1] = p.X[3 * (size_t)pt + 1];
  Xcm[3 * k + 2] = p.X[3 * (size_t)pt + 2];
  if (obs_cm) obs_cm[k] = p.obs_xy[b];
}

// Jcm[k] = J[cm_perm[k]]: the Jacobian rows in camera-major order, 16 B per
// lane, consecutive lanes on consecutive destination pieces (coalesced
// stores, row-contiguous gathers).  Built once per linearization for the PCG
// path, whose camera-side passes then read rows contiguously.
template <int CT>
__global__ __launch_bounds__(kBlock) void permute_rows_kernel(const uint32_t* __restrict__ cm_perm, int64_t n,
                                                               const double* __restrict__ J,
                                                               double* __restrict__ Jcm) {
  constexpr int H = 9 + CT;  // 16-B pieces per block (2 rows of 9 + CT doubles)
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n * H) return;
  const int64_t k = e / H;
  const int piece = (int)(e - k * H);
  const dvec2 v = reinterpret_cast<const dvec2*>(J + (size_t)cm_perm[k] * 2 * H)[piece];
  reinterpret_cast<dvec2*>(Jcm + (size_t)k * 2 * H)[piece] = v;
}

__global__ void add_diag_kernel(const double* __restrict__ lambda_f, const double* __restrict__ x,
                                double* __restrict__ y, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k < n) y[k] += lambda_f[k] * x[k];
}

template <int CT>
__global__ void precond_kernel(DevProblem p, const double* __restrict__ prec_pose,
                               const double* __restrict__ prec_cam, const double* __restrict__ r,
                               double* __restrict__ z) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  const int I = p.num_images, C = p.num_cameras;
  if (k < I) {
    const double* M = prec_pose + 36 * (size_t)k;
    const double* rv = r + 6 * (size_t)k;
    double rr[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) rr[m] = rv[m];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < 6; ++c) s += M[a * 6 + c] * rr[c];
      z[6 * (size_t)k + a] = s;
    }
  } else if (CT > 0 && k < I + C) {
    const int c0 = k - I;
    const double* M = prec_cam + (size_t)CT * CT * c0;
    const size_t o = 6 * (size_t)I + (size_t)CT * c0;
    double rr[CT > 0 ? CT : 1];
#pragma unroll
    for (int m = 0; m < CT; ++m) rr[m] = r[o + m];
#pragma unroll
    for (int a = 0; a < CT; ++a) {
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < CT; ++c) s += M[a * CT + c] * rr[c];
      z[o + a] = s;
    }
  }
}

__global__ __launch_bounds__(1024) void dot_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                   int64_t n, double* __restrict__ out) {
  __shared__ double sred[16];
  double v = 0.0;
  for (int64_t k = threadIdx.x; k < n; k += 1024) v += a[k] * b[k];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int k = 0; k < 16; ++k) s += sred[k];
    out[0] = s;
  }
}

__global__ void axpy_kernel(double* __restrict__ y, const double* __restrict__ x, const double* num,
                            const double* den, double sign, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k < n) y[k] += sign * (num[0] / den[0]) * x[k];
}

__global__ void xpby_kernel(double* __restrict__ pv, const double* __restrict__ z, const double* num,
                            const double* den, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k < n) pv[k] = z[k] + (num[0] / den[0]) * pv[k];
}

// The CG step of ConjugateGradientsSolver (Ceres 2.1, restated): alpha =
// rho / pq, x += alpha p and (update_r) r -= alpha q — taken only when the
// iteration gets that far in Ceres: rho (and beta = rho / rho_prev, when
// given) neither 0 nor inf, pq > 0 and finite, alpha finite.  Otherwise x
// and r stay, and the host (which reads the same scalars) ends the solve
// with FAILURE or NO_CONVERGENCE.
__device__ inline bool cg_zero_or_inf(double v) { return v == 0.0 || isinf(v) || isnan(v); }
__global__ void cg_step_kernel(double* __restrict__ x, const double* __restrict__ pv, double* __restrict__ r,
                               const double* __restrict__ q, const double* rho, const double* rho_prev,
                               const double* pq, int update_r, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const double rh = rho[0], d = pq[0];
  if (cg_zero_or_inf(rh) || (rho_prev && cg_zero_or_inf(rh / rho_prev[0]))) return;
  if (!(d > 0.0) || isinf(d)) return;
  const double alpha = rh / d;
  if (isinf(alpha)) return;
  x[k] = x[k] + alpha * pv[k];
  if (update_r) r[k] = r[k] - alpha * q[k];
}

// Raw camera-side gradient g_f += sum J_f' r (tangent, unscaled) of every
// reduced block over the image-aligned camera-major tiles, one atomic flush
// per tile (the gradient tolerance test: TrustRegionMinimizer::
// EvaluateGradientAndJacobian).
template <int CT>
__global__ __launch_bounds__(kBlock) void grad_f_kernel(DevProblem p, const DevTile* __restrict__ tiles,
                                                         const uint32_t* __restrict__ cm_perm,
                                                         const double2* __restrict__ rr,
                                                         const double* __restrict__ J, double* __restrict__ g,
                                                         double* __restrict__ part) {
  constexpr int F = 6 + CT, W = 9 + CT;
  __shared__ double sred[4 * F];
  const DevTile tile = tiles[blockIdx.x];
  double acc[F];
#pragma unroll
  for (int m = 0; m < F; ++m) acc[m] = 0.0;
  for (uint32_t k = threadIdx.x; k < tile.count; k += kBlock) {
    const uint32_t b = cm_perm[tile.start + k];
    const double* Jb = J + (size_t)b * 2 * W;
    const double2 r = rr[b];
#pragma unroll
    for (int m = 0; m < 6; ++m) acc[m] += Jb[m] * r.x + Jb[W + m] * r.y;
#pragma unroll
    for (int m = 0; m < CT; ++m) acc[6 + m] += Jb[9 + m] * r.x + Jb[W + 9 + m] * r.y;
  }
  block_reduce<F>(acc, sred);
  const int k = threadIdx.x;
  if (k >= F) return;
  if (part) {
    part[(size_t)blockIdx.x * kTilePartStride + k] = sred[k];
    return;
  }
  const uint32_t img = tile.image, cam = p.img_cam[img];
  if (k < 6 ? !(p.img_flags[img] & 1u) : !p.cam_var[cam]) return;
  atomicAdd(g + fslot(p, img, cam, k), sred[k]);
}

__device__ inline void atomic_max_nonneg(double* out, double v) {
  atomicMax(reinterpret_cast<unsigned long long*>(out), (unsigned long long)__double_as_longlong(v));
}

// |x - Plus(x, -g)|_inf over the image and camera blocks (qvec on the
// QuaternionManifold, tvec / intrinsics under their SubsetManifolds) into
// out[0] (as the bit pattern of a non-negative double: atomicMax).
__global__ void grad_max_f_kernel(DevProblem p, const double* __restrict__ g, double* out) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  double mx = 0.0;
  if (k < p.num_images) {
    const uint32_t fl = p.img_flags[k];
    if (fl & 1u) {
      const double* a = p.qt + 8 * (size_t)k;
      const double* gk = g + 6 * (size_t)k;
      const double q[4] = {a[0], a[1], a[2], a[3]};
      const double d[3] = {-gk[0], -gk[1], -gk[2]};
      double qn[4];
      quat_plus(q, d, qn);
      for (int m = 0; m < 4; ++m) mx = fmax(mx, fabs(q[m] - qn[m]));
      for (int m = 0; m < 3; ++m)
        if (!((fl >> (1 + m)) & 1u)) mx = fmax(mx, fabs(a[4 + m] - (a[4 + m] + -gk[3 + m])));
    }
  } else if (k < p.num_images + p.num_cameras) {
    const int c = k - p.num_images;
    if (p.cam_var[c]) {
      const double* a = p.cam + 8 * (size_t)c;
      const double* gc = g + 6 * (size_t)p.num_images + (size_t)p.ct * c;
      const unsigned cm = cam_tangent_mask(p.cam_model[c], p.refine_mask);
      int t = 0;
      for (int m = 0; m < 8; ++m)
        if ((cm >> m) & 1u) {
          mx = fmax(mx, fabs(a[m] - (a[m] + -gc[t])));
          ++t;
        }
    }
  } else {
    return;
  }
  if (mx > 0.0) atomic_max_nonneg(out, mx);
}

// The same over the variable points (g_p from the point blocks Vg).
// Grid-stride over the variable points (a few workgroups per CU), one
// atomic max per workgroup: one per wave over 1M points serialised ~16k
// atomics on one address (185 us at C4).
__global__ __launch_bounds__(kBlock) void grad_max_points_kernel(DevProblem p, const DevPoint* __restrict__ vp,
                                                                 int64_t npv, const double* __restrict__ Vg,
                                                                 double* out) {
  __shared__ double smax[kBlock / 64];
  double mx = 0.0;
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < npv; k += (int64_t)gridDim.x * kBlock) {
    const uint32_t pt = vp[k].point;
    const double* gp = Vg + 9 * (size_t)pt + 6;
    const double* X = p.X + 3 * (size_t)pt;
#pragma unroll
    for (int m = 0; m < 3; ++m) mx = fmax(mx, fabs(X[m] - (X[m] + -gp[m])));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off, 64));
  if ((threadIdx.x & 63) == 0) smax[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = smax[0];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) m = fmax(m, smax[w]);
    if (m > 0.0) atomic_max_nonneg(out, m);
  }
}

// Ceres' state vector over the variable blocks, ambient coordinates: |x|^2
// and |x - x_c|^2 (ParameterToleranceReached's x_norm and step_norm).  Images
// and cameras counted when with_f (rank 0 of a multi-rank solve), points
// always (each rank its own).  Per-workgroup partials: out[b] (|x|^2) and
// out[gridDim.x + b] (|x - x_c|^2), summed in a fixed order afterwards.
__global__ __launch_bounds__(1024) void state_norms_kernel(DevProblem p, const double* __restrict__ qt_c,
                                                           const double* __restrict__ cam_c,
                                                           const double* __restrict__ X_c, int with_f,
                                                           double* __restrict__ out) {
  __shared__ double sred[2][16];
  double vx = 0.0, vd = 0.0;
  const int64_t nf_items = with_f ? (int64_t)p.num_images + p.num_cameras : 0;
  const int64_t n = nf_items + p.num_points;
  const int64_t stride = (int64_t)gridDim.x * 1024;
  for (int64_t k = (int64_t)blockIdx.x * 1024 + threadIdx.x; k < n; k += stride) {
    const double* a = nullptr;
    const double* b = nullptr;
    int cnt = 0;
    if (k < p.num_images && with_f) {
      if (p.img_flags[k] & 1u) {
        a = p.qt + 8 * k;
        b = qt_c + 8 * k;
        cnt = 7;
      }
    } else if (k < nf_items) {
      const int64_t c = k - p.num_images;
      if (p.cam_var[c]) {
        a = p.cam + 8 * c;
        b = cam_c + 8 * c;
        cnt = num_params(p.cam_model[c]);
      }
    } else {
      const int64_t q = k - nf_items;
      if (p.pt_var[q]) {
        a = p.X + 3 * q;
        b = X_c + 3 * q;
        cnt = 3;
      }
    }
    for (int m = 0; m < cnt; ++m) {
      const double d = a[m] - b[m];
      vx += a[m] * a[m];
      vd += d * d;
    }
  }
  vx = wave_sum(vx);
  vd = wave_sum(vd);
  if ((threadIdx.x & 63) == 0) {
    sred[0][threadIdx.x >> 6] = vx;
    sred[1][threadIdx.x >> 6] = vd;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int k = 0; k < 16; ++k) s += sred[threadIdx.x][k];
    out[threadIdx.x * gridDim.x + blockIdx.x] = s;
  }
}

template <int CT>
__global__ __launch_bounds__(kBlock) void backsub_kernel(DevProblem p, const DevPoint* __restrict__ vp,
                                                          int64_t npv, const double* __restrict__ J,
                                                          const double* __restrict__ Vg,
                                                          const double* __restrict__ Vinv,
                                                          const double* __restrict__ df,
                                                          double* __restrict__ dX) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= npv) return;
  const DevPoint d = vp[k];
  const int W = 9 + CT;
  const double* g = Vg + 9 * (size_t)d.point + 6;
  double t[3] = {g[0], g[1], g[2]};
  for (uint32_t m = 0; m < d.count; ++m) {
    const uint32_t b = d.start + m;
    const double* Jb = J + (size_t)b * 2 * W;
    double e[2];
    load_jf_x<CT>(p, Jb, p.obs_img[b], df, e);
#pragma unroll
    for (int n = 0; n < 3; ++n) t[n] += Jb[6 + n] * e[0] + Jb[W + 6 + n] * e[1];
  }
  const double* vi = Vinv + 6 * (size_t)d.point;
  const double Vi[6] = {vi[0], vi[1], vi[2], vi[3], vi[4], vi[5]};
  double o[3];
  sym3_mul(Vi, t, o);
#pragma unroll
  for (int n = 0; n < 3; ++n) dX[3 * (size_t)d.point + n] = -o[n];
}

// Back substitution fused with the model cost change: one pass over a
// variable point's blocks gives e_a = J_f,a df, dX_p = -V_p^-1 (g_p + sum
// J_p,a' e_a), and the point's share of the model cost change
//   -sum_a [(J_a d).r_a + |J_a d|^2 / 2],  J_a d = e_a + J_p,a dX_p
//   = -(sum e.r + dX.g_p + sum |e|^2 / 2 + dX.sum J_p'e + dX' V_p dX / 2)
// (V_p, g_p undamped from point_normal), so J is read once instead of twice.
// Per-wave partials into partial[k / 64]; blocks of constant points are
// added by model_cost_const_kernel.
template <int CT>
__global__ __launch_bounds__(kBlock) void backsub_cost_kernel(DevProblem p, const DevPoint* __restrict__ vp,
                                                               int64_t npv, const double* __restrict__ J,
                                                               const double2* __restrict__ rr,
                                                               const double* __restrict__ Vg,
                                                               const double* __restrict__ Vinv,
                                                               const double* __restrict__ df,
                                                               double* __restrict__ dX,
                                                               double* __restrict__ partial) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double model = 0.0;
  if (k < npv) {
    const DevPoint d = vp[k];
    const int W = 9 + CT;
    const double* g = Vg + 9 * (size_t)d.point;
    double te[3] = {0.0, 0.0, 0.0};
    double see = 0.0, ser = 0.0;
    for (uint32_t m = 0; m < d.count; ++m) {
      const uint32_t b = d.start + m;
      const double* Jb = J + (size_t)b * 2 * W;
      double e[2];
      load_jf_x<CT>(p, Jb, p.obs_img[b], df, e);
      const double2 r = rr[b];
#pragma unroll
      for (int n = 0; n < 3; ++n) te[n] += Jb[6 + n] * e[0] + Jb[W + 6 + n] * e[1];
      see += e[0] * e[0] + e[1] * e[1];
      ser += e[0] * r.x + e[1] * r.y;
    }
    const double t[3] = {g[6] + te[0], g[7] + te[1], g[8] + te[2]};
    const double* vi = Vinv + 6 * (size_t)d.point;
    const double Vi[6] = {vi[0], vi[1], vi[2], vi[3], vi[4], vi[5]};
    double o[3];
    sym3_mul(Vi, t, o);
    const double x[3] = {-o[0], -o[1], -o[2]};
#pragma unroll
    for (int n = 0; n < 3; ++n) dX[3 * (size_t)d.point + n] = x[n];
    double Vx[3];
    sym3_mul(g, x, Vx);  // g[0..5] = V_p packed
    const double xg = x[0] * g[6] + x[1] * g[7] + x[2] * g[8];
    const double xte = x[0] * te[0] + x[1] * te[1] + x[2] * te[2];
    const double xVx = x[0] * Vx[0] + x[1] * Vx[1] + x[2] * Vx[2];
    model = -(ser + xg + see / 2.0 + xte + xVx / 2.0);
  }
  const double s = wave_sum(model);
  if ((threadIdx.x & 63) == 0 && k < npv) partial[k >> 6] = s;
}

// Back substitution + model cost change over point chunks (the default):
// chunk c = blocks [chunk[c], chunk[c+1]) of whole points (point-major), at
// most 64 blocks unless one point has more.  One lane per block: the wave
// stages 64 J rows in its LDS slab with coalesced loads (a lane walking its
// own point's rows touches a different line per lane and instruction: the
// per-point loop of backsub_cost_kernel ran 1.33 ms at C4), forms
// e = J_f df, the block's share -(e.r + |e|^2/2) of the model cost change and
// t_b = J_p' e; the first lane of each variable point sums its points' t_b in
// lane order (deterministic), then dX_p = -V_p^-1 (g_p + t) and the point's
// terms -(dX.g_p + dX.t + dX' V_p dX / 2).  Blocks of constant points only
// add their share.  One cost partial per chunk.
// PP: the implicit Schur product's point pass instead (x = the CG vector):
// w_p = V_p^-1 sum_a J_p,a' (J_f,a x), no cost terms (schur_point_pass's
// per-point loop, on chunks).
template <int CT, bool PP = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void backsub_chunk_kernel(DevProblem p, const uint32_t* __restrict__ chunk,
                                                                int nchunks, const double* __restrict__ J,
                                                                const double2* __restrict__ rr,
                                                                const double* __restrict__ Vg,
                                                                const double* __restrict__ Vinv,
                                                                const double* __restrict__ df,
                                                                double* __restrict__ dX,
                                                                double* __restrict__ partial) {
  constexpr int W = 9 + CT, W2 = 2 * W, LS = W2 | 1;
  // rows staged 32 at a time (7.9 KB per wave at OPENCV, 39 KB per
  // workgroup: four workgroups per CU; a 64-row slab allowed two)
  __shared__ double sl[(kBlock / 64) * 32 * LS];
  __shared__ double stv[kBlock / 64][64 * 3];
  __shared__ uint32_t spt[kBlock / 64][64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* slab = sl + wv * 32 * LS;
  double* tvs = stv[wv];
  uint32_t* wpt = spt[wv];
  const int c = blockIdx.x * (kBlock / 64) + wv;
  if (c >= nchunks) return;  // wave-uniform
  const uint32_t b0 = chunk[c], b1 = chunk[c + 1];
  const bool multi = b1 - b0 > 64u;  // one point with more than 64 blocks
  double model = 0.0;
  double carry[3] = {0.0, 0.0, 0.0};
  uint32_t carry_pt = 0;
  bool carry_var = false;
  auto finalize = [&](uint32_t pt, const double t[3]) {
    const double* vi = Vinv + 6 * (size_t)pt;
    if constexpr (PP) {
      const double Vi[6] = {vi[0], vi[1], vi[2], vi[3], vi[4], vi[5]};
      double wv[3];
      sym3_mul(Vi, t, wv);
#pragma unroll
      for (int n = 0; n < 3; ++n) dX[3 * (size_t)pt + n] = wv[n];
      return;
    }
    const double* g = Vg + 9 * (size_t)pt;
    const double Vi[6] = {vi[0], vi[1], vi[2], vi[3], vi[4], vi[5]};
    const double tt[3] = {g[6] + t[0], g[7] + t[1], g[8] + t[2]};
    double o[3];
    sym3_mul(Vi, tt, o);
    const double x[3] = {-o[0], -o[1], -o[2]};
#pragma unroll
    for (int n = 0; n < 3; ++n) dX[3 * (size_t)pt + n] = x[n];
    double Vx[3];
    sym3_mul(g, x, Vx);  // g[0..5] = V_p packed (undamped)
    model -= x[0] * g[6] + x[1] * g[7] + x[2] * g[8] + x[0] * t[0] + x[1] * t[1] + x[2] * t[2] +
             (x[0] * Vx[0] + x[1] * Vx[1] + x[2] * Vx[2]) / 2.0;
  };
  for (uint32_t s0 = b0; s0 < b1; s0 += 64) {
    const int live = (int)min(64u, b1 - s0);
    const bool on = lane < live;
    const uint32_t b = s0 + (on ? lane : 0);
    const uint32_t pt = p.obs_pt[b];
    const bool var = on && p.pt_var[pt] != 0;
    double te[3] = {0.0, 0.0, 0.0};
    // each half: lane l takes residual row l / 32 of block l % 32; the two
    // rows' t terms meet by a cross-half swizzle at the block's own lane
    const int bi = lane & 31, rw = lane >> 5;
    for (int h = 0; h < 2; ++h) {
      const int live_h = min(32, live - 32 * h);
      if (live_h <= 0) break;  // wave-uniform
      wave_load_rows_u<W2, LS, 32>(J + (size_t)(s0 + 32 * h) * W2, slab, live_h);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      double tr[3] = {0.0, 0.0, 0.0};
      if (bi < live_h) {
        const uint32_t bb = s0 + 32 * h + bi;
        const double* row = slab + bi * LS + rw * W;
        const uint32_t img = p.obs_img[bb];
        const double* xi = df + 6 * (size_t)img;
        const double* xc = df + 6 * (size_t)p.num_images + (size_t)CT * p.img_cam[img];
        double e = 0.0;
#pragma unroll
        for (int m = 0; m < 6; ++m) e += row[m] * xi[m];
#pragma unroll
        for (int m = 0; m < CT; ++m) e += row[9 + m] * xc[m];
        if constexpr (!PP) {
          const double2 r = rr[bb];
          model -= e * (rw ? r.y : r.x) + e * e / 2.0;
        }
#pragma unroll
        for (int n = 0; n < 3; ++n) tr[n] = row[6 + n] * e;
      }
#pragma unroll
      for (int n = 0; n < 3; ++n) {
        const double o = __shfl_xor(tr[n], 32);
        if (rw == h) te[n] = tr[n] + o;  // row 0 + row 1
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    if (!var) te[0] = te[1] = te[2] = 0.0;
    // segmented sum: t_b and the point id per lane
    double* tv = tvs + lane * 3;
    tv[0] = te[0];
    tv[1] = te[1];
    tv[2] = te[2];
    wpt[lane] = on ? pt : 0xffffffffu;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const bool head = var && (lane == 0 || wpt[lane - 1] != pt);
    if (head) {
      double t[3] = {te[0], te[1], te[2]};
      for (int l = lane + 1; l < live && wpt[l] == pt; ++l) {
        t[0] += tvs[l * 3];
        t[1] += tvs[l * 3 + 1];
        t[2] += tvs[l * 3 + 2];
      }
      if (multi) {
        carry[0] += t[0];
        carry[1] += t[1];
        carry[2] += t[2];
        carry_pt = pt;
        carry_var = true;
      } else {
        finalize(pt, t);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  if (multi && carry_var) finalize(carry_pt, carry);  // lane 0
  if constexpr (!PP) {
    const double s = wave_sum(model);
    if (lane == 0) partial[c] = s;
  }
}

// Model cost change of the blocks of constant points (no point step).
template <int CT>
__global__ __launch_bounds__(kBlock) void model_cost_const_kernel(DevProblem p, const double2* __restrict__ rr,
                                                                   const double* __restrict__ J,
                                                                   const double* __restrict__ df,
                                                                   double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double v = 0.0;
  bool any = false;
  if (i < p.nb && !p.pt_var[p.obs_pt[i]]) {
    const double* Jb = J + (size_t)i * 2 * (9 + CT);
    double e[2];
    load_jf_x<CT>(p, Jb, p.obs_img[i], df, e);
    const double2 r = rr[i];
    v = -(e[0] * (r.x + e[0] / 2.0) + e[1] * (r.y + e[1] / 2.0));
    any = true;
  }
  const double s = wave_sum(v);
  const bool wave_any = __any(any);  // voted with every lane active
  if ((threadIdx.x & 63) == 0 && wave_any) atomicAdd(out, s);
}

template <int CT>
__global__ __launch_bounds__(kBlock) void model_cost_kernel(DevProblem p, const double2* __restrict__ rr,
                                                             const double* __restrict__ J,
                                                             const double* __restrict__ df,
                                                             const double* __restrict__ dX,
                                                             double* __restrict__ partial) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double v = 0.0;
  if (i < p.nb) {
    const int W = 9 + CT;
    const double* Jb = J + (size_t)i * 2 * W;
    double e[2];
    load_jf_x<CT>(p, Jb, p.obs_img[i], df, e);
    const uint32_t pt = p.obs_pt[i];
    if (p.pt_var[pt]) {
      const double dx[3] = {dX[3 * (size_t)pt], dX[3 * (size_t)pt + 1], dX[3 * (size_t)pt + 2]};
#pragma unroll
      for (int row = 0; row < 2; ++row)
        e[row] += Jb[row * W + 6] * dx[0] + Jb[row * W + 7] * dx[1] + Jb[row * W + 8] * dx[2];
    }
    const double2 r = rr[i];
    v = -(e[0] * (r.x + e[0] / 2.0) + e[1] * (r.y + e[1] / 2.0));
  }
  const double s = wave_sum(v);  // per-wave partial (reproj_grid)
  if ((threadIdx.x & 63) == 0 && i < p.nb) partial[i >> 6] = s;
}

__global__ void plus_images_kernel(DevProblem p, const double* __restrict__ df, const double* __restrict__ qt,
                                   double* __restrict__ qt_out) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= p.num_images) return;
  const double* a = qt + 8 * (size_t)k;
  double* o = qt_out + 8 * (size_t)k;
  if (!(p.img_flags[k] & 1u)) {
    for (int m = 0; m < 8; ++m) o[m] = a[m];
    return;
  }
  const double* d = df + 6 * (size_t)k;
  const double q[4] = {a[0], a[1], a[2], a[3]};
  const double dr[3] = {d[0], d[1], d[2]};
  double qn[4];
  quat_plus(q, dr, qn);
  o[0] = qn[0]; o[1] = qn[1]; o[2] = qn[2]; o[3] = qn[3];
  o[4] = a[4] + d[3];
  o[5] = a[5] + d[4];
  o[6] = a[6] + d[5];
  o[7] = 0.0;
}

__global__ void plus_cameras_kernel(DevProblem p, const double* __restrict__ df, const double* __restrict__ cam,
                                    double* __restrict__ cam_out) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= p.num_cameras) return;
  const double* a = cam + 8 * (size_t)k;
  double* o = cam_out + 8 * (size_t)k;
  for (int m = 0; m < 8; ++m) o[m] = a[m];
  if (!p.cam_var[k]) return;
  // the camera's refined intrinsics, in parameter order, occupy the first
  // slots of its p.ct-wide block (SubsetManifold::Plus)
  const double* d = df + 6 * (size_t)p.num_images + (size_t)p.ct * k;
  const unsigned cm = cam_tangent_mask(p.cam_model[k], p.refine_mask);
  int c = 0;
  for (int m = 0; m < 8; ++m)
    if ((cm >> m) & 1u) {
      o[m] = a[m] + d[c];
      ++c;
    }
}

__global__ void plus_points_kernel(DevProblem p, const double* __restrict__ dX, const double* __restrict__ X,
                                   double* __restrict__ X_out) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= p.num_points) return;
  const bool var = p.pt_var[k] != 0;
#pragma unroll
  for (int m = 0; m < 3; ++m) X_out[3 * k + m] = X[3 * k + m] + (var ? dX[3 * k + m] : 0.0);
}

// |a|^2 + |b|^2; with gridDim.x > 1 every workgroup writes its partial to
// out[blockIdx.x] (a second one-workgroup launch, sum_kernel, adds them in a
// fixed order: deterministic).
__global__ __launch_bounds__(1024) void sqnorm2_kernel(const double* __restrict__ a, int64_t na,
                                                       const double* __restrict__ b, int64_t nb2,
                                                       double* __restrict__ out) {
  __shared__ double sred[16];
  double v = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 1024;
  for (int64_t k = (int64_t)blockIdx.x * 1024 + threadIdx.x; k < na; k += stride) v += a[k] * a[k];
  for (int64_t k = (int64_t)blockIdx.x * 1024 + threadIdx.x; k < nb2; k += stride) v += b[k] * b[k];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int k = 0; k < 16; ++k) s += sred[k];
    out[blockIdx.x] = s;
  }
}

// ---------------------------------------------------------------------------
// Explicit reduced camera system S = U + Lambda - sum_p W_p V_p^-1 W_p'
// (the system Ceres' DENSE_SCHUR / SPARSE_SCHUR factorise exactly).
// ---------------------------------------------------------------------------

// U = sum J_f' J_f, reduced per image-aligned tile (one flush per tile).
template <int CT>
__global__ __launch_bounds__(kBlock) void dense_u_kernel(DevProblem p, const DevTile* __restrict__ tiles,
                                                          const uint32_t* __restrict__ cm_perm,
                                                          const double* __restrict__ J, double* __restrict__ S) {
  constexpr int F = 6 + CT;
  constexpr int NV = F * (F + 1) / 2;
  __shared__ double sred[4 * NV];
  const DevTile tile = tiles[blockIdx.x];
  const int W = 9 + CT;
  double acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.0;
  for (uint32_t k = threadIdx.x; k < tile.count; k += kBlock) {
    const uint32_t b = cm_perm[tile.start + k];
    const double* Jb = J + (size_t)b * 2 * W;
    double jf[2][F];
#pragma unroll
    for (int row = 0; row < 2; ++row) {
#pragma unroll
      for (int m = 0; m < 6; ++m) jf[row][m] = Jb[row * W + m];
#pragma unroll
      for (int m = 0; m < CT; ++m) jf[row][6 + m] = Jb[row * W + 9 + m];
    }
    int o = 0;
#pragma unroll
    for (int a = 0; a < F; ++a)
#pragma unroll
      for (int c = a; c < F; ++c, ++o) acc[o] += jf[0][a] * jf[0][c] + jf[1][a] * jf[1][c];
  }
  block_reduce<NV>(acc, sred);
  const int k = threadIdx.x;
  if (k < NV) {
    int a = 0, rem = k;
    while (rem >= F - a) { rem -= F - a; ++a; }
    const int c = a + rem;
    const uint32_t img = tile.image, cam = p.img_cam[img];
    const bool pv = p.img_flags[img] & 1u, cv = p.cam_var[cam] != 0;
    const bool va = a < 6 ? pv : cv, vc = c < 6 ? pv : cv;
    if (va && vc) {
      const int64_t ra = fslot(p, img, cam, a), rc = fslot(p, img, cam, c);
      const double v = sred[k];
      // upper triangle (row <= col) only: rocSOLVER reads the column-major lower
      if (ra <= rc)
        atomicAdd(S + ra * p.lds + rc, v);
      else
        atomicAdd(S + rc * p.lds + ra, v);
    }
  }
}

// ---------------------------------------------------------------------------
// Explicit reduced camera system, Schur term.
//
// S -= sum_p W_p V_p^-1 W_p' is accumulated per image pair: with the damped
// point block factored as V^-1 = Linv' Linv, every observation a carries
// Z_a = W_a Linv' (F x 3, W_a = J_f,a' J_p,a), and the image-pair block is
// S_ij -= sum over co-observed points of Z_a Z_b'.  That is a GEMM with
// K = 3 per pair: one v_mfma_f64_16x16x4f64 per pair (F <= 14 padded to 16,
// K = 3 padded to 4) over a bucketed pair list built once at setup.
// ---------------------------------------------------------------------------

// Z_a (k-major: Z[b][k*F + m]) of every block of a variable point; zero for
// blocks of constant points.  J rows are read and Z rows written through the
// wave's LDS slab (coalesced 8-B-per-lane transfers).
// PERM (zorder 1): Z's row i is the block at camera-major position i
// (cm_perm[i]; its J row gathered), so one image's Z rows are one contiguous
// range and a pair tile's gathers stay inside two such ranges.
template <int CT, bool PERM = false>
__global__ __launch_bounds__(kBlock) void schur_z_kernel(DevProblem p, const double* __restrict__ J,
                                                          const double* __restrict__ Linv, double* __restrict__ Z,
                                                          const uint32_t* __restrict__ cm_perm = nullptr,
                                                          const uint32_t* __restrict__ cm_ptv = nullptr) {
  constexpr int F = 6 + CT, W = 9 + CT, W2 = 2 * W, LS = W2 | 1;
  constexpr int ZN = 3 * F, ZS = ZN | 1;
  constexpr int SL = (LS > ZS ? LS : ZS) * 64;
  __shared__ double sl[(kBlock / 64) * SL];
  double* slab = sl + (threadIdx.x >> 6) * SL;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t wb0 = i - lane;
  const int live = wb0 >= p.nb ? 0 : (p.nb - wb0 < 64 ? (int)(p.nb - wb0) : 64);
  if constexpr (PERM)
    wave_gather_rows_u<W2, LS, 64>(J, i < p.nb ? cm_perm[i] : 0u, slab, live);
  else
    wave_load_rows_u<W2, LS, 64>(J + wb0 * W2, slab, live);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  double jf[2][F], jp[2][3];
  {
    const double* row = slab + lane * LS;
#pragma unroll
    for (int rw = 0; rw < 2; ++rw) {
#pragma unroll
      for (int m = 0; m < 6; ++m) jf[rw][m] = row[rw * W + m];
#pragma unroll
      for (int m = 0; m < 3; ++m) jp[rw][m] = row[rw * W + 6 + m];
#pragma unroll
      for (int m = 0; m < CT; ++m) jf[rw][6 + m] = row[rw * W + 9 + m];
    }
  }
  double L[6] = {0, 0, 0, 0, 0, 0};
  if (i < p.nb) {
    if constexpr (PERM) {
      const uint32_t pt = cm_ptv[i];
      if (pt != 0xffffffffu) {
#pragma unroll
        for (int m = 0; m < 6; ++m) L[m] = Linv[6 * (size_t)pt + m];
      }
    } else {
      const uint32_t pt = p.obs_pt[i];
      if (p.pt_var[pt]) {
#pragma unroll
        for (int m = 0; m < 6; ++m) L[m] = Linv[6 * (size_t)pt + m];
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  double* zr = slab + lane * ZS;
#pragma unroll
  for (int m = 0; m < F; ++m) {
    const double w0 = jf[0][m] * jp[0][0] + jf[1][m] * jp[1][0];
    const double w1 = jf[0][m] * jp[0][1] + jf[1][m] * jp[1][1];
    const double w2 = jf[0][m] * jp[0][2] + jf[1][m] * jp[1][2];
    zr[m] = w0 * L[0];
    zr[F + m] = w0 * L[1] + w1 * L[2];
    zr[2 * F + m] = w0 * L[3] + w1 * L[4] + w2 * L[5];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  wave_readout<ZN, ZS, ZN>(slab, Z + wb0 * ZN, live);
}

// Store one pair tile's 16 x 16 accumulator (the v_mfma_f64_16x16x4f64 D
// layout) into S: through the deterministic route's partial slot, as the S
// block's only writer, or by float atomics (pf.pslot null).
template <int F>
__device__ __forceinline__ void pair_tile_store(const DevProblem& p, const DevPairTile& tl, int t, int lane,
                                                const double (&acc)[4], double* __restrict__ S, const PairFlush& pf) {
  if (pf.pslot) {
    const int32_t ps = pf.pslot[t];
    if (ps >= 0) {  // summed with the block's other tiles (schur_pairs_flush_kernel)
#pragma unroll
      for (int r = 0; r < 4; ++r) pf.part[(size_t)ps * 256 + r * 64 + lane] = acc[r];
      return;
    }
  }
  const uint32_t ia = tl.ia, ib = tl.ib;
  const uint32_t ca = p.img_cam[ia], cb = p.img_cam[ib];
  const bool pa = p.img_flags[ia] & 1u, pb = p.img_flags[ib] & 1u;
  const bool cva = p.cam_var[ca] != 0, cvb = p.cam_var[cb] != 0;
  const int ncol = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int mrow = 4 * r + (lane >> 4);  // v_mfma_f64_16x16x4f64 D layout (measured): D[4r + l/16][l%16]
    if (mrow >= F || ncol >= F) continue;
    const bool va = mrow < 6 ? pa : cva, vb = ncol < 6 ? pb : cvb;
    if (!va || !vb) continue;
    const int64_t ra = fslot(p, ia, ca, mrow), rb = fslot(p, ib, cb, ncol);
    const double v = acc[r];
    if (pf.pslot) {  // the block's only tile (ia != ib, cameras not shared): ra != rb, one writer
      double* e = S + (ra < rb ? ra * p.lds + rb : rb * p.lds + ra);
      *e -= v;
      continue;
    }
    if (tl.self) {
      if (ra <= rb) atomicAdd(S + ra * p.lds + rb, -v);
    } else if (ra < rb) {
      atomicAdd(S + ra * p.lds + rb, -v);
    } else if (ra > rb) {
      atomicAdd(S + rb * p.lds + ra, -v);
    } else {
      atomicAdd(S + ra * p.lds + ra, -2.0 * v);
    }
  }
}

// One wavefront per image-pair tile: acc = sum over the tile's pairs of
// Z_a Z_b' (16x16 f64 MFMA accumulator), then -acc into the upper triangle
// (row <= col, row-major = rocSOLVER's column-major lower) of S.
// Cross tiles hold pairs a != b: a mirrored entry lands on the same upper
// element, a diagonal one counts twice.  Self tiles hold a == b.
// XMAP: XCD-aware order — workgroup b runs on XCD b % 8; each XCD gets a
// contiguous range of tiles (tiles sorted by first image, so one image's Z
// rows stay in that XCD's L2 while its pairs stream by).  Else dispatch order
// (image-block-ordered tiles: every XCD sweeps the same image block at once).
// NTB: second-image (b-side) rows loaded nontemporal, so the streaming b-side
// does not evict the first image's rows an XCD keeps in its L2 (variant 5).
template <int CT, bool XMAP = true, bool NTB = false, bool SELF1 = false>
__global__ __launch_bounds__(kBlock) void schur_pairs_kernel(DevProblem p, const DevPairTile* __restrict__ tiles,
                                                              int ntiles, const uint2* __restrict__ pairs,
                                                              const double* __restrict__ Z, double* __restrict__ S,
                                                              PairFlush pf) {
  constexpr int F = 6 + CT, ZN = 3 * F;
  const int G = (ntiles + 3) / 4;
  const int per = (G + 7) / 8;
  const int b = blockIdx.x;
  const int lb = XMAP ? (b % 8) * per + b / 8 : b;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = lb * 4 + wv;
  if (lb >= G || t >= ntiles) return;
  const DevPairTile tl = tiles[t];
  if (tl.count == 0) return;  // padding tile (variant 5)
  const int lane = threadIdx.x & 63;
  const int m = lane & 15, k = lane >> 4;
  const bool on = m < F && k < 3;
  const int off = on ? k * F + m : 0;
  typedef double dvec4 __attribute__((ext_vector_type(4)));
  dvec4 acc = {0.0, 0.0, 0.0, 0.0};
  const uint32_t cnt = tl.count;
  const uint2* pl = pairs + tl.start;
  uint32_t n = 0;
  if (tl.self && SELF1) {
    // self tile: a == b, one load per pair (a branch-free form of these
    // loops, 8 pairs' loads issued behind one scalar load of their indices,
    // measured the same: 5.15 ms, profiles/r6i_ab_schur_pairs_self_flat.log)
    for (; n + 4 <= cnt; n += 4) {
      uint32_t pa[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) pa[u] = pl[n + u].x;
      double va[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) va[u] = on ? Z[(size_t)pa[u] * ZN + off] : 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va[u], va[u], acc, 0, 0, 0);
    }
  }
  for (; n + 4 <= cnt; n += 4) {
    uint2 pr[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) pr[u] = pl[n + u];
    double va[4], vb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      va[u] = on ? Z[(size_t)pr[u].x * ZN + off] : 0.0;
      if constexpr (NTB)
        vb[u] = on ? __builtin_nontemporal_load(Z + (size_t)pr[u].y * ZN + off) : 0.0;
      else
        vb[u] = on ? Z[(size_t)pr[u].y * ZN + off] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va[u], vb[u], acc, 0, 0, 0);
  }
  for (; n < cnt; ++n) {
    const uint2 pr = pl[n];
    const double va = on ? Z[(size_t)pr.x * ZN + off] : 0.0;
    double vb = 0.0;
    if constexpr (NTB)
      vb = on ? __builtin_nontemporal_load(Z + (size_t)pr.y * ZN + off) : 0.0;
    else
      vb = on ? Z[(size_t)pr.y * ZN + off] : 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va, vb, acc, 0, 0, 0);
  }
  const double accv[4] = {acc[0], acc[1], acc[2], acc[3]};
  pair_tile_store<F>(p, tl, t, lane, accv, S, pf);
}

// Z_a's entry (k, m) formed from block a's J row and its point's Linv, with
// schur_z_kernel's operation sequence: W_a = J_f,a' J_p,a (column m of the
// camera side: pose 0..5 at J columns 0..5, intrinsics at 9..), Z_a = W_a
// Linv'.  row: the block's 2 x W J rows; L: the packed lower Linv (zero for a
// constant point).
template <int W>
__device__ __forceinline__ double z_from_j(const double* __restrict__ row, int col, int k, const double (&L)[6]) {
  const double a0 = row[col], a1 = row[W + col];
  const double w0 = a0 * row[6] + a1 * row[W + 6];
  if (k == 0) return w0 * L[0];
  const double w1 = a0 * row[7] + a1 * row[W + 7];
  if (k == 1) return w0 * L[1] + w1 * L[2];
  const double w2 = a0 * row[8] + a1 * row[W + 8];
  return w0 * L[3] + w1 * L[4] + w2 * L[5];
}

// schur_pairs_variant 7: schur_pairs_kernel without the Z pass — each pair's
// two Z rows are formed in registers from the blocks' J rows (240 B each at
// OPENCV instead of Z's 288 B) and the point's Linv (48 B, shared by the
// pair), so neither Z's 2.9 GB write nor schur_z_kernel's J read happens.
// Dispatch-order tiles (the image-block order of svariant 4).
template <int CT>
__global__ __launch_bounds__(kBlock) void schur_pairs_j_kernel(DevProblem p, const DevPairTile* __restrict__ tiles,
                                                                int ntiles, const uint2* __restrict__ pairs,
                                                                const double* __restrict__ J,
                                                                const double* __restrict__ Linv,
                                                                double* __restrict__ S, PairFlush pf) {
  constexpr int F = 6 + CT, W = 9 + CT, W2 = 2 * W;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = blockIdx.x * 4 + wv;
  if (t >= ntiles) return;
  const DevPairTile tl = tiles[t];
  if (tl.count == 0) return;
  const int lane = threadIdx.x & 63;
  const int m = lane & 15, k = lane >> 4;
  const bool on = m < F && k < 3;
  const int col = m < 6 ? m : 3 + m;  // J column of camera-side tangent m (pose 0..5, intrinsics 9..)
  typedef double dvec4 __attribute__((ext_vector_type(4)));
  dvec4 acc = {0.0, 0.0, 0.0, 0.0};
  const uint32_t cnt = tl.count;
  const uint2* pl = pairs + tl.start;
  constexpr int U = 2;
  uint32_t n = 0;
  for (; n + U <= cnt; n += U) {
    uint2 pr[U];
    uint32_t pt[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      pr[u] = pl[n + u];
      pt[u] = p.obs_pt[pr[u].x];
    }
    double L[U][6];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool v = p.pt_var[pt[u]] != 0;
#pragma unroll
      for (int q = 0; q < 6; ++q) L[u][q] = v ? Linv[6 * (size_t)pt[u] + q] : 0.0;
    }
    double va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va[u] = on ? z_from_j<W>(J + (size_t)pr[u].x * W2, col, k, L[u]) : 0.0;
      vb[u] = on ? z_from_j<W>(J + (size_t)pr[u].y * W2, col, k, L[u]) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va[u], vb[u], acc, 0, 0, 0);
  }
  for (; n < cnt; ++n) {
    const uint2 pr = pl[n];
    const uint32_t pt = p.obs_pt[pr.x];
    double L[6];
    const bool v = p.pt_var[pt] != 0;
#pragma unroll
    for (int q = 0; q < 6; ++q) L[q] = v ? Linv[6 * (size_t)pt + q] : 0.0;
    const double va = on ? z_from_j<W>(J + (size_t)pr.x * W2, col, k, L) : 0.0;
    const double vb = on ? z_from_j<W>(J + (size_t)pr.y * W2, col, k, L) : 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va, vb, acc, 0, 0, 0);
  }
  const double accv[4] = {acc[0], acc[1], acc[2], acc[3]};
  pair_tile_store<F>(p, tl, t, lane, accv, S, pf);
}

// The pair tiles' partial blocks summed per S block in list order and
// subtracted (one workgroup per block, thread (m, n) of the 16 x 16 tile).
// Diagonal blocks (ia == ib) take the upper triangle: a self tile's Z_a Z_a'
// as is, a same-image tile's Z_a Z_b' + its transpose (a pair a != b of one
// image lands on both (m, n) and (n, m)).  Cameras are not shared (the
// condition of the deterministic route), so every (m, n) of an off-diagonal
// block is a distinct S element.
__device__ inline int mfma_d_index(int m, int n) { return (m >> 2) * 64 + ((m & 3) << 4) + n; }

template <int CT>
__global__ __launch_bounds__(256) void schur_pairs_flush_kernel(DevProblem p, PairFlush pf, double* __restrict__ S) {
  constexpr int F = 6 + CT;
  const uint4 d = pf.dest[blockIdx.x];
  const int m = threadIdx.x >> 4, n = threadIdx.x & 15;
  if (m >= F || n >= F) return;
  const uint32_t ia = d.x, ib = d.y;
  if (ia == ib && m > n) return;
  double v = 0.0;
  for (uint32_t k = 0; k < d.w; ++k) {
    const double* a = pf.part + (size_t)(d.z + k) * 256;
    v += (ia == ib && !pf.self[d.z + k]) ? a[mfma_d_index(m, n)] + a[mfma_d_index(n, m)] : a[mfma_d_index(m, n)];
  }
  const uint32_t ca = p.img_cam[ia], cb = p.img_cam[ib];
  const bool va = m < 6 ? (p.img_flags[ia] & 1u) : p.cam_var[ca] != 0;
  const bool vb = n < 6 ? (p.img_flags[ib] & 1u) : p.cam_var[cb] != 0;
  if (!va || !vb) return;
  const int64_t ra = fslot(p, ia, ca, m), rb = fslot(p, ib, cb, n);
  S[ra <= rb ? ra * p.lds + rb : rb * p.lds + ra] -= v;
}

// Shared cameras (PairFlush::odest): one workgroup per run of an owner
// pair's entries, thread (i, j) = element (X_i, Y_j) of the owner-pair block
// (X_i the owner's i-th slot: pose 0..5 or camera 0..ct-1): the run's tile
// partials summed in entry order into opart[run][8 i + j].  A quadrant whose
// owners were swapped contributes its transposed element; an owner paired
// with itself takes the upper triangle, a tile of a != b pairs contributing
// both mirrored entries (twice on the diagonal), a self tile its upper one.
__device__ inline double owner_quadrant_value(const double* __restrict__ g, uint32_t e, int i, int j, bool same) {
  const int q = (e >> 2) & 3;
  const int ro = (q & 2) ? 6 : 0, co = (q & 1) ? 6 : 0;
  const bool sw = (e >> 1) & 1, self = e & 1;
  if (!same) return sw ? g[mfma_d_index(ro + j, co + i)] : g[mfma_d_index(ro + i, co + j)];
  if (self) return g[mfma_d_index(ro + i, co + j)];
  return i == j ? 2.0 * g[mfma_d_index(ro + i, co + i)] : g[mfma_d_index(ro + i, co + j)] + g[mfma_d_index(ro + j, co + i)];
}

__global__ __launch_bounds__(64) void schur_owner_chunk_kernel(DevProblem p, PairFlush pf) {
  const uint4 c = pf.ochunk[blockIdx.x];
  const uint4 d = pf.odest[c.x];
  const int i = threadIdx.x >> 3, j = threadIdx.x & 7;
  const int nx = (d.x & kOwnerCam) ? p.ct : 6, ny = (d.y & kOwnerCam) ? p.ct : 6;
  const bool same = d.x == d.y;
  double v = 0.0;
  if (i < nx && j < ny && !(same && i > j)) {
    for (uint32_t k = 0; k < c.z; ++k) {
      const uint32_t e = pf.oent[c.y + k];
      v += owner_quadrant_value(pf.part + (size_t)(e >> 4) * 256, e, i, j, same);
    }
  }
  pf.opart[(size_t)blockIdx.x * 64 + threadIdx.x] = v;
}

// The owner pair's runs added in run order and subtracted from S once
// (variable owners only: a constant pose or camera has no S slots in use).
__global__ __launch_bounds__(64) void schur_owner_flush_kernel(DevProblem p, PairFlush pf, double* __restrict__ S) {
  const uint4 d = pf.odest[blockIdx.x];
  const int i = threadIdx.x >> 3, j = threadIdx.x & 7;
  const bool xc = d.x & kOwnerCam, yc = d.y & kOwnerCam;
  const uint32_t xi = d.x & ~kOwnerCam, yi = d.y & ~kOwnerCam;
  const int nx = xc ? p.ct : 6, ny = yc ? p.ct : 6;
  if (i >= nx || j >= ny || (d.x == d.y && i > j)) return;
  if (!(xc ? p.cam_var[xi] != 0 : (p.img_flags[xi] & 1u)) || !(yc ? p.cam_var[yi] != 0 : (p.img_flags[yi] & 1u))) return;
  double v = 0.0;
  for (uint32_t k = 0; k < d.w; ++k) v += pf.opart[(size_t)(d.z + k) * 64 + threadIdx.x];
  const int64_t ra = xc ? fslot(p, 0, xi, 6 + i) : fslot(p, xi, 0, i);
  const int64_t rb = yc ? fslot(p, 0, yi, 6 + j) : fslot(p, yi, 0, j);
  S[ra <= rb ? ra * p.lds + rb : rb * p.lds + ra] -= v;
}

// schur_pairs_variant 6: per block the record JG_a = [J_f,a (2 x F, row-major),
// G_a = Linv J_p,a' (3 x 2), zero pad] of jg_width(F) doubles (256 B at F <=
// 13: two aligned 128-B lines, where a Z row of 3 F doubles spans three), so
// that Z_a Z_b' = J_f,a' (G_a' G_b) J_f,b: a pair's two records cost four line
// requests instead of six.
__host__ __device__ constexpr int jg_width(int F) { return ((2 * F + 6 + 15) / 16) * 16; }

template <int CT>
__global__ __launch_bounds__(kBlock) void schur_jg_kernel(DevProblem p, const double* __restrict__ J,
                                                           const double* __restrict__ Linv, double* __restrict__ JG) {
  constexpr int F = 6 + CT, W = 9 + CT, W2 = 2 * W, LS = W2 | 1;
  constexpr int RW = jg_width(F), RS = RW | 1;
  constexpr int SL = (LS > RS ? LS : RS) * 64;
  __shared__ double sl[(kBlock / 64) * SL];
  double* slab = sl + (threadIdx.x >> 6) * SL;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t wb0 = i - lane;
  const int live = wb0 >= p.nb ? 0 : (p.nb - wb0 < 64 ? (int)(p.nb - wb0) : 64);
  wave_load_rows_u<W2, LS, 64>(J + wb0 * W2, slab, live);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  double jf[2][F], jp[2][3];
  {
    const double* row = slab + lane * LS;
#pragma unroll
    for (int rw = 0; rw < 2; ++rw) {
#pragma unroll
      for (int m = 0; m < 6; ++m) jf[rw][m] = row[rw * W + m];
#pragma unroll
      for (int m = 0; m < 3; ++m) jp[rw][m] = row[rw * W + 6 + m];
#pragma unroll
      for (int m = 0; m < CT; ++m) jf[rw][6 + m] = row[rw * W + 9 + m];
    }
  }
  double L[6] = {0, 0, 0, 0, 0, 0};
  if (i < p.nb) {
    const uint32_t pt = p.obs_pt[i];
    if (p.pt_var[pt]) {
#pragma unroll
      for (int m = 0; m < 6; ++m) L[m] = Linv[6 * (size_t)pt + m];
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  double* o = slab + lane * RS;
#pragma unroll
  for (int rw = 0; rw < 2; ++rw)
#pragma unroll
    for (int m = 0; m < F; ++m) o[rw * F + m] = jf[rw][m];
#pragma unroll
  for (int rw = 0; rw < 2; ++rw) {
    o[2 * F + rw] = L[0] * jp[rw][0];
    o[2 * F + 2 + rw] = L[1] * jp[rw][0] + L[2] * jp[rw][1];
    o[2 * F + 4 + rw] = L[3] * jp[rw][0] + L[4] * jp[rw][1] + L[5] * jp[rw][2];
  }
#pragma unroll
  for (int m = 2 * F + 6; m < RW; ++m) o[m] = 0.0;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  wave_readout<RW, RS, RW>(slab, JG + wb0 * RW, live);
}

// Variant 6 of schur_pairs_kernel: two pairs per v_mfma_f64_16x16x4f64 (K
// slots 0, 1 the first pair's two residual rows, 2, 3 the second's), per
// pair acc += J_f,a' T with T = (G_a' G_b) J_f,b: lane (m, k) loads J_f,a[k
// & 1][m] and J_f,b[0..1][m]; the pairs' G blocks are wave-uniform.
template <int CT>
__global__ __launch_bounds__(kBlock) void schur_pairs_jg_kernel(DevProblem p, const DevPairTile* __restrict__ tiles,
                                                                 int ntiles, const uint2* __restrict__ pairs,
                                                                 const double* __restrict__ JG,
                                                                 double* __restrict__ S) {
  constexpr int F = 6 + CT, RW = jg_width(F);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = blockIdx.x * 4 + wv;
  if (t >= ntiles) return;
  const DevPairTile tl = tiles[t];
  if (tl.count == 0) return;
  const int lane = threadIdx.x & 63;
  const int m = lane & 15, k = lane >> 4;
  const int slot = k >> 1, r = k & 1;
  const bool on = m < F;
  const int mm = on ? m : 0;
  typedef double dvec4 __attribute__((ext_vector_type(4)));
  dvec4 acc = {0.0, 0.0, 0.0, 0.0};
  const uint32_t cnt = tl.count;
  const uint2* pl = pairs + tl.start;
#pragma unroll 2
  for (uint32_t n = 0; n < cnt; n += 2) {
    const uint2 pa = pl[n];
    const bool two = n + 1 < cnt;
    const uint2 pb = two ? pl[n + 1] : pa;
    // wave-uniform: both pairs' G blocks
    const uint32_t a0 = __builtin_amdgcn_readfirstlane(pa.x), b0 = __builtin_amdgcn_readfirstlane(pa.y);
    const uint32_t a1 = __builtin_amdgcn_readfirstlane(pb.x), b1 = __builtin_amdgcn_readfirstlane(pb.y);
    const double* ga = JG + (size_t)(slot ? a1 : a0) * RW;
    const double* gb = JG + (size_t)(slot ? b1 : b0) * RW;
    // this lane's row r of M = G_a' G_b (2 x 2): M[r][s] = sum_c G_a[c][r] G_b[c][s]
    const double g0 = ga[2 * F + r], g1 = ga[2 * F + 2 + r], g2 = ga[2 * F + 4 + r];
    const double m0 = g0 * gb[2 * F] + g1 * gb[2 * F + 2] + g2 * gb[2 * F + 4];
    const double m1 = g0 * gb[2 * F + 1] + g1 * gb[2 * F + 3] + g2 * gb[2 * F + 5];
    const double va = ga[r * F + mm];
    const double vb = m0 * gb[mm] + m1 * gb[F + mm];
    const bool use = on && (slot == 0 || two);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(use ? va : 0.0, use ? vb : 0.0, acc, 0, 0, 0);
  }
  const uint32_t ia = tl.ia, ib = tl.ib;
  const uint32_t ca = p.img_cam[ia], cb = p.img_cam[ib];
  const bool pa_ = p.img_flags[ia] & 1u, pb_ = p.img_flags[ib] & 1u;
  const bool cva = p.cam_var[ca] != 0, cvb = p.cam_var[cb] != 0;
  const int ncol = lane & 15;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int mrow = 4 * q + (lane >> 4);  // v_mfma_f64_16x16x4f64 D layout: D[4q + l/16][l%16]
    if (mrow >= F || ncol >= F) continue;
    const bool va_ = mrow < 6 ? pa_ : cva, vb_ = ncol < 6 ? pb_ : cvb;
    if (!va_ || !vb_) continue;
    const int64_t ra = fslot(p, ia, ca, mrow), rb = fslot(p, ib, cb, ncol);
    const double v = acc[q];
    if (tl.self) {
      if (ra <= rb) atomicAdd(S + ra * p.lds + rb, -v);
    } else if (ra < rb) {
      atomicAdd(S + ra * p.lds + rb, -v);
    } else if (ra > rb) {
      atomicAdd(S + rb * p.lds + ra, -v);
    } else {
      atomicAdd(S + ra * p.lds + ra, -2.0 * v);
    }
  }
}

// schur_pairs_variant 8: the JG records of variant 6 (one 256-B record per
// block at F <= 13: J_f (2 x F) and G = Linv J_p' (3 x 2)), one pair per
// v_mfma_f64_16x16x4f64 with K = 2 (the residual rows; K slots 2, 3 zero):
// acc += J_f,a' (M J_f,b), M = G_a' G_b (2 x 2).  The pair's G blocks are
// wave-uniform (scalar loads, M formed on every lane); per lane a pair costs
// three vector loads (J_f,a[r][m], J_f,b[0..1][n]) from two records — four
// 128-B lines per pair where Z rows take six.
template <int CT, int U>
__global__ __launch_bounds__(kBlock) void schur_pairs_jg1_kernel(DevProblem p, const DevPairTile* __restrict__ tiles,
                                                                  int ntiles, const uint2* __restrict__ pairs,
                                                                  const double* __restrict__ JG,
                                                                  double* __restrict__ S, PairFlush pf) {
  constexpr int F = 6 + CT, RW = jg_width(F);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = blockIdx.x * 4 + wv;
  if (t >= ntiles) return;
  const DevPairTile tl = tiles[t];
  if (tl.count == 0) return;
  const int lane = threadIdx.x & 63;
  const int m = lane & 15, k = lane >> 4;
  const bool on = m < F && k < 2;
  const int mm = m < F ? m : 0;
  const int r = k & 1;
  typedef double dvec4 __attribute__((ext_vector_type(4)));
  dvec4 acc = {0.0, 0.0, 0.0, 0.0};
  const uint32_t cnt = tl.count;
  const uint2* pl = pairs + tl.start;
  auto step = [&](const uint2 pr) {
    const double* ga = JG + (size_t)pr.x * RW;
    const double* gb = JG + (size_t)pr.y * RW;
    // M[r][s] = sum_c G_a[c][r] G_b[c][s] (G[c][s] at 2F + 2c + s)
    const double m0 = ga[2 * F + r] * gb[2 * F] + ga[2 * F + 2 + r] * gb[2 * F + 2] + ga[2 * F + 4 + r] * gb[2 * F + 4];
    const double m1 =
        ga[2 * F + r] * gb[2 * F + 1] + ga[2 * F + 2 + r] * gb[2 * F + 3] + ga[2 * F + 4 + r] * gb[2 * F + 5];
    const double va = ga[r * F + mm];
    const double vb = m0 * gb[mm] + m1 * gb[F + mm];
    return std::pair<double, double>(on ? va : 0.0, on ? vb : 0.0);
  };
  uint32_t n = 0;
  for (; n + U <= cnt; n += U) {
    uint2 pr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint2 q = pl[n + u];
      pr[u] = make_uint2(__builtin_amdgcn_readfirstlane(q.x), __builtin_amdgcn_readfirstlane(q.y));
    }
    double va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const auto v = step(pr[u]);
      va[u] = v.first;
      vb[u] = v.second;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va[u], vb[u], acc, 0, 0, 0);
  }
  for (; n < cnt; ++n) {
    const uint2 q = pl[n];
    const auto v = step(make_uint2(__builtin_amdgcn_readfirstlane(q.x), __builtin_amdgcn_readfirstlane(q.y)));
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v.first, v.second, acc, 0, 0, 0);
  }
  const double accv[4] = {acc[0], acc[1], acc[2], acc[3]};
  pair_tile_store<F>(p, tl, t, lane, accv, S, pf);
}

// As schur_pairs_kernel, latency-hidden: the tile's pair list is staged once
// in the wave's LDS slot (read back as broadcasts, no dependent global load
// per pair), and the Z rows of U pairs are requested one step ahead, so the
// next step's 2U gathers are in flight while this step's MFMAs run.
template <int CT, int U>
__global__ __launch_bounds__(kBlock) void schur_pairs_pipelined_kernel(DevProblem p, const DevPairTile* __restrict__ tiles,
                                                                       int ntiles, const uint2* __restrict__ pairs,
                                                                       const double* __restrict__ Z,
                                                                       double* __restrict__ S) {
  constexpr int F = 6 + CT, ZN = 3 * F;
  __shared__ uint2 spl[kBlock / 64][kPairTile];
  const int G = (ntiles + 3) / 4;
  const int per = (G + 7) / 8;
  const int b = blockIdx.x;
  const int lb = (b % 8) * per + b / 8;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = lb * 4 + wv;
  if (lb >= G || t >= ntiles) return;
  const DevPairTile tl = tiles[t];
  const int lane = threadIdx.x & 63;
  const int m = lane & 15, k = lane >> 4;
  const bool on = m < F && k < 3;
  const int off = on ? k * F + m : 0;
  const int cnt = (int)tl.count;
  const uint2* pl = pairs + tl.start;
  uint2* sp = spl[wv];
  for (int n = lane; n < cnt; n += 64) sp[n] = pl[n];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  typedef double dvec4 __attribute__((ext_vector_type(4)));
  dvec4 acc = {0.0, 0.0, 0.0, 0.0};
  double va[U], vb[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint2 pr = sp[u < cnt ? u : 0];
    const bool ld = on && u < cnt;
    va[u] = ld ? Z[(size_t)pr.x * ZN + off] : 0.0;
    vb[u] = ld ? Z[(size_t)pr.y * ZN + off] : 0.0;
  }
  for (int n0 = 0; n0 < cnt; n0 += U) {
    double na[U], nb[U];
    const int n1 = n0 + U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int n = n1 + u;
      const uint2 pr = sp[n < cnt ? n : 0];
      const bool ld = on && n < cnt;
      na[u] = ld ? Z[(size_t)pr.x * ZN + off] : 0.0;
      nb[u] = ld ? Z[(size_t)pr.y * ZN + off] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va[u], vb[u], acc, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va[u] = na[u];
      vb[u] = nb[u];
    }
  }
  const uint32_t ia = tl.ia, ib = tl.ib;
  const uint32_t ca = p.img_cam[ia], cb = p.img_cam[ib];
  const bool pa = p.img_flags[ia] & 1u, pb = p.img_flags[ib] & 1u;
  const bool cva = p.cam_var[ca] != 0, cvb = p.cam_var[cb] != 0;
  const int ncol = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int mrow = 4 * r + (lane >> 4);
    if (mrow >= F || ncol >= F) continue;
    const bool xa = mrow < 6 ? pa : cva, xb = ncol < 6 ? pb : cvb;
    if (!xa || !xb) continue;
    const int64_t ra = fslot(p, ia, ca, mrow), rb = fslot(p, ib, cb, ncol);
    const double v = acc[r];
    if (tl.self) {
      if (ra <= rb) atomicAdd(S + ra * p.lds + rb, -v);
    } else if (ra < rb) {
      atomicAdd(S + ra * p.lds + rb, -v);
    } else if (ra > rb) {
      atomicAdd(S + rb * p.lds + ra, -v);
    } else {
      atomicAdd(S + ra * p.lds + ra, -2.0 * v);
    }
  }
}

// Damping on the diagonal; identity on slots that are not parameters.
__global__ void dense_finalize_kernel(DevProblem p, const double* __restrict__ lambda_f, double* __restrict__ S) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= p.nf) return;
  bool var;
  if (k < 6 * (int64_t)p.num_images) {
    var = p.img_flags[k / 6] & 1u;
  } else if (k >= p.cyl0) {
    var = p.cyl_var != 0;
  } else {
    var = p.cam_var[(k - 6 * (int64_t)p.num_images) / (p.ct > 0 ? p.ct : 1)] != 0;
  }
  if (var) {
    S[k * p.lds + k] += lambda_f[k];
  } else {
    S[k * p.lds + k] = 1.0;
  }
}

template <typename F>
void dispatch_ct(int ct, F&& f) {
  switch (ct) {
    case 0: f(std::integral_constant<int, 0>{}); break;
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    case 6: f(std::integral_constant<int, 6>{}); break;
    case 7: f(std::integral_constant<int, 7>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    default: break;
  }
}

inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

}  // namespace

// cost partials of the reprojection kernels: one per 64 blocks
int reproj_grid(int64_t nb) { return (int)grid_for(nb, 64); }

// Reads the reprojection kernel's streamed inputs (observations, image /
// point ids, points; 16 B per lane, grid-stride, four loads in flight per
// lane) and drops the values: they land in the memory-side cache, so the
// reprojection kernel behind it meets HBM with its write stream alone
// (linearize_warm_inputs).  One launch of few workgroups (one per CU): it
// runs beside the semantic deferred pass and should take as little of the
// CUs' wave slots as it can.  The sink is written only for an impossible sum.
struct TouchRanges {
  const uint4* ptr[5];
  int64_t n16[5];
};

template <int U>
__global__ __launch_bounds__(256) void touch_kernel(TouchRanges t, unsigned* sink) {
  unsigned acc = 0u;
  const int64_t stride = (int64_t)gridDim.x * 256;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const uint4* a = t.ptr[q];
    const int64_t n = t.n16[q];
    int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; k + (U - 1) * stride < n; k += U * stride) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = a[k + u * stride];  // U loads in flight per lane
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].w;
    }
    for (; k < n; k += stride) acc ^= a[k].x;
  }
  if (acc == 0x9e3779b9u && t.n16[0] < 0) *sink = acc;
}

void launch_touch_inputs(const DevProblem& p, unsigned* sink, hipStream_t s, int mask, int wgs, int unroll) {
  // mask bits: 1 observations, 2 image ids, 4 point ids, 8 points; the ids
  // in the layout the kernel reads (packed: both in obs_ids + wave_pt0)
  TouchRanges t{};
#ifdef MI_BA_AB_VARIANTS
  const bool packed = ((kJacProduction & 8192) != 0 || p.jvariant == 43) && p.obs_ids;
#else
  const bool packed = (kJacProduction & 8192) != 0 && p.obs_ids;
#endif
  const int64_t nw = (p.nb + 63) / 64;
  const void* ptrs[5] = {p.obs_xy, packed ? (const void*)p.obs_ids : (const void*)p.obs_img,
                         packed ? (const void*)p.wave_pt0 : (const void*)p.obs_pt, nullptr, p.X};
  const int64_t bytes[5] = {p.nb * 16, p.nb * 4, packed ? nw * 4 : p.nb * 4, 0, p.num_points * 24};
  const int bit[5] = {1, 2, 4, 4, 8};
  for (int q = 0; q < 5; ++q) {
    t.ptr[q] = reinterpret_cast<const uint4*>(ptrs[q]);
    t.n16[q] = ptrs[q] && (mask & bit[q]) ? bytes[q] / 16 : 0;
  }
  if (wgs <= 0) {  // one workgroup per CU
    int dev = 0;
    wgs = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&wgs, hipDeviceAttributeMultiprocessorCount, dev) ||
        wgs <= 0)
      wgs = 256;
  }
  if (unroll >= 8)
    hipLaunchKernelGGL(touch_kernel<8>, dim3(wgs), dim3(256), 0, s, t, sink);
  else
    hipLaunchKernelGGL(touch_kernel<4>, dim3(wgs), dim3(256), 0, s, t, sink);
}

void launch_reproj_jacobian(const DevProblem& p, double2* r, double* J, double* cost_partial, hipStream_t s) {
  if (p.nb == 0) return;
  const unsigned g = grid_for(p.nb, kBlock);
  if (p.model == kMixedModels) {
    dispatch_ct(p.ct, [&](auto c) {
      constexpr int CT = decltype(c)::value;
      if (p.loss_type == kLossTrivial)
        hipLaunchKernelGGL((reproj_jacobian_kernel<kMixedModels, 0, 0, kJacPasses, kJacProduction, 4, kBlock, CT>), dim3(g),
                           dim3(kBlock), 0, s, p, r, J, cost_partial);
      else
        hipLaunchKernelGGL((reproj_jacobian_kernel<kMixedModels, 0, 1, kJacPasses, kJacProduction, 4, kBlock, CT>), dim3(g),
                           dim3(kBlock), 0, s, p, r, J, cost_partial);
    });
    return;
  }
  dispatch_model(p.model, [&](auto m) {
    constexpr int M = decltype(m)::value;
    auto go = [&](auto rf) {
      constexpr int RF = decltype(rf)::value;
      auto launch = [&](auto loss) {
        constexpr int LOSS = decltype(loss)::value;
#ifdef MI_BA_AB_VARIANTS
        if constexpr (M == kOpenCV && RF == 5 && LOSS == 0) {
          // A/B and roofline-decomposition builds of the C4 shape (tools/ab_jacobian.py)
          switch (p.jvariant) {
            case 1:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 1, kJacProduction>), dim3(g), dim3(kBlock), 0, s, p, r, J,
                                 cost_partial);
              return;
            case 2:  // two slab passes (production before the closed-form rotation columns)
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction>), dim3(g), dim3(kBlock), 0, s, p, r, J,
                                 cost_partial);
              return;
            case 4:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 4, kJacProduction>), dim3(g), dim3(kBlock), 0, s, p, r, J,
                                 cost_partial);
              return;
            case 20:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, 0>), dim3(g), dim3(kBlock), 0, s, p, r, J,
                                 cost_partial);
              return;
            case 21:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, 24>), dim3(g), dim3(kBlock), 0, s, p, r, J,
                                 cost_partial);
              return;
            case 26:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction | 256>), dim3(g), dim3(kBlock), 0, s, p,
                                 r, J, cost_partial);
              return;
            case 27:  // plain (temporal) 16-B J stores
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction & ~8>), dim3(g), dim3(kBlock), 0, s,
                                 p, r, J, cost_partial);
              return;
            case 24:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction, 4, 64>), dim3(grid_for(p.nb, 64)),
                                 dim3(64), 0, s, p, r, J, cost_partial);
              return;
            case 25:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction, 4, 128>),
                                 dim3(grid_for(p.nb, 128)), dim3(128), 0, s, p, r, J, cost_partial);
              return;
            case 23:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacR1>), dim3(g), dim3(kBlock), 0, s, p, r, J,
                                 cost_partial);
              return;
            case 22:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction | 4>), dim3(g), dim3(kBlock), 0, s, p, r, J,
                                 cost_partial);
              return;
            // occupancy study: per-lane records (64), J slab in NP passes, WPE waves/SIMD
            case 30:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction, 5>), dim3(g), dim3(kBlock), 0, s, p, r, J,
                                 cost_partial);
              return;
            case 31:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction | 64, 4>), dim3(g), dim3(kBlock), 0, s, p, r,
                                 J, cost_partial);
              return;
            case 32:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 4, kJacProduction | 64, 5>), dim3(g), dim3(kBlock), 0, s, p, r,
                                 J, cost_partial);
              return;
            case 33:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 4, kJacProduction | 64, 6>), dim3(g), dim3(kBlock), 0, s, p, r,
                                 J, cost_partial);
              return;
            case 34:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 4, kJacProduction | 64, 8>), dim3(g), dim3(kBlock), 0, s, p, r,
                                 J, cost_partial);
              return;
            case 35:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction | 64, 6>), dim3(g), dim3(kBlock), 0, s, p, r,
                                 J, cost_partial);
              return;
            case 36:  // closed-form rotation columns
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction | 512>), dim3(g), dim3(kBlock), 0, s,
                                 p, r, J, cost_partial);
              return;
            case 42:  // A/B: closed form without the unit-quaternion check
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 1, kJacProduction | 4096>), dim3(g), dim3(kBlock), 0,
                                 s, p, r, J, cost_partial);
              return;
            case 37:  // closed-form rotation columns, R X through the rotation matrix
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction | 512 | 1024>), dim3(g), dim3(kBlock),
                                 0, s, p, r, J, cost_partial);
              return;
            case 38:  // closed-form rotation columns, raised-priority store bursts
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction | 512 | 256>), dim3(g), dim3(kBlock),
                                 0, s, p, r, J, cost_partial);
              return;
            case 39:  // closed-form rotation columns, 5 waves per SIMD
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction | 512, 5>), dim3(g), dim3(kBlock),
                                 0, s, p, r, J, cost_partial);
              return;
            case 9:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction | 1>), dim3(g), dim3(kBlock), 0, s, p, r, J,
                                 cost_partial);
              return;
            case 10:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, 2, kJacProduction | 2>), dim3(g), dim3(kBlock), 0, s, p, r, J,
                                 cost_partial);
              return;
            // roofline decomposition of the production shape (one slab pass):
            // 11 = store-only (obs read, r + J rows written, no arithmetic),
            // 12 = no J store (everything but the J write)
            case 11:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, kJacPasses, kJacProduction | 2>), dim3(g), dim3(kBlock),
                                 0, s, p, r, J, cost_partial);
              return;
            case 12:
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, kJacPasses, kJacProduction | 1>), dim3(g), dim3(kBlock),
                                 0, s, p, r, J, cost_partial);
              return;
            case 43:  // packed ids (obs_ids + wave_pt0; slower in the bench step)
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, kJacPasses, kJacProduction | 8192>), dim3(g),
                                 dim3(kBlock), 0, s, p, r, J, cost_partial);
              return;
            case 13:  // R and the unit-q test from the image record (per image, not per block)
              hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, 0, kJacPasses, kJacProduction | 2048>), dim3(g),
                                 dim3(kBlock), 0, s, p, r, J, cost_partial);
              return;
            default:
              break;
          }
        }
#endif
        hipLaunchKernelGGL((reproj_jacobian_kernel<M, RF, LOSS, kJacPasses, kJacProduction>), dim3(g), dim3(kBlock), 0,
                           s, p, r, J, cost_partial);
      };
      if (p.loss_type == kLossTrivial)
        launch(std::integral_constant<int, 0>{});
      else
        launch(std::integral_constant<int, 1>{});
    };
    switch (p.refine_mask & 7) {
      case 0: go(std::integral_constant<int, 0>{}); break;
      case 1: go(std::integral_constant<int, 1>{}); break;
      case 2: go(std::integral_constant<int, 2>{}); break;
      case 3: go(std::integral_constant<int, 3>{}); break;
      case 4: go(std::integral_constant<int, 4>{}); break;
      case 5: go(std::integral_constant<int, 5>{}); break;
      case 6: go(std::integral_constant<int, 6>{}); break;
      default: go(std::integral_constant<int, 7>{}); break;
    }
  });
}

void launch_pack_images(const DevProblem& p, double* rec, hipStream_t s, double* zero, int nzero) {
  const int64_t n = std::max<int64_t>(p.num_images, zero ? nzero : 0);
  if (n == 0) return;
  hipLaunchKernelGGL(pack_images_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, p, rec, zero,
                     zero ? nzero : 0);
}

void launch_reproj_cost(const DevProblem& p, const double* qt, const double* cam, const double* X,
                        double* cost_partial, hipStream_t s) {
  if (p.nb == 0) return;
  const unsigned g = grid_for(p.nb, kBlock);
  if (p.model == kMixedModels) {
    hipLaunchKernelGGL(reproj_cost_kernel<kMixedModels>, dim3(g), dim3(kBlock), 0, s, p, qt, cam, X, cost_partial);
    return;
  }
  dispatch_model(p.model, [&](auto m) {
    constexpr int M = decltype(m)::value;
    hipLaunchKernelGGL(reproj_cost_kernel<M>, dim3(g), dim3(kBlock), 0, s, p, qt, cam, X, cost_partial);
  });
}

void launch_sum2(const double* p1, int64_t n1, double* out1, double* scratch1, const double* p2, int64_t n2,
                 double* out2, hipStream_t s) {
  hipLaunchKernelGGL(sum2_kernel, dim3(kSumGroups + kSumGroups2), dim3(256), 0, s, p1, n1, out1, scratch1, p2, n2,
                     out2);
}

// With scratch the list is always summed by the 64-workgroup pass (the order
// sum2_kernel gives the same list, so the initial, model and trial costs of
// the reprojection partials are summed alike at every size); the single
// workgroup only serves lists without scratch.
void launch_sum(const double* partial, int64_t n, double* out, hipStream_t s, double* scratch) {
  if (scratch) {
    hipLaunchKernelGGL(sum_multi_kernel, dim3(kSumGroups), dim3(256), 0, s, partial, n, out, scratch,
                       reinterpret_cast<unsigned*>(scratch + kSumGroups));
    return;
  }
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(1024), 0, s, partial, n, out);
}

void launch_point_normal(const DevProblem& p, const DevPoint* vp, int64_t npv, const double2* r, const double* J,
                         double* Vg, hipStream_t s, const uint32_t* chunks, int nchunks) {
  if (npv == 0) return;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    if (chunks && nchunks > 0)
      hipLaunchKernelGGL(point_normal_chunk_kernel<CT>, dim3(grid_for(nchunks, kBlock / 64)), dim3(kBlock), 0, s, p,
                         chunks, nchunks, r, J, Vg);
    else
      hipLaunchKernelGGL(point_normal_kernel<CT>, dim3(grid_for(npv, kBlock)), dim3(kBlock), 0, s, vp, npv, r, J, Vg);
  });
}

void launch_point_prepare(const DevProblem& p, const DevPoint* vp, int64_t npv, const double* Vg,
                          double* scale_p, double* diag_p, double* Vinv, double* Linv, double* q, int first,
                          int reuse_diag, double radius, hipStream_t s) {
  if (npv == 0) return;
  hipLaunchKernelGGL(point_prepare_kernel, dim3(grid_for(npv, kBlock)), dim3(kBlock), 0, s, vp, npv, Vg,
                     scale_p, diag_p, Vinv, Linv, q, first, reuse_diag, radius);
}

void launch_fblock_dense(const DevProblem& p, const DevTile* tiles, int ntiles, const uint32_t* cm_perm,
                         const uint32_t* cm_ptv, const double2* r, const double* J, const double* q, double* b,
                         double* udiag, double* S, hipStream_t s, const TileOwners* own) {
  if (ntiles == 0) return;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
#ifdef MI_BA_AB_VARIANTS
    if (p.fvariant == 1) {  // LDS-staged rows + MFMA: 1.30 vs 1.23 ms at C4 (profiles/r3_ab_fblock_fused_rhs.jsonl)
      hipLaunchKernelGGL(fblock_mfma_kernel<CT>, dim3(ntiles), dim3(kBlock), 0, s, p, tiles, cm_perm, r, J, q, b,
                         udiag, S);
      return;
    }
#endif
    hipLaunchKernelGGL(fblock_dense_kernel<CT>, dim3(ntiles), dim3(kBlock), 0, s, p, tiles, cm_perm, cm_ptv, r, J, q,
                       b, udiag, S, own ? own->part : nullptr);
    if (own) {
      constexpr int F = 6 + CT, NU = F * (F + 1) / 2;
      static_assert(NU + F <= kTilePartStride, "tile partial stride");
      launch_owner_flush(FlushDense{p, S, b, udiag, F, NU}, *own, NU + F, p, s);
    }
  });
}

void launch_fblock(const DevProblem& p, const DevTile* tiles, int ntiles, const uint32_t* cm_perm,
                   const double2* r, const double* J, const double* Jcm, const double* Vg, const double* Vinv,
                   double* pose_blk, double* cam_blk, double* b, double* udiag, hipStream_t s, const TileOwners* own) {
  if (ntiles == 0) return;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
#ifdef MI_BA_AB_VARIANTS
    if (p.fvariant == 2) {  // one lane per block (tools build)
      hipLaunchKernelGGL(fblock_kernel<CT>, dim3(ntiles), dim3(kBlock), 0, s, p, tiles, cm_perm, r, J, Jcm, Vg, Vinv,
                         pose_blk, cam_blk, b, udiag);
      return;
    }
#endif
    hipLaunchKernelGGL(fblock_pair_kernel<CT>, dim3(ntiles), dim3(kBlock), 0, s, p, tiles, cm_perm, r, J, Jcm, Vg,
                         Vinv, pose_blk, cam_blk, b, udiag, own ? own->part : nullptr);
    if (own) {
      constexpr int NH = CT > 6 ? CT : 6, NS = sym_size(NH), NA = NS + 2 * NH;
      static_assert(2 * NA <= kTilePartStride, "tile partial stride");
      launch_owner_flush(FlushPair{p, pose_blk, cam_blk, b, udiag, NH, NS, NA}, *own, 2 * NA, p, s);
    }
  });
}

void launch_gather_cm(const DevProblem& p, const uint32_t* cm_perm, int64_t n, double* Xcm, double2* obs_cm,
                      hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_cm_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, p, cm_perm, n, Xcm, obs_cm);
}

void launch_permute_rows(const DevProblem& p, const uint32_t* cm_perm, int64_t n, const double* J, double* Jcm,
                         hipStream_t s) {
  if (n == 0) return;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    hipLaunchKernelGGL(permute_rows_kernel<CT>, dim3((unsigned)grid_for(n * (9 + CT), kBlock)), dim3(kBlock), 0, s,
                       cm_perm, n, J, Jcm);
  });
}

void launch_fblock_finalize(const DevProblem& p, const double* pose_blk, const double* cam_blk,
                            const double* udiag, double* scale_f, double* diag_f, double* lambda_f,
                            double* prec_pose, double* prec_cam, double* b, int first, int reuse_diag,
                            double radius, hipStream_t s) {
  const int n = p.num_images + p.num_cameras;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    hipLaunchKernelGGL(fblock_finalize_kernel<CT>, dim3(grid_for(n, 64)), dim3(64), 0, s, p, pose_blk, cam_blk,
                       udiag, scale_f, diag_f, lambda_f, prec_pose, prec_cam, b, first, reuse_diag, radius);
  });
}

void launch_schur_product(const DevProblem& p, const DevPoint* vp, int64_t npv, const DevTile* tiles,
                          int ntiles, const uint32_t* cm_perm, const double* J, const double* Vinv,
                          const double* lambda_f, const double* x, double* w, double* y, hipStream_t s,
                          const uint32_t* chunks, int nchunks, const uint32_t* cm_ptv, const double* Jcm,
                          bool staged, const double* Xcm, const double2* obs_cm, const TileOwners* own) {
  (void)hipMemsetAsync(y, 0, sizeof(double) * p.nf, s);
  double* part = own ? own->part : nullptr;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    if (Xcm && chunks && cm_ptv && (p.loss_type == 0 || obs_cm)) {
      // matrix-free passes (no J read)
      auto go = [&](auto loss) {
        constexpr int LOSS = decltype(loss)::value;
        if (npv > 0 && nchunks > 0)
          hipLaunchKernelGGL((pcg_point_pass_mf<CT, LOSS>), dim3(grid_for(nchunks, kBlock / 64)), dim3(kBlock), 0, s,
                             p, chunks, nchunks, Vinv, x, w);
        if (ntiles > 0)
          hipLaunchKernelGGL((pcg_camera_pass_mf<CT, LOSS>), dim3(ntiles), dim3(kBlock), 0, s, p, tiles, cm_ptv, Xcm,
                             obs_cm, x, w, y, part);
      };
      if (p.loss_type == 0)
        go(std::integral_constant<int, 0>{});
      else
        go(std::integral_constant<int, 1>{});
      if (own && ntiles > 0) launch_owner_flush(FlushFVec{p, y}, *own, 6 + CT, p, s);
      return;
    }
    if (npv > 0 && chunks && nchunks > 0)
      hipLaunchKernelGGL((backsub_chunk_kernel<CT, true>), dim3(grid_for(nchunks, kBlock / 64)), dim3(kBlock), 0, s,
                         p, chunks, nchunks, J, nullptr, nullptr, Vinv, x, w, nullptr);
    else if (npv > 0)
      hipLaunchKernelGGL(schur_point_pass<CT>, dim3(grid_for(npv, kBlock)), dim3(kBlock), 0, s, p, vp, npv, J,
                         Vinv, x, w);
    if (ntiles > 0 && Jcm && cm_ptv && staged)
      hipLaunchKernelGGL(schur_f_rows_kernel<CT>, dim3(ntiles), dim3(kBlock), 0, s, p, tiles, cm_ptv, Jcm, x, w, y,
                         part);
    else if (ntiles > 0)
      hipLaunchKernelGGL(schur_f_pass<CT>, dim3(ntiles), dim3(kBlock), 0, s, p, tiles, cm_perm, cm_ptv, J, Jcm, x, w,
                         y, part);
    if (own && ntiles > 0) launch_owner_flush(FlushFVec{p, y}, *own, 6 + CT, p, s);
  });
  if (lambda_f)
    hipLaunchKernelGGL(add_diag_kernel, dim3(grid_for(p.nf, kBlock)), dim3(kBlock), 0, s, lambda_f, x, y, p.nf);
}

void launch_precond(const DevProblem& p, const double* prec_pose, const double* prec_cam, const double* r,
                    double* z, hipStream_t s) {
  const int n = p.num_images + p.num_cameras;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    hipLaunchKernelGGL(precond_kernel<CT>, dim3(grid_for(n, 64)), dim3(64), 0, s, p, prec_pose, prec_cam, r, z);
  });
}

void launch_finalize_n(int width, int n, const double* blk, const double* udiag, double* scale_f, double* diag_f,
                       double* lambda_f, double* prec, double* b, int var, int first, int reuse_diag, double radius,
                       hipStream_t s) {
  if (n <= 0) return;
  if (width == 7)
    hipLaunchKernelGGL(finalize_n_kernel<7>, dim3(grid_for(n, 64)), dim3(64), 0, s, n, blk, udiag, scale_f, diag_f,
                       lambda_f, prec, b, var, first, reuse_diag, radius);
  else
    hipLaunchKernelGGL(finalize_n_kernel<8>, dim3(grid_for(n, 64)), dim3(64), 0, s, n, blk, udiag, scale_f, diag_f,
                       lambda_f, prec, b, var, first, reuse_diag, radius);
}

void launch_precond_n(int width, int n, const double* prec, const double* r, double* z, hipStream_t s) {
  if (n <= 0) return;
  if (width == 7)
    hipLaunchKernelGGL(precond_n_kernel<7>, dim3(grid_for(n, 64)), dim3(64), 0, s, n, prec, r, z);
  else
    hipLaunchKernelGGL(precond_n_kernel<8>, dim3(grid_for(n, 64)), dim3(64), 0, s, n, prec, r, z);
}

void launch_dot(const double* a, const double* b, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(dot_kernel, dim3(1), dim3(1024), 0, s, a, b, n, out);
}

void launch_axpy(double* y, const double* x, const double* num, const double* den, double sign, int64_t n,
                 hipStream_t s) {
  hipLaunchKernelGGL(axpy_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, y, x, num, den, sign, n);
}

void launch_xpby(double* pv, const double* z, const double* num, const double* den, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(xpby_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, pv, z, num, den, n);
}

void launch_backsub(const DevProblem& p, const DevPoint* vp, int64_t npv, const double* J, const double* Vg,
                    const double* Vinv, const double* df, double* dX, hipStream_t s) {
  if (npv == 0) return;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    hipLaunchKernelGGL(backsub_kernel<CT>, dim3(grid_for(npv, kBlock)), dim3(kBlock), 0, s, p, vp, npv, J, Vg,
                       Vinv, df, dX);
  });
}

int64_t launch_backsub_chunks(const DevProblem& p, const uint32_t* chunk, int nchunks, const double* J,
                              const double2* r, const double* Vg, const double* Vinv, const double* df, double* dX,
                              double* partial, hipStream_t s) {
  if (nchunks <= 0) return 0;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    hipLaunchKernelGGL(backsub_chunk_kernel<CT>, dim3(grid_for(nchunks, kBlock / 64)), dim3(kBlock), 0, s, p, chunk,
                       nchunks, J, r, Vg, Vinv, df, dX, partial);
  });
  return nchunks;
}

int64_t launch_backsub_cost(const DevProblem& p, const DevPoint* vp, int64_t npv, const double* J, const double2* r,
                            const double* Vg, const double* Vinv, const double* df, double* dX, double* partial,
                            bool const_blocks, hipStream_t s) {
  (void)hipMemsetAsync(partial, 0, sizeof(double), s);
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    if (npv > 0)
      hipLaunchKernelGGL(backsub_cost_kernel<CT>, dim3(grid_for(npv, kBlock)), dim3(kBlock), 0, s, p, vp, npv, J,
                         r, Vg, Vinv, df, dX, partial);
    if (p.nb > 0 && const_blocks)
      hipLaunchKernelGGL(model_cost_const_kernel<CT>, dim3(grid_for(p.nb, kBlock)), dim3(kBlock), 0, s, p, r, J,
                         df, partial);
  });
  return std::max<int64_t>(1, (npv + 63) / 64);
}

void launch_model_cost(const DevProblem& p, const double2* r, const double* J, const double* df, const double* dX,
                       double* partial, hipStream_t s) {
  if (p.nb == 0) return;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    hipLaunchKernelGGL(model_cost_kernel<CT>, dim3(grid_for(p.nb, kBlock)), dim3(kBlock), 0, s, p, r, J, df, dX,
                       partial);
  });
}

void launch_plus(const DevProblem& p, const double* df, const double* dX, const double* qt, const double* cam,
                 const double* X, double* qt_out, double* cam_out, double* X_out, hipStream_t s) {
  hipLaunchKernelGGL(plus_images_kernel, dim3(grid_for(p.num_images, 64)), dim3(64), 0, s, p, df, qt, qt_out);
  hipLaunchKernelGGL(plus_cameras_kernel, dim3(grid_for(p.num_cameras, 64)), dim3(64), 0, s, p, df, cam, cam_out);
  if (p.num_points > 0)
    hipLaunchKernelGGL(plus_points_kernel, dim3(grid_for(p.num_points, kBlock)), dim3(kBlock), 0, s, p, dX, X,
                       X_out);
}

void launch_dense_schur(const DevProblem& p, const DevTile* tiles, int ntiles, const uint32_t* cm_perm,
                        const uint32_t* cm_ptv, const double* J, const double* Linv, double* Z, const DevPairTile* ptiles, int nptiles,
                        const uint2* pairs, double* S, bool with_u, hipStream_t s, const PairFlush* pflush) {
  const PairFlush nof{nullptr, nullptr, nullptr, nullptr, 0};
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    if (with_u && ntiles > 0)
      hipLaunchKernelGGL(dense_u_kernel<CT>, dim3(ntiles), dim3(kBlock), 0, s, p, tiles, cm_perm, J, S);
#ifdef MI_BA_AB_VARIANTS
    if (nptiles > 0 && p.nb > 0 && (p.svariant == 8 || p.svariant == 9)) {
      // JG records, one pair per MFMA (K = 2), image-block tile order
      const PairFlush& pf = pflush ? *pflush : nof;
      hipLaunchKernelGGL(schur_jg_kernel<CT>, dim3(grid_for(p.nb, kBlock)), dim3(kBlock), 0, s, p, J, Linv, Z);
      if (p.svariant == 8)
        hipLaunchKernelGGL((schur_pairs_jg1_kernel<CT, 4>), dim3((nptiles + 3) / 4), dim3(kBlock), 0, s, p, ptiles,
                           nptiles, pairs, Z, S, pf);
      else
        hipLaunchKernelGGL((schur_pairs_jg1_kernel<CT, 8>), dim3((nptiles + 3) / 4), dim3(kBlock), 0, s, p, ptiles,
                           nptiles, pairs, Z, S, pf);
      if (pf.pslot && pf.ndest > 0)
        hipLaunchKernelGGL(schur_pairs_flush_kernel<CT>, dim3(pf.ndest), dim3(256), 0, s, p, pf, S);
      return;
    }
#endif
    if (nptiles > 0 && p.nb > 0 && p.svariant == 6) {
      // JG records + two pairs per MFMA, image-block tile order (dispatch order)
      hipLaunchKernelGGL(schur_jg_kernel<CT>, dim3(grid_for(p.nb, kBlock)), dim3(kBlock), 0, s, p, J, Linv, Z);
      hipLaunchKernelGGL(schur_pairs_jg_kernel<CT>, dim3((nptiles + 3) / 4), dim3(kBlock), 0, s, p, ptiles, nptiles,
                         pairs, Z, S);
    } else if (nptiles > 0 && p.nb > 0) {
#ifdef MI_BA_AB_VARIANTS
      // Z rows in image order (zorder 1, tools build): schur_pairs 5.76 vs
      // 5.64 ms and schur_z 1.28 vs 1.01 ms per C4 launch (the J rows
      // gathered), profiles/r6g_ab_schur_z_image_order.md
      if (p.svariant != 7 && p.zorder)
        hipLaunchKernelGGL((schur_z_kernel<CT, true>), dim3(grid_for(p.nb, kBlock)), dim3(kBlock), 0, s, p, J, Linv, Z,
                           cm_perm, cm_ptv);
      else
#endif
      if (p.svariant != 7)
        hipLaunchKernelGGL(schur_z_kernel<CT>, dim3(grid_for(p.nb, kBlock)), dim3(kBlock), 0, s, p, J, Linv, Z,
                           nullptr, nullptr);
      const int G = (nptiles + 3) / 4;
      const int grid = ((G + 7) / 8) * 8;  // whole XCD stripes (extra workgroups exit)
#ifdef MI_BA_AB_VARIANTS
      if (p.svariant == 1)
        hipLaunchKernelGGL((schur_pairs_pipelined_kernel<CT, 8>), dim3(grid), dim3(kBlock), 0, s, p, ptiles, nptiles,
                           pairs, Z, S);
      else if (p.svariant == 2)
        hipLaunchKernelGGL((schur_pairs_pipelined_kernel<CT, 4>), dim3(grid), dim3(kBlock), 0, s, p, ptiles, nptiles,
                           pairs, Z, S);
      else if (p.svariant == 3)
        hipLaunchKernelGGL((schur_pairs_pipelined_kernel<CT, 16>), dim3(grid), dim3(kBlock), 0, s, p, ptiles, nptiles,
                           pairs, Z, S);
      else
#endif
#ifdef MI_BA_AB_VARIANTS
      if (p.svariant == 7) {
        // Z formed in the pair kernel from J + Linv (no schur_z pass)
        const PairFlush& pf = pflush ? *pflush : nof;
        hipLaunchKernelGGL((schur_pairs_j_kernel<CT>), dim3(G), dim3(kBlock), 0, s, p, ptiles, nptiles, pairs, J, Linv,
                           S, pf);
        if (pf.pslot && pf.ndest > 0)
          hipLaunchKernelGGL(schur_pairs_flush_kernel<CT>, dim3(pf.ndest), dim3(256), 0, s, p, pf, S);
      } else if (p.svariant == 5)
        hipLaunchKernelGGL((schur_pairs_kernel<CT, false, true>), dim3(G), dim3(kBlock), 0, s, p, ptiles, nptiles,
                           pairs, Z, S, nof);
      else
#endif
      if (p.svariant == 4) {
        // pflush: the image-block tile order's deterministic route
        const PairFlush& pf = pflush ? *pflush : nof;
        // self tiles with one Z load per pair: 5.11-5.15 vs 5.38 ms per C4
        // launch (profiles/r6i_ab_schur_pairs_self_flat.log); the duplicate
        // load of a self pair's row was an L2 request of its own.  Z rows
        // padded to 64-B multiples measured slower (pairs 5.26 vs 5.12 ms, Z
        // pass 1.61 vs 0.96 ms, profiles/r6j_ab_schur_z_align.log)
        if (p.sself1)
          hipLaunchKernelGGL((schur_pairs_kernel<CT, false, false, true>), dim3(grid), dim3(kBlock), 0, s, p, ptiles,
                             nptiles, pairs, Z, S, pf);
        else
          hipLaunchKernelGGL((schur_pairs_kernel<CT, false>), dim3(grid), dim3(kBlock), 0, s, p, ptiles, nptiles, pairs,
                             Z, S, pf);
        if (pf.pslot && pf.odest) {
          if (pf.nochunk > 0) {
            hipLaunchKernelGGL(schur_owner_chunk_kernel, dim3(pf.nochunk), dim3(64), 0, s, p, pf);
            hipLaunchKernelGGL(schur_owner_flush_kernel, dim3(pf.nodest), dim3(64), 0, s, p, pf, S);
          }
        } else if (pf.pslot && pf.ndest > 0) {
          hipLaunchKernelGGL(schur_pairs_flush_kernel<CT>, dim3(pf.ndest), dim3(256), 0, s, p, pf, S);
        }
      } else {
        hipLaunchKernelGGL(schur_pairs_kernel<CT>, dim3(grid), dim3(kBlock), 0, s, p, ptiles, nptiles, pairs, Z, S,
                           nof);
      }
    }
  });
}

void launch_dense_finalize(const DevProblem& p, const double* lambda_f, double* S, hipStream_t s) {
  hipLaunchKernelGGL(dense_finalize_kernel, dim3(grid_for(p.nf, kBlock)), dim3(kBlock), 0, s, p, lambda_f, S);
}

void launch_sqnorm2(const double* a, int64_t na, const double* b, int64_t nb2, double* out, double* scratch,
                    hipStream_t s) {
  const int64_t n = na + nb2;
  if (n < (1 << 16) || !scratch) {
    hipLaunchKernelGGL(sqnorm2_kernel, dim3(1), dim3(1024), 0, s, a, na, b, nb2, out);
    return;
  }
  // one CU streams ~30 GB/s: 3M-entry step vectors took 0.79 ms in one
  // workgroup; spread over up to kReduceBlocks workgroups, then add the
  // partials
  const unsigned g = (unsigned)std::min<int64_t>(kReduceBlocks, (n + 4095) / 4096);
  hipLaunchKernelGGL(sqnorm2_kernel, dim3(g), dim3(1024), 0, s, a, na, b, nb2, scratch);
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(1024), 0, s, scratch, (int64_t)g, out);
}

void launch_cg_step(double* x, const double* pv, double* r, const double* q, const double* rho,
                    const double* rho_prev, const double* pq, bool update_r, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(cg_step_kernel, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, x, pv, r, q, rho, rho_prev, pq,
                     update_r ? 1 : 0, n);
}

void launch_grad_f(const DevProblem& p, const DevTile* tiles, int ntiles, const uint32_t* cm_perm, const double2* r,
                   const double* J, double* g, hipStream_t s, const TileOwners* own) {
  if (ntiles == 0) return;
  dispatch_ct(p.ct, [&](auto c) {
    constexpr int CT = decltype(c)::value;
    hipLaunchKernelGGL(grad_f_kernel<CT>, dim3(ntiles), dim3(kBlock), 0, s, p, tiles, cm_perm, r, J, g,
                       own ? own->part : nullptr);
    if (own) launch_owner_flush(FlushFVec{p, g}, *own, 6 + CT, p, s);
  });
}

void launch_grad_max_f(const DevProblem& p, const double* g, double* out, hipStream_t s) {
  const int n = p.num_images + p.num_cameras;
  if (n > 0) hipLaunchKernelGGL(grad_max_f_kernel, dim3(grid_for(n, 64)), dim3(64), 0, s, p, g, out);
}

void launch_grad_max_points(const DevProblem& p, const DevPoint* vp, int64_t npv, const double* Vg, double* out,
                            hipStream_t s) {
  if (npv > 0)
    hipLaunchKernelGGL(grad_max_points_kernel, dim3((unsigned)std::min<int64_t>(grid_for(npv, kBlock), 1024)),
                       dim3(kBlock), 0, s, p, vp, npv, Vg, out);
}

void launch_state_norms(const DevProblem& p, const double* qt_c, const double* cam_c, const double* X_c, bool with_f,
                        double* out, double* scratch, hipStream_t s) {
  const int64_t n = (with_f ? (int64_t)p.num_images + p.num_cameras : 0) + p.num_points;
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(kReduceBlocks / 2, (n + 4095) / 4096));
  hipLaunchKernelGGL(state_norms_kernel, dim3(g), dim3(1024), 0, s, p, qt_c, cam_c, X_c, with_f ? 1 : 0, scratch);
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(1024), 0, s, scratch, (int64_t)g, out);
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(1024), 0, s, scratch + g, (int64_t)g, out + 1);
}

}  // namespace miba
