// CholeskyQR panel of the band reduction (the default panel; gpmi_band_api.hip
// falls back to the Householder panel of gpmi_band.hip when it reports failure).
//
// The Householder panel QR needs one grid-wide reduction per column (128 per
// panel, ~7.6 us each across CUs). This panel needs three: shifted CholeskyQR3
// (Fukaya, Kannan, Nakatsukasa, Yamamoto, Yanagisawa, SIAM J. Sci. Comput. 42
// (2020) A477) orthonormalises the m x 128 panel P = Q R with three Gram /
// Cholesky / triangular-solve passes, the first with the shift
// s = 11 (m b + b (b + 1)) u ||P||_F^2 so that it cannot break down for
// cond(P) < 1/u; then Householder reconstruction (Ballard, Demmel, Grigori,
// Jacquelin, Knight, Nguyen, IPDPS 2014) turns Q into the compact-WY form the
// rest of the reduction consumes: LU without pivoting of Q - [S; 0], with
// S_ii = -sign of the running pivot (|pivot| >= 1), gives Q - [S; 0] = V U with V
// unit lower trapezoidal (the Householder vectors), tau_i = -U_ii S_ii, and
// (I - V T V^T)^T P = [S R; 0]. Only the 128 x 128 top block of Q needs the
// sequential LU; the rows below are V_2 = Q_2 U^-1, one MFMA tile product each.
//
// Kernels (one panel; host sequence in gpmi_band_api.hip: cq_panel):
//   cq_gram_kernel     (m/64 tiles)     Gram partials of P's row tiles (packed lower)
//   cq_reduce_kernel                    G = sum of the partials
//   cq_chol_kernel     (1 workgroup)    L = chol(G [+ s I]), L^-1; failure flag
//   cq_apply_kernel    (m/64 tiles)     Q = Src L^-T and the Gram partials of Q
//   (passes 0 and 1; then reduce)
//   cq_recon_kernel    (1 workgroup)    third factor, Q3's top block, its LU with
//                                       signs, U^-1, tau, C = U^-T M3
//   cq_apply_kernel    (m/64 - 2)       V2 = Q2 C^T below the top block
//   cq_top_kernel      (after the       top block of every panel above the diagonal:
//                       reduction)      S R, R = L3^T L2^T L1^T, one workgroup each
// Failure (a non-positive pivot in any pass, or a third-pass factor farther than
// CQ_TOL from I, i.e. a second-pass Q that is not yet nearly orthonormal) sets the
// panel's failure flag before anything is written to the panel; the guarded
// Householder panel (hh_panel_kernel with that flag) then factors the untouched
// panel on the device (or, past its single-launch size, the host redoes the
// reduction with Householder panels). Numerics
// checked on Matern matrices first in numpy (tools/cholqr_proto.py).

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gpmi_internal.h"
#include "gpmi_device.h"
#include "gpmi_lds_chol.h"
#include "gpmi_band.h"
#include "gpmi_tile.h"

#ifndef GPMI_CQ_STAMPS
#define GPMI_CQ_STAMPS 0   // probe builds: phase stamps of one cq_recon_kernel call (printf)
#endif

namespace gpmi {

#if GPMI_CQ_STAMPS
__device__ int g_cq_calls;
#define CQST(i) \
  if (cst) cs[i] = wall_clock64()
#else
#define CQST(i)
#endif

constexpr double CQ_TOL = 1e-2;   // third pass: max |L3 - I| accepted

// A 128 x 128 row-major matrix in registers: thread t holds the pairs
// e = it * 256 + t (row e >> 6, columns 2 (e & 63) and +1), every load in flight.
__device__ __forceinline__ void load_regs(const double* __restrict__ G, d2 (&v)[32]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 32; ++it) v[it] = *reinterpret_cast<const d2*>(G + 2 * (it * 256 + t));
}

// ||G - I||_F^2 over the workgroup (every thread gets the sum); sred: 4 doubles.
__device__ __forceinline__ double frob_dev2(const d2 (&v)[32], double* sred) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  double s = 0.0;
#pragma unroll
  for (int it = 0; it < 32; ++it) {
    const int e = it * 256 + t, r = e >> 6, c = (e & 63) * 2;
    const double d0 = v[it][0] - (r == c ? 1.0 : 0.0);
    const double d1 = v[it][1] - (r == c + 1 ? 1.0 : 0.0);
    s += d0 * d0 + d1 * d1;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) sred[w] = s;
  __syncthreads();
  const double tot = ((sred[0] + sred[1]) + sred[2]) + sred[3];
  __syncthreads();
  return tot;
}

// First-order inverse Cholesky factor of G = I + E: I - E_l, E_l = stril(E) + diag(E)/2.
__device__ __forceinline__ double fo_entry(double g, int r, int c) {
  return r > c ? -g : (r == c ? 1.0 - 0.5 * (g - 1.0) : 0.0);
}

// out (row-major 128 x 128) = the lower triangle of the LDS block S (row stride DL),
// zeros above: two doubles per store, eight rows' LDS reads in flight together (one
// element per iteration waited out each LDS read: ~4 us per block).
__device__ __forceinline__ void store_lower_pairs(const double* S, double* __restrict__ out) {
  const int t = threadIdx.x;
#pragma unroll 8
  for (int it = 0; it < 32; ++it) {
    const int e = it * 256 + t, r = e >> 6, c = (e & 63) * 2;
    const d2 v = *reinterpret_cast<const d2*>(&S[r * DL + c]);
    *reinterpret_cast<d2*>(out + 2 * e) = d2{c <= r ? v[0] : 0.0, c + 1 <= r ? v[1] : 0.0};
  }
}

// L = chol(G + shift I) (lower), L^-1 (lower), both row-major 128 x 128 with
// zeros above the diagonal. pass 0 adds the shift coef * trace(G); pass 2
// checks L against I.
// First-order pass (pass > 0, ||G - I||_F <= tau_fo): G = I + E with E tiny, so
// L = I + E_l + O(E^2), E_l = stril(E) + diag(E) / 2, and the applied factor is
// Linv = I - E_l: the new Q's orthogonality error is O(||E||^2) (the next pass,
// or none for the last at tau_fo <= 3e-8, removes it). fo[pass] records the
// choice; cq_top_kernel then forms L = Linv^-1 (LDS triangular inverse), so
// P = Q (L1 L2 L3)^T stays exact to rounding. Lout is not written then.
__global__ __launch_bounds__(256) void cq_chol_kernel(const double* __restrict__ G, int pass,
                                                      double coef, double tau_fo,
                                                      double* __restrict__ Lout,
                                                      double* __restrict__ Linv,
                                                      int* __restrict__ fo,
                                                      int* __restrict__ fail,
                                                      unsigned* __restrict__ ctr) {
  __shared__ __attribute__((aligned(16))) double Ls[TS * DL];
  __shared__ double Aux[TS * RLD];
  __shared__ double sdiag[TS];
  __shared__ double sred[4];
  __shared__ int s_fail;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) s_fail = 0;
  if (pass == 0 && t < 128) ctr[t] = 0u;   // the guarded Householder panel's counter
  d2 v[32];
  load_regs(G, v);
  double shift = 0.0;
  if (pass == 0) {
    double d = t < TS ? G[t * TS + t] : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off);
    if (lane == 0) sred[w] = d;
    __syncthreads();
    shift = coef * (((sred[0] + sred[1]) + sred[2]) + sred[3]);
  } else if (tau_fo > 0.0) {
    // NaN takes the exact path (and fails there)
    if (frob_dev2(v, sred) <= tau_fo * tau_fo) {
#pragma unroll
      for (int it = 0; it < 32; ++it) {
        const int e = it * 256 + t, r = e >> 6, c = (e & 63) * 2;
        *reinterpret_cast<d2*>(Linv + 2 * e) =
            d2{fo_entry(v[it][0], r, c), fo_entry(v[it][1], r, c + 1)};
      }
      if (t == 0) fo[pass] = 1;
      return;
    }
  }
  if (t == 0) fo[pass] = 0;
#pragma unroll
  for (int it = 0; it < 32; ++it) {
    const int e = it * 256 + t, r = e >> 6, c = (e & 63) * 2;
    Ls[r * DL + c] = (c <= r) ? v[it][0] + (c == r ? shift : 0.0) : 0.0;
    Ls[r * DL + c + 1] = (c + 1 <= r) ? v[it][1] + (c + 1 == r ? shift : 0.0) : 0.0;
  }
  __syncthreads();
  lds_chol_block(Ls, Aux, sdiag, &s_fail);
  __syncthreads();
  int bad = s_fail;
  double dev = 0.0;
  // lower part out two doubles per store, eight rows' LDS reads in flight together
#pragma unroll 8
  for (int it = 0; it < 32; ++it) {
    const int e = it * 256 + t, r = e >> 6, c = (e & 63) * 2;
    const d2 v = *reinterpret_cast<const d2*>(&Ls[r * DL + c]);
    const d2 o = {c <= r ? v[0] : 0.0, c + 1 <= r ? v[1] : 0.0};
    *reinterpret_cast<d2*>(Lout + 2 * e) = o;
    if (pass == 2)
      dev = fmax(dev, fmax(fabs(o[0] - (c == r ? 1.0 : 0.0)), fabs(o[1] - (c + 1 == r ? 1.0 : 0.0))));
  }
  if (pass == 2) {
    // a NaN fails the test too (!(dev <= tol))
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dev = fmax(dev, __shfl_xor(dev, off));
    if (!(dev <= CQ_TOL)) bad = 1;
  }
  if (bad && lane == 0) __hip_atomic_store(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();   // every thread is done reading L before the inverse overwrites it
  lds_inv_block(Ls, Aux);
  __syncthreads();
  store_lower_pairs(Ls, Linv);
}

// Row tiles of 64: m / 64 workgroups of two per CU (67.6 KB of LDS each), so the
// fp64 MFMA work (~307 GFLOP/s per CU) spreads over the whole chip. Gram partials
// are packed: the 36 lower 16 x 16 tiles (ti >= tj) of the symmetric 128 x 128
// block, tile q = ti (ti + 1) / 2 + tj, 256 doubles each.
constexpr int RT = 64;           // rows per tile
constexpr int T_LD = TS + 4;     // LDS row stride of a staged 64 x 128 tile
constexpr int GPK = 36 * 256;    // doubles per packed Gram partial

__device__ __forceinline__ void tri_tile(int q, int* ti, int* tj) {
  int i = 0;
  while ((i + 1) * (i + 2) / 2 <= q) ++i;
  *ti = i;
  *tj = q - i * (i + 1) / 2;
}

// Stage the 64 x 128 row tile S0 (stride lds) into LDS (stride T_LD).
__device__ __forceinline__ void stage_rows(const double* __restrict__ S0, int64_t lds,
                                           double* T) {
  const int t = threadIdx.x;
  d2 v[16];
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int e = it * 256 + t;
    v[it] = *reinterpret_cast<const d2*>(S0 + (int64_t)(e >> 6) * lds + (e & 63) * 2);
  }
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int e = it * 256 + t;
    *reinterpret_cast<d2*>(T + (e >> 6) * T_LD + (e & 63) * 2) = v[it];
  }
}

// Packed lower Gram partial T^T T of the staged 64 x 128 tile; wave w forms the
// 16 x 16 tiles q = w, w + 4, .. (9 each), 16 k-steps over the 64 rows.
__device__ __forceinline__ void lds_tile_gram(const double* T, double* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  for (int q = w; q < 36; q += 4) {
    int ti, tj;
    tri_tile(q, &ti, &tj);
    d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < RT / 4; ++kk) {
      const double* row = T + (kk * 4 + fk) * T_LD;
      acc = mfma64(row[ti * 16 + fr], row[tj * 16 + fr], acc);
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) part[q * 256 + (fk + 4 * rr) * 16 + fr] = acc[rr];
  }
}

// part[tile] = packed lower Gram of Src's 64-row tile blockIdx.x.
__global__ __launch_bounds__(256, 2) void cq_gram_kernel(const double* __restrict__ Src,
                                                         int64_t lds,
                                                         double* __restrict__ part) {
  extern __shared__ double cq_dyn[];
  stage_rows(Src + (int64_t)blockIdx.x * RT * lds, lds, cq_dyn);
  __syncthreads();
  lds_tile_gram(cq_dyn, part + (int64_t)blockIdx.x * GPK);
}

// G (128 x 128, symmetric, row-major) = sum over the np packed partials, fixed
// order; 64 packed elements per workgroup, each summed by its four waves over the
// partials p = w (mod 4) (eight loads in flight per lane), the four sums combined in
// a fixed order; each element is written to both mirror positions.
__global__ __launch_bounds__(256) void cq_reduce_kernel(const double* __restrict__ part, int np,
                                                        double* __restrict__ G) {
  __shared__ double red[4][64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int e = blockIdx.x * 64 + lane;   // < GPK
  double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int p = w;
  for (; p + 28 < np; p += 32) {
    double x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = part[(int64_t)(p + 4 * q) * GPK + e];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += x[q];
  }
  for (int q = 0; p < np; p += 4, ++q) acc[q] += part[(int64_t)p * GPK + e];
  red[w][lane] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (w == 0) {
    const double v = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    int ti, tj;
    tri_tile(e >> 8, &ti, &tj);
    const int r = ti * 16 + ((e >> 4) & 15), c = tj * 16 + (e & 15);
    G[r * TS + c] = v;
    G[c * TS + r] = v;
  }
}

// Dst[tile] = Src[tile] M^T for the 64-row tile blockIdx.x (M lower, row-major):
// with M = L^-1 this is Src L^-T = Src R^-1; with M = U^-T M3 it is the final
// V2 = Q2 M3^T U^-1. Wave w forms the output column blocks w and 7 - w (k-steps
// 4 (cb + 1) each: M is lower) for all four 16-row blocks; its M fragments are
// loaded from global (L2) once, all in flight, and the tile from LDS. With
// part, also the packed Gram partial of Dst[tile] (the next pass's Gram).
// Src may equal Dst (in place): each workgroup reads its rows before storing them.
__global__ __launch_bounds__(256, 2) void cq_apply_kernel(const double* Src, int64_t lds,
                                                          double* Dst, int64_t ldd,
                                                          const double* __restrict__ M,
                                                          double* __restrict__ part,
                                                          const int* __restrict__ skip) {
  extern __shared__ double cq_dyn[];
  if (skip && __hip_atomic_load(skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * RT;
  const int cb0 = w, cb1 = 7 - w;
  // M fragments of both column blocks: b0[kk] = M[cb0*16 + fr][4 kk + fk]
  double b0[16], b1[32];
#pragma unroll
  for (int kk = 0; kk < 16; ++kk)
    b0[kk] = kk < 4 * (cb0 + 1) ? M[(cb0 * 16 + fr) * TS + kk * 4 + fk] : 0.0;
#pragma unroll
  for (int kk = 0; kk < 32; ++kk)
    b1[kk] = kk < 4 * (cb1 + 1) ? M[(cb1 * 16 + fr) * TS + kk * 4 + fk] : 0.0;
  stage_rows(Src + r0 * lds, lds, cq_dyn);
  __syncthreads();
  d4 acc0[4], acc1[4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    acc0[rb] = d4{0.0, 0.0, 0.0, 0.0};
    acc1[rb] = d4{0.0, 0.0, 0.0, 0.0};
  }
  // column block cb0 <= 3: k-steps < 16; cb1 >= 4: k-steps < 32
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    if (kk < 4 * (cb0 + 1)) {
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
        acc0[rb] = mfma64(cq_dyn[(rb * 16 + fr) * T_LD + kk * 4 + fk], b0[kk], acc0[rb]);
    }
  }
#pragma unroll
  for (int kk = 0; kk < 32; ++kk) {
    if (kk < 4 * (cb1 + 1)) {
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
        acc1[rb] = mfma64(cq_dyn[(rb * 16 + fr) * T_LD + kk * 4 + fk], b1[kk], acc1[rb]);
    }
  }
  double* D0 = Dst + r0 * ldd;
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = rb * 16 + fk + 4 * rr;
      D0[(int64_t)row * ldd + cb0 * 16 + fr] = acc0[rb][rr];
      D0[(int64_t)row * ldd + cb1 * 16 + fr] = acc1[rb][rr];
    }
  if (!part) return;
  __syncthreads();   // every wave is done reading the source tile
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = rb * 16 + fk + 4 * rr;
      cq_dyn[row * T_LD + cb0 * 16 + fr] = acc0[rb][rr];
      cq_dyn[row * T_LD + cb1 * 16 + fr] = acc1[rb][rr];
    }
  __syncthreads();
  lds_tile_gram(cq_dyn, part + (int64_t)blockIdx.x * GPK);
}

// Third pass + reconstruction (one workgroup). From G3 = Q2^T Q2 (Q2 the second
// pass's Q) the third factor M3 = L3^-1 (exact LDS Cholesky, or first order when
// ||G3 - I||_F <= tau_fo), then Q3's top block Q3t = Q2t M3^T, then the LU without
// pivoting of Q3t - S, S_ii = -sign of the running pivot, blocked by 16 in LDS:
//   per column block: the tall panel (rows j0.., 16 columns) with the rows in
//   registers over the four waves (pivot rows by readlane), U12 = L11^-1 A12 by forward
//   substitution (one thread per column), then A22 -= L21 U12 on fp64 MFMA.
// Outputs: V1 (strictly lower: the Householder vectors' top rows, into the top
// block of the panel P), S, tau = -diag(U) S, L3 / M3 (Lx3 / Linv3, for
// cq_top_kernel), and C = U^-T M3 (lower), so that the rows below the top block
// are V2 = Q2 M3^T U^-1 = Q2 C^T in one cq_apply_kernel pass (Q3 itself is never
// formed below the top block).
__global__ __launch_bounds__(256) void cq_recon_kernel(const double* __restrict__ Q2,
                                                       const double* __restrict__ G3,
                                                       double tau_fo,
                                                       double* __restrict__ P, int64_t lda,
                                                       double* __restrict__ S,
                                                       double* __restrict__ tau,
                                                       double* __restrict__ Lx3,
                                                       double* __restrict__ Linv3,
                                                       double* __restrict__ C,
                                                       int* __restrict__ fo,
                                                       int* __restrict__ fail,
                                                       double* __restrict__ US) {
  __shared__ __attribute__((aligned(16))) double A[TS * DL];
  __shared__ double Aux[TS * RLD];
  __shared__ double sS[TS];
  __shared__ double sdiag[TS];
  __shared__ double sred[4];
  __shared__ int s_fail;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  // an earlier pass failed: leave the panel untouched for the Householder panel
  if (__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
#if GPMI_CQ_STAMPS
  unsigned long long cs[10] = {0};
  bool cst = false;
  if (t == 0) {
    const int call = atomicAdd(&g_cq_calls, 1);
    cst = call == 20 || call == 110;
  }
#endif
  CQST(0);
  if (t == 0) s_fail = 0;
  // ---- M3 = L3^-1 into A (lower) and Linv3
  d2 v[32];
  load_regs(G3, v);
  const bool first_order = frob_dev2(v, sred) <= tau_fo * tau_fo;
  if (first_order) {
#pragma unroll
    for (int it = 0; it < 32; ++it) {
      const int e = it * 256 + t, r = e >> 6, c = (e & 63) * 2;
      A[r * DL + c] = fo_entry(v[it][0], r, c);
      A[r * DL + c + 1] = fo_entry(v[it][1], r, c + 1);
    }
    if (t == 0) fo[2] = 1;
  } else {
#pragma unroll
    for (int it = 0; it < 32; ++it) {
      const int e = it * 256 + t, r = e >> 6, c = (e & 63) * 2;
      A[r * DL + c] = (c <= r) ? v[it][0] : 0.0;
      A[r * DL + c + 1] = (c + 1 <= r) ? v[it][1] : 0.0;
    }
    __syncthreads();
    lds_chol_block(A, Aux, sdiag, &s_fail);
    __syncthreads();
    int bad = s_fail;
    double dev = 0.0;
    for (int e = t; e < TS * TS; e += 256) {
      const int r = e >> 7, c = e & 127;
      const double v = (c <= r) ? A[r * DL + c] : 0.0;
      Lx3[e] = v;
      dev = fmax(dev, fabs(v - (c == r ? 1.0 : 0.0)));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dev = fmax(dev, __shfl_xor(dev, off));
    if (!(dev <= CQ_TOL)) bad = 1;   // NaN included
    __syncthreads();
    if (bad && lane == 0) s_fail = 1;
    __syncthreads();
    if (s_fail) {
      if (t == 0) __hip_atomic_store(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    lds_inv_block(A, Aux);
    if (t == 0) fo[2] = 0;
  }
  __syncthreads();
  CQST(1);
  store_lower_pairs(A, Linv3);
  CQST(2);
  // ---- Q3t = Q2t M3^T (M3 lower: output column block cb needs k < 16 (cb + 1)): wave
  // w forms the column blocks w and 7 - w of all eight row blocks, 9 of the 36 units
  // of work each (a split by quadrants gives two waves 2/3 of it). Q2t's loads are
  // issued first (all in flight), M3's fragments of the wave's two column blocks go
  // to registers, then Q2t replaces M3 in LDS and the products read it from there.
  // The same MFMA sequence per output element (k ascending).
  {
    d2 q2[32];
#pragma unroll
    for (int it = 0; it < 32; ++it) q2[it] = *reinterpret_cast<const d2*>(Q2 + 2 * (it * 256 + t));
    const int cb0 = w, cb1 = 7 - w;
    double b0[16], b1[32];
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
      b0[kk] = kk < 4 * (cb0 + 1) ? A[(cb0 * 16 + fr) * DL + kk * 4 + fk] : 0.0;
#pragma unroll
    for (int kk = 0; kk < 32; ++kk)
      b1[kk] = kk < 4 * (cb1 + 1) ? A[(cb1 * 16 + fr) * DL + kk * 4 + fk] : 0.0;
    __syncthreads();   // every wave has its M3 fragments
#pragma unroll
    for (int it = 0; it < 32; ++it) {
      const int e = it * 256 + t, r = e >> 6, c = (e & 63) * 2;
      A[r * DL + c] = q2[it][0];
      A[r * DL + c + 1] = q2[it][1];
    }
    __syncthreads();
    d4 acc0[8], acc1[8];
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      acc0[rb] = d4{0.0, 0.0, 0.0, 0.0};
      acc1[rb] = d4{0.0, 0.0, 0.0, 0.0};
    }
#pragma unroll
    for (int kk = 0; kk < 32; ++kk) {
      if (kk < 4 * (cb1 + 1)) {
#pragma unroll
        for (int rb = 0; rb < 8; ++rb) {
          const double a = A[(rb * 16 + fr) * DL + kk * 4 + fk];
          if (kk < 4 * (cb0 + 1)) acc0[rb] = mfma64(a, b0[kk < 16 ? kk : 0], acc0[rb]);
          acc1[rb] = mfma64(a, b1[kk], acc1[rb]);
        }
      }
    }
    __syncthreads();   // every wave is done reading Q2t from A
#pragma unroll
    for (int rb = 0; rb < 8; ++rb)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        A[(rb * 16 + fk + 4 * rr) * DL + cb0 * 16 + fr] = acc0[rb][rr];
        A[(rb * 16 + fk + 4 * rr) * DL + cb1 * 16 + fr] = acc1[rb][rr];
      }
  }
  __syncthreads();
  CQST(3);
  for (int jb = 0; jb < NDB; ++jb) {
    const int j0 = jb * DB;
    // ---- tall panel (columns j0 .. j0 + 15) on all four waves: lanes 0-15 of every
    // wave hold the diagonal block's rows (each wave factors them redundantly, so
    // the pivot rows come by readlane, no exchange), lanes 16-63 hold rows
    // j0 + 16 + 4 (lane - 16) + w below it
    {
      const int row = lane < DB ? j0 + lane : j0 + DB + 4 * (lane - DB) + w;
      const bool live = row < TS;
      double pa[DB];
#pragma unroll
      for (int k = 0; k < DB; ++k) pa[k] = live ? A[row * DL + j0 + k] : 0.0;
#pragma unroll
      for (int j = 0; j < DB; ++j) {
        double prow[DB];
#pragma unroll
        for (int k = j; k < DB; ++k) prow[k] = readlane_d(pa[k], j);
        const double s = prow[j] >= 0.0 ? -1.0 : 1.0;
        const double u = prow[j] - s;   // |u| = |pivot| + 1
        const double rinv = 1.0 / u;
        if (lane == j) pa[j] = u;
        if (lane > j) {
          const double l = pa[j] * rinv;
          pa[j] = l;
#pragma unroll
          for (int k = j + 1; k < DB; ++k) pa[k] -= l * prow[k];
        }
        if (w == 0 && lane == 0) sS[j0 + j] = s;
      }
      __syncthreads();   // every wave read its rows before any wave writes back
      if (live && (lane >= DB || w == 0)) {
#pragma unroll
        for (int k = 0; k < DB; ++k) A[row * DL + j0 + k] = pa[k];
      }
    }
    __syncthreads();
    if (jb + 1 == NDB) break;
    // ---- U12 = L11^-1 A12: one thread per column right of the block; L11 (120
    // values, the same for every thread) read from LDS up front, not inside the
    // dependent substitution chain
    {
      const int c = j0 + DB + t;
      if (c < TS) {
        double x[DB], l11[DB * (DB - 1) / 2];
#pragma unroll
        for (int r = 0; r < DB; ++r) x[r] = A[(j0 + r) * DL + c];
#pragma unroll
        for (int r = 1; r < DB; ++r)
#pragma unroll
          for (int p = 0; p < r; ++p) l11[r * (r - 1) / 2 + p] = A[(j0 + r) * DL + j0 + p];
#pragma unroll
        for (int r = 1; r < DB; ++r) {
          double s = x[r];
#pragma unroll
          for (int p = 0; p < r; ++p) s -= l11[r * (r - 1) / 2 + p] * x[p];
          x[r] = s;
        }
#pragma unroll
        for (int r = 1; r < DB; ++r) A[(j0 + r) * DL + c] = x[r];
      }
    }
    __syncthreads();
    // ---- A22 -= L21 U12 over the (7 - jb)^2 trailing 16 x 16 tiles
    {
      const int nt = NDB - 1 - jb;
      for (int q = w; q < nt * nt; q += 4) {
        const int r0 = (jb + 1 + q / nt) * DB, c0 = (jb + 1 + q % nt) * DB;
        d4 acc;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[rr] = A[(r0 + fk + 4 * rr) * DL + c0 + fr];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const double av = A[(r0 + fr) * DL + j0 + 4 * kk + fk];
          const double bv = A[(j0 + 4 * kk + fk) * DL + c0 + fr];
          acc = mfma64_neg(av, bv, acc);
        }
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) A[(r0 + fk + 4 * rr) * DL + c0 + fr] = acc[rr];
      }
    }
    __syncthreads();
  }
  CQST(4);
  // V1 (strictly lower, into the panel's top block) and U S (for cq_t_kernel) out, two
  // doubles per store, eight rows' LDS reads in flight together; the signs / tau
#pragma unroll 8
  for (int it = 0; it < 32; ++it) {
    const int e = it * 256 + t, r = e >> 6, c = (e & 63) * 2;
    const d2 v = *reinterpret_cast<const d2*>(&A[r * DL + c]);
    double* pr = P + (int64_t)r * lda + c;
    if (c + 1 < r) *reinterpret_cast<d2*>(pr) = v;
    else if (c < r) pr[0] = v[0];
    if (US)
      *reinterpret_cast<d2*>(US + 2 * e) =
          d2{c >= r ? v[0] * sS[c] : 0.0, c + 1 >= r ? v[1] * sS[c + 1] : 0.0};
  }
  if (t < TS) {
    S[t] = sS[t];
    tau[t] = -A[t * DL + t] * sS[t];
  }
  if (t == 0) fo[3] = 1;   // this panel's R is formed by cq_top_kernel
  __syncthreads();
  // U^T into the lower triangle (each lower slot is written by the one thread
  // that reads its mirror), then U^-T by the LDS triangular inverse
  // (upper entries read, lower written: disjoint, so eight reads go out before the writes)
  for (int it0 = 0; it0 < TS * TS / 256; it0 += 8) {
    double u[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = (it0 + q) * 256 + t, r = e >> 7, c = e & 127;
      u[q] = r > c ? A[c * DL + r] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = (it0 + q) * 256 + t, r = e >> 7, c = e & 127;
      if (r > c) A[r * DL + c] = u[q];
    }
  }
  __syncthreads();
  CQST(5);
  lds_diag_inv_lower(A, Aux);
  __syncthreads();
  lds_inv_block(A, Aux);
  __syncthreads();
  CQST(6);
  // ---- C = U^-T M3 (lower x lower): A operand from LDS, M3 from global (Linv3,
  // written above by this workgroup)
  {
    d4 acc[4][4];
    zero_tile(acc);
    const int wr = w >> 1, wc = w & 1;
    const int kmax = wr * 64 + 64;   // U^-T rows wr*64.. have k <= row
    for (int k0 = 0; k0 < kmax; k0 += 32) {
      double b[8][4];   // the chunk's M3 operands in flight together
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) b[q][j] = Linv3[(k0 + 4 * q + fk) * TS + wc * 64 + j * 16 + fr];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = k0 + 4 * q + fk;
        double a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wr * 64 + i * 16 + fr;   // above the diagonal A still holds U
          a[i] = k <= row ? A[row * DL + k] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma64(a[i], b[q][j], acc[i][j]);
      }
    }
    store_tile(C, TS, acc, 1.0);
  }
#if GPMI_CQ_STAMPS
  CQST(7);
  if (cst)
    printf("cq_recon (10ns): M3 %llu  Linv3 %llu  Q3t %llu  LU %llu  V1/U^T %llu  inv %llu  C %llu\n",
           cs[1] - cs[0], cs[2] - cs[1], cs[3] - cs[2], cs[4] - cs[3], cs[5] - cs[4],
           cs[6] - cs[5], cs[7] - cs[6]);
#endif
}

// The panel's compact-WY T straight from the reconstruction (one workgroup, on a
// stream of its own beside the rest of the chain): from (I - V T V^T) [S; 0] = Q and
// Q - [S; 0] = V U, U = -T V1^T S, so T = -U S V1^-T (V1 the unit lower top block of
// V, S = diag(+-1)). It replaces the V^T V pass and the inverse of tbuild_kernel,
// which had to wait for the whole V (vcopy) and, for the last panels, delayed the
// X T product. A failed panel (the Householder fallback owns it) is left to
// tbuild_kernel. V1^-1 by the LDS triangular inverse, written to W; then
// T = -(U S) (V1^-1)^T as one 128^3 MFMA tile product (upper x upper: the zeros
// below the diagonal come out exactly).
__global__ __launch_bounds__(256) void cq_t_kernel(const double* __restrict__ P, int64_t lda,
                                                   const double* __restrict__ US,
                                                   double* __restrict__ W,
                                                   double* __restrict__ T,
                                                   const int* __restrict__ fail) {
  __shared__ double buf[TS * DL + TS * RLD];
  double* Ls = buf;
  double* Aux = buf + TS * DL;
  const int t = threadIdx.x;
  if (__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  for (int e = t; e < TS * TS; e += 256) {
    const int r = e >> 7, c = e & 127;
    Ls[r * DL + c] = c < r ? P[(int64_t)r * lda + c] : (c == r ? 1.0 : 0.0);
  }
  __syncthreads();
  lds_diag_inv_lower(Ls, Aux);
  __syncthreads();
  lds_inv_block(Ls, Aux);
  __syncthreads();
  for (int e = t; e < TS * TS; e += 256) {
    const int r = e >> 7, c = e & 127;
    W[e] = c <= r ? Ls[r * DL + c] : 0.0;
  }
  __threadfence();
  __syncthreads();   // W complete (the product reads it from L2); Ls free for the stages
  d4 acc[4][4];
  zero_tile(acc);
  gemm_tile<KFAST, KFAST, true>(US, TS, W, TS, TS, buf, acc);
  store_tile(T, TS, acc, 1.0);
}

// The top 128 x 128 block above the diagonal of every CholeskyQR panel, one
// workgroup per panel after the whole reduction: R = (L1 L2 L3)^T, then
// P[r][c] = S_r R[r][c] (c >= r) (the vectors below the diagonal are written by
// cq_recon_kernel). A first-order pass's L is the exact inverse of its applied
// factor Linv (LDS triangular inverse). Per panel p: Lx / Linv at p * 3 * 128^2,
// S at p * 128, flags at p * 8 (flag[3] = 1: the panel's CholeskyQR succeeded), the
// panel at Ab + (p + 1) * 128 * lda + p * 128; scr: 128^2 per panel.
__global__ __launch_bounds__(256) void cq_top_kernel(double* __restrict__ Lx,
                                                     const double* __restrict__ Linv,
                                                     const int* __restrict__ flags,
                                                     const double* __restrict__ S,
                                                     double* __restrict__ scr,
                                                     double* __restrict__ Ab, int64_t lda) {
  __shared__ double pool[TS * DL + TS * RLD];   // LDS inverse, or the gemm_tile stages
  __shared__ double sS[TS];
  const int t = threadIdx.x, p = blockIdx.x;
  const int* fl = flags + 8 * p;
  if (!fl[3]) return;
  double* L = Lx + (int64_t)p * 3 * TS * TS;
  const double* Li = Linv + (int64_t)p * 3 * TS * TS;
  double* sc = scr + (int64_t)p * TS * TS;
  if (t < TS) sS[t] = S[p * TS + t];
  for (int k = 1; k < 3; ++k) {
    if (!fl[k]) continue;
    double* Ls = pool;
    double* Aux = pool + TS * DL;
    for (int e = t; e < TS * TS; e += 256) {
      const int r = e >> 7, c = e & 127;
      Ls[r * DL + c] = (c <= r) ? Li[k * TS * TS + e] : 0.0;
    }
    __syncthreads();
    lds_diag_inv_lower(Ls, Aux);
    __syncthreads();
    lds_inv_block(Ls, Aux);
    __syncthreads();
    for (int e = t; e < TS * TS; e += 256) {
      const int r = e >> 7, c = e & 127;
      L[k * TS * TS + e] = (c <= r) ? Ls[r * DL + c] : 0.0;
    }
    __syncthreads();
  }
  d4 acc[4][4];
  zero_tile(acc);
  // acc[r][c] = sum_k L1[r][k] L2[k][c]
  gemm_tile<KFAST, KSLOW, false>(L, TS, L + TS * TS, TS, TS, pool, acc);
  store_tile(sc, TS, acc, 1.0);
  __syncthreads();
  zero_tile(acc);
  gemm_tile<KFAST, KSLOW, false>(sc, TS, L + 2 * TS * TS, TS, TS, pool, acc);
  store_tile(sc, TS, acc, 1.0);   // M = L1 L2 L3 (lower); R = M^T
  __syncthreads();
  double* P = Ab + (int64_t)(p + 1) * TS * lda + (int64_t)p * TS;
  for (int e = t; e < TS * TS; e += 256) {
    const int r = e >> 7, c = e & 127;
    if (c >= r) P[(int64_t)r * lda + c] = sS[r] * sc[c * TS + r];
  }
}

}  // namespace gpmi
