// Batched blocked Cholesky of K + eta_b I on gfx950 fp64 MFMA, with the
// forward substitution of a resident RHS block, logdet and Gram partials fused
// into the factorization loop.
//
// Replaces, per eta, the reference's dense numerics behind the MixedCorrelation
// duck type:
//   MixedCorrelation.logdet   gaussian_proc/_mixed_correlation/mixed_correlation.py:221-274
//   MixedCorrelation.solve    mixed_correlation.py:280-299 -> _linear_solver.py:71
//                             (scipy.linalg.solve(assume_a='pos') = LAPACK ?posv)
// which the reference runs 2-3 times per DirectLikelihood.log_likelihood
// (_direct_likelihood.py:59,62,332); here one factorization serves all of them.
//
// Algorithm (lower, row-major A, 128-wide diagonal blocks, outer panels of
// S sub-panels, see gpmi_api.hip): per sub-panel k
//   diag_block_kernel : L_kk = chol(A_kk) in LDS, Linv_kk = L_kk^-1, logdet
//                       partial, y_k = Linv_kk r_k, u_k = Linv_kk^T y_k, Gram y_k^T y_k
//   panel_kernel      : L_ik = A_ik Linv_kk^T  and  r_i -= A_ik u_k  (= L_ik y_k)
//   syrk_kernel       : A_ij -= sum_p L_ip L_jp^T over the lower-triangular tiles
// All three are batched over the eta values (blockIdx.y / blockIdx.x = member).

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gpmi_internal.h"

#include "gpmi_device.h"

namespace gpmi {

// ---------------------------------------------------------------------------
// A_b = K + eta_b * I on the lower-triangular 128-tiles (diagonal tiles whole) of
// the first wc tile columns (tri_decode's band enumeration). K is read once per
// launch and written to every batch member. The shift is applied only to the
// first n diagonal entries; pads stay identity.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void shift_copy_kernel(
    const double* __restrict__ K, int64_t ldk, double* __restrict__ A, int64_t lda,
    int64_t sA, const double* __restrict__ etas, int nb, int64_t n, int wc) {
  int I, J;
  tri_decode(blockIdx.x, wc, &I, &J);
  const int t = threadIdx.x;
  for (int e = t; e < TS * TS / 2; e += 256) {
    const int r = e >> 6, c = (e & 63) * 2;
    const int64_t gi = (int64_t)I * TS + r, gj = (int64_t)J * TS + c;
    const d2 v = *reinterpret_cast<const d2*>(K + gi * ldk + gj);
    for (int b = 0; b < nb; ++b) {
      d2 o = v;
      if (gi < n) {
        if (gi == gj) o[0] += etas[b];
        if (gi == gj + 1) o[1] += etas[b];
      }
      *reinterpret_cast<d2*>(A + b * sA + gi * lda + gj) = o;
    }
  }
}

// ---------------------------------------------------------------------------
// Panel: for row tile I = kb + 1 + blockIdx.x of member b = blockIdx.y:
//   L_Ik = A_Ik Linv_kk^T (in place)  and  r_I -= A_Ik u_k.
// ---------------------------------------------------------------------------
#ifndef GPMI_PROBE_PANEL_NO_RHS
#define GPMI_PROBE_PANEL_NO_RHS 0
#endif
__global__ __launch_bounds__(256, 2) void panel_kernel(BatchPtrs P, int64_t lda, int kb) {
  __shared__ double smem[4 * STAGE + TS * RLD];
  double* sA = smem;
  double* sB = smem + 2 * STAGE;
  double* sU = smem + 4 * STAGE;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  const int b = blockIdx.y;
  const int I = kb + 1 + blockIdx.x;
  double* A = P.A + b * P.sA;
  const double* U = P.U + b * P.sU;
  if (!GPMI_PROBE_PANEL_NO_RHS) {
    d2 v[4];
#pragma unroll
    for (int it = 0; it < 4; ++it)
      v[it] = *reinterpret_cast<const d2*>(U + 2 * (it * 256 + t));
#pragma unroll
    for (int it = 0; it < 4; ++it) *reinterpret_cast<d2*>(&sU[2 * (it * 256 + t)]) = v[it];
  }
  double* Aik = A + (int64_t)I * TS * lda + (int64_t)kb * TS;
  const double* Li = P.Linv + b * P.sL + (int64_t)kb * TS * TS;
  d4 acc[4][4];
  d4 racc[2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  racc[0] = racc[1] = d4{0.0, 0.0, 0.0, 0.0};
#if GPMI_PROBE_PANEL_NO_RHS
  // timing probe only (wrong results): the panel without its RHS operand, the bound on
  // what folding r_I -= L_Ik y_k into the SYRK could save (round 6, verdict item 7)
  tile_mma<false>(Aik, lda, Li, TS, TS, sA, sB, acc, sU, racc);
#else
  tile_mma<true>(Aik, lda, Li, TS, TS, sA, sB, acc, sU, racc);
#endif
  // C/D map of v_mfma_f64_16x16x4f64: row = (lane>>4) + 4*r, col = lane&15.
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Aik[(int64_t)(wr * 64 + i * 16 + fk + 4 * r) * lda + wc * 64 + j * 16 + fr] =
            acc[i][j][r];
  double* R = P.R + b * P.sR + (int64_t)I * TS * RLD;
#if GPMI_PROBE_PANEL_NO_RHS
  return;
#endif
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      R[(wr * 64 + wc * 32 + h * 16 + fk + 4 * r) * RLD + fr] -= racc[h][r];
}

// ---------------------------------------------------------------------------
// Trailing update on a band of tile columns [tc0, tc0 + w) over tile rows
// [tc0, tc0 + t): A_IJ -= sum_{p in [p0, p0+kdim)} A_Ip A_Jp^T, J <= I.
// blockIdx.y = batch member.
// ---------------------------------------------------------------------------
// Ksrc (the first trailing update of a factorization): C is read from the shared K
// instead of the member's copy, with eta_b added on the diagonal of its first n rows,
// so A_b = K + eta_b I is never copied for the tiles right of the first outer panel.
__global__ __launch_bounds__(256, 2) void syrk_kernel(double* A, int64_t lda, int64_t sA,
                                                      int tc0, int w, int t, int p0,
                                                      int kdim, const uint32_t* order,
                                                      const double* __restrict__ Ksrc,
                                                      const double* __restrict__ etas,
                                                      int64_t n) {
  __shared__ double smem[4 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1, fr = lane & 15, fk = lane >> 4;
  const int q = xcd_remap(blockIdx.x, gridDim.x);
  int i, j;
  if (order) {
    // host-built grouped order (row groups, column-major inside a group): the
    // tiles in flight on one XCD share a few row and column slabs in its L2
    const uint32_t o = order[q];
    i = (int)(o >> 16);
    j = (int)(o & 0xffffu);
  } else {
    tri_decode(q, w, &i, &j);
  }
  (void)t;
  const int I = tc0 + i, J = tc0 + j;
  double* Ab = A + blockIdx.y * sA;
  const double* P1 = Ab + (int64_t)I * TS * lda + p0;
  const double* P2 = Ab + (int64_t)J * TS * lda + p0;
  // The C tile is loaded into the accumulators up front (its latency overlaps
  // the first operand stage) and the update runs as acc += (-P1) P2^T, so the
  // epilogue is store-only.
  double* C = Ab + (int64_t)I * TS * lda + (int64_t)J * TS;
  const double* Cin = Ksrc ? Ksrc + (int64_t)I * TS * lda + (int64_t)J * TS : C;
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[a][c][r] = Cin[(int64_t)(wr * 64 + a * 16 + fk + 4 * r) * lda + wc * 64 + c * 16 + fr];
  if (Ksrc && I == J && wr == wc) {
    // diagonal entries: a == c, row fk + 4 r == column fr
    const double eta = etas[blockIdx.y];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (fk + 4 * r == fr && (int64_t)I * TS + wr * 64 + a * 16 + fr < n) acc[a][a][r] += eta;
  }
  d4 dummy[2];
  tile_mma<false, true>(P1, lda, P2, lda, kdim, smem, smem + 2 * STAGE, acc, nullptr, dummy);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(int64_t)(wr * 64 + a * 16 + fk + 4 * r) * lda + wc * 64 + c * 16 + fr] = acc[a][c][r];
}

// out[b][0] = logdet = sum of block partials; out[b][1 + e] = Gram entry e (16x16).
__global__ __launch_bounds__(256) void finalize_kernel(BatchPtrs P, int nt, double* out,
                                                       int out_ld) {
  const int b = blockIdx.x, t = threadIdx.x;
  double g = 0.0;
  for (int k = 0; k < nt; ++k) g += P.gram[b * P.sG + (int64_t)k * 256 + t];
  out[b * out_ld + 1 + t] = g;
  if (t == 0) {
    double s = 0.0;
    for (int k = 0; k < nt; ++k) s += P.logdiag[b * P.sLD + k];
    out[b * out_ld] = s;
  }
}

// ---------------------------------------------------------------------------
// Backward substitution L^T X = Y (Y = forward-substituted R), step kb
// (descending). Every workgroup recomputes x_kb = Linv_kb^T y_kb in LDS;
// workgroup j < kb then applies y_j -= L_{kb,j}^T x_kb; workgroup 0 stores x_kb.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bwd_step_kernel(BatchPtrs P, int64_t lda, int kb,
                                                       double* X, int64_t sX) {
  __shared__ double Ys[TS * RLD];
  __shared__ double Xs[TS * RLD];
  const int t = threadIdx.x, b = blockIdx.y, jblk = blockIdx.x;
  const int row = t & 127, half = t >> 7;
  double* R = P.R + b * P.sR;
  const double* A = P.A + b * P.sA;
  const double* Li = P.Linv + b * P.sL + (int64_t)kb * TS * TS;
  for (int e = t; e < TS * RLD; e += 256) Ys[e] = R[(int64_t)kb * TS * RLD + e];
  __syncthreads();
  {
    double xv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) xv[q] = 0.0;
    for (int r = row; r < TS; ++r) {
      const double l = Li[r * TS + row];
#pragma unroll
      for (int q = 0; q < 8; ++q) xv[q] += l * Ys[r * RLD + half * 8 + q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) Xs[row * RLD + half * 8 + q] = xv[q];
  }
  __syncthreads();
  if (jblk == 0) {
    double* Xb = X + b * sX + (int64_t)kb * TS * RLD;
    for (int e = t; e < TS * RLD; e += 256) Xb[e] = Xs[e];
  }
  if (kb == 0) return;
  // y_j[c][q] -= sum_r L_{kb,j}[r][c] x[r][q]
  const double* Lkj = A + (int64_t)kb * TS * lda + (int64_t)jblk * TS;
  const int c = row;
  double yv[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) yv[q] = 0.0;
  for (int r = 0; r < TS; ++r) {
    const double l = Lkj[(int64_t)r * lda + c];
#pragma unroll
    for (int q = 0; q < 8; ++q) yv[q] += l * Xs[r * RLD + half * 8 + q];
  }
  double* Yj = R + (int64_t)jblk * TS * RLD;
#pragma unroll
  for (int q = 0; q < 8; ++q) Yj[c * RLD + half * 8 + q] -= yv[q];
}

// y[:, c] = K x[:, c]  (one wave per row, lanes stride the columns of K).
__global__ __launch_bounds__(256) void gemv_sym_kernel(const double* __restrict__ K,
                                                       int64_t ldk, int64_t n,
                                                       const double* __restrict__ x,
                                                       int64_t ldx, int ncol,
                                                       double* __restrict__ y, double eta,
                                                       int exponent) {
  (void)eta;
  (void)exponent;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  for (int c = 0; c < ncol; ++c) {
    double s = 0.0;
    for (int64_t j = lane; j < n; j += 64) s += K[row * ldk + j] * x[j * ldx + c];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) y[row * ldx + c] = s;
  }
}

// Per-block partial sums of trace(K) and ||K||_F^2 (host adds the partials).
__global__ __launch_bounds__(256) void trace_kernel(const double* __restrict__ K, int64_t ldk,
                                                    int64_t n, double* __restrict__ out) {
  __shared__ double s0[256], s1[256];
  const int t = threadIdx.x;
  const int64_t row = blockIdx.x;
  double a = 0.0, f = 0.0;
  if (row < n) {
    if (t == 0) a = K[row * ldk + row];
    for (int64_t j = t; j < n; j += 256) {
      const double v = K[row * ldk + j];
      f += v * v;
    }
  }
  s0[t] = a;
  s1[t] = f;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) {
      s0[t] += s0[t + off];
      s1[t] += s1[t + off];
    }
    __syncthreads();
  }
  if (t == 0) {
    out[2 * row] = s0[0];
    out[2 * row + 1] = s1[0];
  }
}

}  // namespace gpmi

namespace gpmi {

// Forward substitution step kb with a cached factor (L y = r, descending blocks
// already done): every workgroup recomputes y_kb = Linv_kb r_kb in LDS;
// workgroup 0 stores it, workgroup i > 0 applies r_{kb+i} -= L_{kb+i,kb} y_kb.
__global__ __launch_bounds__(256) void fwd_step_kernel(BatchPtrs P, int64_t lda, int kb) {
  __shared__ double Rs[TS * RLD];
  __shared__ double Ys[TS * RLD];
  const int t = threadIdx.x, b = blockIdx.y, iblk = blockIdx.x;
  const int row = t & 127, half = t >> 7;
  double* R = P.R + b * P.sR;
  const double* A = P.A + b * P.sA;
  const double* Li = P.Linv + b * P.sL + (int64_t)kb * TS * TS;
  for (int e = t; e < TS * RLD; e += 256) Rs[e] = R[(int64_t)kb * TS * RLD + e];
  __syncthreads();
  {
    double yv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) yv[q] = 0.0;
    for (int p = 0; p <= row; ++p) {
      const double l = Li[row * TS + p];
#pragma unroll
      for (int q = 0; q < 8; ++q) yv[q] += l * Rs[p * RLD + half * 8 + q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) Ys[row * RLD + half * 8 + q] = yv[q];
  }
  __syncthreads();
  if (iblk == 0) {
    for (int e = t; e < TS * RLD; e += 256) R[(int64_t)kb * TS * RLD + e] = Ys[e];
    return;
  }
  const int I = kb + iblk;
  const double* Lik = A + (int64_t)I * TS * lda + (int64_t)kb * TS;
  double yv[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) yv[q] = 0.0;
  for (int c = 0; c < TS; ++c) {
    const double l = Lik[(int64_t)row * lda + c];
#pragma unroll
    for (int q = 0; q < 8; ++q) yv[q] += l * Ys[c * RLD + half * 8 + q];
  }
  double* Ri = R + (int64_t)I * TS * RLD;
#pragma unroll
  for (int q = 0; q < 8; ++q) Ri[row * RLD + half * 8 + q] -= yv[q];
}

}  // namespace gpmi
