// Banded Cholesky of B + eta I by block cyclic reduction (odd-even elimination):
// the likelihood terms of the band path with every CU busy even for one eta.
//
// band_chol_kernel (gpmi_band.hip) walks the nt = n_pad / 128 block steps in
// sequence, one workgroup per eta: 128 steps of a 128 x 128 LDS Cholesky chain
// (~9.6 ms at N = 16384 whatever the eta count), so a call with few eta (the
// optimizer's one (sigma, eta) at a time, the per-rank block of a strong-scaled
// curve) leaves most CUs idle. Here each level of the reduction eliminates every
// odd block of the current block-tridiagonal matrix independently and forms the
// Schur complement on the even blocks (numpy prototype tools/bcr_proto.py):
//   odd i:   L_i = chol(D_i), Linv_i, Z_i = Linv_i Y_i,            bcr_chol_kernel
//            logdet += 2 sum log diag L_i, G += Z_i^T Z_i
//            W_l = Linv_i F_{i-1},  W_r = Linv_i F_i^T              bcr_w_kernel
//   even j:  D_j' = D_j - W_r(j-1)^T W_r(j-1) - W_l(j+1)^T W_l(j+1)  bcr_upd_kernel
//            Y_j' = Y_j - W_r(j-1)^T Z_{j-1} - W_l(j+1)^T Z_{j+1}
//            F_{j/2}' = -W_r(j+1)^T W_l(j+1)
// (F_i = B_{i+1,i}: upper triangular at level 0, full after). ceil(log2 nt)
// levels of three launches, each with (blocks x eta) workgroups; it is a block
// Cholesky factorization of the odd-even permuted matrix, so logdet and
// Y^T (B + eta I)^-1 Y are exact to rounding (not bit-identical to the sequential
// order). Every sum has a fixed order: per-block partials (logdet, Z^T Z,
// failure) are reduced by bcr_final_kernel in original block order.
//
// Replaces, like band_chol_kernel, the per-eta logdet + 2 solves of the
// reference's 'eigenvalue' operator (mixed_correlation.py:239-248,
// _direct_likelihood.py:59,62,332).

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gpmi_internal.h"
#include "gpmi_device.h"
#include "gpmi_lds_chol.h"
#include "gpmi_band.h"
#include "gpmi_tile.h"

namespace gpmi {

// Level-0 couplings F_i = triu(B_{i+1,i}) (the lower part of the stored tile holds
// Householder vectors), shared by every eta. grid (nt - 1).
__global__ __launch_bounds__(256) void bcr_f0_kernel(const double* __restrict__ Ab, int64_t lda,
                                                     double* __restrict__ F0) {
  const int i = blockIdx.x;
  const double* src = Ab + (int64_t)(i + 1) * TS * lda + (int64_t)i * TS;
  double* dst = F0 + (int64_t)i * TS * TS;
  for (int e = threadIdx.x; e < TS * TS; e += 256) {
    const int r = e >> 7, c = e & 127;
    dst[e] = c >= r ? src[(int64_t)r * lda + c] : 0.0;
  }
}

// Eliminate block p = first + 2 blockIdx.x of level `lvl` for eta blockIdx.y:
// D_p (level 0: the stored diagonal tile + eta I; else Din) -> L, Linv (to Lout
// when lout), Z = Linv Y_p (to Zall at the block's original index o = p << lvl),
// the block's logdet, Z^T Z and failure partials (original index o).
__global__ __launch_bounds__(256) void bcr_chol_kernel(
    const double* __restrict__ Ab, int64_t lda, const double* __restrict__ etas, int lvl, int first,
    const double* __restrict__ Din, int64_t sD, const double* __restrict__ Yin, int64_t sY,
    double* __restrict__ Lout, int64_t sL, int lout, double* __restrict__ Zall, int64_t sZ,
    double* __restrict__ logd, double* __restrict__ gpart, int* __restrict__ failv, int nt,
    int64_t n) {
  __shared__ double Ls[TS * DL];
  __shared__ double Aux[TS * RLD];
  __shared__ double sdiag[TS];
  __shared__ double sred[2];
  __shared__ int s_fail;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int e = blockIdx.y;
  const int p = first + 2 * blockIdx.x;
  const int o = p << lvl;   // original block index
  if (lvl == 0) {
    const double eta = etas[e];
    const double* src = Ab + (int64_t)p * TS * lda + (int64_t)p * TS;
    for (int q = t; q < TS * TS; q += 256) {
      const int r = q >> 7, c = q & 127;
      Ls[r * DL + c] = (c <= r) ? src[(int64_t)r * lda + c] + (r == c ? eta : 0.0) : 0.0;
    }
  } else {
    const double* src = Din + e * sD + (int64_t)p * TS * TS;
    for (int q = t; q < TS * TS; q += 256) {
      const int r = q >> 7, c = q & 127;
      Ls[r * DL + c] = (c <= r) ? src[q] : 0.0;
    }
  }
  // Y_p -> Aux (k-major [128][16])
  const double* ysrc = Yin + e * sY + (int64_t)p * TS * RLD;
  for (int q = t; q < TS * RLD; q += 256) Aux[q] = ysrc[q];
  if (t == 0) s_fail = 0;
  __syncthreads();
  // keep Y in registers: lds_chol_block uses Aux as scratch
  d4 Rr[2];
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = slot == 0 ? w : NDB - 1 - w;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) Rr[slot][rr] = Aux[(ti * DB + fk + 4 * rr) * RLD + fr];
  }
  __syncthreads();
  lds_chol_block(Ls, Aux, sdiag, &s_fail);
  if (w < 2) {
    double v = ((int64_t)o * TS + t < n) ? log(sdiag[t]) : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) sred[w] = v;
  }
  __syncthreads();
  if (t == 0) {
    logd[(int64_t)e * nt + o] = 2.0 * (sred[0] + sred[1]);
    failv[(int64_t)e * nt + o] = s_fail ? o * TS + s_fail : 0;
  }
  lds_inv_block(Ls, Aux);
  __syncthreads();
  if (lout) {
    double* dst = Lout + e * sL + (int64_t)o * TS * TS;
    for (int q = t; q < TS * TS; q += 256) {
      const int r = q >> 7, c = q & 127;
      dst[q] = (c <= r) ? Ls[r * DL + c] : 0.0;
    }
  }
  // Y back to Aux, then Z = Linv Y (the lower-triangular k-tiles only)
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = slot == 0 ? w : NDB - 1 - w;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) Aux[(ti * DB + fk + 4 * rr) * RLD + fr] = Rr[slot][rr];
  }
  __syncthreads();
  d4 Zv[2];
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = slot == 0 ? w : NDB - 1 - w;
    d4 a0 = {0.0, 0.0, 0.0, 0.0}, a1 = {0.0, 0.0, 0.0, 0.0};
    for (int kt = 0; kt <= ti; ++kt) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double av = Ls[(ti * DB + fr) * DL + kt * DB + 4 * kk + fk];
        const double bv = Aux[(kt * DB + 4 * kk + fk) * RLD + fr];
        if (kk & 1) a1 = mfma64(av, bv, a1);
        else a0 = mfma64(av, bv, a0);
      }
    }
    Zv[slot] = a0 + a1;
  }
  __syncthreads();
  double* zdst = Zall + e * sZ + (int64_t)o * TS * RLD;
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = slot == 0 ? w : NDB - 1 - w;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int r = ti * DB + fk + 4 * rr;
      Aux[r * RLD + fr] = Zv[slot][rr];
      zdst[r * RLD + fr] = Zv[slot][rr];
    }
  }
  __syncthreads();
  // Z^T Z over this wave's two 16-row slices, the waves summed in order
  d4 G = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kt = 2 * w + h;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const double v = Aux[(kt * DB + 4 * kk + fk) * RLD + fr];
      G = mfma64(v, v, G);
    }
  }
  d4* sg = reinterpret_cast<d4*>(Ls);
  __syncthreads();
  sg[w * 64 + lane] = G;
  __syncthreads();
  if (w == 0) {
    const d4 Gs = ((sg[lane] + sg[64 + lane]) + sg[128 + lane]) + sg[192 + lane];
    double* gd = gpart + ((int64_t)e * nt + o) * RLD * RLD;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) gd[(fk + 4 * rr) * RLD + fr] = Gs[rr];
  }
}

// W of odd block p = 1 + 2 (bx >> 1): which = bx & 1:
//   0: W_l = Linv_p F_{p-1};  1: W_r = Linv_p F_p^T (only when p + 1 < m).
// F: level 0 the shared F0 (sF = 0), else Fin. Linv and W are stored by the block's
// original index (p << lvl): every level's factor survives for the solves of
// bcr_back_kernel / bcr_rhs_*.
__device__ __forceinline__ void bcr_w_role(int bx, const double* __restrict__ Lin, int64_t sL,
                                           const double* __restrict__ Fin, int64_t sF,
                                           double* __restrict__ W, int64_t sW, int m, int lvl,
                                           double* smem) {
  const int e = blockIdx.y;
  const int h = bx >> 1, which = bx & 1;
  const int p = 1 + 2 * h;
  const int o = p << lvl;
  if (which == 1 && p + 1 >= m) return;
  const double* L = Lin + e * sL + (int64_t)o * TS * TS;
  d4 acc[4][4];
  zero_tile(acc);
  if (which == 0)
    gemm_tile<KFAST, KSLOW, false>(L, TS, Fin + e * sF + (int64_t)(p - 1) * TS * TS, TS, TS, smem,
                                   acc);
  else
    gemm_tile<KFAST, KFAST, false>(L, TS, Fin + e * sF + (int64_t)p * TS * TS, TS, TS, smem, acc);
  store_tile(W + e * sW + ((int64_t)o * 2 + which) * TS * TS, TS, acc, 1.0);
}

// Tangent of the eliminated block's inverse factor (defined with the tangent kernels
// below): dLinv = -Phi(Linv dD Linv^T) Linv.
__device__ void bcr_dfac_role(const double* __restrict__ L, int64_t sL,
                              const double* __restrict__ dDin, int64_t sdD,
                              double* __restrict__ scr, int64_t sS, double* __restrict__ dL,
                              int lvl, int p, double* smem);

// bcr_w_role for bx < 2 nodd (nodd = m / 2); with tangents (dL != nullptr) the
// workgroups bx - 2 nodd < nodd form the same blocks' dLinv beside them (level m == 1:
// the last level's single block, p = 0).
__global__ __launch_bounds__(256, 2) void bcr_w_kernel(const double* __restrict__ Lin, int64_t sL,
                                                       const double* __restrict__ Fin, int64_t sF,
                                                       double* __restrict__ W, int64_t sW,
                                                       int m, int lvl,
                                                       const double* __restrict__ dDin,
                                                       int64_t sdD, double* __restrict__ scr,
                                                       double* __restrict__ dL) {
  __shared__ double smem[4 * GSTAGE];
  const int nodd = m / 2;
  const int bx = blockIdx.x;
  if (bx < 2 * nodd) {
    bcr_w_role(bx, Lin, sL, Fin, sF, W, sW, m, lvl, smem);
    return;
  }
  const int d = bx - 2 * nodd;
  bcr_dfac_role(Lin, sL, dDin, sdD, scr, sW, dL, lvl, m == 1 ? 0 : 1 + 2 * d, smem);
}

// dW of odd block p = 1 + 2 (bx >> 1), which = bx & 1 as bcr_w_role (defined below).
__device__ void bcr_dw_role(int bx, const double* __restrict__ L, const double* __restrict__ dL,
                            int64_t sL, const double* __restrict__ Fin, int64_t sF,
                            const double* __restrict__ dFin, int64_t sdF, double* __restrict__ dW,
                            int64_t sW, int m, int lvl, double* smem);

// Even block j = 2 (bx / 3) of an m-block level: which = bx % 3:
//   0: D_j',  1: F_{j/2}' = -W_r(j+1)^T W_l(j+1)  (only when j + 2 < m),
//   2: Y_j' = Y_j - W_r(j-1)^T Z_{j-1} - W_l(j+1)^T Z_{j+1} (its own workgroup: the
//      scalar 128 x 16 update no longer follows the D' products).
// W pairs of odd block i at W[(i << lvl) * 2 + {0: l, 1: r}]; Z of odd block i at
// its original index (i << lvl) in Zall. With tangents (dW != nullptr) the workgroups
// bx - 3 neven < 2 nodd form the level's dW (bcr_dw_role) beside them.
__global__ __launch_bounds__(256, 2) void bcr_upd_kernel(
    const double* __restrict__ Ab, int64_t lda, const double* __restrict__ etas, int lvl,
    const double* __restrict__ Din, int64_t sD, const double* __restrict__ Yin, int64_t sY,
    const double* __restrict__ W, int64_t sW, const double* __restrict__ Zall, int64_t sZ,
    double* __restrict__ Dout, double* __restrict__ Fout, double* __restrict__ Yout, int64_t sO,
    int64_t sOY, int m, const double* __restrict__ L, const double* __restrict__ dL, int64_t sL,
    const double* __restrict__ Fin, int64_t sF, const double* __restrict__ dFin, int64_t sdF,
    double* __restrict__ dW) {
  __shared__ double smem[4 * GSTAGE];
  const int neven = (m + 1) / 2;
  if ((int)blockIdx.x >= 3 * neven) {
    bcr_dw_role(blockIdx.x - 3 * neven, L, dL, sL, Fin, sF, dFin, sdF, dW, sW, m, lvl, smem);
    return;
  }
  const int e = blockIdx.y;
  const int h = blockIdx.x / 3, which = blockIdx.x % 3;
  const int j = 2 * h;
  const double* We = W + e * sW;
  const bool left = j >= 1, right = j + 1 < m;
  if (which == 2) {
    // Y_j' = Y_j - W_r(j-1)^T Z_{j-1} - W_l(j+1)^T Z_{j+1}: thread (row r, 8 columns)
    const int t = threadIdx.x, r = t >> 1, c0 = (t & 1) * 8;
    const double* ysrc = Yin + e * sY + (int64_t)j * TS * RLD;
    double y[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) y[q] = ysrc[r * RLD + c0 + q];
    for (int side = 0; side < 2; ++side) {
      if (side == 0 && !left) continue;
      if (side == 1 && !right) continue;
      const int i = side == 0 ? j - 1 : j + 1;
      const double* Wm = We + ((int64_t)(i << lvl) * 2 + (side == 0 ? 1 : 0)) * TS * TS;
      const double* Z = Zall + e * sZ + (int64_t)(i << lvl) * TS * RLD;
      for (int k = 0; k < TS; ++k) {
        const double wv = Wm[k * TS + r];
#pragma unroll
        for (int q = 0; q < 8; ++q) y[q] -= wv * Z[k * RLD + c0 + q];
      }
    }
    double* ydst = Yout + e * sOY + (int64_t)h * TS * RLD;
#pragma unroll
    for (int q = 0; q < 8; ++q) ydst[r * RLD + c0 + q] = y[q];
    return;
  }
  d4 acc[4][4];
  if (which == 1) {
    if (j + 2 >= m) return;
    const double* Wl = We + ((int64_t)((j + 1) << lvl) * 2 + 0) * TS * TS;
    const double* Wr = We + ((int64_t)((j + 1) << lvl) * 2 + 1) * TS * TS;
    zero_tile(acc);
    gemm_tile_rr<true>(Wr, true, Wl, true, smem, acc);
    store_tile(Fout + e * sO + (int64_t)h * TS * TS, TS, acc, 1.0);
    return;
  }
  if (lvl == 0) {
    load_tile(Ab + (int64_t)j * TS * lda + (int64_t)j * TS, lda, acc);
    const double eta = etas[e];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (wr * 64 + a * 16 + fk + 4 * r == wc * 64 + c * 16 + fr) acc[a][c][r] += eta;
  } else {
    load_tile(Din + e * sD + (int64_t)j * TS * TS, TS, acc);
  }
  // W_r(j-1)^T W_r(j-1), then W_l(j+1)^T W_l(j+1): a rolled loop (one inlined product)
#pragma unroll 1
  for (int q = 0; q < 2; ++q) {
    if (q == 0 ? !left : !right) continue;
    const double* Wm = We + ((int64_t)((q == 0 ? j - 1 : j + 1) << lvl) * 2 + (q == 0 ? 1 : 0)) *
                                TS * TS;
    gemm_tile_rr<true>(Wm, true, Wm, true, smem, acc);
  }
  store_tile(Dout + e * sO + (int64_t)h * TS * TS, TS, acc, 1.0);
}

// out[e][0] = logdet (original block order), out[e][1 + a * 16 + c] = sum of the
// blocks' Z^T Z, info[e] = the first failing block's pivot code. grid (neta).
__global__ __launch_bounds__(256) void bcr_final_kernel(const double* __restrict__ logd,
                                                        const double* __restrict__ gpart,
                                                        const int* __restrict__ failv, int nt,
                                                        double* __restrict__ out, int out_ld,
                                                        int* __restrict__ info) {
  const int e = blockIdx.x, t = threadIdx.x;
  double g = 0.0;
  for (int o = 0; o < nt; ++o) g += gpart[((int64_t)e * nt + o) * RLD * RLD + t];
  out[(int64_t)e * out_ld + 1 + t] = g;
  if (t == 0) {
    double s = 0.0;
    int f = 0;
    for (int o = 0; o < nt; ++o) {
      s += logd[(int64_t)e * nt + o];
      if (!f) f = failv[(int64_t)e * nt + o];
    }
    out[(int64_t)e * out_ld] = s;
    info[e] = f;
  }
}

// ---------------------------------------------------------------------------
// Derivative terms (ProfileLikelihood der1 / der2, _profile_likelihood.py:91-192:
// G2 = Y^T (B + eta I)^-2 Y, G3 = Y^T (B + eta I)^-3 Y) from the stored levels:
// back substitution X = (B + eta I)^-1 Y from the last level down,
//   x_i = Linv_i^T (Z_i - W_l(i) x_{i-1} - W_r(i) x_{i+1}),   G2 = sum X_o^T X_o,
// then the forward elimination again with X as the right-hand side,
//   Z'_i = Linv_i Y'_i,  Y'_j -= W_r(j-1)^T Z'_{j-1} + W_l(j+1)^T Z'_{j+1},
//   G3 = sum Z'^T Z' (= X^T (B + eta I)^-1 X).
// Blocks by original index; 128 x 16 products as plain FMAs (thread = row, 8 columns).
// ---------------------------------------------------------------------------

// Z^T Z of a 128 x 16 block in LDS (row stride RLD) into g[256], fixed order.
__device__ __forceinline__ void block_gram(const double* Zs, double* g) {
  const int t = threadIdx.x, a = t >> 4, c = t & 15;
  double acc = 0.0;
  for (int k = 0; k < TS; ++k) acc += Zs[k * RLD + a] * Zs[k * RLD + c];
  g[t] = acc;
}

// Odd blocks p = first + 2 blockIdx.x of level lvl (first 0: the last level's single
// block): x_p -> Xall[o], X_o^T X_o -> g2part[o].
__global__ __launch_bounds__(256) void bcr_back_kernel(
    const double* __restrict__ L, int64_t sL, const double* __restrict__ W, int64_t sW,
    const double* __restrict__ Zall, int64_t sZ, double* __restrict__ Xall,
    double* __restrict__ g2part, int nt, int lvl, int first, int m) {
  __shared__ double xs[2][TS * RLD];
  __shared__ double vs[TS * RLD];
  const int t = threadIdx.x, r = t >> 1, c0 = (t & 1) * 8;
  const int e = blockIdx.y;
  const int p = first + 2 * blockIdx.x;
  const int o = p << lvl;
  const double* Z = Zall + e * sZ + (int64_t)o * TS * RLD;
  const bool left = first == 1, right = first == 1 && p + 1 < m;
  const double* Xe = Xall + e * sZ;
  for (int q = t; q < TS * RLD; q += 256) {
    xs[0][q] = left ? Xe[(int64_t)((p - 1) << lvl) * TS * RLD + q] : 0.0;
    xs[1][q] = right ? Xe[(int64_t)((p + 1) << lvl) * TS * RLD + q] : 0.0;
  }
  __syncthreads();
  double v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = Z[r * RLD + c0 + q];
  for (int side = 0; side < 2; ++side) {
    if ((side == 0 && !left) || (side == 1 && !right)) continue;
    const double* Wm = W + e * sW + ((int64_t)o * 2 + side) * TS * TS + (int64_t)r * TS;
    const double* x = xs[side];
    for (int k = 0; k < TS; ++k) {
      const double wv = Wm[k];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] -= wv * x[k * RLD + c0 + q];
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) vs[r * RLD + c0 + q] = v[q];
  __syncthreads();
  // x = Linv^T v (Linv lower: rows k >= r of column r)
  const double* Lm = L + e * sL + (int64_t)o * TS * TS;
  double x[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] = 0.0;
  for (int k = r; k < TS; ++k) {
    const double lv = Lm[k * TS + r];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] += lv * vs[k * RLD + c0 + q];
  }
  __syncthreads();
  double* Xo = Xall + e * sZ + (int64_t)o * TS * RLD;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    Xo[r * RLD + c0 + q] = x[q];
    vs[r * RLD + c0 + q] = x[q];
  }
  __syncthreads();
  block_gram(vs, g2part + ((int64_t)e * nt + o) * RLD * RLD);
}

// Forward elimination of a right-hand side, odd blocks p = first + 2 blockIdx.x:
// Z'_o = Linv_o Y'_p -> Zp[o], Z'^T Z' -> g3part[o]. Yin: the level's blocks (level 0:
// Xall, blocks by original index = level index).
__global__ __launch_bounds__(256) void bcr_rhs_odd_kernel(
    const double* __restrict__ L, int64_t sL, const double* __restrict__ Yin, int64_t sY,
    double* __restrict__ Zp, int64_t sZ, double* __restrict__ g3part, int nt, int lvl,
    int first) {
  __shared__ double ys[TS * RLD];
  const int t = threadIdx.x, r = t >> 1, c0 = (t & 1) * 8;
  const int e = blockIdx.y;
  const int p = first + 2 * blockIdx.x;
  const int o = p << lvl;
  const double* Y = Yin + e * sY + (int64_t)p * TS * RLD;
  for (int q = t; q < TS * RLD; q += 256) ys[q] = Y[q];
  __syncthreads();
  const double* Lm = L + e * sL + (int64_t)o * TS * TS + (int64_t)r * TS;
  double z[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) z[q] = 0.0;
  for (int k = 0; k <= r; ++k) {
    const double lv = Lm[k];
#pragma unroll
    for (int q = 0; q < 8; ++q) z[q] += lv * ys[k * RLD + c0 + q];
  }
  __syncthreads();
  double* Zo = Zp + e * sZ + (int64_t)o * TS * RLD;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    Zo[r * RLD + c0 + q] = z[q];
    ys[r * RLD + c0 + q] = z[q];
  }
  __syncthreads();
  block_gram(ys, g3part + ((int64_t)e * nt + o) * RLD * RLD);
}

// Even blocks j = 2 blockIdx.x of an m-block level: Y'_j - W_r(j-1)^T Z'_{j-1}
// - W_l(j+1)^T Z'_{j+1} -> Yout[j / 2].
__global__ __launch_bounds__(256) void bcr_rhs_even_kernel(
    const double* __restrict__ W, int64_t sW, const double* __restrict__ Zp, int64_t sZ,
    const double* __restrict__ Yin, int64_t sY, double* __restrict__ Yout, int64_t sOY, int lvl,
    int m) {
  const int t = threadIdx.x, r = t >> 1, c0 = (t & 1) * 8;
  const int e = blockIdx.y;
  const int j = 2 * blockIdx.x;
  const double* Y = Yin + e * sY + (int64_t)j * TS * RLD;
  double y[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) y[q] = Y[r * RLD + c0 + q];
  for (int side = 0; side < 2; ++side) {
    if ((side == 0 && j < 1) || (side == 1 && j + 1 >= m)) continue;
    const int i = side == 0 ? j - 1 : j + 1;
    const double* Wm = W + e * sW + ((int64_t)(i << lvl) * 2 + (side == 0 ? 1 : 0)) * TS * TS;
    const double* Z = Zp + e * sZ + (int64_t)(i << lvl) * TS * RLD;
    for (int k = 0; k < TS; ++k) {
      const double wv = Wm[k * TS + r];
#pragma unroll
      for (int q = 0; q < 8; ++q) y[q] -= wv * Z[k * RLD + c0 + q];
    }
  }
  double* yd = Yout + e * sOY + (int64_t)blockIdx.x * TS * RLD;
#pragma unroll
  for (int q = 0; q < 8; ++q) yd[r * RLD + c0 + q] = y[q];
}

// der[e][0:256] = sum_o g2part, der[e][256:512] = sum_o g3part (original block order).
__global__ __launch_bounds__(256) void bcr_der_final_kernel(const double* __restrict__ g2part,
                                                            const double* __restrict__ g3part,
                                                            int nt, double* __restrict__ der) {
  const int e = blockIdx.x, t = threadIdx.x;
  double a = 0.0, b = 0.0;
  for (int o = 0; o < nt; ++o) {
    a += g2part[((int64_t)e * nt + o) * RLD * RLD + t];
    b += g3part[((int64_t)e * nt + o) * RLD * RLD + t];
  }
  der[(int64_t)e * 2 * RLD * RLD + t] = a;
  der[(int64_t)e * 2 * RLD * RLD + RLD * RLD + t] = b;
}

// ---------------------------------------------------------------------------
// trace((B + eta I)^-1) by selected inversion down the reduction tree (round 5):
// the factor above is a block Cholesky of the odd-even permuted matrix, in which
// block p of level l (odd) is eliminated before its two neighbours l = p - 1,
// r = p + 1 of that level, with L_{l,p} = W_l^T and L_{r,p} = W_r^T (bcr_w_kernel).
// The Takahashi recurrences (Takahashi, Fagan and Chin 1973; Erisman and Tinney,
// Comm. ACM 18 (1975) 177) need only the inverse's blocks on the factor's pattern:
//   X_s  = W_s^T Linv_p                          s in {l, r}
//   Z_sp = -(Z_sl X_l + Z_sr X_r)                                bcr_sinv_off_kernel
//   Z_pp = Linv_p^T Linv_p - X_l^T Z_lp - X_r^T Z_rp              bcr_sinv_diag_kernel
// top-down from the last level's single block (Z = Linv^T Linv), level by level,
// every node of a level independent (numpy prototype tools/bcr_sinv_proto.py: the
// diagonal blocks equal inv(A)'s to 1e-16). X_s and Linv_p^T Linv_p depend on the
// factor only, so ONE launch forms them for every block of every level before the
// top-down pass (bcr_sinv_pre_kernel; round 6, with the tangents below: the level
// loop keeps two launches of <= 2 products (<= 4 with tangents) per level, against
// three of 1 / 2 / 3 (+ 2 / 4 / 6) before). The parents' coupling Z_lr is the
// off-diagonal block their own elimination produced one level up: l' = (p - 1) / 2
// and r' = l' + 1 there; if r' is odd it is Z_{l', r'} = Zo[o_r][0], else l' is odd and
// Z_lr = Zo[o_l][1]^T. tr Z_pp over the rows < n (the identity pad is decoupled) per
// block, summed in block order by bcr_sinv_final_kernel. This replaces the eigenvalue
// sums sum_i (lambda_i + eta)^-1 of the reference's 'eigenvalue' traceinv
// (mixed_correlation.py:172-181) without the eigenvalues: O(n b^2) per eta.
// Blocks by original index o = p << l: Zd[o] (diagonal), Zo[o][2] (Z_lp, Z_rp), X[o][2].
//
// trace((B + eta I)^-2) without eigenvalues (round 6): -d/deta trace((B + eta I)^-1)
// by forward-mode differentiation of the factor and of the selected inversion
// (numpy prototype tools/bcr_dsinv_proto.py). Every block carries its eta-tangent
// (d/deta); level 0: dD = I, dF = 0.
// Factor (with bcr_w / bcr_upd of the level, as extra workgroups of their launches):
//   M_p     = Phi(Linv_p dD_p Linv_p^T)   Phi: strict lower + half diagonal   bcr_dfac_role
//   dLinv_p = -M_p Linv_p                 (S = L L^T, dS = dL L^T + L dL^T)
//   dW_l    = dLinv_p F_{p-1} + Linv_p dF_{p-1}                               bcr_dw_role
//   dW_r    = dLinv_p F_p^T   + Linv_p dF_p^T
//   dD_j'   = dD_j - (dW_r^T W_r + W_r^T dW_r)(j-1) - (dW_l^T W_l + W_l^T dW_l)(j+1)
//   dF_j/2' = -(dW_r^T W_l + W_r^T dW_l)(j+1)                                 bcr_dupd
// Selected inversion (extra workgroups of the launches above):
//   dX_s  = dW_s^T Linv_p + W_s^T dLinv_p
//   dZ_sp = -(dZ_sl X_l + Z_sl dX_l + dZ_sr X_r + Z_sr dX_r)
//   dZ_pp = dLinv^T Linv + Linv^T dLinv - dX_l^T Z_lp - X_l^T dZ_lp
//           - dX_r^T Z_rp - X_r^T dZ_rp
// trace((B + eta I)^-2) = -sum_p tr dZ_pp over the rows < n. This replaces the
// eigenvalue sums sum_i (lambda_i + eta)^-2 of the reference's 'eigenvalue'
// traceinv(eta, exponent=2) (mixed_correlation.py:172-181), which the direct
// Hessian (_direct_likelihood.py:224) and the profiled der2
// (_profile_likelihood.py:168) call: O(n b^2) per eta, about three times the
// selected inversion's products.
// ---------------------------------------------------------------------------

// the diagonal elements of a 128 x 128 accumulator tile (C/D map of load_tile):
// acc += v on the diagonal
__device__ __forceinline__ void tile_add_diag(d4 (&acc)[4][4], double v) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  if (wr != wc) return;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (fk + 4 * r == fr) acc[a][a][r] += v;
}

// sum over the rows < n of the tile's diagonal (block o), to trpart (scaled by sign);
// smem: 4 doubles of scratch
__device__ __forceinline__ void tile_trace(const d4 (&acc)[4][4], int o, int64_t n, double sign,
                                           double* smem, double* trpart) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  double v = 0.0;
  if (wr == wc)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 64 + a * 16 + fk + 4 * r;
        if (fk + 4 * r == fr && (int64_t)o * TS + row < n) v += acc[a][a][r];
      }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if (lane == 0) smem[w] = v;
  __syncthreads();
  if (t == 0) *trpart = sign * ((smem[0] + smem[1]) + (smem[2] + smem[3]));
}

// Block o's level, its index p there and the level's block count (m0 = nt blocks at
// level 0, ceil(m / 2) each level up; o = 0 is the root, at level L with m = 1).
__device__ __forceinline__ void bcr_node(int o, int nt, int L, int& lvl, int& p, int& m) {
  lvl = o == 0 ? L : __builtin_ctz(o);
  p = o >> lvl;
  m = nt;
  for (int l = 0; l < lvl; ++l) m = (m + 1) >> 1;
}

// Every eliminated block's factor-only terms, before the top-down pass. Workgroup
// bx: block o = bx / (3 + 3 ntan), role = bx % (3 + 3 ntan) (roles 3-5: tangents):
//   0: X_l = W_l^T Linv   1: X_r = W_r^T Linv (p + 1 < m)   2: Zd = Linv^T Linv
//   3: dX_l               4: dX_r                           5: dZd = dLinv^T Linv + Linv^T dLinv
// The root (o = 0) has roles 2 and 5 only, and its trace (it is final).
__global__ __launch_bounds__(256, 2) void bcr_sinv_pre_kernel(
    const double* __restrict__ L, const double* __restrict__ dL, int64_t sL,
    const double* __restrict__ W, const double* __restrict__ dW, int64_t sW,
    double* __restrict__ X, double* __restrict__ dX, int64_t sX, double* __restrict__ Zd,
    double* __restrict__ dZd, int64_t sZd, double* __restrict__ trpart,
    double* __restrict__ dtrpart, int nt, int nlev, int64_t n, int ntan) {
  __shared__ double smem[4 * GSTAGE];
  const int e = blockIdx.y;
  const int o = blockIdx.x / (3 + 3 * ntan), role = blockIdx.x % (3 + 3 * ntan);
  int lvl, p, m;
  bcr_node(o, nt, nlev, lvl, p, m);
  if (o == 0 && role != 2 && role != 5) return;
  if ((role == 1 || role == 4) && p + 1 >= m) return;
  const int64_t lo = e * sL + (int64_t)o * TS * TS;
  const double* Lo = L + lo;
  const bool tan = role >= 3;
  const int side = (role % 3) == 1 ? 1 : 0;
  const int64_t wo = e * sW + ((int64_t)o * 2 + side) * TS * TS;
  d4 acc[4][4];
  zero_tile(acc);
  const int nterm = tan ? 2 : 1;
#pragma unroll 1
  for (int t = 0; t < nterm; ++t) {
    const double* A;
    const double* Bm;
    if (role % 3 == 2) {   // Linv^T Linv;  dLinv^T Linv + Linv^T dLinv
      A = (tan && t == 0) ? dL + lo : Lo;
      Bm = (tan && t == 1) ? dL + lo : Lo;
    } else {               // W_s^T Linv;   dW_s^T Linv + W_s^T dLinv
      A = (tan && t == 0) ? dW + wo : W + wo;
      Bm = (tan && t == 1) ? dL + lo : Lo;
    }
    gemm_tile<KSLOW, KSLOW, false>(A, TS, Bm, TS, TS, smem, acc);
  }
  if (role % 3 == 2) {
    store_tile((tan ? dZd : Zd) + e * sZd + (int64_t)o * TS * TS, TS, acc, 1.0);
    if (o == 0)
      tile_trace(acc, 0, n, tan ? -1.0 : 1.0, smem, (tan ? dtrpart : trpart) + (int64_t)e * nt);
  } else {
    store_tile((tan ? dX : X) + e * sX + ((int64_t)o * 2 + side) * TS * TS, TS, acc, 1.0);
  }
}

// Z_sp (and with tangents, ntan = 1, dZ_sp) of the odd blocks p = 1 + 2 h of level
// lvl: workgroup bx = (2 + 2 ntan) h + 2 tan + side (grid (2 + 2 ntan) nodd).
//   Z_lp  = -(Z_ll X_l + Z_lr X_r)            Z_rp = -(Z_rl X_l + Z_rr X_r)
//   dZ_lp = -(dZ_ll X_l + Z_ll dX_l + dZ_lr X_r + Z_lr dX_r), dZ_rp likewise.
// The products run in a rolled loop on the runtime-layout product (the coupling Z_lr
// is stored directly or transposed): one inlined product per kernel.
__global__ __launch_bounds__(256, 2) void bcr_sinv_off_kernel(
    const double* __restrict__ Zd, const double* __restrict__ dZd, int64_t sZd,
    double* __restrict__ Zo, double* __restrict__ dZo, int64_t sZo,
    const double* __restrict__ X, const double* __restrict__ dX, int64_t sX, int m, int lvl,
    int ntan) {
  __shared__ double smem[4 * GSTAGE];
  const int e = blockIdx.y;
  const int R = 2 + 2 * ntan;
  const int h = blockIdx.x / R, tan = (blockIdx.x % R) >> 1, side = blockIdx.x & 1;
  const int p = 1 + 2 * h;
  const bool right = p + 1 < m;
  if (side == 1 && !right) return;
  const int o = p << lvl, ol = (p - 1) << lvl, orr = (p + 1) << lvl;
  const double* Xl = X + e * sX + ((int64_t)o * 2 + 0) * TS * TS;
  const double* Xr = Xl + TS * TS;
  const double* dXl = dX + e * sX + ((int64_t)o * 2 + 0) * TS * TS;
  const double* dXr = dXl + TS * TS;
  // the parents' coupling: stored as Z_lr (r' odd one level up) or Z_rl (l' odd)
  int64_t qlr = 0;
  bool lr_direct = true;
  if (right) {
    const int lp = (p - 1) >> 1;
    if ((lp + 1) & 1) {
      qlr = ((int64_t)orr * 2 + 0) * TS * TS;   // Z_{l', r'}
    } else {
      qlr = ((int64_t)ol * 2 + 1) * TS * TS;    // Z_{r', l'}
      lr_direct = false;
    }
  }
  const double* Mlr = Zo + e * sZo + qlr;
  const double* dMlr = dZo + e * sZo + qlr;
  const int64_t qd = e * sZd + (int64_t)(side == 0 ? ol : orr) * TS * TS;
  d4 acc[4][4];
  zero_tile(acc);
  // terms in order: the X_l pair, then the X_r pair; the primal has one term per pair
  const int per = tan ? 2 : 1;
#pragma unroll 1
  for (int t = 0; t < 2 * per; ++t) {
    const bool xl = t < per;
    if (side == 0 && !xl && !right) break;
    const bool diag = (side == 0) == xl;                // Z_ll (side 0) / Z_rr (side 1)
    const bool dz = tan && ((t % per) == 0);            // the term with the Z tangent
    const bool dx = tan && !dz;                         // the term with the X tangent
    const double* M = diag ? (dz ? dZd : Zd) + qd : (dz ? dMlr : Mlr);
    const bool trans = diag ? false : (side == 0 ? !lr_direct : lr_direct);
    const double* Xs = xl ? (dx ? dXl : Xl) : (dx ? dXr : Xr);
    gemm_tile_ra<true>(M, trans, Xs, smem, acc);
  }
  store_tile((tan ? dZo : Zo) + e * sZo + ((int64_t)o * 2 + side) * TS * TS, TS, acc, 1.0);
}

// Z_pp (and with ntan = 1 dZ_pp) of the odd blocks p = 1 + 2 h, workgroup
// bx = (1 + ntan) h + tan, from the
// pre-pass terms: Z_pp = Zd_pre - X_l^T Z_lp - X_r^T Z_rp, dZ_pp = dZd_pre
// - dX_l^T Z_lp - X_l^T dZ_lp - dX_r^T Z_rp - X_r^T dZ_rp; their traces (rows < n;
// the tangent's negated: -tr dZ_pp = tr (B + eta I)^-2 of the block).
__global__ __launch_bounds__(256, 2) void bcr_sinv_diag_kernel(
    const double* __restrict__ X, const double* __restrict__ dX, int64_t sX,
    const double* __restrict__ Zo, const double* __restrict__ dZo, int64_t sZo,
    double* __restrict__ Zd, double* __restrict__ dZd, int64_t sZd, double* __restrict__ trpart,
    double* __restrict__ dtrpart, int nt, int64_t n, int m, int lvl, int ntan) {
  __shared__ double smem[4 * GSTAGE];
  const int e = blockIdx.y;
  const int p = 1 + 2 * (blockIdx.x / (1 + ntan)), tan = blockIdx.x % (1 + ntan);
  const int o = p << lvl;
  double* Zdst = (tan ? dZd : Zd) + e * sZd + (int64_t)o * TS * TS;
  d4 acc[4][4];
  load_tile(Zdst, TS, acc);
  const int per = tan ? 2 : 1;
  const int nterm = (p + 1 < m ? 2 : 1) * per;
#pragma unroll 1
  for (int t = 0; t < nterm; ++t) {
    const int64_t q = ((int64_t)o * 2 + t / per) * TS * TS;
    const bool dxt = tan && (t % per) == 0;   // dX_s^T Z_sp, then X_s^T dZ_sp
    const double* A = (dxt ? dX : X) + e * sX + q;
    const double* Bm = ((tan && !dxt) ? dZo : Zo) + e * sZo + q;
    gemm_tile<KSLOW, KSLOW, true>(A, TS, Bm, TS, TS, smem, acc);
  }
  store_tile(Zdst, TS, acc, 1.0);
  tile_trace(acc, o, n, tan ? -1.0 : 1.0, smem, (tan ? dtrpart : trpart) + (int64_t)e * nt + o);
}

// tr[e] = sum_o trpart[e][o] in block order.
__global__ void bcr_sinv_final_kernel(const double* __restrict__ trpart, int nt,
                                      double* __restrict__ tr, int neta) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= neta) return;
  double sum = 0.0;
  for (int o = 0; o < nt; ++o) sum += trpart[(int64_t)e * nt + o];
  tr[e] = sum;
}

// ---------------------------------------------------------------------------
// Factor tangents (the roles bcr_w_kernel / bcr_upd_kernel run beside the primal
// workgroups, and bcr_dupd_kernel).
// ---------------------------------------------------------------------------

// dLinv of eliminated block p of level lvl. dD: level 0 the identity, else dDin's
// blocks by level index. scr (per block 2 x 128^2, by original index) holds Linv dD
// and M: the three products run in one workgroup, through global memory (written,
// then read by the same workgroup after a barrier).
__device__ void bcr_dfac_role(const double* __restrict__ L, int64_t sL,
                              const double* __restrict__ dDin, int64_t sdD,
                              double* __restrict__ scr, int64_t sS, double* __restrict__ dL,
                              int lvl, int p, double* smem) {
  const int e = blockIdx.y;
  const int o = p << lvl;
  const double* Lo = L + e * sL + (int64_t)o * TS * TS;
  double* T = scr + e * sS + (int64_t)o * 2 * TS * TS;
  double* Mm = T + TS * TS;
  d4 acc[4][4];
  const double* Tsrc = Lo;   // Linv dD (dD = I at level 0)
  if (lvl > 0) {
    zero_tile(acc);
    gemm_tile<KFAST, KSLOW, false>(Lo, TS, dDin + e * sdD + (int64_t)p * TS * TS, TS, TS, smem,
                                   acc);
    store_tile(T, TS, acc, 1.0);
    __syncthreads();
    Tsrc = T;
  }
  zero_tile(acc);
  gemm_tile<KFAST, KFAST, false>(Tsrc, TS, Lo, TS, TS, smem, acc);   // (Linv dD) Linv^T
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wr * 64 + a * 16 + fk + 4 * r, col = wc * 64 + c * 16 + fr;
          acc[a][c][r] = col > row ? 0.0 : (col == row ? 0.5 * acc[a][c][r] : acc[a][c][r]);
        }
  }
  store_tile(Mm, TS, acc, 1.0);
  __syncthreads();
  zero_tile(acc);
  gemm_tile<KFAST, KSLOW, true>(Mm, TS, Lo, TS, TS, smem, acc);     // -M Linv
  store_tile(dL + e * sL + (int64_t)o * TS * TS, TS, acc, 1.0);
}

// dW of odd block p = 1 + 2 (bx >> 1), which = bx & 1 as bcr_w_role. F / dF: level 0
// the shared F0 (sF = 0) and dF = 0 (dFin unused), else the level's.
__device__ void bcr_dw_role(int bx, const double* __restrict__ L, const double* __restrict__ dL,
                            int64_t sL, const double* __restrict__ Fin, int64_t sF,
                            const double* __restrict__ dFin, int64_t sdF, double* __restrict__ dW,
                            int64_t sW, int m, int lvl, double* smem) {
  const int e = blockIdx.y;
  const int h = bx >> 1, which = bx & 1;
  const int p = 1 + 2 * h;
  const int o = p << lvl;
  if (which == 1 && p + 1 >= m) return;
  const int64_t lo = e * sL + (int64_t)o * TS * TS;
  const int fi = which == 0 ? p - 1 : p;
  const double* F = Fin + e * sF + (int64_t)fi * TS * TS;
  const double* dF = dFin + e * sdF + (int64_t)fi * TS * TS;
  d4 acc[4][4];
  zero_tile(acc);
  const int nterm = lvl > 0 ? 2 : 1;
  // (accumulated negated: the product form of bcr_upd_kernel's other roles, one
  // inlined product per kernel; the sign is flipped at the store)
#pragma unroll 1
  for (int t = 0; t < nterm; ++t)   // . F_{p-1} (which 0) or . F_p^T (which 1)
    gemm_tile_rr<true>(t == 0 ? dL + lo : L + lo, false, t == 0 ? F : dF, which == 0, smem, acc);
  store_tile(dW + e * sW + ((int64_t)o * 2 + which) * TS * TS, TS, acc, -1.0);
}

// dD_j' / dF_{j/2}' of the even blocks j = 2 (bx >> 1), which = bx & 1.
__global__ __launch_bounds__(256, 2) void bcr_dupd_kernel(
    const double* __restrict__ W, const double* __restrict__ dW, int64_t sW,
    const double* __restrict__ dDin, int64_t sdD, double* __restrict__ dDout,
    double* __restrict__ dFout, int64_t sO, int m, int lvl) {
  __shared__ double smem[4 * GSTAGE];
  const int e = blockIdx.y;
  const int h = blockIdx.x >> 1, which = blockIdx.x & 1;
  const int j = 2 * h;
  const double* We = W + e * sW;
  const double* dWe = dW + e * sW;
  d4 acc[4][4];
  if (which == 1) {
    if (j + 2 >= m) return;
    const int64_t ol = ((int64_t)((j + 1) << lvl) * 2 + 0) * TS * TS;
    const int64_t orr = ((int64_t)((j + 1) << lvl) * 2 + 1) * TS * TS;
    zero_tile(acc);
#pragma unroll 1
    for (int t = 0; t < 2; ++t)   // -(dW_r^T W_l + W_r^T dW_l)
      gemm_tile<KSLOW, KSLOW, true>((t == 0 ? dWe : We) + orr, TS, (t == 0 ? We : dWe) + ol, TS,
                                    TS, smem, acc);
    store_tile(dFout + e * sO + (int64_t)h * TS * TS, TS, acc, 1.0);
    return;
  }
  if (lvl == 0) {
    zero_tile(acc);
    tile_add_diag(acc, 1.0);
  } else {
    load_tile(dDin + e * sdD + (int64_t)j * TS * TS, TS, acc);
  }
  // (dW_r^T W_r + W_r^T dW_r)(j - 1), then (dW_l^T W_l + W_l^T dW_l)(j + 1), in a
  // rolled loop (straight-line, the four products spilled)
  const int64_t ql = ((int64_t)((j - 1) << lvl) * 2 + 1) * TS * TS;
  const int64_t qr = ((int64_t)((j + 1) << lvl) * 2 + 0) * TS * TS;
#pragma unroll 1
  for (int t = 0; t < 4; ++t) {
    if (t < 2 ? j < 1 : j + 1 >= m) continue;
    const int64_t q = t < 2 ? ql : qr;
    gemm_tile<KSLOW, KSLOW, true>((t & 1) ? We + q : dWe + q, TS, (t & 1) ? dWe + q : We + q, TS,
                                  TS, smem, acc);
  }
  store_tile(dDout + e * sO + (int64_t)h * TS * TS, TS, acc, 1.0);
}

}  // namespace gpmi
