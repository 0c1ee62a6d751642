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

// W of odd block p = 1 + 2 (blockIdx.x >> 1): which = blockIdx.x & 1:
//   0: W_l = Linv_p F_{p-1};  1: W_r = Linv_p F_p^T (only when p + 1 < m).
// F: level 0 the shared F0 (sF = 0), else Fin. Linv and W are stored by the block's
// original index (p << lvl): every level's factor survives for the solves of
// bcr_back_kernel / bcr_rhs_*.
__global__ __launch_bounds__(256, 2) void bcr_w_kernel(const double* __restrict__ Lin, int64_t sL,
                                                       const double* __restrict__ Fin, int64_t sF,
                                                       double* __restrict__ W, int64_t sW,
                                                       int m, int lvl) {
  __shared__ double smem[4 * GSTAGE];
  const int e = blockIdx.y;
  const int h = blockIdx.x >> 1, which = blockIdx.x & 1;
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

// Even block j = 2 (blockIdx.x >> 1) of an m-block level: which = blockIdx.x & 1:
//   0: D_j' (and Y_j'),  1: F_{j/2}' = -W_r(j+1)^T W_l(j+1)  (only when j + 2 < m).
// W pairs of odd block i at W[(i << lvl) * 2 + {0: l, 1: r}]; Z of odd block i at
// its original index (i << lvl) in Zall.
__global__ __launch_bounds__(256, 2) void bcr_upd_kernel(
    const double* __restrict__ Ab, int64_t lda, const double* __restrict__ etas, int lvl,
    const double* __restrict__ Din, int64_t sD, const double* __restrict__ Yin, int64_t sY,
    const double* __restrict__ W, int64_t sW, const double* __restrict__ Zall, int64_t sZ,
    double* __restrict__ Dout, double* __restrict__ Fout, double* __restrict__ Yout, int64_t sO,
    int64_t sOY, int m) {
  __shared__ double smem[4 * GSTAGE];
  const int e = blockIdx.y;
  const int h = blockIdx.x >> 1, which = blockIdx.x & 1;
  const int j = 2 * h;
  const double* We = W + e * sW;
  d4 acc[4][4];
  if (which == 1) {
    if (j + 2 >= m) return;
    const double* Wl = We + ((int64_t)((j + 1) << lvl) * 2 + 0) * TS * TS;
    const double* Wr = We + ((int64_t)((j + 1) << lvl) * 2 + 1) * TS * TS;
    zero_tile(acc);
    gemm_tile<KSLOW, KSLOW, true>(Wr, TS, Wl, TS, TS, smem, acc);
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
  const bool left = j >= 1, right = j + 1 < m;
  if (left) {
    const double* Wr = We + ((int64_t)((j - 1) << lvl) * 2 + 1) * TS * TS;
    gemm_tile<KSLOW, KSLOW, true>(Wr, TS, Wr, TS, TS, smem, acc);
  }
  if (right) {
    const double* Wl = We + ((int64_t)((j + 1) << lvl) * 2 + 0) * TS * TS;
    gemm_tile<KSLOW, KSLOW, true>(Wl, TS, Wl, TS, TS, smem, acc);
  }
  store_tile(Dout + e * sO + (int64_t)h * TS * TS, TS, acc, 1.0);
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
//   X_s  = W_s^T Linv_p                          s in {l, r}     bcr_sinv_x_kernel
//   Z_sp = -(Z_sl X_l + Z_sr X_r)                                bcr_sinv_off_kernel
//   Z_pp = Linv_p^T Linv_p - X_l^T Z_lp - X_r^T Z_rp              bcr_sinv_diag_kernel
// top-down from the last level's single block (Z = Linv^T Linv), level by level,
// every node of a level independent (numpy prototype tools/bcr_sinv_proto.py: the
// diagonal blocks equal inv(A)'s to 1e-16). The parents' coupling Z_lr is the
// off-diagonal block their own elimination produced one level up: l' = (p - 1) / 2
// and r' = l' + 1 there; if r' is odd it is Z_{l', r'} = Zo[o_r][0], else l' is odd and
// Z_lr = Zo[o_l][1]^T. tr Z_pp over the rows < n (the identity pad is decoupled) per
// block, summed in block order by bcr_sinv_final_kernel. This replaces the eigenvalue
// sums sum_i (lambda_i + eta)^-1 of the reference's 'eigenvalue' traceinv
// (mixed_correlation.py:172-181) without the eigenvalues: O(n b^2) per eta.
// Blocks by original index o = p << l: Zd[o] (diagonal), Zo[o][2] (Z_lp, Z_rp), X[o][2].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void bcr_sinv_x_kernel(const double* __restrict__ L,
                                                            int64_t sL,
                                                            const double* __restrict__ W,
                                                            int64_t sW, double* __restrict__ X,
                                                            int64_t sX, int m, int lvl) {
  __shared__ double smem[4 * GSTAGE];
  const int e = blockIdx.y;
  const int h = blockIdx.x >> 1, side = blockIdx.x & 1;
  const int p = 1 + 2 * h;
  const int o = p << lvl;
  if (side == 1 && p + 1 >= m) return;
  d4 acc[4][4];
  zero_tile(acc);
  // X_s = W_s^T Linv_p
  gemm_tile<KSLOW, KSLOW, false>(W + e * sW + ((int64_t)o * 2 + side) * TS * TS, TS,
                                 L + e * sL + (int64_t)o * TS * TS, TS, TS, smem, acc);
  store_tile(X + e * sX + ((int64_t)o * 2 + side) * TS * TS, TS, acc, 1.0);
}

// acc -= op(M) Xs, op(M) = M (KFAST) or M^T (KSLOW)
__device__ __forceinline__ void sinv_sub(const double* M, bool trans, const double* Xs,
                                         double* smem, d4 (&acc)[4][4]) {
  if (trans)
    gemm_tile<KSLOW, KSLOW, true>(M, TS, Xs, TS, TS, smem, acc);
  else
    gemm_tile<KFAST, KSLOW, true>(M, TS, Xs, TS, TS, smem, acc);
}

__global__ __launch_bounds__(256, 2) void bcr_sinv_off_kernel(
    const double* __restrict__ Zd, int64_t sZd, double* __restrict__ Zo, int64_t sZo,
    const double* __restrict__ X, int64_t sX, int m, int lvl) {
  __shared__ double smem[4 * GSTAGE];
  const int e = blockIdx.y;
  const int h = blockIdx.x >> 1, side = blockIdx.x & 1;
  const int p = 1 + 2 * h;
  const bool right = p + 1 < m;
  if (side == 1 && !right) return;
  const int o = p << lvl, ol = (p - 1) << lvl, orr = (p + 1) << lvl;
  const double* Zde = Zd + e * sZd;
  const double* Zoe = Zo + e * sZo;
  const double* Xe = X + e * sX;
  const double* Xl = Xe + ((int64_t)o * 2 + 0) * TS * TS;
  const double* Xr = Xe + ((int64_t)o * 2 + 1) * TS * TS;
  // the parents' coupling: stored as Z_lr (r' odd one level up) or Z_rl (l' odd)
  const double* Mlr = nullptr;
  bool lr_direct = true;
  if (right) {
    const int lp = (p - 1) >> 1;
    if ((lp + 1) & 1) {
      Mlr = Zoe + ((int64_t)orr * 2 + 0) * TS * TS;   // Z_{l', r'}
    } else {
      Mlr = Zoe + ((int64_t)ol * 2 + 1) * TS * TS;    // Z_{r', l'}
      lr_direct = false;
    }
  }
  d4 acc[4][4];
  zero_tile(acc);
  if (side == 0) {
    sinv_sub(Zde + (int64_t)ol * TS * TS, false, Xl, smem, acc);   // Z_ll X_l
    if (right) sinv_sub(Mlr, !lr_direct, Xr, smem, acc);         // Z_lr X_r
  } else {
    sinv_sub(Mlr, lr_direct, Xl, smem, acc);                       // Z_rl X_l
    sinv_sub(Zde + (int64_t)orr * TS * TS, false, Xr, smem, acc);  // Z_rr X_r
  }
  store_tile(Zo + e * sZo + ((int64_t)o * 2 + side) * TS * TS, TS, acc, 1.0);
}

// Z_pp and tr Z_pp (rows < n) of the odd blocks p = 1 + 2 blockIdx.x of level lvl, or
// (root != 0) the last level's single block 0.
__global__ __launch_bounds__(256, 2) void bcr_sinv_diag_kernel(
    const double* __restrict__ L, int64_t sL, const double* __restrict__ X, int64_t sX,
    const double* __restrict__ Zo, int64_t sZo, double* __restrict__ Zd, int64_t sZd,
    double* __restrict__ trpart, int nt, int64_t n, int m, int lvl, int root) {
  __shared__ double smem[4 * GSTAGE];
  const int e = blockIdx.y;
  const int p = root ? 0 : 1 + 2 * blockIdx.x;
  const int o = p << lvl;
  const double* Lo = L + e * sL + (int64_t)o * TS * TS;
  d4 acc[4][4];
  zero_tile(acc);
  gemm_tile<KSLOW, KSLOW, false>(Lo, TS, Lo, TS, TS, smem, acc);   // Linv^T Linv
  if (!root) {
    const double* Xe = X + e * sX;
    const double* Zoe = Zo + e * sZo;
    gemm_tile<KSLOW, KSLOW, true>(Xe + ((int64_t)o * 2) * TS * TS, TS,
                                  Zoe + ((int64_t)o * 2) * TS * TS, TS, TS, smem, acc);
    if (p + 1 < m)
      gemm_tile<KSLOW, KSLOW, true>(Xe + ((int64_t)o * 2 + 1) * TS * TS, TS,
                                    Zoe + ((int64_t)o * 2 + 1) * TS * TS, TS, TS, smem, acc);
  }
  store_tile(Zd + e * sZd + (int64_t)o * TS * TS, TS, acc, 1.0);
  // the trace: diagonal elements (row = wr 64 + a 16 + fk + 4 r == col = wc 64 + a 16 + fr)
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
  if (t == 0) trpart[(int64_t)e * nt + o] = (smem[0] + smem[1]) + (smem[2] + smem[3]);
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

}  // namespace gpmi
