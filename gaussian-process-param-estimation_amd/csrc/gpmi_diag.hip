// Diagonal-block step of the blocked Cholesky (one 256-thread workgroup per
// batch member, the 128x128 block resident in LDS):
//
//   L_kk = chol(A_kk)              blocked by 16: in-register 16x16 factor (wave 0,
//                                  rsq + Newton pivots, no divisions), 16-wide panel
//                                  solve, MFMA trailing update
//   Linv_kk = L_kk^-1              column blocks in parallel over the 4 waves,
//                                  X_ij = -X_ii sum_k L_ik X_kj on fp64 MFMA with the
//                                  X column held in registers
//   logdet partial = 2 sum log diag(L_kk)   (logs taken in parallel at the end)
//   y_k = Linv r_k, u_k = Linv^T y_k (feeds r_i -= L_ik y_k in the panel kernel),
//   Gram partial y_k^T y_k         all on fp64 MFMA
//
// f64 MFMA 16x16x4 maps: A[i = lane&15][k = lane>>4], B[k = lane>>4][j = lane&15],
// C/D: lane holds rows (lane>>4) + 4 r (r = 0..3) of column lane&15. The C/D
// register r of a tile is therefore the B fragment of k-step r of the same tile,
// which chains the inverse products without an LDS round trip.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gpmi_device.h"
#include "gpmi_lds_chol.h"

namespace gpmi {

#ifdef GPMI_DIAG_STAMPS
__device__ unsigned long long g_diag_stamps[64];
#define STAMP(i)                                                        \
  do {                                                                  \
    if (blockIdx.x == 0 && threadIdx.x == 0)                            \
      g_diag_stamps[i] = __builtin_amdgcn_s_memtime();                  \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

__global__ __launch_bounds__(256) void diag_block_kernel(BatchPtrs P, int64_t lda, int kb,
                                                         int nt) {
  __shared__ double Ls[TS * DL];     // the block: L, then Linv
  __shared__ double Aux[TS * RLD];   // inv(L_jj) blocks [8][16][16], then the RHS block
  __shared__ double sdiag[TS];       // diag(L) for the deferred logdet
  __shared__ double sred[2];
  __shared__ int s_fail;
  (void)nt;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int b = blockIdx.x;
  const int64_t k0 = (int64_t)kb * TS;
  double* A = P.A + b * P.sA;
  double* R = P.R + b * P.sR;

  STAMP(0);
  if (t == 0) s_fail = 0;
  // 128 KB block: all 32 loads of a thread in flight before the first LDS write
  {
    d2 v[32];
#pragma unroll
    for (int it = 0; it < 32; ++it) {
      const int e = it * 256 + t;
      const int r = e >> 6, c = (e & 63) * 2;
      v[it] = *reinterpret_cast<const d2*>(A + (k0 + r) * lda + k0 + c);
    }
#pragma unroll
    for (int it = 0; it < 32; ++it) {
      const int e = it * 256 + t;
      const int r = e >> 6, c = (e & 63) * 2;
      Ls[r * DL + c] = (c <= r) ? v[it][0] : 0.0;
      Ls[r * DL + c + 1] = (c + 1 <= r) ? v[it][1] : 0.0;
    }
  }
  __syncthreads();
  STAMP(1);

  lds_chol_block(Ls, Aux, sdiag, &s_fail);

  // logdet partial: logs of the 128 pivots in parallel (waves 0, 1)
  if (w < 2) {
    double v = log(sdiag[t]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) sred[w] = v;
  }
  // L (upper triangle is zero) back to the working matrix
  for (int e = t; e < TS * TS / 2; e += 256) {
    const int r = e >> 6, c = (e & 63) * 2;
    d2 v;
    v[0] = Ls[r * DL + c];
    v[1] = Ls[r * DL + c + 1];
    *reinterpret_cast<d2*>(A + (k0 + r) * lda + k0 + c) = v;
  }
  STAMP(26);
  // ---- inverse: diagonal blocks X_ii = inv(L_ii), then column blocks per wave
  __syncthreads();
  if (t == 0) {
    P.logdiag[b * P.sLD + kb] = 2.0 * (sred[0] + sred[1]);
    if (s_fail && P.info[b] == 0) P.info[b] = (int)k0 + s_fail;
  }
  lds_inv_block(Ls, Aux);
  {
    d2 v[4];
#pragma unroll
    for (int it = 0; it < 4; ++it)
      v[it] = *reinterpret_cast<const d2*>(R + k0 * RLD + 2 * (it * 256 + t));
#pragma unroll
    for (int it = 0; it < 4; ++it) *reinterpret_cast<d2*>(&Aux[2 * (it * 256 + t)]) = v[it];
  }
  __syncthreads();
  STAMP(27);
  double* Li = P.Linv + b * P.sL + (int64_t)kb * TS * TS;
  for (int e = t; e < TS * TS / 2; e += 256) {
    const int r = e >> 6, c = (e & 63) * 2;
    d2 v;
    v[0] = Ls[r * DL + c];
    v[1] = Ls[r * DL + c + 1];
    *reinterpret_cast<d2*>(Li + r * TS + c) = v;
  }
  STAMP(28);
  // ---- RHS: y = Linv r_k ; u = Linv^T y ; Gram = y^T y. Wave w owns row tiles
  // w and 7 - w (balanced chains), each chain split over two accumulators.
  d4 Y0, Y1;
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
    if (slot == 0) Y0 = a0 + a1;
    else Y1 = a0 + a1;
  }
  __syncthreads();
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = slot == 0 ? w : NDB - 1 - w;
    const d4 Yv = slot == 0 ? Y0 : Y1;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = ti * DB + fk + 4 * rr;
      Aux[row * RLD + fr] = Yv[rr];
      R[(k0 + row) * RLD + fr] = Yv[rr];
    }
  }
  __syncthreads();
  double* U = P.U + b * P.sU;
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int tc = slot == 0 ? w : NDB - 1 - w;
    d4 a0 = {0.0, 0.0, 0.0, 0.0}, a1 = {0.0, 0.0, 0.0, 0.0};
    for (int kt = tc; kt < NDB; ++kt) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double av = Ls[(kt * DB + 4 * kk + fk) * DL + tc * DB + fr];
        const double bv = Aux[(kt * DB + 4 * kk + fk) * RLD + fr];
        if (kk & 1) a1 = mfma64(av, bv, a1);
        else a0 = mfma64(av, bv, a0);
      }
    }
    const d4 acc = a0 + a1;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) U[(tc * DB + fk + 4 * rr) * RLD + fr] = acc[rr];
  }
  {
    // Gram partial over this wave's two k-tiles, reduced through LDS (reuses Ls)
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
    __syncthreads();   // every wave is done reading Ls
    d4* sg = reinterpret_cast<d4*>(Ls);
    sg[w * 64 + lane] = G;
    __syncthreads();
    if (w == 0) {
      const d4 Gs = ((sg[lane] + sg[64 + lane]) + sg[128 + lane]) + sg[192 + lane];
      double* gp = P.gram + b * P.sG + (int64_t)kb * 256;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) gp[(fk + 4 * rr) * 16 + fr] = Gs[rr];
    }
  }
  STAMP(29);
}

}  // namespace gpmi
