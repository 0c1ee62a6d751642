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

constexpr int DB = 16;         // inner block
constexpr int NDB = TS / DB;   // 8
constexpr int DL = 130;        // LDS row stride in doubles (conflict-free MFMA A reads)

// Broadcast a double from a compile-time-uniform source lane (v_readlane, no LDS).
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// 1/sqrt(d) to double precision: hardware estimate + two Newton steps.
__device__ __forceinline__ double rsqrt_nr(double d) {
  double r = __builtin_amdgcn_rsq(d);
  r = r * (1.5 - 0.5 * d * r * r);
  r = r * (1.5 - 0.5 * d * r * r);
  return r;
}

// Column block J of X = L^-1 (rows J..7), X_JJ already in the LDS diagonal tile.
// Xc[i - J] holds X_iJ in C/D layout (= B-operand layout, k = row).
template <int J>
__device__ __forceinline__ void inv_colblock(const double* Ls, d4 (&Xc)[NDB - J], int fr,
                                             int fk) {
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) Xc[0][rr] = Ls[(J * DB + fk + 4 * rr) * DL + J * DB + fr];
#pragma unroll
  for (int i = J + 1; i < NDB; ++i) {
    d4 T0 = {0.0, 0.0, 0.0, 0.0}, T1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = J; k < i; ++k) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double av = Ls[(i * DB + fr) * DL + k * DB + 4 * kk + fk];
        if (kk & 1) T1 = mfma64(av, Xc[k - J][kk], T1);
        else T0 = mfma64(av, Xc[k - J][kk], T0);
      }
    }
    const d4 T = T0 + T1;
    d4 Xt = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const double av = -Ls[(i * DB + fr) * DL + i * DB + 4 * kk + fk];
      Xt = mfma64(av, T[kk], Xt);
    }
    Xc[i - J] = Xt;
  }
}

template <int J>
__device__ __forceinline__ void store_colblock(double* Ls, const d4 (&Xc)[NDB - J], int fr,
                                               int fk) {
#pragma unroll
  for (int i = J; i < NDB; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) Ls[(i * DB + fk + 4 * rr) * DL + J * DB + fr] = Xc[i - J][rr];
}

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

  for (int jb = 0; jb < NDB; ++jb) {
    const int j0 = jb * DB;
    // ---- F1: factor and invert the 16x16 diagonal block in registers (wave 0)
    if (w == 0) {
      const int r = lane >> 2, g = lane & 3;
      double a[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = Ls[(j0 + r) * DL + j0 + 4 * g + k];
      double myrinv = 0.0;
#pragma unroll
      for (int j = 0; j < DB; ++j) {
        const int sk = j & 3, sg = j >> 2;
        const double d = readlane_d(a[sk], (j << 2) | sg);
        const double crj = __shfl(a[sk], (r << 2) | sg);
        double lcj[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) lcj[k] = __shfl(a[sk], ((4 * g + k) << 2) | sg);
        const double rinv = rsqrt_nr(d);
        const double ljj = d * rinv;
        if (lane == 0) {
          if (!(d > 0.0) && s_fail == 0) s_fail = j0 + j + 1;
          sdiag[j0 + j] = ljj;
        }
        if (r == j) myrinv = rinv;
        const double lrj = (r > j) ? crj * rinv : ((r == j) ? ljj : 0.0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int c = 4 * g + k;
          if (c > j && c <= r) a[k] -= lrj * (lcj[k] * rinv);
        }
        if (g == sg) a[sk] = lrj;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) Ls[(j0 + r) * DL + j0 + 4 * g + k] = a[k];
      // X = inv(L_jj): row p of X is final once the rows above it are.
      double lrow[DB];   // L[r][p], p = 0..15
#pragma unroll
      for (int p = 0; p < DB; ++p) lrow[p] = __shfl(a[p & 3], (r << 2) | (p >> 2));
      double s[4] = {0.0, 0.0, 0.0, 0.0}, x[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int p = 0; p < DB; ++p) {
        if (r == p) {
#pragma unroll
          for (int k = 0; k < 4; ++k) x[k] = (((4 * g + k) == p ? 1.0 : 0.0) - s[k]) * myrinv;
        }
        double xp[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) xp[k] = __shfl(x[k], (p << 2) | g);
        if (r > p) {
#pragma unroll
          for (int k = 0; k < 4; ++k) s[k] += lrow[p] * xp[k];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) Aux[jb * 256 + r * 16 + 4 * g + k] = x[k];
    }
    __syncthreads();
    STAMP(2 + 3 * jb);
    // ---- F2: panel rows below: L[i][j0 + c] = sum_p A[i][j0 + p] X[c][p]
    {
      const int row = j0 + DB + (t >> 1), h = t & 1;
      double av[DB];
      if (row < TS) {
#pragma unroll
        for (int p = 0; p < DB; ++p) av[p] = Ls[row * DL + j0 + p];
      }
      __syncthreads();
      if (row < TS) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const double* xr = &Aux[jb * 256 + (8 * h + c) * 16];
          double o = 0.0;
#pragma unroll
          for (int p = 0; p < DB; ++p) o += av[p] * xr[p];
          Ls[row * DL + j0 + 8 * h + c] = o;
        }
      }
    }
    __syncthreads();
    STAMP(3 + 3 * jb);
    // ---- F3: trailing update of tiles (ti, tj), jb < tj <= ti < 8, K = 16 (MFMA)
    {
      const int m = NDB - 1 - jb;               // trailing tiles per side
      const int ntile = m * (m + 1) / 2;
      for (int q = w; q < ntile; q += 4) {
        int ti = 0;
        while ((ti + 1) * (ti + 2) / 2 <= q) ++ti;
        const int tj = q - ti * (ti + 1) / 2;
        const int r0 = (jb + 1 + ti) * DB, c0 = (jb + 1 + tj) * DB;
        d4 acc;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[rr] = Ls[(r0 + fk + 4 * rr) * DL + c0 + fr];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const double av = -Ls[(r0 + fr) * DL + j0 + 4 * kk + fk];
          const double bv = Ls[(c0 + fr) * DL + j0 + 4 * kk + fk];
          acc = mfma64(av, bv, acc);
        }
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) Ls[(r0 + fk + 4 * rr) * DL + c0 + fr] = acc[rr];
      }
    }
    __syncthreads();
    STAMP(4 + 3 * jb);
  }

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
  for (int e = t; e < NDB * 256; e += 256) {
    const int jb = e >> 8, r = (e >> 4) & 15, c = e & 15;
    Ls[(jb * DB + r) * DL + jb * DB + c] = Aux[e];
  }
  __syncthreads();
  if (t == 0) {
    P.logdiag[b * P.sLD + kb] = 2.0 * (sred[0] + sred[1]);
    if (s_fail && P.info[b] == 0) P.info[b] = (int)k0 + s_fail;
  }
  // balanced column-block ownership: {0}, {1,7}, {2,6}, {3,4,5}
  if (w == 0) {
    d4 X0[8];
    inv_colblock<0>(Ls, X0, fr, fk);
    __syncthreads();
    store_colblock<0>(Ls, X0, fr, fk);
  } else if (w == 1) {
    d4 X1[7], X7[1];
    inv_colblock<1>(Ls, X1, fr, fk);
    inv_colblock<7>(Ls, X7, fr, fk);
    __syncthreads();
    store_colblock<1>(Ls, X1, fr, fk);
    store_colblock<7>(Ls, X7, fr, fk);
  } else if (w == 2) {
    d4 X2[6], X6[2];
    inv_colblock<2>(Ls, X2, fr, fk);
    inv_colblock<6>(Ls, X6, fr, fk);
    __syncthreads();
    store_colblock<2>(Ls, X2, fr, fk);
    store_colblock<6>(Ls, X6, fr, fk);
  } else {
    d4 X3[5], X4[4], X5[3];
    inv_colblock<3>(Ls, X3, fr, fk);
    inv_colblock<4>(Ls, X4, fr, fk);
    inv_colblock<5>(Ls, X5, fr, fk);
    __syncthreads();
    store_colblock<3>(Ls, X3, fr, fk);
    store_colblock<4>(Ls, X4, fr, fk);
    store_colblock<5>(Ls, X5, fr, fk);
  }
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
