// 128x128 SPD block factorization and inversion in LDS, shared by the
// diagonal-block kernel of the blocked Cholesky (gpmi_diag.hip) and the banded
// Cholesky of the band path (gpmi_band.hip). One 256-thread workgroup.
//
//   lds_chol_block : Ls (lower, row stride DL) <- L = chol(Ls), blocked by 16:
//                    in-register 16x16 factor (wave 0, rsq + Newton pivots),
//                    16-wide panel solve, MFMA trailing update. inv(L_jj) of the
//                    eight 16x16 diagonal blocks are left in Aux[8][16][16],
//                    diag(L) in sdiag, the first non-positive pivot (1-based)
//                    in *s_fail.
//   lds_inv_block  : Ls <- L^-1 (lower), column blocks in parallel over the 4
//                    waves, X_ij = -X_ii sum_k L_ik X_kj on fp64 MFMA with the X
//                    column held in registers.
//
// f64 MFMA 16x16x4 maps: A[i = lane&15][k = lane>>4], B[k = lane>>4][j = lane&15],
// C/D: lane holds rows (lane>>4) + 4 r (r = 0..3) of column lane&15.
#pragma once

#include "gpmi_device.h"

namespace gpmi {

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

#ifndef GPMI_CHOL_STAMPS
#define GPMI_CHOL_STAMPS 0   // probe builds: per-block phase stamps of one lds_chol_block call
#endif
#if GPMI_CHOL_STAMPS
__device__ int g_chol_calls;
#endif

// Lanes of one wave exchanging values through LDS: the write must stay before the
// read (the compiler, reasoning per lane, could otherwise forward or hoist). LDS
// executes one wave's instructions in order, so no s_barrier is needed.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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


// F1 of block jb (wave 0): factor the 16x16 diagonal block in registers and
// invert it into Aux[jb][16][16]; diag(L) to sdiag, first bad pivot to *s_fail.
// Lane r (and its mirrors r + 16, r + 32, r + 48, which only compute) holds row r
// of the block and column r of X = L^-1. Pivot step j takes the pivot and the
// column below it from the lanes that hold them by v_readlane (scalar registers:
// every lane sees them, no LDS round trip, no barrier); row r's update and the
// right-looking substitution of X's column r (s_i += L_ij X_jr, X_jr =
// (delta_jr - s_j) / L_jj, in ascending j as the row-wise substitution) use the
// same values. The arithmetic of every element is that of the round-4 quad /
// LDS-exchange version: the same results.
__device__ __forceinline__ void f1_factor(double* Ls, double* Aux, double* sdiag, int* s_fail,
                                          int jb) {
  const int lane = threadIdx.x & 63;
  const int j0 = jb * DB;
  const int r = lane & 15;
  double a[DB];
#pragma unroll
  for (int k = 0; k < DB; ++k) a[k] = Ls[(j0 + r) * DL + j0 + k];
  double s[DB], x[DB];
#pragma unroll
  for (int k = 0; k < DB; ++k) s[k] = x[k] = 0.0;
  int fail = 0;
#pragma unroll
  for (int j = 0; j < DB; ++j) {
    const double d = readlane_d(a[j], j);
    double col[DB];
#pragma unroll
    for (int c = j + 1; c < DB; ++c) col[c] = readlane_d(a[j], c);
    const double rinv = rsqrt_nr(d);
    const double ljj = d * rinv;
    if (!(d > 0.0) && fail == 0) fail = j0 + j + 1;   // d is wave-uniform
    if (lane == 0) sdiag[j0 + j] = ljj;
    const double lrj = (r > j) ? a[j] * rinv : ((r == j) ? ljj : 0.0);
    a[j] = lrj;
    // X column r: row j final, then its contribution to the rows below
    x[j] = ((r == j ? 1.0 : 0.0) - s[j]) * rinv;
    // row r's update, unpredicated: the entries right of the diagonal (c > r) take
    // garbage that nothing reads (they are zeroed when the block is stored)
#pragma unroll
    for (int c = j + 1; c < DB; ++c) {
      const double lc = col[c] * rinv;
      a[c] -= lrj * lc;
      s[c] += lc * x[j];
    }
  }
  if (lane == 0 && fail && *s_fail == 0) *s_fail = fail;
  if (lane < DB) {
#pragma unroll
    for (int k = 0; k < DB; ++k) Ls[(j0 + r) * DL + j0 + k] = k <= r ? a[k] : 0.0;
#pragma unroll
    for (int i = 0; i < DB; ++i) Aux[jb * 256 + i * 16 + r] = x[i];
  }
}

// F3 tile q of the trailing update after block jb: (ti, tj), jb < tj <= ti < 8, K = 16.
__device__ __forceinline__ void f3_tile(double* Ls, int jb, int q, int fr, int fk) {
  const int j0 = jb * DB;
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

// Blocked by 16 with a look-ahead: wave 0 updates trailing tile 0 (the next
// diagonal block) and factors it (F1 of jb + 1) while waves 1-3 update the other
// trailing tiles, so F3 hides behind the F1 chain. The two lanes of an F2 row are
// in one wave (LDS order: both read the row before either writes it).
__device__ __forceinline__ void lds_chol_block(double* Ls, double* Aux, double* sdiag,
                                               int* s_fail) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
#if GPMI_CHOL_STAMPS
  unsigned long long cs[NDB + 1][3];
  bool cst = false;
  if (t == 0 && blockIdx.x == 0) cst = atomicAdd(&g_chol_calls, 1) == 2;
#define CHST(jb, i) \
  if (cst) cs[jb][i] = wall_clock64()
#else
#define CHST(jb, i)
#endif
  CHST(0, 2);
  if (w == 0) f1_factor(Ls, Aux, sdiag, s_fail, 0);
  CHST(0, 1);
  for (int jb = 0; jb < NDB; ++jb) {
    const int j0 = jb * DB;
    __syncthreads();   // F1 of jb done
    CHST(jb, 0);
    // ---- F2: panel rows below: L[i][j0 + c] = sum_p A[i][j0 + p] X[c][p]
    {
      const int row = j0 + DB + (t >> 1), h = t & 1;
      if (row < TS) {
        double av[DB];
#pragma unroll
        for (int p = 0; p < DB; ++p) av[p] = Ls[row * DL + j0 + p];
        wave_lds_sync();   // both lanes of the row read it before either writes
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
    CHST(jb + 1, 1);
    // ---- F3 (+ F1 of jb + 1 on wave 0)
    const int m = NDB - 1 - jb;               // trailing tiles per side
    const int ntile = m * (m + 1) / 2;
    if (w == 0) {
      if (ntile > 0) {
        f3_tile(Ls, jb, 0, fr, fk);
        wave_lds_sync();   // the tile written by other lanes of this wave
        f1_factor(Ls, Aux, sdiag, s_fail, jb + 1);
        CHST(jb + 1, 2);
      }
    } else {
      for (int q = w; q < ntile; q += 3) f3_tile(Ls, jb, q, fr, fk);
    }
  }
  __syncthreads();
#if GPMI_CHOL_STAMPS
  if (cst)
    for (int jb = 1; jb < NDB; ++jb)
      printf("lds_chol jb=%d (10ns): F2 %llu  F3t0+F1 %llu  wait %llu\n", jb - 1,
             cs[jb][1] - cs[jb - 1][0], cs[jb][2] - cs[jb][1], cs[jb][0] - cs[jb][2]);
#endif
}

// Aux[8][16][16] <- inverses of the eight 16 x 16 diagonal blocks of the lower
// triangular Ls (non-unit diagonal), by forward substitution; wave w inverts
// blocks w and w + 4. Lane (r, g) holds row r, columns 4g..4g+3 of the inverse.
__device__ __forceinline__ void lds_diag_inv_lower(const double* Ls, double* Aux) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int j0 = (w + 4 * h) * DB;
    const int r = lane >> 2, g = lane & 3;
    double lrow[DB];
#pragma unroll
    for (int p = 0; p < DB; ++p) lrow[p] = Ls[(j0 + r) * DL + j0 + p];
    const double rinv = 1.0 / Ls[(j0 + r) * DL + j0 + r];
    double s[4] = {0.0, 0.0, 0.0, 0.0}, x[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int p = 0; p < DB; ++p) {
      if (r == p) {
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = (((4 * g + k) == p ? 1.0 : 0.0) - s[k]) * rinv;
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
    for (int k = 0; k < 4; ++k) Aux[(j0 / DB) * 256 + r * 16 + 4 * g + k] = x[k];
  }
}

__device__ __forceinline__ void lds_inv_block(double* Ls, const double* Aux) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  for (int e = t; e < NDB * 256; e += 256) {
    const int jb = e >> 8, r = (e >> 4) & 15, c = e & 15;
    Ls[(jb * DB + r) * DL + jb * DB + c] = Aux[e];
  }
  __syncthreads();
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
}

}  // namespace gpmi
