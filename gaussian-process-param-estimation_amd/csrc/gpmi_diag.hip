// Diagonal-block step of the blocked Cholesky (one 256-thread workgroup per
// batch member, the 128x128 block resident in LDS):
//
//   L_kk = chol(A_kk)              blocked by 16: in-register 16x16 factor (wave 0),
//                                  16-wide panel solve, MFMA trailing update
//   Linv_kk = L_kk^-1              blocked: X_ii = inv(L_ii) from the factor step,
//                                  X_ij = -X_ii sum_k L_ik X_kj on fp64 MFMA
//   logdet partial = 2 sum log diag(L_kk)
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

constexpr int DB = 16;         // inner block
constexpr int NDB = TS / DB;   // 8
constexpr int DL = 130;        // LDS row stride in doubles (conflict-free MFMA A reads)

__device__ __forceinline__ double sel4(const double (&a)[4], int k) {
  return k == 0 ? a[0] : (k == 1 ? a[1] : (k == 2 ? a[2] : a[3]));
}

__global__ __launch_bounds__(256) void diag_block_kernel(BatchPtrs P, int64_t lda, int kb,
                                                         int nt) {
  __shared__ double Ls[TS * DL];     // the block: L, then Linv
  __shared__ double Aux[TS * RLD];   // inv(L_jj) blocks [8][16][16], then the RHS block
  __shared__ int s_fail;
  (void)nt;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int b = blockIdx.x;
  const int64_t k0 = (int64_t)kb * TS;
  double* A = P.A + b * P.sA;
  double* R = P.R + b * P.sR;

  if (t == 0) s_fail = 0;
  for (int e = t; e < TS * TS / 2; e += 256) {
    const int r = e >> 6, c = (e & 63) * 2;
    const d2 v = *reinterpret_cast<const d2*>(A + (k0 + r) * lda + k0 + c);
    Ls[r * DL + c] = (c <= r) ? v[0] : 0.0;
    Ls[r * DL + c + 1] = (c + 1 <= r) ? v[1] : 0.0;
  }
  __syncthreads();

  double logsum = 0.0;   // meaningful in lane 0 of wave 0
  for (int jb = 0; jb < NDB; ++jb) {
    const int j0 = jb * DB;
    // ---- F1: factor and invert the 16x16 diagonal block in registers (wave 0)
    if (w == 0) {
      const int r = lane >> 2, g = lane & 3;
      double a[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = Ls[(j0 + r) * DL + j0 + 4 * g + k];
#pragma unroll
      for (int j = 0; j < DB; ++j) {
        const int sk = j & 3, sg = j >> 2;
        const double d = __shfl(a[sk], (j << 2) | sg);
        const double ljj = sqrt(d);
        const double inv = 1.0 / ljj;
        if (lane == 0) {
          if (!(d > 0.0) && s_fail == 0) s_fail = j0 + j + 1;
          logsum += log(ljj);
        }
        const double crj = __shfl(a[sk], (r << 2) | sg);
        const double lrj = (r > j) ? crj * inv : ((r == j) ? ljj : 0.0);
        double lcj[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) lcj[k] = __shfl(a[sk], ((4 * g + k) << 2) | sg) * inv;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int c = 4 * g + k;
          if (c > j && c <= r) a[k] -= lrj * lcj[k];
        }
        if (g == sg) a[sk] = lrj;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) Ls[(j0 + r) * DL + j0 + 4 * g + k] = a[k];
      // X = inv(L_jj): row p of X is final once the rows above it are.
      const double mydiag = (g == (r >> 2)) ? sel4(a, r & 3) : 0.0;
      const double lrr = __shfl(mydiag, (r << 2) | (r >> 2));
      double s[4] = {0.0, 0.0, 0.0, 0.0}, x[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int p = 0; p < DB; ++p) {
        if (r == p) {
#pragma unroll
          for (int k = 0; k < 4; ++k) x[k] = (((4 * g + k) == p ? 1.0 : 0.0) - s[k]) / lrr;
        }
        double xp[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) xp[k] = __shfl(x[k], (p << 2) | g);
        const double lrp = __shfl(a[p & 3], (r << 2) | (p >> 2));
        if (r > p) {
#pragma unroll
          for (int k = 0; k < 4; ++k) s[k] += lrp * xp[k];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) Aux[jb * 256 + r * 16 + 4 * g + k] = x[k];
    }
    __syncthreads();
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
  }

  if (t == 0) {
    P.logdiag[b * P.sLD + kb] = 2.0 * logsum;
    if (s_fail && P.info[b] == 0) P.info[b] = (int)k0 + s_fail;
  }
  // L (upper triangle is zero) back to the working matrix
  for (int e = t; e < TS * TS / 2; e += 256) {
    const int r = e >> 6, c = (e & 63) * 2;
    d2 v;
    v[0] = Ls[r * DL + c];
    v[1] = Ls[r * DL + c + 1];
    *reinterpret_cast<d2*>(A + (k0 + r) * lda + k0 + c) = v;
  }
  // ---- inverse: diagonal blocks X_ii = inv(L_ii)
  for (int e = t; e < NDB * 256; e += 256) {
    const int jb = e >> 8, r = (e >> 4) & 15, c = e & 15;
    Ls[(jb * DB + r) * DL + jb * DB + c] = Aux[e];
  }
  __syncthreads();
  for (int i = 1; i < NDB; ++i) {
    d4 X0 = {0.0, 0.0, 0.0, 0.0}, X1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int slot = 0; slot < 2; ++slot) {
      const int j = w + 4 * slot;
      if (j < i) {
        d4 T = {0.0, 0.0, 0.0, 0.0};
        for (int k = j; k < i; ++k) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const double av = Ls[(i * DB + fr) * DL + k * DB + 4 * kk + fk];
            const double bv = Ls[(k * DB + 4 * kk + fk) * DL + j * DB + fr];
            T = mfma64(av, bv, T);
          }
        }
        d4 Xt = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const double av = -Ls[(i * DB + fr) * DL + i * DB + 4 * kk + fk];
          Xt = mfma64(av, T[kk], Xt);
        }
        if (slot == 0) X0 = Xt; else X1 = Xt;
      }
    }
    __syncthreads();
#pragma unroll
    for (int slot = 0; slot < 2; ++slot) {
      const int j = w + 4 * slot;
      if (j < i) {
        const d4 Xt = slot == 0 ? X0 : X1;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) Ls[(i * DB + fk + 4 * rr) * DL + j * DB + fr] = Xt[rr];
      }
    }
    __syncthreads();
  }
  double* Li = P.Linv + b * P.sL + (int64_t)kb * TS * TS;
  for (int e = t; e < TS * TS / 2; e += 256) {
    const int r = e >> 6, c = (e & 63) * 2;
    d2 v;
    v[0] = Ls[r * DL + c];
    v[1] = Ls[r * DL + c + 1];
    *reinterpret_cast<d2*>(Li + r * TS + c) = v;
  }
  // ---- RHS: y = Linv r_k ; u = Linv^T y ; Gram = y^T y
  for (int e = t; e < TS * RLD; e += 256) Aux[e] = R[k0 * RLD + e];
  __syncthreads();
  d4 Y0 = {0.0, 0.0, 0.0, 0.0}, Y1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = w + 4 * slot;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int kt = 0; kt <= ti; ++kt) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double av = Ls[(ti * DB + fr) * DL + kt * DB + 4 * kk + fk];
        const double bv = Aux[(kt * DB + 4 * kk + fk) * RLD + fr];
        acc = mfma64(av, bv, acc);
      }
    }
    if (slot == 0) Y0 = acc; else Y1 = acc;
  }
  __syncthreads();
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = w + 4 * slot;
    const d4 acc = slot == 0 ? Y0 : Y1;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = ti * DB + fk + 4 * rr;
      Aux[row * RLD + fr] = acc[rr];
      R[(k0 + row) * RLD + fr] = acc[rr];
    }
  }
  __syncthreads();
  double* U = P.U + b * P.sU;
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int tc = w + 4 * slot;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int kt = tc; kt < NDB; ++kt) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double av = Ls[(kt * DB + 4 * kk + fk) * DL + tc * DB + fr];
        const double bv = Aux[(kt * DB + 4 * kk + fk) * RLD + fr];
        acc = mfma64(av, bv, acc);
      }
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) U[(tc * DB + fk + 4 * rr) * RLD + fr] = acc[rr];
  }
  if (w == 0) {
    d4 G = {0.0, 0.0, 0.0, 0.0};
    for (int kt = 0; kt < NDB; ++kt) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double v = Aux[(kt * DB + 4 * kk + fk) * RLD + fr];
        G = mfma64(v, v, G);
      }
    }
    double* gp = P.gram + b * P.sG + (int64_t)kb * 256;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) gp[(fk + 4 * rr) * 16 + fr] = G[rr];
  }
}

}  // namespace gpmi
