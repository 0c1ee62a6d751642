// Band path: one orthogonal reduction of the correlation matrix to symmetric
// band form, K = Q B Q^T with bandwidth 128, then every eta is a banded
// Cholesky of B + eta I (K + eta I = Q (B + eta I) Q^T for every eta).
//
// This is the device form of the reference's one-time spectral setup
// (MixedCorrelation.__init__ with imate_method='eigenvalue' runs eigh(K) once,
// gaussian_proc/_mixed_correlation/mixed_correlation.py:76-79, so that every
// later logdet / traceinv is cheap, :172-181,239-248). Here the once-per-K work
// is the band reduction (4/3 n^3 flops, fp64 MFMA), after which one likelihood
// evaluation costs O(n b^2) instead of the O(n^3) factorization per eta:
//   logdet(K + eta I)            = logdet(B + eta I)
//   R^T (K + eta I)^-1 R         = Y^T (B + eta I)^-1 Y,   Y = Q^T R (once per RHS)
//
// Stage 1 (dense -> band), per panel j of 128 columns (rows r0 = 128 (j + 1) on):
//   hh_col_kernel x 128    Householder QR of the m x 128 panel, one launch per
//                          column (partial sums of the next column published per
//                          workgroup; the panel rows live in registers)
//   vcopy + tn_partial/reduce + tbuild    V (unit lower) and the compact-WY T:
//                          T = (diag(1/tau) + striu(V^T V))^-1 (LDS MFMA inverse)
//   symm -> psum -> xt     X = A22 V T (A22 lower-stored: transposed tile reads above
//                          the diagonal), split-K partials summed deterministically
//   tn_partial/reduce(V,X) -> z -> w      W = X - 1/2 V (T^T V^T X)
//   syr2k                  A22 -= W V^T + V W^T on the lower tiles (kdim 256)
// Stage 2 (per eta, band_chol_kernel): one workgroup per eta walks the 128-blocks:
//   D_k = B_kk + eta I - C_k C_k^T;  L_kk = chol(D_k), Linv_kk (LDS, shared with
//   the diagonal-block kernel, gpmi_lds_chol.h);  y_k = Linv_kk (Y_k - C_k y_{k-1});
//   C_{k+1} = E_k Linv_kk^T with E_k = triu(B_{k+1,k}); logdet and Gram y^T y
//   accumulated in registers. Nothing leaves the workgroup until the end.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gpmi_internal.h"
#include "gpmi_device.h"
#include "gpmi_lds_chol.h"
#include "gpmi_band.h"
#include "gpmi_tile.h"

#ifndef GPMI_BAND_STAMPS
#define GPMI_BAND_STAMPS 0   // probe builds: phase stamps of band_chol_kernel (printf)
#endif

namespace gpmi {

// ---------------------------------------------------------------------------
// Householder QR of the m x 128 panel P (row-major, ld lda), column c.
// Workgroup g owns panel rows [128 g, 128 g + 128) (8 waves x 16 rows, lanes
// over the columns, two columns per lane); its rows are loaded into registers
// before the reduction of the previous launch's partials completes.
// Inputs (written by launch c - 1): part[c & 1][g'] = partial sums over the rows
// of workgroup g' of x_i P_ij (j >= c, x = column c, rows >= c) and, at [128],
// of x_i^2 (rows > c); pivrow[c & 1] = row c of the panel.
// Reflector (LAPACK dlarfg convention): alpha = -sign(x0) ||x||,
// tau = (alpha - x0) / alpha, v = x / (x0 - alpha) with v_c = 1; tau = 0 when the
// sub-column is exactly zero. w_j = v^T P_j = (S_j - alpha P_cj) / (x0 - alpha).
// Then P_ij -= tau v_i w_j (j > c), column c <- (alpha; v), and the partials of
// column c + 1 are published. c = -1 publishes the partials of column 0 only.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(HH_THREADS) void hh_col_kernel(double* __restrict__ P, int64_t lda,
                                                      int m, int c, double* __restrict__ part,
                                                      double* __restrict__ pivrow,
                                                      double* __restrict__ tau) {
  __shared__ double sacc[HH_WAVES][HH_PART_LD];
  const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int j0 = lane, j1 = lane + 64;
  const int rbase = g * HH_ROWS + w * HH_RPW;
  // every independent load first: own rows, the pivot row, the partial records
  double p0[HH_RPW], p1[HH_RPW];
#pragma unroll
  for (int q = 0; q < HH_RPW; ++q) {
    const int i = rbase + q;
    p0[q] = 0.0;
    p1[q] = 0.0;
    if (i < m && i >= c) {
      const double* row = P + (int64_t)i * lda;
      if (j0 >= c) p0[q] = row[j0];
      if (j1 >= c) p1[q] = row[j1];
    }
  }
  double tau_c = 0.0, scale = 0.0, alpha = 0.0, w0 = 0.0, w1 = 0.0;
  if (c >= 0) {
    const double pv0 = pivrow[(c & 1) * TS + j0];
    const double pv1 = pivrow[(c & 1) * TS + j1];
    const double* pp = part + (size_t)(c & 1) * HH_MAXG * HH_PART_LD;
    double s0 = 0.0, s1 = 0.0, sn = 0.0;
#pragma unroll 4
    for (int u = 0; u < HH_MAXG / HH_WAVES; ++u) {
      const int q = w + HH_WAVES * u;
      if (q < G) {
        s0 += pp[q * HH_PART_LD + j0];
        s1 += pp[q * HH_PART_LD + j1];
        sn += pp[q * HH_PART_LD + 128];
      }
    }
    sacc[w][j0] = s0;
    sacc[w][j1] = s1;
    if (lane == 0) sacc[w][128] = sn;
    __syncthreads();
    double S0 = 0.0, S1 = 0.0, nb2 = 0.0;
#pragma unroll
    for (int q = 0; q < HH_WAVES; ++q) {
      S0 += sacc[q][j0];
      S1 += sacc[q][j1];
      nb2 += sacc[q][128];
    }
    // the reflector, computed identically by every thread (no broadcast step)
    const double x0 = readlane_d(c < 64 ? pv0 : pv1, c & 63);
    if (nb2 > 0.0) {
      const double nrm = sqrt(x0 * x0 + nb2);
      alpha = x0 >= 0.0 ? -nrm : nrm;
      tau_c = (alpha - x0) / alpha;
      scale = 1.0 / (x0 - alpha);
    } else {
      alpha = x0;
    }
    if (g == 0 && t == 0) tau[c] = tau_c;
    if (j0 > c) w0 = (S0 - alpha * pv0) * scale;
    if (j1 > c) w1 = (S1 - alpha * pv1) * scale;
  }
  const bool act = tau_c != 0.0;
  const int c1 = c + 1;
  double a0 = 0.0, a1 = 0.0, nb = 0.0;
#pragma unroll
  for (int q = 0; q < HH_RPW; ++q) {
    const int i = rbase + q;
    if (i >= m || i < c) continue;
    double* row = P + (int64_t)i * lda;
    if (act) {
      const double xc = readlane_d(c < 64 ? p0[q] : p1[q], c & 63);
      const double vi = (i == c) ? 1.0 : xc * scale;
      const double tv = tau_c * vi;
      p0[q] -= tv * w0;
      p1[q] -= tv * w1;
      if (j0 == c) p0[q] = (i == c) ? alpha : vi;
      if (j1 == c) p1[q] = (i == c) ? alpha : vi;
      if (j0 >= c) row[j0] = p0[q];
      if (j1 >= c) row[j1] = p1[q];
    }
    if (c1 < TS && i >= c1) {
      const double x = readlane_d(c1 < 64 ? p0[q] : p1[q], c1 & 63);
      a0 += x * p0[q];
      a1 += x * p1[q];
      if (i > c1) nb += x * x;
      if (i == c1) {
        if (j0 >= c1) pivrow[(c1 & 1) * TS + j0] = p0[q];
        if (j1 >= c1) pivrow[(c1 & 1) * TS + j1] = p1[q];
      }
    }
  }
  if (c1 >= TS) return;
  __syncthreads();
  sacc[w][j0] = a0;
  sacc[w][j1] = a1;
  if (lane == 0) sacc[w][128] = nb;
  __syncthreads();
  if (t <= 128 && t >= c1) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < HH_WAVES; ++q) s += sacc[q][t];
    part[((size_t)(c1 & 1) * HH_MAXG + g) * HH_PART_LD + t] = s;
  }
}

// ---------------------------------------------------------------------------
// The same panel QR in ONE launch (G <= HH_PANEL_MAXG workgroups, one per CU,
// all co-resident): the panel rows stay in registers for all 128 columns and
// the per-column reduction is exchanged inside the launch. Hand-off (the
// write-through form of the guide's publish/consume recipe): every partial
// record and pivot-row word is stored sc1 (agent-scope relaxed atomic store),
// each storing wave drains vmcnt, the workgroup barrier follows, then ONE lane
// adds to the monotonic counter (agent scope; 8 shards, one per g % 8). Consumers:
// every wave polls the shards with sc1 loads until their sum reaches G (c + 1)
// and then reads the records with sc1 loads only. Records are double-buffered by column
// parity: a workgroup publishing column c + 1 has seen every workgroup publish
// column c, i.e. finish reading the slot it overwrites. Every spin is bounded
// (spin_limit polls); a timeout sets *err, every workgroup leaves, and the host
// redoes the reduction with the per-column launches (hh_col_kernel).
// counter[0..127] must be zero at launch (the host memsets it per panel).
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(HH_THREADS) void hh_panel_kernel(double* __restrict__ P,
                                                              int64_t lda, int m,
                                                              double* __restrict__ part,
                                                              double* __restrict__ pivrow,
                                                              unsigned* __restrict__ counter,
                                                              double* __restrict__ tau,
                                                              int* __restrict__ err,
                                                              unsigned spin_limit,
                                                              const int* __restrict__ guard,
                                                              double* __restrict__ Uv,
                                                              int64_t ldu) {
  const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int j0 = lane, j1 = lane + 64;
  const int rbase = g * HH_ROWS + w * HH_RPW;
  // the panel's reflectors into U[.][128:256] (vcopy_kernel's layout), from P's rows
  // (a CholeskyQR panel) or from the registers (this kernel's own)
  auto copy_v = [&](const double* p0, const double* p1) {
#pragma unroll
    for (int q = 0; q < HH_RPW; ++q) {
      const int i = rbase + q;
      if (i < m) {
        double* u = Uv + (int64_t)i * ldu + TS;
        u[j0] = i > j0 ? p0[q] : (i == j0 ? 1.0 : 0.0);
        u[j1] = i > j1 ? p1[q] : (i == j1 ? 1.0 : 0.0);
      }
    }
  };
  // guarded form (after a CholeskyQR panel): run only if that panel failed
  if (guard && !__hip_atomic_load(guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
    if (Uv) {
      double v0[HH_RPW], v1[HH_RPW];
#pragma unroll
      for (int q = 0; q < HH_RPW; ++q) {
        const int i = rbase + q;
        v0[q] = i < m ? P[(int64_t)i * lda + j0] : 0.0;
        v1[q] = i < m ? P[(int64_t)i * lda + j1] : 0.0;
      }
      copy_v(v0, v1);
    }
    return;
  }
  extern __shared__ double dyn_lds[];   // sized by the host to keep one workgroup per CU
  double(*sacc)[HH_PART_LD] = reinterpret_cast<double(*)[HH_PART_LD]>(dyn_lds);
  __shared__ int s_bail;
  double p0[HH_RPW], p1[HH_RPW];
#pragma unroll
  for (int q = 0; q < HH_RPW; ++q) {
    const int i = rbase + q;
    p0[q] = 0.0;
    p1[q] = 0.0;
    if (i < m) {
      const double* row = P + (int64_t)i * lda;
      p0[q] = row[j0];
      p1[q] = row[j1];
    }
  }
  if (t == 0) s_bail = 0;
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
      part, (short)0, (int)(2 * HH_MAXG * HH_PART_LD * sizeof(double)), 0x00020000);
  // publish the partials of column c1 (slot c1 & 1) from the registers
  auto publish = [&](int c1) {
    double a0 = 0.0, a1 = 0.0, nb = 0.0;
#pragma unroll
    for (int q = 0; q < HH_RPW; ++q) {
      const int i = rbase + q;
      if (i >= m || i < c1) continue;
      const double x = readlane_d(c1 < 64 ? p0[q] : p1[q], c1 & 63);
      a0 += x * p0[q];
      a1 += x * p1[q];
      if (i > c1) nb += x * x;
      if (i == c1) {
        if (j0 >= c1) st_sc1(pivrow + (c1 & 1) * TS + j0, p0[q]);
        if (j1 >= c1) st_sc1(pivrow + (c1 & 1) * TS + j1, p1[q]);
      }
    }
    __syncthreads();   // sacc is free (previous readers done)
    sacc[w][j0] = a0;
    sacc[w][j1] = a1;
    if (lane == 0) sacc[w][128] = nb;
    __syncthreads();
    if (t <= 128 && t >= c1) {
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < HH_WAVES; ++q) s += sacc[q][t];
      st_sc1(part + ((size_t)(c1 & 1) * HH_MAXG + g) * HH_PART_LD + t, s);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // arrival on this workgroup's shard (8 shards, 64 bytes apart: fan-in <= G / 8)
    if (t == 0)
      __hip_atomic_fetch_add(counter + 16 * (g & 7), 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  };
  publish(0);
  for (int c = 0; c < TS; ++c) {
    // wait until every workgroup has published column c: each wave polls the 8
    // shards itself (lane k < 8 reads shard k) and loads only after its own poll
    {
      const unsigned target = (unsigned)G * (unsigned)(c + 1);
      unsigned spins = 0;
      for (;;) {
        unsigned v = 0;
        if (lane < 8) v = __hip_atomic_load(counter + 16 * lane, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int off = 4; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (__builtin_amdgcn_readfirstlane(v) >= target) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > spin_limit ||
            ((spins & 1023u) == 0 &&
             __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
          if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_bail = 1;
          break;
        }
      }
    }
    // records of slot c & 1: lane l reads columns (2l, 2l + 1) of every record this
    // wave owns with 16-byte sc1 loads, all in flight together; lane 0 also reads
    // the x^2 sum at [128]
    const uint32_t slot_off = (uint32_t)((c & 1) * HH_MAXG * HH_PART_LD * 8);
    const double pv0 = ld_sc1(pivrow + (c & 1) * TS + j0);
    const double pv1 = ld_sc1(pivrow + (c & 1) * TS + j1);
    d2 rv[HH_PANEL_MAXG / HH_WAVES];
    double rn[HH_PANEL_MAXG / HH_WAVES];
#pragma unroll
    for (int u = 0; u < HH_PANEL_MAXG / HH_WAVES; ++u) {
      const int q = w + HH_WAVES * u;
      rv[u] = d2{0.0, 0.0};
      rn[u] = 0.0;
      if (q < G) {
        const uint32_t roff = slot_off + (uint32_t)(q * HH_PART_LD * 8);
        // only the columns right of c enter the update: lanes left of it skip the load
        if (2 * lane + 1 > c)
          rv[u] = __builtin_bit_cast(
              d2, __builtin_amdgcn_raw_buffer_load_b128(prs, roff + 16 * lane, 0, 16));
        if (lane == 0) rn[u] = ld_sc1(part + (roff >> 3) + 128);
      }
    }
    d2 sv = {0.0, 0.0};
    double sn = 0.0;
#pragma unroll
    for (int u = 0; u < HH_PANEL_MAXG / HH_WAVES; ++u) {
      sv += rv[u];
      sn += rn[u];
    }
    sacc[w][2 * lane] = sv[0];
    sacc[w][2 * lane + 1] = sv[1];
    if (lane == 0) sacc[w][128] = sn;
    __syncthreads();
    // a timed-out wave reached this barrier too (its loads read stale but valid
    // memory); every wave sees s_bail here and the workgroup leaves together
    if (s_bail) return;
    double S0 = 0.0, S1 = 0.0, nb2 = 0.0;
#pragma unroll
    for (int q = 0; q < HH_WAVES; ++q) {
      S0 += sacc[q][j0];
      S1 += sacc[q][j1];
      nb2 += sacc[q][128];
    }
    const double x0 = readlane_d(c < 64 ? pv0 : pv1, c & 63);
    double tau_c = 0.0, scale = 0.0, alpha = x0;
    if (nb2 > 0.0) {
      const double nrm = sqrt(x0 * x0 + nb2);
      alpha = x0 >= 0.0 ? -nrm : nrm;
      tau_c = (alpha - x0) / alpha;
      scale = 1.0 / (x0 - alpha);
    }
    if (g == 0 && t == 0) tau[c] = tau_c;
    if (tau_c != 0.0) {
      const double w0 = (j0 > c) ? (S0 - alpha * pv0) * scale : 0.0;
      const double w1 = (j1 > c) ? (S1 - alpha * pv1) * scale : 0.0;
#pragma unroll
      for (int q = 0; q < HH_RPW; ++q) {
        const int i = rbase + q;
        if (i >= m || i < c) continue;
        const double xc = readlane_d(c < 64 ? p0[q] : p1[q], c & 63);
        const double vi = (i == c) ? 1.0 : xc * scale;
        const double tv = tau_c * vi;
        p0[q] -= tv * w0;
        p1[q] -= tv * w1;
        if (j0 == c) p0[q] = (i == c) ? alpha : vi;
        if (j1 == c) p1[q] = (i == c) ? alpha : vi;
      }
    }
    if (c + 1 < TS) publish(c + 1);
  }
#pragma unroll
  for (int q = 0; q < HH_RPW; ++q) {
    const int i = rbase + q;
    if (i < m) {
      double* row = P + (int64_t)i * lda;
      row[j0] = p0[q];
      row[j1] = p1[q];
    }
  }
  if (Uv) copy_v(p0, p1);
}

// U[r0 + i][128 + q] = V[i][q] (unit lower trapezoidal), i < m.
__global__ __launch_bounds__(256) void vcopy_kernel(const double* __restrict__ P, int64_t lda,
                                                    int m, double* __restrict__ U, int64_t ldu) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t i = e >> 7;
  const int q = (int)(e & 127);
  if (i >= m) return;
  const double v = (i > q) ? P[i * lda + q] : (i == q ? 1.0 : 0.0);
  U[i * ldu + TS + q] = v;
}

// part[ch] = P1[rows]^T P2[rows] (128 x 128), rows = [ch * TN_CH, +TN_CH) of m.
__global__ __launch_bounds__(256, 2) void tn_partial_kernel(const double* __restrict__ P1,
                                                            int64_t ld1,
                                                            const double* __restrict__ P2,
                                                            int64_t ld2, int m,
                                                            double* __restrict__ part,
                                                            const int* __restrict__ only_if) {
  __shared__ double smem[4 * GSTAGE];
  if (only_if && *only_if == 0) return;
  const int ch = blockIdx.x;
  const int i0 = ch * TN_CH, kd = min(TN_CH, m - i0);
  d4 acc[4][4];
  zero_tile(acc);
  gemm_tile<KSLOW, KSLOW, false>(P1 + (int64_t)i0 * ld1, ld1, P2 + (int64_t)i0 * ld2, ld2, kd,
                                 smem, acc);
  store_tile(part + (int64_t)ch * TS * TS, TS, acc, 1.0);
}

// out = scale * sum_ch part[ch] (128 x 128), fixed order: 64 elements per
// workgroup, each summed by its four waves over ch = w (mod 4) (eight loads in
// flight per lane), the four sums combined in a fixed order.
__global__ __launch_bounds__(256) void tn_reduce_kernel(const double* __restrict__ part, int nch,
                                                        double* __restrict__ out, double scale,
                                                        const int* __restrict__ only_if) {
  __shared__ double red[4][64];
  if (only_if && *only_if == 0) return;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int e = blockIdx.x * 64 + lane;
  double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int c = w;
  for (; c + 28 < nch; c += 32) {
    double x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = part[(int64_t)(c + 4 * q) * TS * TS + e];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += x[q];
  }
  for (int q = 0; c < nch; c += 4, ++q) acc[q] += part[(int64_t)c * TS * TS + e];
  red[w][lane] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (w == 0) out[e] = scale * ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]));
}

// Compact-WY T (upper) of the panel's 128 reflectors, one workgroup:
//   T = (diag(1/tau) + striu(V^T V))^-1 = (Lm^-1)^T,  Lm = diag(1/tau) + stril(V^T V),
// which equals LAPACK's forward recurrence T[0:c, c] = -tau_c T[0:c, 0:c] (V^T V)[0:c, c].
// Lm^-1 reuses the LDS block inverse of the Cholesky kernels (16 x 16 diagonal
// blocks by forward substitution, then MFMA column blocks). An identity reflector
// (tau_c = 0) is decoupled: unit diagonal, no coupling, and T_cc = 0.
__device__ __forceinline__ void tbuild_body(const double* __restrict__ VtV,
                                            const double* __restrict__ tau,
                                            double* __restrict__ T, double* Ls, double* Aux,
                                            double* stau) {
  const int t = threadIdx.x;
  if (t < TS) stau[t] = tau[t];
  __syncthreads();
  for (int e = t; e < TS * TS; e += 256) {
    const int r = e >> 7, c = e & 127;
    double v = 0.0;
    if (c == r) v = stau[r] != 0.0 ? 1.0 / stau[r] : 1.0;
    else if (c < r && stau[r] != 0.0 && stau[c] != 0.0) v = VtV[e];
    Ls[r * DL + c] = v;
  }
  __syncthreads();
  // inverses of the eight 16 x 16 diagonal blocks (wave w: blocks w and w + 4)
  lds_diag_inv_lower(Ls, Aux);
  __syncthreads();
  lds_inv_block(Ls, Aux);
  __syncthreads();
  for (int e = t; e < TS * TS; e += 256) {
    const int r = e >> 7, c = e & 127;
    double v = 0.0;
    if (r <= c && !(r == c && stau[c] == 0.0)) v = Ls[c * DL + r];
    T[e] = v;
  }
}

__global__ __launch_bounds__(256) void tbuild_kernel(const double* __restrict__ VtV,
                                                     const double* __restrict__ tau,
                                                     double* __restrict__ T,
                                                     const int* __restrict__ only_if) {
  __shared__ double Ls[TS * DL];
  __shared__ double Aux[TS * RLD];
  __shared__ double stau[TS];
  if (only_if && *only_if == 0) return;
  tbuild_body(VtV, tau, T, Ls, Aux, stau);
}

// T of a CholeskyQR panel that fell back to the Householder panel (flag set), in ONE
// workgroup: V^T V over the m rows (the tn_partial products chunk by chunk into one
// accumulator), then tbuild_body. Slow (one CU), but it runs only for a failed
// panel; for every other panel it is one launch that exits at once (round 5: it
// replaces the three guarded launches tn_partial / tn_reduce / tbuild, whose ~15 us
// of no-op launches on the side stream delayed X T of the chain-bound late panels).
__global__ __launch_bounds__(256) void t_fallback_kernel(const double* __restrict__ V,
                                                         int64_t ldv, int m,
                                                         const double* __restrict__ tau,
                                                         double* __restrict__ VtV,
                                                         double* __restrict__ T,
                                                         const int* __restrict__ only_if) {
  __shared__ double Ls[TS * DL];   // also the product's LDS stages (4 GSTAGE <= TS DL)
  __shared__ double Aux[TS * RLD];
  __shared__ double stau[TS];
  static_assert(4 * GSTAGE <= TS * DL, "t_fallback_kernel: staging exceeds Ls");
  if (*only_if == 0) return;
  d4 acc[4][4];
  zero_tile(acc);
  for (int i0 = 0; i0 < m; i0 += TN_CH)
    gemm_tile<KSLOW, KSLOW, false>(V + (int64_t)i0 * ldv, ldv, V + (int64_t)i0 * ldv, ldv,
                                   min(TN_CH, m - i0), Ls, acc);
  store_tile(VtV, TS, acc, 1.0);
  __threadfence_block();
  __syncthreads();
  tbuild_body(VtV, tau, T, Ls, Aux, stau);
}

// Split-K symmetric product: Xp[il][ch] = sum_{J in chunk ch} A22_IJ V_J, with
// A22_IJ = A_IJ (J <= I, stored) or A_JI^T (J > I, read transposed).
__global__ __launch_bounds__(256, 2) void symm_kernel(const double* __restrict__ A, int64_t lda,
                                                      const double* __restrict__ U, int64_t ldu,
                                                      int tr0, int mt, int chunk,
                                                      double* __restrict__ Xp) {
  __shared__ double smem[4 * GSTAGE];
  const int il = blockIdx.x, ch = blockIdx.y, nch = gridDim.y;
  const int I = tr0 + il;
  const int jl0 = ch * chunk, jl1 = min(mt, (ch + 1) * chunk);
  const int jsplit = min(jl1, max(jl0, il + 1));   // tiles [jl0, jsplit) have J <= I
  d4 acc[4][4];
  zero_tile(acc);
  for (int jl = jl0; jl < jsplit; ++jl) {
    const int J = tr0 + jl;
    gemm_tile<KFAST, KSLOW, false>(A + (int64_t)I * TS * lda + (int64_t)J * TS, lda,
                                   U + (int64_t)J * TS * ldu + TS, ldu, TS, smem, acc);
  }
  for (int jl = jsplit; jl < jl1; ++jl) {
    const int J = tr0 + jl;
    gemm_tile<KSLOW, KSLOW, false>(A + (int64_t)J * TS * lda + (int64_t)I * TS, lda,
                                   U + (int64_t)J * TS * ldu + TS, ldu, TS, smem, acc);
  }
  store_tile(Xp + ((int64_t)il * nch + ch) * TS * TS, TS, acc, 1.0);
}

// X[tile il] = sum_ch Xp[il][ch]   (elementwise, 2 doubles per thread)
__global__ __launch_bounds__(256) void psum_kernel(const double* __restrict__ Xp, int nch,
                                                   double* __restrict__ X) {
  const int il = blockIdx.y;
  const int e = (blockIdx.x * 256 + threadIdx.x) * 2;
  d2 s = {0.0, 0.0};
  // the split-K partials' loads in flight eight at a time, summed in order (the
  // same sums as one load at a time)
  for (int c0 = 0; c0 < nch; c0 += 8) {
    d2 x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      x[q] = c0 + q < nch
                 ? *reinterpret_cast<const d2*>(Xp + ((int64_t)il * nch + c0 + q) * TS * TS + e)
                 : d2{0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (c0 + q < nch) s += x[q];
  }
  *reinterpret_cast<d2*>(X + (int64_t)il * TS * TS + e) = s;
}

// The serial steps between the SYMM and the look-ahead on quadrant workgroups
// (blockIdx.y = the 64 x 64 quadrant, gemm_quad2): each is one 128^3 product per output
// tile, whose MFMA chain bounds one workgroup (~14 us at the CU's fp64 rate plus the
// staging); four workgroups per tile run a quarter of it each, all operand loads in
// flight at once.
// X2_I = X_I T (out of place: the quadrants of a row read all of X_I).
__global__ __launch_bounds__(256, 2) void xt_q_kernel(const double* __restrict__ X,
                                                      const double* __restrict__ T,
                                                      double* __restrict__ X2) {
  __shared__ double smem[Q2_SMEM];
  const int q = blockIdx.y;
  const int64_t off = (int64_t)blockIdx.x * TS * TS;
  d4 acc[2][2];
  zero_quad(acc);
  gemm_quad2<KFAST, KSLOW, false, TS>(X + off, TS, T, TS, smem, acc, q >> 1, q & 1);
  store_quad(X2 + off, TS, acc, 1.0, q >> 1, q & 1);
}

// part[ch] = P1[rows]^T P2[rows] as tn_partial_kernel, one quadrant per workgroup.
__global__ __launch_bounds__(256, 2) void tn_partial_q_kernel(const double* __restrict__ P1,
                                                              int64_t ld1,
                                                              const double* __restrict__ P2,
                                                              int64_t ld2, int m,
                                                              double* __restrict__ part) {
  __shared__ double smem[Q2_SMEM];
  const int ch = blockIdx.x, q = blockIdx.y;
  const int i0 = ch * TN_CH;   // (m is a multiple of TN_CH = 128)
  d4 acc[2][2];
  zero_quad(acc);
  gemm_quad2<KSLOW, KSLOW, false, TN_CH>(P1 + (int64_t)i0 * ld1, ld1, P2 + (int64_t)i0 * ld2,
                                         ld2, smem, acc, q >> 1, q & 1);
  store_quad(part + (int64_t)ch * TS * TS, TS, acc, 1.0, q >> 1, q & 1);
}

// Zh = 1/2 T^T M (four workgroups).
__global__ __launch_bounds__(256) void z_q_kernel(const double* __restrict__ T,
                                                  const double* __restrict__ M,
                                                  double* __restrict__ Zh) {
  __shared__ double smem[Q2_SMEM];
  const int q = blockIdx.x;
  d4 acc[2][2];
  zero_quad(acc);
  gemm_quad2<KSLOW, KSLOW, false, TS>(T, TS, M, TS, smem, acc, q >> 1, q & 1);
  store_quad(Zh, TS, acc, 0.5, q >> 1, q & 1);
}

// W_I = X_I - V_I Zh -> U[rows I][0:128] and U[rows I][256:384].
__global__ __launch_bounds__(256, 2) void w_q_kernel(const double* __restrict__ X,
                                                     double* __restrict__ U, int64_t ldu,
                                                     const double* __restrict__ Zh) {
  __shared__ double smem[Q2_SMEM];
  const int il = blockIdx.x, q = blockIdx.y;
  double* Ui = U + (int64_t)il * TS * ldu;
  d4 acc[2][2];
  load_quad(X + (int64_t)il * TS * TS, TS, acc, q >> 1, q & 1);
  gemm_quad2<KFAST, KSLOW, true, TS>(Ui + TS, ldu, Zh, TS, smem, acc, q >> 1, q & 1);
  store_quad(Ui, ldu, acc, 1.0, q >> 1, q & 1);
  store_quad(Ui + 2 * TS, ldu, acc, 1.0, q >> 1, q & 1);
}

// Tile column 0 of the trailing update (the next panel's columns, look-ahead):
// A_I0 -= [W_I V_I] [V_0 W_0]^T, one quadrant per workgroup.
// Ksrc (the first panel's update): C is read from K, the reduction's source, instead of
// A, so A never needs K's copy right of tile column 0.
__global__ __launch_bounds__(256, 2) void syr2k_col_q_kernel(double* __restrict__ A, int64_t lda,
                                                             const double* __restrict__ U,
                                                             int64_t ldu, int tr0,
                                                             const double* __restrict__ Ksrc) {
  __shared__ double smem[Q2_SMEM];
  const int I = tr0 + blockIdx.x, q = blockIdx.y;
  const int64_t off = (int64_t)I * TS * lda + (int64_t)tr0 * TS;
  double* C = A + off;
  d4 acc[2][2];
  load_quad((Ksrc ? Ksrc : A) + off, lda, acc, q >> 1, q & 1);
  gemm_quad2<KFAST, KFAST, true, 2 * TS>(U + (int64_t)I * TS * ldu, ldu,
                                         U + (int64_t)tr0 * TS * ldu + TS, ldu, smem, acc,
                                         q >> 1, q & 1);
  store_quad(C, lda, acc, 1.0, q >> 1, q & 1);
}

// A_IJ -= [W_I V_I] [V_J W_J]^T on the lower tiles of the trailing mt x mt tiles.
__device__ __forceinline__ void syr2k_tile(double* __restrict__ A, int64_t lda,
                                           const double* __restrict__ U, int64_t ldu, int I, int J,
                                           double* smem) {
  double* C = A + (int64_t)I * TS * lda + (int64_t)J * TS;
  d4 acc[4][4];
  load_tile(C, lda, acc);
  gemm_tile<KFAST, KFAST, true>(U + (int64_t)I * TS * ldu, ldu, U + (int64_t)J * TS * ldu + TS,
                                ldu, 2 * TS, smem, acc);
  store_tile(C, lda, acc, 1.0);
}

// Every lower tile of the trailing mt x mt block (XCD-aware order; no look-ahead).
__global__ __launch_bounds__(256, 2) void syr2k_kernel(double* __restrict__ A, int64_t lda,
                                                       const double* __restrict__ U,
                                                       int64_t ldu, int tr0, int mt) {
  __shared__ double smem[4 * GSTAGE];
  int i, j;
  tri_decode(xcd_remap(blockIdx.x, gridDim.x), mt, &i, &j);
  syr2k_tile(A, lda, U, ldu, tr0 + i, tr0 + j, smem);
}

// Look-ahead: the lower tiles right of tile column 0, looped over by a capped
// grid so that CUs stay free for the next panel's QR. With `order` (the
// (mt - 1)-triangle in row groups, column-major inside a group, packed
// (i << 16) | j): XCD x (workgroups b = x mod 8) takes the x-th contiguous eighth
// of the list, its workgroups striding through it together, so the tiles in
// flight on one XCD share a few W / V row slabs in its L2 (without: consecutive
// tiles of the triangle land on different XCDs and every XCD streams all of U).
__global__ __launch_bounds__(256, 2) void syr2k_rest_kernel(double* __restrict__ A, int64_t lda,
                                                            const double* __restrict__ U,
                                                            int64_t ldu, int tr0, int mt,
                                                            const uint32_t* __restrict__ order) {
  __shared__ double smem[4 * GSTAGE];
  const int ntiles = (mt - 1) * mt / 2;
  if (order && gridDim.x >= 8) {   // (every XCD needs a workgroup for its eighth)
    const int nwg = gridDim.x, x = blockIdx.x & 7, l = blockIdx.x >> 3;
    const int nx = (nwg >> 3) + (x < (nwg & 7) ? 1 : 0);   // workgroups on XCD x
    const int c0 = (int)((int64_t)ntiles * x / 8), c1 = (int)((int64_t)ntiles * (x + 1) / 8);
    for (int q = c0 + l; q < c1; q += nx) {
      const uint32_t o = order[q];
      syr2k_tile(A, lda, U, ldu, tr0 + 1 + (int)(o >> 16), tr0 + 1 + (int)(o & 0xffffu), smem);
    }
    return;
  }
  for (int q = blockIdx.x; q < ntiles; q += gridDim.x) {
    int i, j;
    tri_decode(q, mt - 1, &i, &j);
    syr2k_tile(A, lda, U, ldu, tr0 + i + 1, tr0 + j + 1, smem);
  }
}

// Look-ahead SYR2K that leaves whole CUs to the next panel's chain: a persistent
// tile loop of ONE workgroup per CU (launch_bounds (256, 1): every wave owns a
// SIMD's 512 registers), so a grid of NCU - F workgroups leaves F CUs with nothing
// of it and the chain's single-workgroup kernels (cq_chol, cq_recon: 280-400
// registers, 150 KB of LDS) run there at once instead of after the SYR2K drains.
// One workgroup per CU keeps the two-per-CU throughput by software pipelining
// (tools/probe/syr2k_probe.hip rest_pipe: 0.716 of the fp64 peak at k = 256, as two
// plain workgroups per CU): while tile q runs its 16 k-steps, 4 of the 64 per-lane C
// values of tile q + grid are loaded and 4 of tile q - grid's results are stored per
// step, and the last step stages tile q + grid's first operand slab. Tiles as
// syr2k_rest_kernel (the triangle right of tile column 0, from tile row tr0 + 1).
//
// With cnt (dynamic tiles): the launch's workgroup b starts on tile b (filler = 0)
// and every further tile is nmain + a ticket of *cnt, drawn by thread 0 half-way
// through the tile before the one it is for and passed on through LDS (the tile's
// C loads need it a tile ahead; the atomic's return is waited for where it is
// drawn, ~1 us of one wave per tile: the same reduction time as static tiles
// without the filler, 141.0 ms). A filler launch (filler = 1, on the chain's
// stream after the chain) draws every tile from *cnt: the CUs the chain had to
// itself join the update once it ends. *cnt is zeroed before the launch.
__global__ __launch_bounds__(256, 1) void syr2k_pipe_kernel(double* __restrict__ A, int64_t lda,
                                                            const double* __restrict__ U,
                                                            int64_t ldu, int tr0, int mt,
                                                            int* __restrict__ cnt, int nmain,
                                                            int filler,
                                                            const double* __restrict__ Ksrc) {
  __shared__ double smem[4 * GSTAGE + 2];
  int* stk = reinterpret_cast<int*>(smem + 4 * GSTAGE);   // [0] next ticket, [1] first
  constexpr int KD = 2 * TS;
  constexpr int NS = KD / BK;
  constexpr int PER = (64 + NS - 1) / NS;   // C values per lane per step
  const int ntiles = (mt - 1) * mt / 2;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int q = blockIdx.x, qn = q + gridDim.x;
  if (cnt) {
    if (t == 0) {
      const int a = filler ? nmain + atomicAdd(cnt, 1) : q;
      stk[1] = a;
      stk[0] = a < ntiles ? nmain + atomicAdd(cnt, 1) : ntiles;
    }
    __syncthreads();
    q = stk[1];
    qn = stk[0];
    __syncthreads();
  }
  if (q >= ntiles) return;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  double* sA = smem;
  double* sB = smem + 2 * GSTAGE;
  auto tile_ptrs = [&](int qq, double** C, const double** P1, const double** P2) {
    int i, j;
    tri_decode(qq, mt - 1, &i, &j);
    const int I = tr0 + 1 + i, J = tr0 + 1 + j;
    *C = A + (int64_t)I * TS * lda + (int64_t)J * TS;
    *P1 = U + (int64_t)I * TS * ldu;
    *P2 = U + (int64_t)J * TS * ldu + TS;
  };
  const int64_t coff = (int64_t)(wr * 64 + fk) * lda + wc * 64 + fr;
  auto cidx = [&](int e) -> int64_t {   // e = a * 16 + c * 4 + r
    return (int64_t)((e >> 4) * 16 + 4 * (e & 3)) * lda + ((e >> 2) & 3) * 16;
  };
  // C tiles are read from Ksrc when given (the first panel's update; the same offsets)
  auto csrc = [&](const double* c) -> const double* { return Ksrc ? Ksrc + (c - A) : c; };
  d4 acc[4][4], cn[4][4], po[4][4];
  double* Cq;
  const double *P1, *P2;
  tile_ptrs(q, &Cq, &P1, &P2);
  load_tile(csrc(Cq), lda, acc);
  d2 ra[4], rb[4];
  gl_op<KFAST>(P1, ldu, 0, ra);
  gl_op<KFAST>(P2, ldu, 0, rb);
  st_op<KFAST>(sA, ra);
  st_op<KFAST>(sB, rb);
  __syncthreads();
  double* Cp = nullptr;
  bool has_p = false;
  int tk = 0;
  while (true) {
    const bool has_n = qn < ntiles;
    double* Cn = nullptr;
    const double *N1 = nullptr, *N2 = nullptr;
    if (has_n) tile_ptrs(qn, &Cn, &N1, &N2);
    const double* Cns = has_n ? csrc(Cn) : nullptr;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int cur = s & 1;
      const double* cA = sA + cur * GSTAGE;
      const double* cB = sB + cur * GSTAGE;
      const bool ld = s + 1 < NS || has_n;
      // the ticket before this step's loads (its return is waited for at once: the
      // value goes to an AGPR; ~1 us of wave 0 per tile)
      if (cnt && t == 0 && has_n) {
        if (s == NS / 2) tk = atomicAdd(cnt, 1);
        if (s == NS - 1) stk[0] = nmain + tk;
      }
      if (s + 1 < NS) {
        gl_op<KFAST>(P1, ldu, (s + 1) * BK, ra);
        gl_op<KFAST>(P2, ldu, (s + 1) * BK, rb);
      } else if (has_n) {
        gl_op<KFAST>(N1, ldu, 0, ra);
        gl_op<KFAST>(N2, ldu, 0, rb);
      }
      if (has_n) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int e = s * PER + u;
          if (e < 64) cn[e >> 4][(e >> 2) & 3][e & 3] = Cns[coff + cidx(e)];
        }
      }
      if (has_p) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int e = s * PER + u;
          if (e < 64) Cp[coff + cidx(e)] = po[e >> 4][(e >> 2) & 3][e & 3];
        }
      }
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = fr_op<KFAST>(cA, wr * 64 + i * 16 + fr, kk * 4 + fk);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = fr_op<KFAST>(cB, wc * 64 + j * 16 + fr, kk * 4 + fk);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma64_neg(a[i], b[j], acc[i][j]);
      }
      if (ld) {
        st_op<KFAST>(sA + (cur ^ 1) * GSTAGE, ra);
        st_op<KFAST>(sB + (cur ^ 1) * GSTAGE, rb);
      }
      __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        po[a][c] = acc[a][c];
        acc[a][c] = cn[a][c];
      }
    Cp = Cq;
    has_p = true;
    if (!has_n) break;
    q = qn;
    qn = cnt ? stk[0] : q + gridDim.x;   // (written before the last step's barrier)
    Cq = Cn;
    P1 = N1;
    P2 = N2;
  }
#pragma unroll
  for (int e = 0; e < 64; ++e) Cp[coff + cidx(e)] = po[e >> 4][(e >> 2) & 3][e & 3];
}

// ---------------------------------------------------------------------------
// Y <- Q_j^T Y for one panel (Y rows r0.., 16 columns): Y -= V (T^T (V^T Y)).
// V is read from the reduced matrix (unit lower trapezoidal below the band).
//   qt_partial : workgroup g: part[g] = V[rows]^T Y[rows] over QT_ROWS rows
//   qt_reduce  : a = sum_g part[g] (128 x 16), 8 workgroups
//   qt_tb      : b = T^T a (one workgroup)
//   qt_apply   : Y[rows] -= V[rows] b
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void qt_partial_kernel(const double* __restrict__ P,
                                                         int64_t lda, int m,
                                                         const double* __restrict__ Y,
                                                         double* __restrict__ part) {
  __shared__ double sy[QT_ROWS * RLD];
  const int g = blockIdx.x, t = threadIdx.x;
  const int i0 = g * QT_ROWS, i1 = min(m, i0 + QT_ROWS);
  for (int e = t; e < QT_ROWS * RLD; e += 256)
    sy[e] = (i0 + e / RLD < i1) ? Y[(int64_t)i0 * RLD + e] : 0.0;
  __syncthreads();
  const int a = t & 127, h = t >> 7;
  double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int i = i0; i < i1; ++i) {
    const double v = (i > a) ? P[(int64_t)i * lda + a] : (i == a ? 1.0 : 0.0);
    const double* yr = sy + (i - i0) * RLD + 8 * h;
#pragma unroll
    for (int q = 0; q < 8; ++q) s[q] += v * yr[q];
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) part[((int64_t)g * TS + a) * RLD + 8 * h + q] = s[q];
}

// a[e] = sum_g part[g][e], e < 128 * 16 (fixed order)
__global__ __launch_bounds__(256) void qt_reduce_kernel(const double* __restrict__ part, int G,
                                                        double* __restrict__ a) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  double s = 0.0;
  for (int g = 0; g < G; ++g) s += part[(int64_t)g * TS * RLD + e];
  a[e] = s;
}

// b = T^T a  (128 x 16, one workgroup; T upper triangular)
__global__ __launch_bounds__(256) void qt_tb_kernel(const double* __restrict__ a,
                                                    const double* __restrict__ T,
                                                    double* __restrict__ b) {
  __shared__ double sa[TS * RLD];
  const int t = threadIdx.x;
  for (int e = t; e < TS * RLD; e += 256) sa[e] = a[e];
  __syncthreads();
  const int k = t & 127, h = t >> 7;
  double o[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int r = 0; r <= k; ++r) {
    const double tv = T[r * TS + k];
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] += tv * sa[r * RLD + 8 * h + q];
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) b[k * RLD + 8 * h + q] = o[q];
}

// Y[i] -= V[i] b for the QT_ROWS rows of this workgroup (4 threads per row, 4
// columns each; the row of V is staged through LDS).
__global__ __launch_bounds__(256) void qt_apply_kernel(const double* __restrict__ P, int64_t lda,
                                                       int m, double* __restrict__ Y,
                                                       const double* __restrict__ b) {
  __shared__ double sb[TS * RLD];
  __shared__ double sv[QT_ROWS * (TS + 1)];
  const int t = threadIdx.x;
  const int i0 = blockIdx.x * QT_ROWS, i1 = min(m, i0 + QT_ROWS);
  for (int e = t; e < TS * RLD; e += 256) sb[e] = b[e];
  for (int e = t; e < QT_ROWS * TS; e += 256) {
    const int r = e >> 7, a = e & 127, i = i0 + r;
    double v = 0.0;
    if (i < i1) v = (i > a) ? P[(int64_t)i * lda + a] : (i == a ? 1.0 : 0.0);
    sv[r * (TS + 1) + a] = v;
  }
  __syncthreads();
  const int r = t >> 2, c4 = (t & 3) * 4;
  const int i = i0 + r;
  if (i >= i1) return;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  const double* vr = sv + r * (TS + 1);
  for (int a = 0; a < TS; ++a) {
    const double v = vr[a];
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q] += v * sb[a * RLD + c4 + q];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) Y[(int64_t)i * RLD + c4 + q] -= s[q];
}

// Tile row I of the subdiagonal factor block C = E Linv^T (band_chol_kernel):
// E = triu(B_{k+1,k}) (global) and Linv^T are upper triangular, so C is, and
// tile (I, j), j >= I, sums only the k-tiles q = I..j (120 of the 512 tile
// products of a full 128^3 product). The wave's E fragments of row I are all
// loaded first (one batch of global loads), Linv is read from LDS.
template <int I>
__device__ __forceinline__ void c_row(const double* __restrict__ E, int64_t lda, const double* Ls,
                                      d4 (&Ct)[NDB - I], int fr, int fk) {
  double ef[NDB - I][4];
#pragma unroll
  for (int q = I; q < NDB; ++q)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int r = I * DB + fr, qk = q * DB + 4 * kk + fk;
      ef[q - I][kk] = (q > I || r <= qk) ? E[(int64_t)r * lda + qk] : 0.0;
    }
#pragma unroll
  for (int j = I; j < NDB; ++j) {
    d4 a0 = {0.0, 0.0, 0.0, 0.0}, a1 = {0.0, 0.0, 0.0, 0.0};
    const int c = j * DB + fr;
#pragma unroll
    for (int q = I; q <= j; ++q)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int qk = q * DB + 4 * kk + fk;
        const double bv = (q < j || qk <= c) ? Ls[c * DL + qk] : 0.0;
        if (kk & 1) a1 = mfma64(ef[q - I][kk], bv, a1);
        else a0 = mfma64(ef[q - I][kk], bv, a0);
      }
    Ct[j - I] = a0 + a1;
  }
}

// Row I of C into Ls (zeros left of the diagonal tile).
template <int I>
__device__ __forceinline__ void c_store(double* Ls, const d4 (&Ct)[NDB - I], int fr, int fk) {
#pragma unroll
  for (int j = 0; j < NDB; ++j)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      Ls[(I * DB + fk + 4 * rr) * DL + j * DB + fr] = (j < I) ? 0.0 : Ct[j - I < 0 ? 0 : j - I][rr];
}

// Ls (Linv) <- C = E Linv^T. Tile rows per wave {0}, {1,6}, {2,5}, {3,4,7}:
// 36 / 31 / 27 / 26 tile products. Ends with a workgroup barrier.
__device__ __forceinline__ void c_rows(const double* __restrict__ E, int64_t lda, double* Ls,
                                       int w, int fr, int fk) {
  if (w == 0) {
    d4 C0[8];
    c_row<0>(E, lda, Ls, C0, fr, fk);
    __syncthreads();   // every wave is done with Linv
    c_store<0>(Ls, C0, fr, fk);
  } else if (w == 1) {
    d4 C1[7], C6[2];
    c_row<1>(E, lda, Ls, C1, fr, fk);
    c_row<6>(E, lda, Ls, C6, fr, fk);
    __syncthreads();
    c_store<1>(Ls, C1, fr, fk);
    c_store<6>(Ls, C6, fr, fk);
  } else if (w == 2) {
    d4 C2[6], C5[3];
    c_row<2>(E, lda, Ls, C2, fr, fk);
    c_row<5>(E, lda, Ls, C5, fr, fk);
    __syncthreads();
    c_store<2>(Ls, C2, fr, fk);
    c_store<5>(Ls, C5, fr, fk);
  } else {
    d4 C3[5], C4[4], C7[1];
    c_row<3>(E, lda, Ls, C3, fr, fk);
    c_row<4>(E, lda, Ls, C4, fr, fk);
    c_row<7>(E, lda, Ls, C7, fr, fk);
    __syncthreads();
    c_store<3>(Ls, C3, fr, fk);
    c_store<4>(Ls, C4, fr, fk);
    c_store<7>(Ls, C7, fr, fk);
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Banded Cholesky of B + eta I per workgroup (eta = etas[blockIdx.x]) with the
// forward substitution of Y, logdet and Gram. B = the reduced matrix: diagonal
// tiles (full) and the upper triangles of the subdiagonal tiles (bandwidth 128).
// out[e][0] = logdet (rows < n only; the identity pad is decoupled),
// out[e][1 + a * 16 + c] = (L^-1 Y)^T (L^-1 Y); info[e] = first bad pivot.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void band_chol_kernel(const double* __restrict__ B,
                                                        int64_t lda, int nt, int64_t n,
                                                        const double* __restrict__ Y,
                                                        const double* __restrict__ etas,
                                                        double* __restrict__ out, int out_ld,
                                                        int* __restrict__ info,
                                                        double* __restrict__ fac,
                                                        double* __restrict__ ysol) {
  __shared__ double Ls[TS * DL];
  __shared__ double Aux[TS * RLD];
  __shared__ double sdiag[TS];
  __shared__ double sred[2];
  __shared__ int s_fail;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int e = blockIdx.x;
  const double eta = etas[e];
#if GPMI_BAND_STAMPS
  unsigned long long bst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define BSTAMP(i) \
  if (e == 0 && (k == 8 || k == 64) && t == 0) bst[i] = wall_clock64()
#define BSTAMP_PRINT() \
  if (e == 0 && (k == 8 || k == 64) && t == 0)                                          \
    printf("band_chol k=%d stamps(10ns): chol %llu ld %llu inv %llu y %llu C %llu r %llu D %llu\n", \
           k, bst[1] - bst[0], bst[2] - bst[1], bst[3] - bst[2], bst[4] - bst[3],          \
           bst[5] - bst[4], bst[6] - bst[5], bst[7] - bst[6])
#else
#define BSTAMP(i)
#define BSTAMP_PRINT()
#endif
  // optional factor store for band_der_kernel: [nt][2][128][128] per eta
  double* const fac_e = fac ? fac + (int64_t)e * nt * 2 * TS * TS : nullptr;
  double* const ysol_e = ysol ? ysol + (int64_t)e * nt * TS * RLD : nullptr;
  double logdet = 0.0;
  int fail = 0;
  d4 Gacc = {0.0, 0.0, 0.0, 0.0};
  d4 Rr[2];
  // D_0 = B_00 + eta I (lower), r_0 = Y_0
  for (int q = t; q < TS * TS; q += 256) {
    const int r = q >> 7, c = q & 127;
    Ls[r * DL + c] = (c <= r) ? B[(int64_t)r * lda + c] + (r == c ? eta : 0.0) : 0.0;
  }
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = slot == 0 ? w : NDB - 1 - w;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) Rr[slot][rr] = Y[(int64_t)(ti * DB + fk + 4 * rr) * RLD + fr];
  }
  if (t == 0) s_fail = 0;
  __syncthreads();
  for (int k = 0; k < nt; ++k) {
    BSTAMP(0);
    // B_{k+1,k+1} + eta I on this wave's 9 lower 16x16 tiles, loaded now so the
    // loads complete during the block factorization (the D update below)
    const int64_t g1 = (int64_t)(k + 1) * TS;
    d4 S[9];
    if (k + 1 < nt) {
#pragma unroll
      for (int s9 = 0; s9 < 9; ++s9) {
        const int qt = w + 4 * s9;
        int ti = 0;
        while ((ti + 1) * (ti + 2) / 2 <= qt) ++ti;
        const int tj = qt - ti * (ti + 1) / 2;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int r = ti * DB + fk + 4 * rr, c = tj * DB + fr;
          S[s9][rr] = B[(g1 + r) * lda + g1 + c] + (r == c ? eta : 0.0);
        }
      }
    }
    lds_chol_block(Ls, Aux, sdiag, &s_fail);
    BSTAMP(1);
    if (w < 2) {
      double v = ((int64_t)k * TS + t < n) ? log(sdiag[t]) : 0.0;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0) sred[w] = v;
    }
    __syncthreads();
    if (t == 0) {
      logdet += 2.0 * (sred[0] + sred[1]);
      if (s_fail && !fail) fail = k * TS + s_fail;
      s_fail = 0;
    }
    BSTAMP(2);
    lds_inv_block(Ls, Aux);
    __syncthreads();
    BSTAMP(3);
    if (fac_e) {
      double* dst = fac_e + (int64_t)(2 * k) * TS * TS;
      for (int q = t; q < TS * TS; q += 256) {
        const int r = q >> 7, c = q & 127;
        dst[q] = (c <= r) ? Ls[r * DL + c] : 0.0;
      }
    }
    // r_k -> Aux (k-major [128][16])
#pragma unroll
    for (int slot = 0; slot < 2; ++slot) {
      const int ti = slot == 0 ? w : NDB - 1 - w;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) Aux[(ti * DB + fk + 4 * rr) * RLD + fr] = Rr[slot][rr];
    }
    __syncthreads();
    // y_k = Linv r_k
    d4 Yv[2];
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
      Yv[slot] = a0 + a1;
    }
    __syncthreads();
#pragma unroll
    for (int slot = 0; slot < 2; ++slot) {
      const int ti = slot == 0 ? w : NDB - 1 - w;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) Aux[(ti * DB + fk + 4 * rr) * RLD + fr] = Yv[slot][rr];
    }
    __syncthreads();
    if (ysol_e)
      for (int q = t; q < TS * RLD; q += 256) ysol_e[(int64_t)k * TS * RLD + q] = Aux[q];
    // Gram += y^T y over this wave's two 16-row slices
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kt = 2 * w + h;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double v = Aux[(kt * DB + 4 * kk + fk) * RLD + fr];
        Gacc = mfma64(v, v, Gacc);
      }
    }
    BSTAMP(4);
    if (k + 1 == nt) break;
    // C = E_k Linv^T, E_k = triu(B_{k+1,k}): upper triangular, like both factors
    // (tile rows per wave: c_rows)
    c_rows(B + (int64_t)(k + 1) * TS * lda + (int64_t)k * TS, lda, Ls, w, fr, fk);
    BSTAMP(5);
    if (fac_e) {
      double* dst = fac_e + (int64_t)(2 * k + 1) * TS * TS;
      for (int q = t; q < TS * TS; q += 256) dst[q] = Ls[(q >> 7) * DL + (q & 127)];
    }
    // r_{k+1} = Y_{k+1} - C y_k
#pragma unroll
    for (int slot = 0; slot < 2; ++slot) {
      const int ti = slot == 0 ? w : NDB - 1 - w;
      d4 a0;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) a0[rr] = Y[(g1 + ti * DB + fk + 4 * rr) * RLD + fr];
      for (int kt = ti; kt < NDB; ++kt) {   // C upper triangular
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const double av = -Ls[(ti * DB + fr) * DL + kt * DB + 4 * kk + fk];
          const double bv = Aux[(kt * DB + 4 * kk + fk) * RLD + fr];
          a0 = mfma64(av, bv, a0);
        }
      }
      Rr[slot] = a0;
    }
    BSTAMP(6);
    // D_{k+1} = B_{k+1,k+1} + eta I - C C^T on the 36 lower 16x16 tiles (9 per wave)
#pragma unroll
    for (int s9 = 0; s9 < 9; ++s9) {
      const int qt = w + 4 * s9;
      int ti = 0;
      while ((ti + 1) * (ti + 2) / 2 <= qt) ++ti;
      const int tj = qt - ti * (ti + 1) / 2;
      const int r0 = ti * DB, c0 = tj * DB;
      d4 a = S[s9];
      for (int kq = 4 * ti; kq < TS / 4; ++kq) {   // C rows of tile ti: columns >= r0
        const double av = -Ls[(r0 + fr) * DL + 4 * kq + fk];
        const double bv = Ls[(c0 + fr) * DL + 4 * kq + fk];
        a = mfma64(av, bv, a);
      }
      S[s9] = a;
    }
    __syncthreads();   // every wave is done with C
#pragma unroll
    for (int s9 = 0; s9 < 9; ++s9) {
      const int qt = w + 4 * s9;
      int ti = 0;
      while ((ti + 1) * (ti + 2) / 2 <= qt) ++ti;
      const int tj = qt - ti * (ti + 1) / 2;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        Ls[(ti * DB + fk + 4 * rr) * DL + tj * DB + fr] = S[s9][rr];
    }
    __syncthreads();
    BSTAMP(7);
    BSTAMP_PRINT();
  }
  __syncthreads();
  d4* sg = reinterpret_cast<d4*>(Ls);
  sg[w * 64 + lane] = Gacc;
  __syncthreads();
  if (w == 0) {
    const d4 Gs = ((sg[lane] + sg[64 + lane]) + sg[128 + lane]) + sg[192 + lane];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) out[(int64_t)e * out_ld + 1 + (fk + 4 * rr) * RLD + fr] = Gs[rr];
  }
  if (t == 0) {
    out[(int64_t)e * out_ld] = logdet;
    info[e] = fail;
  }
}

// ---------------------------------------------------------------------------
// Higher inverse powers for the eta-derivatives (ProfileLikelihood der1 / der2,
// _profile_likelihood.py:91-192, need R^T (K + eta I)^-p R for p = 2, 3):
// with the factor blocks band_chol_kernel stored (Linv_k at fac[2k], the
// subdiagonal block L_{k+1,k} = C_k at fac[2k+1]) and y = L^-1 Y in ysol,
//   backward  x = L^-T y   (x_k = Linv_k^T (y_k - C_k^T x_{k+1})),  G2 = x^T x
//   forward   u = L^-1 x   (u_k = Linv_k (x_k - C_{k-1} u_{k-1})),  G3 = u^T u
// so G2 = Y^T (B + eta I)^-2 Y and G3 = Y^T (B + eta I)^-3 Y. One workgroup per
// eta; x overwrites y in ysol. der[e][0:256] = G2, der[e][256:512] = G3.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void block_to_ls(const double* __restrict__ src, double* Ls) {
  // all 32 16-byte loads of this thread in flight before the LDS stores
  constexpr int NP = TS * TS / 2 / 256;
  d2 r[NP];
#pragma unroll
  for (int u = 0; u < NP; ++u)
    r[u] = *reinterpret_cast<const d2*>(src + 2 * (u * 256 + threadIdx.x));
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int q = 2 * (u * 256 + threadIdx.x);
    Ls[(q >> 7) * DL + (q & 127)] = r[u][0];
    Ls[(q >> 7) * DL + (q & 127) + 1] = r[u][1];
  }
}

// out[slot] (rows ti * 16 + fk + 4 rr, column fr) = sum_k op(M)[row][k] V[k][fr];
// op(M) = M or M^T of the 128 x 128 block in Ls; M lower (Linv) or upper (C)
// triangular: only the nonzero k-tiles are summed.
constexpr int TRI_LOWER = 1, TRI_UPPER = 2;
template <bool TRANS, int TRI>
__device__ __forceinline__ void ls_mm(const double* Ls, const double* V, d4 (&out)[2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = slot == 0 ? w : NDB - 1 - w;
    int k0 = 0, k1 = NDB;
    if ((TRI == TRI_LOWER) == TRANS) k0 = ti;
    else k1 = ti + 1;
    d4 a0 = {0.0, 0.0, 0.0, 0.0}, a1 = {0.0, 0.0, 0.0, 0.0};
    for (int kt = k0; kt < k1; ++kt) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int row = ti * DB + fr, kx = kt * DB + 4 * kk + fk;
        const double av = TRANS ? Ls[kx * DL + row] : Ls[row * DL + kx];
        const double bv = V[kx * RLD + fr];
        if (kk & 1) a1 = mfma64(av, bv, a1);
        else a0 = mfma64(av, bv, a0);
      }
    }
    out[slot] = a0 + a1;
  }
}

__device__ __forceinline__ void slots_to_aux(const d4 (&v)[2], double* Aux) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = slot == 0 ? w : NDB - 1 - w;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) Aux[(ti * DB + fk + 4 * rr) * RLD + fr] = v[slot][rr];
  }
}

__device__ __forceinline__ void load_slots(const double* __restrict__ src, d4 (&v)[2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int slot = 0; slot < 2; ++slot) {
    const int ti = slot == 0 ? w : NDB - 1 - w;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) v[slot][rr] = src[(ti * DB + fk + 4 * rr) * RLD + fr];
  }
}

__device__ __forceinline__ void gram_acc(const double* Aux, d4& G) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kt = 2 * w + h;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const double v = Aux[(kt * DB + 4 * kk + fk) * RLD + fr];
      G = mfma64(v, v, G);
    }
  }
}

__device__ __forceinline__ void gram_out(d4 G, double* Ls, double* dst) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fk = lane >> 4;
  d4* sg = reinterpret_cast<d4*>(Ls);
  __syncthreads();
  sg[w * 64 + lane] = G;
  __syncthreads();
  if (w == 0) {
    const d4 Gs = ((sg[lane] + sg[64 + lane]) + sg[128 + lane]) + sg[192 + lane];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) dst[(fk + 4 * rr) * RLD + fr] = Gs[rr];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void band_der_kernel(const double* __restrict__ fac, int nt,
                                                       double* __restrict__ ysol,
                                                       double* __restrict__ der) {
  __shared__ double Ls[TS * DL];
  __shared__ double Aux[TS * RLD];
  const int e = blockIdx.x;
  const double* fe = fac + (int64_t)e * nt * 2 * TS * TS;
  double* ye = ysol + (int64_t)e * nt * TS * RLD;
  d4 G2 = {0.0, 0.0, 0.0, 0.0}, G3 = {0.0, 0.0, 0.0, 0.0};
  d4 v[2], p[2];
  // backward: x_k = Linv_k^T (y_k - C_k^T x_{k+1}); Aux holds x_{k+1}
  for (int k = nt - 1; k >= 0; --k) {
    load_slots(ye + (int64_t)k * TS * RLD, v);
    if (k + 1 < nt) {
      block_to_ls(fe + (int64_t)(2 * k + 1) * TS * TS, Ls);
      __syncthreads();
      ls_mm<true, TRI_UPPER>(Ls, Aux, p);   // C_k^T x_{k+1}
#pragma unroll
      for (int q = 0; q < 2; ++q) v[q] -= p[q];
    }
    __syncthreads();
    slots_to_aux(v, Aux);
    block_to_ls(fe + (int64_t)(2 * k) * TS * TS, Ls);
    __syncthreads();
    ls_mm<true, TRI_LOWER>(Ls, Aux, p);
    __syncthreads();
    slots_to_aux(p, Aux);
    __syncthreads();
    for (int q = threadIdx.x; q < TS * RLD; q += 256) ye[(int64_t)k * TS * RLD + q] = Aux[q];
    gram_acc(Aux, G2);
  }
  __syncthreads();
  // forward: u_k = Linv_k (x_k - C_{k-1} u_{k-1}); Aux holds u_{k-1}
  for (int k = 0; k < nt; ++k) {
    load_slots(ye + (int64_t)k * TS * RLD, v);
    if (k > 0) {
      block_to_ls(fe + (int64_t)(2 * k - 1) * TS * TS, Ls);
      __syncthreads();
      ls_mm<false, TRI_UPPER>(Ls, Aux, p);   // C_{k-1} u_{k-1}
#pragma unroll
      for (int q = 0; q < 2; ++q) v[q] -= p[q];
    }
    __syncthreads();
    slots_to_aux(v, Aux);
    block_to_ls(fe + (int64_t)(2 * k) * TS * TS, Ls);
    __syncthreads();
    ls_mm<false, TRI_LOWER>(Ls, Aux, p);
    __syncthreads();
    slots_to_aux(p, Aux);
    __syncthreads();
    gram_acc(Aux, G3);
  }
  gram_out(G2, Ls, der + (int64_t)e * 2 * RLD * RLD);
  gram_out(G3, Ls, der + (int64_t)e * 2 * RLD * RLD + RLD * RLD);
}

}  // namespace gpmi
