// Sparse path kernels: CSR SpMM with the K + eta I shift, column-blocked dot
// products / Gram-Schmidt updates for a block of Lanczos / CG vectors, and the
// counter-based Rademacher probes. HBM/Infinity-Cache-bound (no MFMA): the
// vector blocks are row-major [n][s] so every CSR nonzero reads s contiguous
// doubles, and every reduction uses a fixed grid and a fixed order
// (bit-reproducible run to run).
//
// Replaces, for a sparse K (reference: imate's 'slq' / 'hutchinson' estimators
// and scipy.sparse.linalg.cg at mixed_correlation.py:138-143,193-209,263-268 and
// _linear_solver.py:57-68): the Krylov primitives of stochastic Lanczos
// quadrature and blocked CG.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gpmi_device.h"

namespace gpmi {

// Y[:, 0:s] = (K + eta I) X[:, 0:s]; one wave per row (blocks of 4 rows,
// contiguous row ranges per XCD so neighbouring rows share X rows in L2). The
// wave loads its row's (column, value) pairs, up to 64 per chunk, in one
// coalesced read and broadcasts them with ds_bpermute to lanes = (slot, column),
// slots = 64 / s nonzeros at a time, four independent gathers per lane; the
// slots are summed with shuffles in a fixed order. (Runs of rows per wave with
// the next row prefetched measured 1.5x slower: fewer waves in flight.) The gathers (nnz * s doubles) come from
// L2 / MALL; HBM sees the CSR arrays once.
// The SPMM_UNR gathers of a lane are issued before any of their products (the
// predicate on the load only): cfg 5 172 -> 140 us per s = 20 launch; eight in flight
// measured slower (194 us).
#ifndef GPMI_SPMM_UNR
#define GPMI_SPMM_UNR 4   // gathers in flight per lane
#endif
constexpr int SPMM_UNR = GPMI_SPMM_UNR;
__device__ __forceinline__ void spmm_chunk(const int myidx, const double myval, int cnt,
                                           const double* __restrict__ X, int64_t ldx, int slots,
                                           int slot, int c, bool on, double (&acc)[4]) {
  // wave-uniform trip count: every lane takes part in every ds_bpermute
  for (int jb = 0; jb < cnt; jb += SPMM_UNR * slots) {
    int ix[SPMM_UNR];
    double vx[SPMM_UNR], g[SPMM_UNR];
#pragma unroll
    for (int u = 0; u < SPMM_UNR; ++u) {
      const int j = (jb + u * slots + slot) & 63;
      ix[u] = __shfl(myidx, j);
      vx[u] = __shfl(myval, j);
    }
#pragma unroll
    for (int u = 0; u < SPMM_UNR; ++u)
      g[u] = (on && jb + u * slots + slot < cnt) ? X[(int64_t)ix[u] * ldx + c] : 0.0;
#pragma unroll
    for (int u = 0; u < SPMM_UNR; ++u)
      if (on && jb + u * slots + slot < cnt) acc[u & 3] += vx[u] * g[u];
  }
}

__global__ __launch_bounds__(256) void csr_spmm_kernel(const int64_t* __restrict__ indptr,
                                                       const int* __restrict__ indices,
                                                       const double* __restrict__ data,
                                                       int64_t n, const double* __restrict__ X,
                                                       int64_t ldx, double* __restrict__ Y,
                                                       int64_t ldy, int s, int slots, double eta) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // contiguous row ranges per XCD: neighbouring rows share X rows in that XCD's L2
  const int64_t row = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 4 + wv;
  if (row >= n) return;
  const int slot = lane / s;
  const int c = lane - slot * s;
  const bool on = slot < slots;
  const int64_t k0 = indptr[row], k1 = indptr[row + 1];
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t kb = k0; kb < k1; kb += 64) {
    const int cnt = (int)((k1 - kb) < 64 ? (k1 - kb) : 64);
    const int myidx = lane < cnt ? indices[kb + lane] : 0;
    const double myval = lane < cnt ? data[kb + lane] : 0.0;
    spmm_chunk(myidx, myval, cnt, X, ldx, slots, slot, c, on, acc);
  }
  const double part = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  double tot = 0.0;
  for (int u = 0; u < slots; ++u) tot += __shfl(part, (c + u * s) & 63);
  if (slot == 0) Y[row * ldy + c] = tot + eta * X[row * ldx + c];
}

// The gather kernel with a lane reading a column pair (16-byte loads): h = s/2 lanes
// per nonzero, slots = 64 / h nonzeros at a time, so a wave instruction covers twice
// the nonzeros of csr_spmm_kernel. Needs s even and X, Y 16-byte aligned with ld = s
// (the host checks). Fixed summation order (not csr_spmm_kernel's: the slots differ).
template <int U>
__global__ __launch_bounds__(256) void csr_spmm_pair_kernel(const int64_t* __restrict__ indptr,
                                                            const int* __restrict__ indices,
                                                            const double* __restrict__ data,
                                                            int64_t n, const double* __restrict__ X,
                                                            double* __restrict__ Y, int s,
                                                            int slots, double eta) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t row = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 4 + wv;
  if (row >= n) return;
  const int h = s >> 1;
  const int slot = lane / h;
  const int c = lane - slot * h;
  const bool on = slot < slots;
  const double2* __restrict__ X2 = reinterpret_cast<const double2*>(X);
  const int64_t k0 = indptr[row], k1 = indptr[row + 1];
  double ax[4] = {0.0, 0.0, 0.0, 0.0}, ay[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t kb = k0; kb < k1; kb += 64) {
    const int cnt = (int)((k1 - kb) < 64 ? (k1 - kb) : 64);
    const int myidx = lane < cnt ? indices[kb + lane] : 0;
    const double myval = lane < cnt ? data[kb + lane] : 0.0;
    for (int jb = 0; jb < cnt; jb += U * slots) {
      int ix[U];
      double vx[U];
      double2 g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = (jb + u * slots + slot) & 63;
        ix[u] = __shfl(myidx, j);
        vx[u] = __shfl(myval, j);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        g[u] = (on && jb + u * slots + slot < cnt) ? X2[(int64_t)ix[u] * h + c]
                                                    : make_double2(0.0, 0.0);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (on && jb + u * slots + slot < cnt) {
          ax[u & 3] += vx[u] * g[u].x;
          ay[u & 3] += vx[u] * g[u].y;
        }
    }
  }
  const double px = (ax[0] + ax[1]) + (ax[2] + ax[3]);
  const double py = (ay[0] + ay[1]) + (ay[2] + ay[3]);
  double tx = 0.0, ty = 0.0;
  for (int u = 0; u < slots; ++u) {
    tx += __shfl(px, (c + u * h) & 63);
    ty += __shfl(py, (c + u * h) & 63);
  }
  if (slot == 0) {
    const double2 xr = X2[row * h + c];
    reinterpret_cast<double2*>(Y)[row * h + c] = make_double2(tx + eta * xr.x, ty + eta * xr.y);
  }
}

template __global__ void csr_spmm_pair_kernel<3>(const int64_t*, const int*, const double*, int64_t,
                                                const double*, double*, int, int, double);

// ---------------------------------------------------------------------------
// X-window SpMM (default). Rows in blocks of WIN_ROWS (64, consecutive in the
// locality order); a block's nonzeros reference a compact set of columns (its
// "window": ~400 in 3D at cfg 5, ~170 in 2D at cfg 4). spmm_window_build_kernel
// (once per operator) sorts and de-duplicates each block's columns into
// wcols[b][0, u_b) and rewrites every nonzero's column as its window position
// (lidx, 16 bit). csr_spmm_win_kernel then stages the block's window rows of X
// (WIN_CS columns at a time) in LDS with one coalesced pass and gathers from LDS:
// the L2 / Infinity Cache gather traffic falls from nnz * s to sum_b u_b * s
// doubles (≈5x at cfg 5). Blocks with more than WIN_MAXM nonzeros or WIN_MAXU
// window columns keep gathering from X (u_b = 0).
// ---------------------------------------------------------------------------
constexpr int WIN_ROWS = 64;
constexpr int WIN_MAXM = 4096;
constexpr int WIN_MAXU = 1024;
constexpr int WIN_CS = 8;

__global__ __launch_bounds__(256) void spmm_window_build_kernel(
    const int64_t* __restrict__ indptr, const int* __restrict__ indices, int64_t n,
    int* __restrict__ wcols, int* __restrict__ ucount, unsigned short* __restrict__ lidx) {
  __shared__ int keys[WIN_MAXM];
  __shared__ int ukeys[WIN_MAXU];
  __shared__ int tsum[256];
  const int t = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int64_t r0 = b * WIN_ROWS, r1 = min(r0 + WIN_ROWS, n);
  const int64_t k0 = indptr[r0], k1 = indptr[r1];
  const int64_t m64 = k1 - k0;
  if (m64 > WIN_MAXM) {
    if (t == 0) ucount[b] = 0;
    return;
  }
  const int m = (int)m64;
  int P = 256;
  while (P < m) P <<= 1;
  for (int i = t; i < P; i += 256) keys[i] = i < m ? indices[k0 + i] : 0x7fffffff;
  __syncthreads();
  // bitonic sort of P keys
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < (P >> 1); i += 256) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const int a = keys[lo], c = keys[hi];
        if ((a > c) == up) {
          keys[lo] = c;
          keys[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  // unique: each thread owns P / 256 consecutive keys; exclusive scan of the counts
  const int per = P / 256, i0 = t * per;
  int cnt = 0;
  for (int i = i0; i < i0 + per; ++i)
    cnt += (i < m && (i == 0 || keys[i] != keys[i - 1])) ? 1 : 0;
  tsum[t] = cnt;
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int q = 0; q < 256; ++q) {
      const int v = tsum[q];
      tsum[q] = acc;
      acc += v;
    }
    ukeys[0] = acc;   // total, read below before the list is written
  }
  __syncthreads();
  const int u = ukeys[0];
  __syncthreads();
  if (u > WIN_MAXU) {
    if (t == 0) ucount[b] = 0;
    return;
  }
  int pos = tsum[t];
  for (int i = i0; i < i0 + per; ++i)
    if (i < m && (i == 0 || keys[i] != keys[i - 1])) {
      ukeys[pos] = keys[i];
      wcols[b * WIN_MAXU + pos] = keys[i];
      ++pos;
    }
  __syncthreads();
  // every nonzero's window position (binary search in the sorted window)
  for (int i = t; i < m; i += 256) {
    const int c = indices[k0 + i];
    int lo = 0, hi = u - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ukeys[mid] < c) lo = mid + 1;
      else hi = mid;
    }
    lidx[k0 + i] = (unsigned short)lo;
  }
  if (t == 0) ucount[b] = u;
}

__global__ __launch_bounds__(256) void csr_spmm_win_kernel(
    const int64_t* __restrict__ indptr, const int* __restrict__ indices,
    const unsigned short* __restrict__ lidx, const double* __restrict__ data, int64_t n,
    const int* __restrict__ wcols, const int* __restrict__ ucount,
    const double* __restrict__ X, int64_t ldx, double* __restrict__ Y, int64_t ldy, int s,
    double eta) {
  // LDS: the window [u][WIN_CS], the block's values, window positions, row starts
  extern __shared__ double smem[];
  const int t = threadIdx.x;
  // consecutive blocks on one XCD: neighbouring windows overlap in its L2
  const int64_t b = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t r0 = b * WIN_ROWS, r1 = min(r0 + WIN_ROWS, n);
  const int nr = (int)(r1 - r0);
  const int u = ucount[b];
  const int64_t k0 = indptr[r0];
  const int c = t & (WIN_CS - 1), rq = t >> 3;   // column in the chunk, row slot (0..31)
  if (u == 0) {
    // window over its limits: gather straight from X
    for (int cc0 = 0; cc0 < s; cc0 += WIN_CS) {
      if (cc0 + c >= s) continue;
      for (int r = rq; r < nr; r += 32) {
        const int64_t row = r0 + r;
        double acc = 0.0;
        for (int64_t k = indptr[row]; k < indptr[row + 1]; ++k)
          acc += data[k] * X[(int64_t)indices[k] * ldx + cc0 + c];
        Y[row * ldy + cc0 + c] = acc + eta * X[row * ldx + cc0 + c];
      }
    }
    return;
  }
  const int m = (int)(indptr[r1] - k0);
  double* win = smem;                                   // [u][WIN_CS]
  double* sval = win + (size_t)u * WIN_CS;              // [m]
  unsigned short* slix = reinterpret_cast<unsigned short*>(sval + m);   // [m]
  int* srow = reinterpret_cast<int*>(slix + ((m + 1) & ~1));            // [WIN_ROWS + 1]
  for (int i = t; i < m; i += 256) {
    sval[i] = data[k0 + i];
    slix[i] = lidx[k0 + i];
  }
  if (t <= nr) srow[t] = (int)(indptr[r0 + t] - k0);
  for (int cc0 = 0; cc0 < s; cc0 += WIN_CS) {
    const int cs = min(WIN_CS, s - cc0);
    const int* wc = wcols + b * WIN_MAXU;
    for (int i = t; i < u * WIN_CS; i += 256) {
      const int e = i >> 3, cj = i & (WIN_CS - 1);
      win[i] = cj < cs ? X[(int64_t)wc[e] * ldx + cc0 + cj] : 0.0;
    }
    __syncthreads();
    if (c < cs) {
      // thread = (row slot rq, column c): rows rq and rq + 32 of the block
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = rq + 32 * h;
        if (r >= nr) break;
        const int ka = srow[r], kb = srow[r + 1];
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        int k = ka;
        for (; k + 4 <= kb; k += 4) {
          a0 += sval[k] * win[slix[k] * WIN_CS + c];
          a1 += sval[k + 1] * win[slix[k + 1] * WIN_CS + c];
          a2 += sval[k + 2] * win[slix[k + 2] * WIN_CS + c];
          a3 += sval[k + 3] * win[slix[k + 3] * WIN_CS + c];
        }
        for (; k < kb; ++k) a0 += sval[k] * win[slix[k] * WIN_CS + c];
        const int64_t row = r0 + r;
        Y[row * ldy + cc0 + c] = ((a0 + a1) + (a2 + a3)) + eta * X[row * ldx + cc0 + c];
      }
    }
    __syncthreads();   // the window is rewritten for the next column chunk
  }
}

// The one-pass window with its staging latency hidden (round 3): the window rows of
// X are gathered with NB loads in flight per thread (16-byte loads for even S; a
// batch covers 8192 doubles, ~410 rows at S = 20), where the round-2 one-pass window
// kernel waited for each 8-byte load before the next (its 3D windows of ~350 rows then took 27
// serialised L2 round trips per thread); the nonzeros' values and window positions
// are read from global memory (the four threads of a row share each; U of them in
// flight per thread), so LDS holds only the window: u S doubles, two workgroups per
// CU up to 80 KB.
template <int S, int U, int TPR>
__global__ __launch_bounds__(64 * TPR) void csr_spmm_wing_kernel(
    const int64_t* __restrict__ indptr, const int* __restrict__ indices,
    const unsigned short* __restrict__ lidx, const double* __restrict__ data, int64_t n,
    const int* __restrict__ wcols, const int* __restrict__ ucount,
    const double* __restrict__ X, double* __restrict__ Y, double eta,
    double* __restrict__ pqp, int dots2, unsigned long long* __restrict__ stamp) {
  extern __shared__ double smem[];
  // TPR threads per row (4: 256-thread blocks, 8: 512), CG columns each
  constexpr int NT = 64 * TPR;
  constexpr int CG = (S + TPR - 1) / TPR;
  constexpr int NB = 4096 / NT;   // loads in flight per thread while staging
  const int t = threadIdx.x;
  // in-step timing (gpmi_sp_set_timing): this workgroup's start and end on the
  // constant wall clock, stored at its end into its own pair of the launch's slot
  // (no atomics, no wait inside the kernel; reduced to the launch's span afterwards)
  const unsigned long long t_start = stamp ? (unsigned long long)wall_clock64() : 0ull;
  const int64_t b = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t r0 = b * WIN_ROWS, r1 = min(r0 + WIN_ROWS, n);
  const int nr = (int)(r1 - r0);
  const int u = ucount[b];
  const int r = t / TPR, g = t % TPR, c0 = g * CG;
  double acc[CG];
#pragma unroll
  for (int j = 0; j < CG; ++j) acc[j] = 0.0;
  if (u == 0) {
    // window over its limits: gather straight from X
    if (r < nr) {
      const int64_t row = r0 + r;
      for (int64_t k = indptr[row]; k < indptr[row + 1]; ++k) {
        const double v = data[k];
        const double* xr = X + (int64_t)indices[k] * S;
#pragma unroll
        for (int j = 0; j < CG; ++j)
          if (c0 + j < S) acc[j] += v * xr[c0 + j];
      }
    }
  } else {
    double* win = smem;   // [u][S]
    const int* wc = wcols + b * WIN_MAXU;
    if (S % 2 == 0) {
      constexpr int H = S / 2;   // 16-byte pairs per row
      const int E2 = u * H;
      for (int base = 0; base < E2; base += NT * NB) {
        d2 v[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const int i = base + q * NT + t;
          v[q] = i < E2 ? *reinterpret_cast<const d2*>(X + (int64_t)wc[i / H] * S + 2 * (i % H))
                        : d2{0.0, 0.0};
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const int i = base + q * NT + t;
          if (i < E2) *reinterpret_cast<d2*>(win + 2 * i) = v[q];
        }
      }
    } else {
      const int E = u * S;
      for (int base = 0; base < E; base += NT * NB) {
        double v[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const int i = base + q * NT + t;
          v[q] = i < E ? X[(int64_t)wc[i / S] * S + i % S] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const int i = base + q * NT + t;
          if (i < E) win[i] = v[q];
        }
      }
    }
    __syncthreads();
    if (r < nr) {
      const int64_t row = r0 + r;
      const int64_t ka = indptr[row], kb = indptr[row + 1];
      // U nonzeros' values and window positions loaded (global, in flight together)
      // before their window reads and products
      int64_t k = ka;
      for (; k + U <= kb; k += U) {
        double v[U];
        int p[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
          v[q] = data[k + q];
          p[q] = (int)lidx[k + q];
        }
#pragma unroll
        for (int q = 0; q < U; ++q) {
          const double* wr = win + p[q] * S + c0;
#pragma unroll
          for (int j = 0; j < CG; ++j)
            if (c0 + j < S) acc[j] += v[q] * wr[j];
        }
      }
      for (; k < kb; ++k) {
        const double v = data[k];
        const double* wr = win + (int)lidx[k] * S + c0;
#pragma unroll
        for (int j = 0; j < CG; ++j)
          if (c0 + j < S) acc[j] += v * wr[j];
      }
    }
  }
  double xy[CG], xx[CG];
#pragma unroll
  for (int j = 0; j < CG; ++j) xy[j] = xx[j] = 0.0;
  if (r < nr) {
    const int64_t row = r0 + r;
#pragma unroll
    for (int j = 0; j < CG; ++j)
      if (c0 + j < S) {
        const double x = X[row * S + c0 + j];
        const double y = acc[j] + eta * x;
        Y[row * S + c0 + j] = y;
        xy[j] = x * y;
        xx[j] = x * x;
      }
  }
  if (pqp) {
    // the block's x . y per column (the Lanczos's u . Ku), rows summed in order:
    // pqp[c][b]; the window's LDS is free once every thread is past its products.
    // dots2 (the Chronopoulos-Gear multi-shift CG, x = r, y = A r): the row
    // [x . y | x . x] of this block at pqp[0 .. 2S)[b] (summed by ms_cg2_reduce_kernel)
    const int WD = dots2 ? 2 * S : S;
    __syncthreads();
    double* red = smem;   // [64][WD]
#pragma unroll
    for (int j = 0; j < CG; ++j)
      if (c0 + j < S) {
        red[r * WD + c0 + j] = xy[j];
        if (dots2) red[r * WD + S + c0 + j] = xx[j];
      }
    __syncthreads();
    if (t < WD) {
      double sum = 0.0;
      for (int q = 0; q < nr; ++q) sum += red[q * WD + t];
      // column-major [WD][nblk]: the per-column sums (lz0_alpha_kernel,
      // ms_cg2_reduce_kernel) read it coalesced
      pqp[(int64_t)t * gridDim.x + b] = sum;
    }
  }
  if (stamp) {
    __syncthreads();
    if (t == 0) {
      const unsigned long long t_end = (unsigned long long)wall_clock64();
      stamp[2 * blockIdx.x] = t_start;
      stamp[2 * blockIdx.x + 1] = t_end;
    }
  }
}

// every width 1 .. 20: the probe and column shards of an N-rank sweep run narrower
// blocks than the single-GPU 20 (Lanczos) / 12 (multi-shift CG): at N = 8 a cfg 5
// rank's 3 probes and 2 columns (round 6; the gather kernels they fell back to
// made cfg 5's rank step 3x slower than the whole single-GPU step)
#define GPMI_WING_INST(S)                                                                \
  template __global__ void csr_spmm_wing_kernel<S, 8, 4>(                                 \
      const int64_t*, const int*, const unsigned short*, const double*, int64_t, const int*, \
      const int*, const double*, double*, double, double*, int, unsigned long long*);
GPMI_WING_INST(1) GPMI_WING_INST(2) GPMI_WING_INST(3) GPMI_WING_INST(4) GPMI_WING_INST(5)
GPMI_WING_INST(6) GPMI_WING_INST(7) GPMI_WING_INST(8) GPMI_WING_INST(9) GPMI_WING_INST(10)
GPMI_WING_INST(11) GPMI_WING_INST(12) GPMI_WING_INST(13) GPMI_WING_INST(14) GPMI_WING_INST(15)
GPMI_WING_INST(16) GPMI_WING_INST(17) GPMI_WING_INST(18) GPMI_WING_INST(19) GPMI_WING_INST(20)
#undef GPMI_WING_INST

// partial[b][j][c] = sum over this block's rows of A_j[i][c] * B[i][c],
// A_j = A + j * strideA, j = blockIdx.y; grid-stride over rows.
__global__ __launch_bounds__(256) void col_dot_partial_kernel(const double* __restrict__ A,
                                                              int64_t strideA,
                                                              const double* __restrict__ B,
                                                              int64_t n, int s,
                                                              double* __restrict__ partial) {
  __shared__ double red[256];
  const int t = threadIdx.x;
  const int rows_per = 256 / s;            // s <= 256
  const int c = t % s, r = t / s;
  const int j = blockIdx.y;
  const double* Aj = A + j * strideA;
  double acc = 0.0;
  if (r < rows_per)
    for (int64_t i = (int64_t)blockIdx.x * rows_per + r; i < n; i += (int64_t)gridDim.x * rows_per)
      acc += Aj[i * s + c] * B[i * s + c];
  red[t] = acc;
  __syncthreads();
  if (t < s) {
    double v = 0.0;
    for (int q = 0; q < rows_per; ++q) v += red[q * s + t];
    partial[((int64_t)blockIdx.x * gridDim.y + j) * s + t] = v;
  }
}

// Fixed-order wave reduction of v over the 64 lanes (xor butterfly).
__device__ __forceinline__ double wave_sum(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// sum_b partial[b * stride + e], b < nblk, by one wave (nblk strided over lanes).
__device__ __forceinline__ double wave_reduce_partials(const double* __restrict__ partial,
                                                       int nblk, int64_t stride, int e) {
  // a lane's partials (b = lane, lane + 64, ...) summed in ascending b, their loads
  // issued eight at a time (the same additions, in the same order, as one at a time)
  const int lane = threadIdx.x & 63;
  double v = 0.0;
  int b = lane;
  for (; b + 7 * 64 < nblk; b += 8 * 64) {
    double x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = partial[(int64_t)(b + q * 64) * stride + e];
#pragma unroll
    for (int q = 0; q < 8; ++q) v += x[q];
  }
  for (; b < nblk; b += 64) v += partial[(int64_t)b * stride + e];
  return wave_sum(v);
}

// out[j][c] = sum_b partial[b][j][c]: one wave per output element (fixed order).
__global__ __launch_bounds__(256) void col_dot_reduce_kernel(const double* __restrict__ partial,
                                                             int nblk, int J, int s,
                                                             double* __restrict__ out) {
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= J * s) return;
  const double v = wave_reduce_partials(partial, nblk, (int64_t)J * s, e);
  if ((threadIdx.x & 63) == 0) out[e] = v;
}

// W[i][c] = alpha * W[i][c] - sum_{j<J} A_j[i][c] * H[j][c]   (H on the device)
// W -= sum_j A_j diag(H_j): two consecutive elements per thread (16-byte loads when
// the vector stride is even), the J vector loads issued four at a time (the same
// per-element order of subtraction as one element per thread)
__global__ __launch_bounds__(256) void col_gs_update_kernel(double* __restrict__ W,
                                                            const double* __restrict__ A,
                                                            int64_t strideA,
                                                            const double* __restrict__ H, int J,
                                                            int64_t n, int s) {
  const int64_t ns = n * s;
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
  if (e >= ns) return;
  if (e + 1 < ns && (strideA & 1) == 0) {
    const int c0 = (int)(e % s), c1 = (c0 + 1 == s) ? 0 : c0 + 1;
    d2 w = *reinterpret_cast<const d2*>(W + e);
    int j = 0;
    for (; j + 4 <= J; j += 4) {
      d2 a[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = *reinterpret_cast<const d2*>(A + (j + q) * strideA + e);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w[0] -= a[q][0] * H[(j + q) * s + c0];
        w[1] -= a[q][1] * H[(j + q) * s + c1];
      }
    }
    for (; j < J; ++j) {
      const d2 a = *reinterpret_cast<const d2*>(A + j * strideA + e);
      w[0] -= a[0] * H[j * s + c0];
      w[1] -= a[1] * H[j * s + c1];
    }
    *reinterpret_cast<d2*>(W + e) = w;
  } else {
    for (int64_t f = e; f < e + 2 && f < ns; ++f) {
      const int c = (int)(f % s);
      double w = W[f];
      for (int j = 0; j < J; ++j) w -= A[j * strideA + f] * H[j * s + c];
      W[f] = w;
    }
  }
}

// Y[i][c] = a[c] * X[i][c] + b[c] * Y[i][c]  (per-column coefficients, device)
__global__ __launch_bounds__(256) void col_axpby_kernel(const double* __restrict__ X,
                                                        double* __restrict__ Y,
                                                        const double* __restrict__ a,
                                                        const double* __restrict__ b,
                                                        int64_t n, int s) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * s) return;
  const int c = (int)(e % s);
  Y[e] = a[c] * X[e] + b[c] * Y[e];
}

// gpmi_sp_cg with its scalars on the device (no host round trip per iteration).
// Step 1: an active column c (act[c]) takes a = rr[c] / pq[c]; x += a p, r -= a q.
// Block 0 flags a non-positive p.q of an active column (the host reads err when it polls).
__global__ __launch_bounds__(256) void cg_xr_kernel(const double* __restrict__ P,
                                                    const double* __restrict__ Q,
                                                    double* __restrict__ X, double* __restrict__ R,
                                                    const double* __restrict__ rr,
                                                    const double* __restrict__ pq,
                                                    const int* __restrict__ act, int64_t n, int s,
                                                    int* __restrict__ err) {
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)s) {
    const int c = threadIdx.x;
    if (act[c] && !(pq[c] > 0.0)) err[0] = 1;
  }
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * s) return;
  const int c = (int)(e % s);
  if (!act[c]) return;
  const double a = rr[c] / pq[c];
  X[e] += a * P[e];
  R[e] -= a * Q[e];
}

// Step 2: p = r + (rrn[c] / rr[c]) p on the active columns. Block 0 writes the next
// iteration's flags (active while sqrt(rrn) > rtol ||b||, the host loop's test) and,
// when any column ran this iteration, the iteration count it + 1.
__global__ __launch_bounds__(256) void cg_p_kernel(const double* __restrict__ R,
                                                   double* __restrict__ P,
                                                   const double* __restrict__ rr,
                                                   const double* __restrict__ rrn,
                                                   const int* __restrict__ act,
                                                   int* __restrict__ act_next,
                                                   const double* __restrict__ thr, int it,
                                                   int* __restrict__ iters, int64_t n, int s) {
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)s) {
    const int c = threadIdx.x;
    act_next[c] = act[c] && (std::sqrt(rrn[c]) > thr[c]);
    if (c == 0) {
      int any = 0;
      for (int k = 0; k < s; ++k) any |= act[k];
      if (any) iters[0] = it + 1;
    }
  }
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * s) return;
  const int c = (int)(e % s);
  if (!act[c]) return;
  P[e] = R[e] + (rrn[c] / rr[c]) * P[e];
}

// First flags: thr = rtol sqrt(rr0), act = sqrt(rr0) > thr.
__global__ void cg_init_kernel(const double* __restrict__ rr, double rtol, int s,
                               double* __restrict__ thr, int* __restrict__ act,
                               int* __restrict__ err, int* __restrict__ iters) {
  const int c = threadIdx.x;
  if (c == 0) {
    err[0] = 0;
    iters[0] = 0;
  }
  if (c >= s) return;
  const double bn = std::sqrt(rr[c]);
  thr[c] = rtol * bn;
  act[c] = bn > rtol * bn;
}

// Lanczos step k scalars on the device (no host round trip): alpha = the two
// CGS2 passes' projections on V_k, beta = ||W||, a column whose beta falls below
// 1e-13 max(1, |alpha|) is dead (invariant subspace: padding from then on).
// Writes alpha/beta[c][k], and the axpby coefficients for V_{k+1} = W / beta
// (ca/cb) and for the next step's W -= beta V_k (na/nb).
__global__ void lanczos_scalar_kernel(const double* __restrict__ H1k,
                                      const double* __restrict__ H2k,
                                      const double* __restrict__ nrm, int s, int k, int steps,
                                      int* __restrict__ dead, double* __restrict__ alpha,
                                      double* __restrict__ beta, double* __restrict__ ca,
                                      double* __restrict__ cb, double* __restrict__ na,
                                      double* __restrict__ nb) {
  const int c = threadIdx.x;
  if (c >= s) return;
  if (k == 0) dead[c] = 0;
  const int dd = dead[c];
  const double a = dd ? 0.0 : (0.0 + H1k[c]) + H2k[c];
  double b = dd ? 0.0 : sqrt(fmax(nrm[c], 0.0));
  if (!dd && !(b > 1e-13 * fmax(1.0, fabs(a)))) {
    dead[c] = 1;
    b = 0.0;
  }
  alpha[(int64_t)c * steps + k] = a;
  beta[(int64_t)c * steps + k] = b;
  ca[c] = b > 0.0 ? 1.0 / b : 0.0;
  cb[c] = 0.0;
  na[c] = -b;
  nb[c] = 1.0;
}

// ---------------------------------------------------------------------------
// Lanczos by the plain three-term recurrence (imate's orthogonalize = 0, its
// default) in three launches per step and one pass over three vectors. The
// vectors are stored unnormalised, u_k = gamma_k v_k (gamma_0 = 1: the probes are
// normalised, gamma_k = beta_{k-1} after). Step k, in the order of
// oracle/sparse.py lanczos(reorth=False) (w = K v_k - beta v_{k-1}; h = v_k . w;
// w -= h v_k):
//   SpMM    y = K u_k, with the 64-row block partials of u_k . y (the window
//           kernel's epilogue, or lz0_dot64_kernel)
//   alpha   per column (one wave each): gamma_k = ||u_k|| from the previous
//           update's partials (= beta_{k-1}, with lanczos_scalar_kernel's breakdown
//           test), alpha_k = h = (u_k . y) / gamma_k^2 - (u_k . u_{k-1}) / gamma_{k-1},
//           and the update's coefficients
//   update  u_{k+1} = y / gamma_k - (gamma_k / gamma_{k-1}) u_{k-1} - (h / gamma_k) u_k,
//           with the 64-row block partials of ||u_{k+1}||^2 and u_{k+1} . u_k
// A last alpha launch (k = steps) forms beta_{steps-1}. Every reduction has a fixed
// order (deterministic). st: [0, s) gamma_k, [s, 2s) gamma_{k-1}; coef [3][s].

// out[c][b] = sum over the 64 rows of block b of X[i][c] Y[i][c] (fixed order;
// column-major, as the window SpMM's epilogue).
__global__ __launch_bounds__(256) void lz0_dot64_kernel(const double* __restrict__ X,
                                                        const double* __restrict__ Y, int64_t n,
                                                        int s, double* __restrict__ out) {
  __shared__ double sp[64 * 32];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  const int rows = (int)min((int64_t)64, n - r0);
  for (int e = t; e < 64 * s; e += 256) {
    const int i = e / s;
    sp[e] = i < rows ? X[r0 * s + e] * Y[r0 * s + e] : 0.0;
  }
  __syncthreads();
  if (t < s) {
    double a = 0.0;
    for (int i = 0; i < 64; ++i) a += sp[i * s + t];
    out[(int64_t)t * gridDim.x + blockIdx.x] = a;
  }
}

__global__ __launch_bounds__(256) void lz0_alpha_kernel(const double* __restrict__ pq,
                                                        const double* __restrict__ pv, int nb,
                                                        int s, int k, int steps,
                                                        double* __restrict__ st,
                                                        int* __restrict__ dead,
                                                        double* __restrict__ alpha,
                                                        double* __restrict__ beta,
                                                        double* __restrict__ coef) {
  // one workgroup per column c: thread t sums blocks b = t, t + 256, ... of the three
  // partial arrays (column-major [column][block]: coalesced; their loads in flight
  // together, eight blocks at a time), then the four waves' sums combine in a fixed
  // order (the round-3 form, one wave per column and one array after the other, took
  // ~44 us at 4096 blocks; with [block][column] rows ~28 us in the cfg 5 step)
  const int c = blockIdx.x, t = threadIdx.x;
  __shared__ double red[3][4];
  const bool has1 = k < steps, has2 = k > 0;
  const double* p1 = pq + (int64_t)c * nb;
  const double* p2 = pv + (int64_t)c * nb;
  const double* p3 = pv + (int64_t)(s + c) * nb;
  double a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int b = t;
  for (; b + 7 * 256 < nb; b += 8 * 256) {
    double x1[8], x2[8], x3[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int bq = b + q * 256;
      x1[q] = has1 ? p1[bq] : 0.0;
      x2[q] = has2 ? p2[bq] : 0.0;
      x3[q] = has2 ? p3[bq] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      a1 += x1[q];
      a2 += x2[q];
      a3 += x3[q];
    }
  }
  for (; b < nb; b += 256) {
    if (has1) a1 += p1[b];
    if (has2) {
      a2 += p2[b];
      a3 += p3[b];
    }
  }
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  a3 = wave_sum(a3);
  const int w = t >> 6;
  if ((t & 63) == 0) {
    red[0][w] = a1;
    red[1][w] = a2;
    red[2][w] = a3;
  }
  __syncthreads();
  if (t != 0) return;
  const double d1 = has1 ? (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]) : 0.0;
  const double nrm2 = has2 ? (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]) : 1.0;
  const double d2 = has2 ? (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]) : 0.0;
  double gam = 1.0, gamp = 1.0;
  if (k == 0) {
    dead[c] = 0;
  } else {
    gamp = st[c];
    double b = dead[c] ? 0.0 : sqrt(fmax(nrm2, 0.0));
    if (!dead[c] && !(b > 1e-13 * fmax(1.0, fabs(alpha[(int64_t)c * steps + k - 1])))) {
      dead[c] = 1;
      b = 0.0;
    }
    beta[(int64_t)c * steps + k - 1] = b;
    gam = b;
  }
  if (k == steps) return;
  st[c] = gam;
  st[s + c] = gamp;
  if (dead[c]) {
    alpha[(int64_t)c * steps + k] = 0.0;
    coef[c] = coef[s + c] = coef[2 * s + c] = 0.0;
    return;
  }
  const double h = d1 / (gam * gam) - (k > 0 ? d2 / gamp : 0.0);
  alpha[(int64_t)c * steps + k] = h;
  coef[c] = 1.0 / gam;
  coef[s + c] = k > 0 ? gam / gamp : 0.0;
  coef[2 * s + c] = h / gam;
}

// u_{k+1} = c1 y - c2 u_{k-1} - c3 u_k per column, and per 64-row block b the partials
// pv[0][c][b] = ||u_{k+1}||^2, pv[1][c][b] = u_{k+1} . u_k (fixed order; column-major).
__global__ __launch_bounds__(256) void lz0_update_kernel(const double* __restrict__ Y,
                                                         const double* __restrict__ Up,
                                                         const double* __restrict__ Uc,
                                                         double* __restrict__ Un,
                                                         const double* __restrict__ coef,
                                                         int64_t n, int s,
                                                         double* __restrict__ pv) {
  __shared__ double sq[64 * 32];
  __shared__ double sx[64 * 32];
  __shared__ double sc[3 * 32];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  const int rows = (int)min((int64_t)64, n - r0);
  const int E = rows * s;   // the block's elements, contiguous from g0
  const int64_t g0 = r0 * s;
  if (t < 3 * s) sc[t] = coef[t];
  for (int e = E + t; e < 64 * s; e += 256) sq[e] = sx[e] = 0.0;
  __syncthreads();
  const bool vec = ((reinterpret_cast<uintptr_t>(Y + g0) | reinterpret_cast<uintptr_t>(Up + g0) |
                     reinterpret_cast<uintptr_t>(Uc + g0) | reinterpret_cast<uintptr_t>(Un + g0)) &
                    15) == 0;
  if (vec) {
    // element pairs as 16-byte loads / stores; the pair's first column c advances by
    // 512 mod s per iteration (no division in the loop)
    const int step = 512 % s;
    int c = (2 * t) % s;
    for (int p = t; 2 * p + 1 < E; p += 256) {
      const int e = 2 * p;
      const d2 y = *reinterpret_cast<const d2*>(Y + g0 + e);
      const d2 up = *reinterpret_cast<const d2*>(Up + g0 + e);
      const d2 uc = *reinterpret_cast<const d2*>(Uc + g0 + e);
      const int c1 = c + 1 == s ? 0 : c + 1;
      const double w0 = sc[c] * y[0] - sc[s + c] * up[0] - sc[2 * s + c] * uc[0];
      const double w1 = sc[c1] * y[1] - sc[s + c1] * up[1] - sc[2 * s + c1] * uc[1];
      *reinterpret_cast<d2*>(Un + g0 + e) = d2{w0, w1};
      sq[e] = w0 * w0;
      sq[e + 1] = w1 * w1;
      sx[e] = w0 * uc[0];
      sx[e + 1] = w1 * uc[1];
      c += step;
      if (c >= s) c -= s;
    }
    if ((E & 1) && t == 0) {
      const int e = E - 1, cc = e % s;
      const double u = Uc[g0 + e];
      const double w = sc[cc] * Y[g0 + e] - sc[s + cc] * Up[g0 + e] - sc[2 * s + cc] * u;
      Un[g0 + e] = w;
      sq[e] = w * w;
      sx[e] = w * u;
    }
  } else {
    for (int e = t; e < E; e += 256) {
      const int c = e % s;
      const int64_t g = g0 + e;
      const double uc = Uc[g];
      const double w = sc[c] * Y[g] - sc[s + c] * Up[g] - sc[2 * s + c] * uc;
      Un[g] = w;
      sq[e] = w * w;
      sx[e] = w * uc;
    }
  }
  __syncthreads();
  if (t < 2 * s) {
    const double* src = t < s ? sq : sx;
    const int c = t < s ? t : t - s;
    double a = 0.0;
    for (int i = 0; i < 64; ++i) a += src[i * s + c];
    pv[(int64_t)t * gridDim.x + blockIdx.x] = a;
  }
}

// ---------------------------------------------------------------------------
// Lanczos with delayed classical Gram-Schmidt reorthogonalisation (DCGS2:
// Bielich, Langou, Thomas, Swirydowicz, Yamazaki, Boman, Parallel Computing 112
// (2022) 102940; numpy prototype tools/dcgs2_proto.py). CGS2 reads the basis four
// times per step (two dot passes, two update passes); here step k reads it twice:
//   y = (K) u_k                                  (SpMM of the once-projected u_k)
//   dots:   s = V^T u_k, t = V^T y, sigma = u.u, tau = u.y   (ONE pass, lz_dots)
//   scalar: rho = sqrt(sigma - s.s) = beta_{k-1}, H[:, k-1] += s (alpha_{k-1}
//           final), Hs = H s (K V s = V_{k+1} H s), h = V_{k+1}^T K v_k from
//           (t, tau, Hs)                                 (lz_scalar)
//   update: v_k = (u - V s) / rho, u_{k+1} = y / rho - V_{k+1} (Hs / rho + h)
//           (ONE pass, both vectors, lz_update)
// Per probe column c; every reduction has a fixed order (deterministic).

// Basis reads of the DCGS2 passes as non-temporal loads when NT (chosen by the host
// for a basis larger than twice the Infinity Cache): the basis (1.26 GB at cfg 5)
// then streams through each pass without evicting the CSR and window rows the SpMMs
// (the Lanczos's own and the multi-shift CG's beside it) reread (cfg 5 Lanczos
// 13.0 -> 11.2 ms); a basis that fits (cfg 4: 0.3 GB) is faster cached.
template <bool NT>
__device__ __forceinline__ double ld_basis(const double* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ d2 ld_basis2(const double* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const d2*>(p));
  return *reinterpret_cast<const d2*>(p);
}

// partial[b][v][c] over this block's rows: v = j0 + q: V_{j0+q} . u; v = J + j0 + q:
// V_{j0+q} . y (Y given); with j0 == 0 also v = 2J: u . u and 2J + 1: u . y.
// Vectors [j0, j0 + LZ_JC) of the J per launch; rows grid-strided, one column per
// thread (256 / s rows per block iteration).
template <bool NT>
__global__ __launch_bounds__(256) void lz_dots_kernel(const double* __restrict__ V, int64_t ns,
                                                      int J, int j0,
                                                      const double* __restrict__ U,
                                                      const double* __restrict__ Y, int64_t n,
                                                      int s, int nv,
                                                      double* __restrict__ partial) {
  __shared__ double red[256];
  const int t = threadIdx.x;
  const int rows_per = 256 / s;
  const int c = t % s, r = t / s;
  const int jc = min(LZ_JC, J - j0);
  double as[LZ_JC], at[LZ_JC];
#pragma unroll
  for (int q = 0; q < LZ_JC; ++q) as[q] = at[q] = 0.0;
  double uu = 0.0, uy = 0.0;
  if (r < rows_per)
    for (int64_t i = (int64_t)blockIdx.x * rows_per + r; i < n;
         i += (int64_t)gridDim.x * rows_per) {
      const int64_t e = i * s + c;
      const double u = U[e];
      const double y = Y ? Y[e] : 0.0;
      double v[LZ_JC];
#pragma unroll
      for (int q = 0; q < LZ_JC; ++q)
        v[q] = q < jc ? ld_basis<NT>(V + (int64_t)(j0 + q) * ns + e) : 0.0;
      uu += u * u;
      uy += u * y;
#pragma unroll
      for (int q = 0; q < LZ_JC; ++q) {
        as[q] += v[q] * u;
        at[q] += v[q] * y;
      }
    }
  // per column: the rows_per threads of column c summed in row order
  auto put = [&](double val, int vi) {
    red[t] = val;
    __syncthreads();
    if (t < s) {
      double acc = 0.0;
      for (int q = 0; q < rows_per; ++q) acc += red[q * s + t];
      partial[((int64_t)blockIdx.x * nv + vi) * s + t] = acc;
    }
    __syncthreads();
  };
  for (int q = 0; q < jc; ++q) {
    put(as[q], j0 + q);
    if (Y) put(at[q], J + j0 + q);
  }
  if (j0 == 0) {
    put(uu, 2 * J);
    put(uy, 2 * J + 1);
  }
}
template __global__ void lz_dots_kernel<false>(const double*, int64_t, int, int, const double*,
                                               const double*, int64_t, int, int, double*);
template __global__ void lz_dots_kernel<true>(const double*, int64_t, int, int, const double*,
                                              const double*, int64_t, int, int, double*);

// Step k's scalars (one workgroup; d = reduced dots [(2k + 2)][s]; per column c:
// H [c][(steps + 2) x (steps + 1)] row-major (H[i][j]: coefficient of v_i in K v_j),
// the update coefficients cv [k][s] (of V_j in v_k, times -1), cu [k + 1][s] (of V_j
// in u_{k+1}, times -1), ir[s] = 1 / rho; alpha / beta [c][steps] as lanczos_scalar;
// inexact[c]: sigma - s.s lost more than six digits to cancellation (rho then
// unreliable; the host reruns the block with CGS2).
// stage: the host gave (2k + 2) s doubles of dynamic LDS, and d is read from there
// (the phases' per-column loops over the dots then wait on LDS, not L2).
__global__ void lz_scalar_kernel(const double* __restrict__ dg, int k, int steps, int s,
                                 double* __restrict__ H, double* __restrict__ cv,
                                 double* __restrict__ cu, double* __restrict__ ir,
                                 double* __restrict__ rho_s, int* __restrict__ dead,
                                 int* __restrict__ inexact, double* __restrict__ alpha,
                                 double* __restrict__ beta, int stage) {
  extern __shared__ double sdots[];
  const int ld = steps + 1;
  const size_t hsz = (size_t)(steps + 2) * ld;
  const int J = k;
  const int t = threadIdx.x;
  if (stage) {
    for (int i = t; i < (2 * J + 2) * s; i += blockDim.x) sdots[i] = dg[i];
    __syncthreads();
  }
  const double* d = stage ? sdots : dg;
  if (t < s) {
    const int c = t;
    if (k == 0) {
      dead[c] = 0;
      inexact[c] = 0;
    }
    double* Hc = H + c * hsz;
    double rho = 1.0;
    if (k > 0) {
      double ss = 0.0;
      for (int j = 0; j < J; ++j) {
        const double sj = d[j * s + c];
        ss += sj * sj;
        Hc[j * ld + (k - 1)] += sj;
      }
      const double sig = d[2 * J * s + c];
      const double dd = sig - ss;
      rho = sqrt(fmax(dd, 0.0));
      const double a = dead[c] ? 0.0 : Hc[(k - 1) * ld + (k - 1)];
      double b = dead[c] ? 0.0 : rho;
      if (!dead[c] && !(b > 1e-13 * fmax(1.0, fabs(a)))) {
        dead[c] = 1;
        b = 0.0;
      } else if (!dead[c] && !(dd >= 1e-6 * sig)) {
        inexact[c] = 1;
      }
      alpha[(int64_t)c * steps + (k - 1)] = a;
      beta[(int64_t)c * steps + (k - 1)] = b;
      if (!dead[c] && k < steps) Hc[k * ld + (k - 1)] = rho;
    }
    rho_s[c] = dead[c] ? 0.0 : rho;
  }
  if (k == steps) return;
  __syncthreads();
  // Hs_i = sum_{j >= i - 1} H[i][j] s_j (H upper Hessenberg), thread per (c, i); into cu
  for (int task = t; task < s * (k + 1); task += blockDim.x) {
    const int c = task % s, i = task / s;
    const double* Hc = H + c * hsz;
    double acc = 0.0;
    for (int j = i > 0 ? i - 1 : 0; j < J; ++j) acc += Hc[i * ld + j] * d[j * s + c];
    cu[i * s + c] = acc;
  }
  __syncthreads();
  if (t < s) {
    const int c = t;
    double* Hc = H + c * hsz;
    const double rho = rho_s[c];
    if (rho == 0.0) {
      for (int j = 0; j < J; ++j) cv[j * s + c] = 0.0;
      for (int i = 0; i <= k; ++i) cu[i * s + c] = 0.0;
      ir[c] = 0.0;
    } else {
      const double inv = 1.0 / rho;
      double st = 0.0;
      for (int j = 0; j < J; ++j) st += d[j * s + c] * d[(J + j) * s + c];
      const double tau = d[(2 * J + 1) * s + c];
      for (int i = 0; i < k; ++i) {
        const double hs = cu[i * s + c];
        const double h = (d[(J + i) * s + c] - hs) * inv;
        Hc[i * ld + k] = h;
        cu[i * s + c] = hs * inv + h;
        cv[i * s + c] = d[i * s + c] * inv;
      }
      const double hsk = cu[k * s + c];
      const double hk = (tau - st) * inv * inv - hsk * inv;
      Hc[k * ld + k] = hk;
      cu[k * s + c] = hsk * inv + hk;
      ir[c] = inv;
    }
  }
}

// v_k = u / rho - sum_{j<k} V_j cv_j;  u <- y / rho - sum_{j<k} V_j cu_j - v_k cu_k;
// V_k = v_k. Two consecutive elements per thread (16-byte loads) in each of NR
// row chunks P pairs apart (P = the grid's thread count, 2 P a multiple of s, so the
// chunks share the thread's two columns and their coefficient loads), the basis
// loads four vectors at a time; the same per-element order of subtraction as one
// element per thread.
template <int NR, bool NT>
__global__ __launch_bounds__(256) void lz_update_kernel(double* __restrict__ V, int64_t ns, int k,
                                                        double* __restrict__ U,
                                                        const double* __restrict__ Y,
                                                        const double* __restrict__ cv,
                                                        const double* __restrict__ cu,
                                                        const double* __restrict__ ir, int s) {
  const int64_t P = (int64_t)gridDim.x * 256;
  const int64_t e0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
  if (e0 >= ns) return;
  const int c0 = (int)(e0 % s), c1 = (c0 + 1 == s) ? 0 : c0 + 1;
  if ((ns & 1) == 0) {
    double v0[NR], v1[NR], w0[NR], w1[NR];
    bool on[NR];
    const double i0 = ir[c0], i1 = ir[c1];
#pragma unroll
    for (int m = 0; m < NR; ++m) {
      const int64_t e = e0 + 2 * P * m;
      on[m] = e < ns;
      const d2 u = on[m] ? *reinterpret_cast<const d2*>(U + e) : d2{0.0, 0.0};
      const d2 y = on[m] ? *reinterpret_cast<const d2*>(Y + e) : d2{0.0, 0.0};
      v0[m] = u[0] * i0;
      v1[m] = u[1] * i1;
      w0[m] = y[0] * i0;
      w1[m] = y[1] * i1;
    }
    int j = 0;
    for (; j + 4 <= k; j += 4) {
      d2 a[4][NR];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int m = 0; m < NR; ++m)
          a[q][m] = on[m] ? ld_basis2<NT>(V + (j + q) * ns + e0 + 2 * P * m)
                          : d2{0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double cv0 = cv[(j + q) * s + c0], cv1 = cv[(j + q) * s + c1];
        const double cu0 = cu[(j + q) * s + c0], cu1 = cu[(j + q) * s + c1];
#pragma unroll
        for (int m = 0; m < NR; ++m) {
          v0[m] -= a[q][m][0] * cv0;
          v1[m] -= a[q][m][1] * cv1;
          w0[m] -= a[q][m][0] * cu0;
          w1[m] -= a[q][m][1] * cu1;
        }
      }
    }
    for (; j < k; ++j) {
      const double cv0 = cv[j * s + c0], cv1 = cv[j * s + c1];
      const double cu0 = cu[j * s + c0], cu1 = cu[j * s + c1];
#pragma unroll
      for (int m = 0; m < NR; ++m) {
        const d2 a = on[m] ? ld_basis2<NT>(V + j * ns + e0 + 2 * P * m)
                           : d2{0.0, 0.0};
        v0[m] -= a[0] * cv0;
        v1[m] -= a[1] * cv1;
        w0[m] -= a[0] * cu0;
        w1[m] -= a[1] * cu1;
      }
    }
    const double ck0 = cu[k * s + c0], ck1 = cu[k * s + c1];
#pragma unroll
    for (int m = 0; m < NR; ++m) {
      if (!on[m]) continue;
      const int64_t e = e0 + 2 * P * m;
      d2 vo, wo;
      vo[0] = v0[m];
      vo[1] = v1[m];
      wo[0] = w0[m] - v0[m] * ck0;
      wo[1] = w1[m] - v1[m] * ck1;
      *reinterpret_cast<d2*>(V + k * ns + e) = vo;
      *reinterpret_cast<d2*>(U + e) = wo;
    }
  } else {
    for (int m = 0; m < NR; ++m)
      for (int64_t f = e0 + 2 * P * m; f < e0 + 2 * P * m + 2 && f < ns; ++f) {
        const int c = (int)(f % s);
        double v = U[f] * ir[c], w = Y[f] * ir[c];
        for (int jj = 0; jj < k; ++jj) {
          const double a = V[jj * ns + f];
          v -= a * cv[jj * s + c];
          w -= a * cu[jj * s + c];
        }
        w -= v * cu[k * s + c];
        V[k * ns + f] = v;
        U[f] = w;
      }
  }
}
template __global__ void lz_update_kernel<4, false>(double*, int64_t, int, double*, const double*,
                                                    const double*, const double*, const double*,
                                                    int);
template __global__ void lz_update_kernel<4, true>(double*, int64_t, int, double*, const double*,
                                                   const double*, const double*, const double*,
                                                   int);

// Normalised Rademacher probes: V[i][c] = +-1/sqrt(n), bit 63 of
// splitmix64(seed * G + (c + c0) * H + i) (matches oracle/sparse.py).
// perm (optional): device row r holds original point perm[r] (locality order of
// gpmi_sp_create_matern); the probe entry follows the original index, so the
// probe set is the same vectors whatever the storage order.
__global__ __launch_bounds__(256) void rademacher_kernel(double* __restrict__ V, int64_t n, int s,
                                                         unsigned long long seed, int c0,
                                                         double scale,
                                                         const int* __restrict__ perm) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * s) return;
  const int64_t i = perm ? (int64_t)perm[e / s] : e / s;
  const int c = (int)(e % s);
  unsigned long long x = seed * 0x9E3779B97F4A7C15ull +
                         (unsigned long long)(c + c0) * 0xD1B54A32D192ED03ull +
                         (unsigned long long)i;
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x = x ^ (x >> 31);
  V[e] = (x >> 63) ? -scale : scale;
}


// ---------------------------------------------------------------------------
// Multi-shift CG Gram: for shifts eta_j = eta_0 + d_j (d_j >= 0) and RHS block
// B [n][s], G_j = B^T (K + eta_j I)^-1 B from ONE blocked CG on K + eta_0 I.
// Every shifted system lives in the same Krylov space (Jegerlehner's CG-M):
// its residual is zeta_j r and its direction p_j = zeta_j r + beta_j p_j', so
// b_c'^T p_j obeys a scalar recurrence driven by b_c'^T r, and
//   G_j[c'][c] = sum_k alpha_j^k (b_c'^T p_j^k)
// needs no per-shift vectors at all. All scalars stay on the device.
//
// Scalar state (device, double): see MsState below; one column c per CG.
// ---------------------------------------------------------------------------
// partial[blk][e]: e = c' * S + c < SA*S -> sum_i B[i][c'] R[i][c]; e = SA*S + c -> R_c . R_c
// (B: [n][SA], the dot columns; R: [n][S], the right-hand sides: SA >= S when the
// RHS columns are a shard of B's).
// One thread per row (grid-stride), the row's S values of R in registers;
// blockIdx.y selects four B columns c' (group 0 also forms R.R), so a thread
// holds at most 4*S + S accumulators. Block sums: wave butterflies, then the
// four waves in order (deterministic).
template <int S>
__global__ __launch_bounds__(256) void ms_dots_partial_kernel(const double* __restrict__ B,
                                                              const double* __restrict__ R,
                                                              int64_t n, int SA,
                                                              double* __restrict__ partial) {
  const int NE = SA * S + S;
  __shared__ double red[4][4 * S + S];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int c0 = blockIdx.y * 4;
  double acc[4][S], rr[S];
#pragma unroll
  for (int c = 0; c < S; ++c) {
    rr[c] = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q][c] = 0.0;
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + t; i < n; i += (int64_t)gridDim.x * 256) {
    double r[S], b[4];
#pragma unroll
    for (int c = 0; c < S; ++c) r[c] = R[i * S + c];
#pragma unroll
    for (int q = 0; q < 4; ++q) b[q] = (c0 + q < SA) ? B[i * SA + c0 + q] : 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int c = 0; c < S; ++c) acc[q][c] += b[q] * r[c];
    if (blockIdx.y == 0) {
#pragma unroll
      for (int c = 0; c < S; ++c) rr[c] += r[c] * r[c];
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int c = 0; c < S; ++c) {
      const double v = wave_sum(acc[q][c]);
      if (lane == 0) red[wv][q * S + c] = v;
    }
#pragma unroll
  for (int c = 0; c < S; ++c) {
    const double v = wave_sum(rr[c]);
    if (lane == 0) red[wv][4 * S + c] = v;
  }
  __syncthreads();
  if (t < 5 * S) {
    const double v = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    if (t < 4 * S) {
      const int q = t / S, c = t - q * S;
      if (c0 + q < SA) partial[(int64_t)blockIdx.x * NE + (c0 + q) * S + c] = v;
    } else if (blockIdx.y == 0) {
      partial[(int64_t)blockIdx.x * NE + SA * S + (t - 4 * S)] = v;
    }
  }
}

// Host-side dispatch over the instantiated widths.
void launch_ms_dots(const double* B, const double* R, int64_t n, int s, double* partial,
                    int nblk, hipStream_t st, int sa) {
  if (sa <= 0) sa = s;
  const dim3 grid(nblk, (sa + 3) / 4), blk(256);
  switch (s) {
#define MS_CASE(k) \
  case k:                                                                                   \
    hipLaunchKernelGGL(ms_dots_partial_kernel<k>, grid, blk, 0, st, B, R, n, sa, partial);    \
    break;
    MS_CASE(1) MS_CASE(2) MS_CASE(3) MS_CASE(4) MS_CASE(5) MS_CASE(6) MS_CASE(7) MS_CASE(8)
    MS_CASE(9) MS_CASE(10) MS_CASE(11) MS_CASE(12) MS_CASE(13) MS_CASE(14) MS_CASE(15)
    MS_CASE(16)
#undef MS_CASE
    default: break;
  }
}

// Multi-shift CG, Chronopoulos-Gear form (round 5): three launches per iteration,
// the SpMM, one reduction and this update, against five for the standard form
// (SpMM, reduce, r update + B^T r, reduce, tail). Iteration k: the SpMM gave
// w_k = (K + eta_0 I) r_k and per-block rows of r_k . w_k and r_k . r_k in its epilogue
// (csr_spmm_wing_kernel dots2, or ms_dots2_kernel); ms_cg2_reduce_kernel summed them,
// and the previous update's B^T r_k rows, into red = [delta[s] | gamma[s] | B^T r_k].
// Every block forms, per column (Chronopoulos and Gear, J. Comput. Appl. Math. 25
// (1989) 153):
//   gamma_k = r_k . r_k, delta_k = r_k . w_k, beta_{k-1} = gamma_k / gamma_{k-1}
//   (0 at k = 0), alpha_k = gamma_k / (delta_k - beta_{k-1} gamma_k / alpha_{k-1}),
// the denominator being p_k^T (K + eta_0 I) p_k (<= 0 flags the column), and the
// stop test gamma_k <= rtol^2 ||b||^2: standard CG's alpha, beta in exact arithmetic
// (numpy check of the whole recurrence: the Gram blocks to 1e-12 of exact solves, the
// same iteration count as a host CG). The vector blocks (1 .. MS_UB) then form, for
// active columns,
//   s_k = w_k + beta_{k-1} s_{k-1}  (= A p_k, p_k = r_k + beta_{k-1} p_{k-1}),
//   r_{k+1} = r_k - alpha_k s_k,
// and the block partials of B^T r_{k+1} on fp64 MFMA into bpart ([neb][MS_UB]),
// which the next iteration's reduction sums. p itself is never formed: the Gram
// blocks need only b . p of the shifted systems, which the shift recurrences carry
// from B^T r (so a pass reads r, w, s and B and writes s and r: six block passes,
// against seven for the standard form's r update and p update). Block 0 does no
// vector work: it takes
// the shift step k - 1 (the zeta / G / b . p recurrences of ms_tail_kernel, which need
// beta_{k-1}, known only now, and B^T r_k), then writes the next scalar state (nxt),
// the batch end state into pinned memory (pin) and the stopping iteration.
// A shift whose zeta fell below this is converged far past any tolerance (its residual
// is zeta times the seed system's): its G is final and its recurrences stop. Without
// the stop, a large shift's zeta (~ (1 + d alpha)^-k) underflows to 0 within the seed's
// iterations and alpha^s = alpha zeta_k / zeta_{k-1} becomes 0 / 0 (round 6: the
// largest eta of cfg 4's curve had a NaN Gram column for the data vector z).
constexpr double MS_ZETA_MIN = 1e-250;

// zeta_k and alpha_{k-1} of shift j for column c (the shifted recurrence of step k - 1
// from the unshifted alpha_{k-1}, alpha_{k-2}, beta_{k-1} in cur).
__device__ __forceinline__ void ms_shift_step(const MsScal& cur, const MsShift& sh,
                                              const double* __restrict__ dshift, int s, int j,
                                              int c, double& zn, double& as) {
  const double a = cur.a[c], ap = cur.a_prev[c], bo = cur.beta[c];
  const double z = sh.z[j * s + c], zp = sh.z_prev[j * s + c];
  const double d = dshift[j];
  zn = z * zp * ap / (a * bo * (zp - z) + zp * ap * (1.0 + d * a));
  as = a * zn / z;
}

// After the last iteration: ms_cg2_update_kernel applies shift step k - 1 during
// iteration k (its b . p update needs beta_k), so a loop that ends at maxiter with
// columns still active has not applied their last step's G update. This applies it
// (G += alpha^s_{k-1} b . p^s for the columns that took step k - 1; one workgroup).
// A no-op when every column had stopped.
__global__ __launch_bounds__(256) void ms_cg2_close_kernel(MsScal cur, MsShift sh,
                                                           const double* __restrict__ dshift,
                                                           int S, int s, int nb) {
  for (int task = threadIdx.x; task < S * s; task += blockDim.x) {
    const int j = task / s, c = task % s;
    if (!cur.active[c]) continue;
    if (!(fabs(sh.z[j * s + c]) >= MS_ZETA_MIN)) continue;   // converged shift
    double zn, as;
    ms_shift_step(cur, sh, dshift, s, j, c, zn, as);
    for (int cp = 0; cp < nb; ++cp) {
      const int e = (j * nb + cp) * s + c;
      sh.g[e] += as * sh.bp[e];
    }
    sh.z_prev[j * s + c] = sh.z[j * s + c];
    sh.z[j * s + c] = zn;
  }
}

__global__ __launch_bounds__(256) void ms_cg2_update_kernel(
    const double* __restrict__ B, double* __restrict__ R, const double* __restrict__ W,
    double* __restrict__ Sv, MsScal cur, MsScal nxt, MsShift sh,
    const double* __restrict__ red_in, double* __restrict__ bpart,
    const double* __restrict__ dshift, int S, int s, int nb, double rtol2, int k, int64_t n,
    MsPin* __restrict__ pin) {
  __shared__ double sd[2 * MS_MAXS];
  __shared__ double sal[MS_MAXS], sbe[MS_MAXS];
  __shared__ int sup[MS_MAXS], sneg[MS_MAXS];
  __shared__ double red[4][16 * 16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t < 2 * s) sd[t] = red_in[t];   // [0, s): r . w, [s, 2s): r . r
  __syncthreads();
  if (t < s) {
    const double delta = sd[t], gamma = sd[s + t];
    const int act = cur.active[t];
    const bool upd = act && !(gamma <= rtol2 * sh.bn2[t]);
    const double be = (k == 0 || !act) ? 0.0 : gamma / cur.rr[t];
    const double den = be == 0.0 ? delta : delta - be * gamma / cur.a[t];
    sbe[t] = be;
    sal[t] = upd ? gamma / den : 0.0;
    sup[t] = upd ? 1 : 0;
    sneg[t] = upd && !(den > 0.0);
  }
  __syncthreads();
  const int neb = nb * s;
  if (blockIdx.x != 0) {
    // ---- vector blocks: s, r and the B^T r_{k+1} block rows ----
    const int vb = blockIdx.x - 1, nvb = gridDim.x - 1;
    const int c = lane & 15, rq = lane >> 4;
    const bool on = c < s, onb = c < nb;
    const double al = on ? sal[c] : 0.0, be = on ? sbe[c] : 0.0;
    const bool up = on && sup[c];
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    constexpr int RG = 4;   // 16 loads in flight per lane
    const int64_t stride = (int64_t)nvb * 16;
    for (int64_t base = (int64_t)vb * 16 + wv * 4; base < n; base += RG * stride) {
      double bv[RG], rv[RG], wv_[RG], sv[RG];
#pragma unroll
      for (int u = 0; u < RG; ++u) {
        const int64_t i = base + u * stride + rq;
        const bool v = on && i < n, w = onb && i < n;
        bv[u] = w ? B[i * nb + c] : 0.0;
        rv[u] = v ? R[i * s + c] : 0.0;
        wv_[u] = v ? W[i * s + c] : 0.0;
        sv[u] = v ? Sv[i * s + c] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < RG; ++u) {
        const int64_t i = base + u * stride + rq;
        double rn = rv[u];
        if (up && i < n) {
          const double sn = wv_[u] + be * sv[u];
          rn = rv[u] - al * sn;
          Sv[i * s + c] = sn;
          R[i * s + c] = rn;
        }
        acc = mfma64(bv[u], rn, acc);
      }
    }
    // C map: row (c') = rq + 4 j, column (c) = lane & 15
#pragma unroll
    for (int j = 0; j < 4; ++j) red[wv][(rq + 4 * j) * 16 + c] = acc[j];
    __syncthreads();
    for (int e = t; e < neb; e += 256) {
      const int cp = e / s, cc = e - cp * s;
      const int idx = cp * 16 + cc;
      bpart[(int64_t)e * nvb + vb] = (red[0][idx] + red[1][idx]) + (red[2][idx] + red[3][idx]);
    }
    return;
  }
  // ---- block 0: shift step k - 1 with B^T r_k = red_in[2s ..], the next state ----
  const double* brd = red_in + 2 * s;
  if (k >= 1)
    for (int task = t; task < S * s; task += blockDim.x) {
      const int j = task / s, c = task % s;
      if (!cur.active[c]) continue;   // step k - 1 not taken by this column
      const double z = sh.z[j * s + c];
      if (!(fabs(z) >= MS_ZETA_MIN)) continue;   // converged shift: G final
      double zn, as;
      ms_shift_step(cur, sh, dshift, s, j, c, zn, as);
      const double bs = sbe[c] * (zn / z) * (zn / z);
      double bpv[MS_MAXS], gv[MS_MAXS];
#pragma unroll
      for (int cp = 0; cp < MS_MAXS; ++cp) {
        const int e = (j * nb + cp) * s + c;
        bpv[cp] = cp < nb ? sh.bp[e] : 0.0;
        gv[cp] = cp < nb ? sh.g[e] : 0.0;
      }
#pragma unroll
      for (int cp = 0; cp < MS_MAXS; ++cp) {
        if (cp >= nb) break;
        const int e = (j * nb + cp) * s + c;
        sh.g[e] = gv[cp] + as * bpv[cp];
        sh.bp[e] = zn * brd[cp * s + c] + bs * bpv[cp];
      }
      sh.z_prev[j * s + c] = z;
      sh.z[j * s + c] = zn;
    }
  if (t < s) {
    const int act = cur.active[t];
    if (act) {
      nxt.rr[t] = sd[s + t];
      nxt.a[t] = sal[t];
      nxt.a_prev[t] = cur.a[t];
      nxt.beta[t] = sbe[t];
    } else {
      nxt.rr[t] = cur.rr[t];
      nxt.a[t] = cur.a[t];
      nxt.a_prev[t] = cur.a_prev[t];
      nxt.beta[t] = cur.beta[t];
    }
    nxt.active[t] = sup[t];
    if (sneg[t]) sh.flags[0] = 1;
  }
  __syncthreads();
  if (t == 0) {
    bool after = false;
    for (int c = 0; c < s; ++c) after = after || sup[c];
    if (!after && sh.it_stop[0] < 0) sh.it_stop[0] = k;   // the first all-stopped iteration
  }
  if (pin && t < s) {   // the batch's end state for the host (pinned, device-mapped)
    pin->rr[t] = cur.active[t] ? sd[s + t] : cur.rr[t];
    pin->act[t] = sup[t];
    if (t == 0) pin->flag = sh.flags[0];
  }
}

// The sums one iteration of ms_cg2_update_kernel needs, one workgroup per output
// element e: e < 2 s the SpMM's block partials of [r . w | r . r] ([2 s][rows_a]),
// else the previous update's block partials of B^T r ([ne_b][rows_b]); column-major,
// so element e's partials are contiguous. Thread t sums partials t, t + 256, ...
// (eight loads in flight), then the four waves in a fixed order.
__global__ __launch_bounds__(256) void ms_cg2_reduce_kernel(const double* __restrict__ pa,
                                                            int rows_a, int s,
                                                            const double* __restrict__ pb,
                                                            int rows_b, int ne_b,
                                                            double* __restrict__ out) {
  __shared__ double w4[4];
  const int e = blockIdx.x, t = threadIdx.x;
  const bool first = e < 2 * s;
  // column-major partials: element e's rows are contiguous (coalesced)
  const int rows = first ? rows_a : rows_b;
  const double* src = first ? pa + (int64_t)e * rows_a : pb + (int64_t)(e - 2 * s) * rows_b;
  (void)ne_b;
  double a = 0.0;
  int b = t;
  for (; b + 7 * 256 < rows; b += 8 * 256) {
    double x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = src[b + q * 256];
#pragma unroll
    for (int q = 0; q < 8; ++q) a += x[q];
  }
  for (; b < rows; b += 256) a += src[b];
  a = wave_sum(a);
  if ((t & 63) == 0) w4[t >> 6] = a;
  __syncthreads();
  if (t == 0) out[e] = (w4[0] + w4[1]) + (w4[2] + w4[3]);
}

// Group rows of x . y and x . x per column ([2s][gridDim.x]: x . y, then x . x) for
// SpMM kinds without the dot epilogue: MS_DOT_BLK blocks, each a contiguous range of
// rows, rows_per = 256 / s rows per block pass, summed in a fixed order.
__global__ __launch_bounds__(256) void ms_dots2_kernel(const double* __restrict__ X,
                                                       const double* __restrict__ Y, int64_t n,
                                                       int s, double* __restrict__ out) {
  __shared__ double red[2][256];
  const int t = threadIdx.x;
  const int rows_per = 256 / s;
  const int c = t % s, r = t / s;
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  double xy = 0.0, xx = 0.0;
  if (r < rows_per)
    for (int64_t i = lo + r; i < hi; i += rows_per) {
      const double x = X[i * s + c], y = Y[i * s + c];
      xy += x * y;
      xx += x * x;
    }
  red[0][t] = xy;
  red[1][t] = xx;
  __syncthreads();
  if (t < s) {
    double a = 0.0, b = 0.0;
    for (int q = 0; q < rows_per; ++q) {
      a += red[0][q * s + t];
      b += red[1][q * s + t];
    }
    out[(int64_t)t * gridDim.x + blockIdx.x] = a;
    out[(int64_t)(s + t) * gridDim.x + blockIdx.x] = b;
  }
}

// Initial scalar state from BR0 = B^T b (= b . p_0 for every shift) and ||b||^2:
// zeta = 1, G = 0, alpha_{-1} = 1 (a, a_prev), beta_{-1} = 0, active = ||b|| > 0.
__global__ void ms_init_kernel(MsScal st, MsShift sh, const double* __restrict__ partial,
                               int nblk, int S, int s, int nb, MsPin* __restrict__ pin2) {
  __shared__ double br[MS_MAXS * MS_MAXS + MS_MAXS];
  const int ne = nb * s + s;
  {
    const int nw = blockDim.x >> 6, wv = threadIdx.x >> 6;
    for (int e = wv; e < ne; e += nw) {
      const double v = wave_reduce_partials(partial, nblk, ne, e);
      if ((threadIdx.x & 63) == 0) br[e] = v;
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  const int j = t / s, c = t % s;
  if (j < S) {
    sh.z[j * s + c] = 1.0;
    sh.z_prev[j * s + c] = 1.0;
    for (int cp = 0; cp < nb; ++cp) {
      const int e = (j * nb + cp) * s + c;
      sh.bp[e] = br[cp * s + c];
      sh.g[e] = 0.0;
    }
  }
  if (t < s) {
    st.rr[t] = br[nb * s + t];
    sh.bn2[t] = br[nb * s + t];
    st.a[t] = 1.0;
    st.a_prev[t] = 1.0;
    st.beta[t] = 0.0;
    st.active[t] = br[nb * s + t] > 0.0 ? 1 : 0;
    pin2[0].bn2[t] = br[nb * s + t];   // the host's stop-rate targets, no readback
    pin2[1].bn2[t] = br[nb * s + t];
  }
  if (t == 0) {
    sh.flags[0] = 0;
    sh.it_stop[0] = -1;
  }
}

// The compaction (MsCompactArgs): blockIdx.y < njob gathers job y, dst[r][c'][v] =
// src[r][map[c']][v] (grid-stride over x); blockIdx.y == njob scatters the dropped
// columns' Grams, gfin[jc][drop_orig[d]] = g[jc][drop[d]], and gathers the new block's
// active flags.
__global__ __launch_bounds__(256) void ms_compact_kernel(MsCompactArgs A) {
  __shared__ int smap[MS_MAXS];
  const int y = blockIdx.y, t = threadIdx.x;
  if (y < A.njob) {
    if (t < A.a) smap[t] = A.map[t];
    __syncthreads();
    const MsCompactJob J = A.job[y];
    const int a = A.a, s = A.s, L = J.L;
    const int64_t total = J.rows * a * L;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + t; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
      const int64_t v = i % L, rc = i / L;
      const int c = (int)(rc % a);
      const int64_t r = rc / a;
      J.dst[i] = J.src[(r * s + smap[c]) * L + v];
    }
    return;
  }
  __shared__ int sdrop[MS_MAXS], sorig[MS_MAXS];
  if (t < A.nd) {
    sdrop[t] = A.drop[t];
    sorig[t] = A.drop_orig[t];
  }
  __syncthreads();
  const int64_t total = A.SN * A.nd;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + t; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t jc = i / A.nd;
    const int d = (int)(i - jc * A.nd);
    A.gfin[jc * A.s0 + sorig[d]] = A.g[jc * A.s + sdrop[d]];
  }
  if (blockIdx.x == 0 && t < A.a) A.act[t] = A.act_src[A.map[t]];
}

// dst[i][c] = src[perm[i]][c] for c < ns_src, 0 for the padding columns up to s
// (perm null: identity): a host block in the caller's row order into the device's
// locality order, on the device.
__global__ __launch_bounds__(256) void rows_gather_kernel(const double* __restrict__ src,
                                                          int ns_src, const int* __restrict__ perm,
                                                          int64_t n, int s,
                                                          double* __restrict__ dst) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * s) return;
  const int64_t i = e / s;
  const int c = (int)(e - i * s);
  const int64_t r = perm ? (int64_t)perm[i] : i;
  dst[e] = c < ns_src ? src[r * ns_src + c] : 0.0;
}

// Row r of the reordered CSR = row perm[r] of the original with every column j
// renamed inv[j] (entries kept in their original order): one wave per row.
__global__ __launch_bounds__(256) void csr_permute_kernel(
    const int64_t* __restrict__ ip, const int* __restrict__ ix, const double* __restrict__ dv,
    const int* __restrict__ perm, const int* __restrict__ inv, int64_t n,
    const int64_t* __restrict__ ip2, int* __restrict__ ix2, double* __restrict__ dv2) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int64_t i = perm[r];
  const int64_t k0 = ip[i], cnt = ip[i + 1] - k0, o = ip2[r];
  for (int64_t q = lane; q < cnt; q += 64) {
    ix2[o + q] = inv[ix[k0 + q]];
    dv2[o + q] = dv[k0 + q];
  }
}

// ---------------------------------------------------------------------------
// Dense operator of the Krylov methods (gpmi_sp_create_dense: 'slq' on a dense K):
// Yp[y] = K[rows, k-split y] X for s <= 16 * CT columns, fp64 MFMA 16x16x4.
// A workgroup owns 64 rows (wave w: rows 16 w .. 16 w + 15) and the k range of
// split y = blockIdx.y (kcs chunks of 64 columns). Per chunk each lane reads 16
// consecutive doubles of its row, K[r0 + (l & 15)][k0 + 16 (l >> 4) + m] (128 B
// per lane, the whole 16 x 64 block per wave), and MFMA m takes k = k0 +
// 16 (l >> 4) + m: a fixed permutation of the k order inside the chunk. The X
// chunk (64 x 16 CT, zero past n and s) is staged in LDS for the four waves,
// double-buffered, with the next chunk's K and X in registers.
// K must have ceil(n / 64) * 64 readable rows and columns (the dense operator's
// n_pad); the partials are summed by dense_mm_reduce_kernel in split order.
// HBM-bound: 8 n^2 bytes of K per launch.
// ---------------------------------------------------------------------------
template <int CT>
__global__ __launch_bounds__(256) void dense_mm_kernel(const double* __restrict__ K, int64_t ldk,
                                                       int64_t n, const double* __restrict__ X,
                                                       int s, int kcs,
                                                       double* __restrict__ Yp) {
  constexpr int XC = 16 * CT;
  constexpr int XU = XC / 4;   // X values per thread per chunk
  __shared__ double sx[2][64][XC + 1];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * 64 + w * 16;
  const int kq = lane >> 4, fr = lane & 15;
  const double* Kr = K + (r0 + fr) * ldk + 16 * kq;
  const int64_t nch = (n + 63) / 64;
  const int64_t c0 = (int64_t)blockIdx.y * kcs, c1 = c0 + kcs < nch ? c0 + kcs : nch;
  d4 acc[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) acc[ct] = d4{0.0, 0.0, 0.0, 0.0};
  // chunk c + 1's K and X are loaded into registers while chunk c computes (the
  // loads' latency, not the MFMA, bounds a chunk otherwise); X goes to the LDS
  // buffer of its parity, one barrier per chunk
  d2 kn[8];
  double xn[XU];
  auto load = [&](int64_t c) {
    const int64_t k0 = c * 64;
#pragma unroll
    for (int q = 0; q < 8; ++q) kn[q] = *reinterpret_cast<const d2*>(Kr + k0 + 2 * q);
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int e = u * 256 + t, kr = e / XC, col = e % XC;
      const int64_t k = k0 + kr;
      xn[u] = (k < n && col < s) ? X[k * s + col] : 0.0;
    }
  };
  if (c0 < c1) load(c0);
  int buf = 0;
  for (int64_t c = c0; c < c1; ++c) {
    d2 kv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) kv[q] = kn[q];
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int e = u * 256 + t;
      sx[buf][e / XC][e % XC] = xn[u];
    }
    __syncthreads();
    if (c + 1 < c1) load(c + 1);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const double a = kv[m >> 1][m & 1];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        acc[ct] = mfma64(a, sx[buf][16 * kq + m][16 * ct + fr], acc[ct]);
    }
    buf ^= 1;
  }
  double* out = Yp + (int64_t)blockIdx.y * n * s;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = r0 + kq + 4 * r;
      const int col = 16 * ct + fr;
      if (row < n && col < s) out[row * s + col] = acc[ct][r];
    }
}
template __global__ void dense_mm_kernel<1>(const double*, int64_t, int64_t, const double*, int,
                                            int, double*);
template __global__ void dense_mm_kernel<2>(const double*, int64_t, int64_t, const double*, int,
                                            int, double*);

// Y = sum_y Yp[y] (split order) + eta X, elementwise over [n][s].
__global__ __launch_bounds__(256) void dense_mm_reduce_kernel(const double* __restrict__ Yp,
                                                              int nsplit, int64_t ns,
                                                              const double* __restrict__ X,
                                                              double eta, double* __restrict__ Y) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= ns) return;
  double v = 0.0;
  for (int y = 0; y < nsplit; ++y) v += Yp[(int64_t)y * ns + e];
  Y[e] = v + eta * X[e];
}

}  // namespace gpmi
