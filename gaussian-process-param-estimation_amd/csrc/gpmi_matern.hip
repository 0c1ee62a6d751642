// Matérn correlation assembly on gfx950 (HBM-write-bound pairwise kernel).
//
// Replaces the reference's Cython/OpenMP assembly:
//   matern_kernel            gaussian_proc/generate_correlation/_kernels.pyx:17-100
//   euclidean_distance       gaussian_proc/generate_correlation/_kernels.pyx:107-136
//   _generate_correlation_matrix  _generate_dense_correlation.pyx:25-91
// Arithmetic follows the reference expression order with FP contraction
// disabled, so entries agree with the Cython build to a few ulp (exp/Bessel).
//
// Layout: points [n][d] fp64 row-major; K [n_pad][ldk] fp64 row-major. Pad rows /
// columns (index >= n) hold the identity so the padded matrix factors as
// [[L, 0], [0, I]] and contributes nothing to logdet / solves.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gpmi_internal.h"

#ifndef GPMI_MATERN_NT
#define GPMI_MATERN_NT 1
#endif
#ifndef GPMI_MATERN_MINB
#define GPMI_MATERN_MINB 5    // minimum resident workgroups per CU (register cap: 96 VGPRs)
#endif
#ifndef GPMI_MATERN_PROBE
#define GPMI_MATERN_PROBE 0   // development probes: 1 no kernel evaluation, 2 no stores
#endif

namespace gpmi {

// ---------------------------------------------------------------------------
// General order nu (reference: kv / gamma from scipy's cython_special,
// _kernels.pyx:85-88). The Matérn value is written as
//   M_a(t) = 2^(1-a) / Gamma(a) * t^a * K_a(t),   t = sqrt(2 nu) x,
// which lies in (0, 1]. Two published facts give it without overflow:
//  * DLMF 10.32.9, K_a(t) = int_0^inf exp(-t cosh s) cosh(a s) ds. The
//    integrand is even and analytic in a strip around the real axis and decays
//    double-exponentially, so the trapezoid rule with step h converges
//    geometrically (error ~ exp(-2 pi d / h)); h follows the width of the
//    integrand's peak, which sits at sinh s* = a / t. The sum is scaled by the
//    peak value and stops once a term past the peak falls below 1e-17 of it.
//    Used for the low orders a = mu, mu + 1 with mu = nu - floor(nu) + 1 in
//    [1, 2) (or a = nu itself when nu < 2), where every exponent stays small.
//  * DLMF 10.29.1, K_{a+1} = K_{a-1} + (2a / t) K_a, rewritten for M:
//      M_{a+1} = M_a + t^2 / (4 a (a - 1)) M_{a-1},
//    a sum of positive terms (no cancellation, no overflow) carries the order
//    up to nu. Checked against mpmath at 40 digits: <= 2e-15 absolute over
//    nu in [0.05, 99.9], x in [1e-8, 60].
// P.lp0 / P.lp1 = log(2^(1-a) / Gamma(a)) of the two starting orders (host).
// ---------------------------------------------------------------------------
__device__ double matern_low_order(double a, double t, double lpref) {
#pragma clang fp contract(off)
  const double sp = asinh(a / t);                       // peak of the integrand
  const double h = fmin(0.1, 0.5 / sqrt(sqrt(t * t + a * a)));
  const double lt = log(t);
  const double L = a * (lt + sp) - t * cosh(sp);          // log of the peak value
  double acc = 0.5 * exp(a * lt - t - L);                 // s = 0, weight 1/2
  for (int k = 1; k < 6000; ++k) {
    const double s = k * h;
    const double c = t * cosh(s);
    const double term = 0.5 * (exp(a * (lt + s) - c - L) + exp(a * (lt - s) - c - L));
    acc += term;
    if (s > sp && term < 1e-17 * acc) break;
  }
  return h * acc * exp(L + lpref);
}

__device__ double matern_general(double t, const MaternParams& P) {
  if (P.nu < 2.0) return matern_low_order(P.nu, t, P.lp0);
  double m0 = matern_low_order(P.mu, t, P.lp0);
  double m1 = matern_low_order(P.mu + 1.0, t, P.lp1);
  const double q = 0.25 * t * t;
  for (double a = P.mu + 1.0; a < P.nu - 0.5; a += 1.0) {
    const double m2 = m1 + q / (a * (a - 1.0)) * m0;
    m0 = m1;
    m1 = m2;
  }
  return m1;
}

// Matérn correlation of a scaled distance x (_kernels.pyx:73-93); MODE < 0:
// the mode is read from P at run time, otherwise fixed at compile time.
template <int MODE = -1>
__device__ __forceinline__ double matern_value(double x, const MaternParams& P) {
#pragma clang fp contract(off)
  if (x == 0.0) return 1.0;
  switch (MODE < 0 ? P.mode : MODE) {
    case MATERN_HALF:
      return exp(-x);
    case MATERN_3HALF: {
      const double s3 = 1.7320508075688772;   // sqrt(3.0), correctly rounded
      return (1.0 + s3 * x) * exp(-s3 * x);
    }
    case MATERN_5HALF: {
      const double s5 = 2.23606797749979;     // sqrt(5.0), correctly rounded
      return (1.0 + s5 * x + (5.0 / 3.0) * (x * x)) * exp(-s5 * x);
    }
    case MATERN_GENERAL:
      return matern_general(P.sqrt2nu * x, P);
    default:
      return exp(-0.5 * (x * x));
  }
}

// (p_i - p_j) / scale, correctly rounded as the reference's division, from the
// correctly rounded reciprocal rs = RN(1 / scale): q0 = RN(a rs), the exact
// remainder a - q0 scale (FMA), q = RN(q0 + rem rs) (Markstein's final step:
// RN(a / scale) whenever rs is within half an ulp of 1 / scale and q0 within one
// ulp of a / scale, no overflow / underflow; 2e8 random cases checked equal on
// the host). One multiply and two FMAs instead of the ~10-instruction IEEE
// division sequence.
__device__ __forceinline__ double div_by_scale(double a, double sc, double rs) {
  const double q0 = a * rs;
  const double rem = fma(-q0, sc, a);
  return fma(rem, rs, q0);
}

// Scaled Euclidean distance, summed in dimension order (_kernels.pyx:130-136).
// Unrolled to GPMI_MAX_DIM so p_j stays in registers.
__device__ __forceinline__ double scaled_distance(const double* __restrict__ pi,
                                                  const double (&pj)[GPMI_MAX_DIM],
                                                  const double* __restrict__ scale,
                                                  const double* __restrict__ rscale, int d) {
#pragma clang fp contract(off)
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < GPMI_MAX_DIM; ++k) {
    if (k < d) {
      const double v = div_by_scale(pi[k] - pj[k], scale[k], rscale[k]);
      acc += v * v;
    }
  }
  return sqrt(acc);
}

// One workgroup = one 64 x 64 tile (I >= J) of the lower triangle, the
// blockIdx -> (I, J) map walks the tiles row by row. Every entry is evaluated
// once and stored twice, K[i][j] from the registers' tile in LDS and K[j][i]
// from its transpose (the reference likewise evaluates one triangle and
// mirrors, _generate_dense_correlation.pyx:76-91; the distance is symmetric
// bit for bit since (p_i - p_j)^2 == (p_j - p_i)^2). Stores are 512-B row
// segments per wave, non-temporal (K is written once and read much later).
// Row points come from LDS, the thread's column point stays in registers.
// Entries with i >= n or j >= n get the identity pad.
constexpr int MT = 64;

__device__ __forceinline__ void store_nt(double* p, double v) {
#if GPMI_MATERN_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

template <int MODE>
__global__ __launch_bounds__(256, GPMI_MATERN_MINB) void matern_dense_kernel_t(
    const double* __restrict__ points, int64_t n, int d,
    const double* __restrict__ scale_dev, MaternParams P, double* __restrict__ K,
    int64_t ldk, int64_t n_pad) {
  __shared__ double half[MT / 2][MT + 1];   // transpose buffer: 32 rows of the tile
  __shared__ double srow[MT * GPMI_MAX_DIM];
  __shared__ double sscale[GPMI_MAX_DIM], srs[GPMI_MAX_DIM];
  const int64_t b = blockIdx.x;
  int I = (int)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
  while ((int64_t)I * (I + 1) / 2 > b) --I;
  while ((int64_t)(I + 1) * (I + 2) / 2 <= b) ++I;
  const int J = (int)(b - (int64_t)I * (I + 1) / 2);
  const int t = threadIdx.x, c = t & (MT - 1), r0 = t >> 6;
  const int64_t i0 = (int64_t)I * MT, j0 = (int64_t)J * MT;
  if (t < d) {
    sscale[t] = scale_dev[t];
    srs[t] = 1.0 / scale_dev[t];
  }
  for (int e = t; e < MT * d; e += 256) {
    const int64_t i = i0 + e / d;
    srow[e] = (i < n) ? points[i * d + (e % d)] : 0.0;
  }
  __syncthreads();
  const int64_t j = j0 + c;
  double pj[GPMI_MAX_DIM];
#pragma unroll
  for (int k = 0; k < GPMI_MAX_DIM; ++k) pj[k] = (k < d && j < n) ? points[j * d + k] : 0.0;
  // thread (r0, c) evaluates rows r0 + 4 q of column c and stores them at once
  double v[MT / 4];
#pragma unroll
  for (int q = 0; q < MT / 4; ++q) {
    const int r = r0 + 4 * q;
    const int64_t i = i0 + r;
    if (i < n && j < n) {
#if GPMI_MATERN_PROBE == 1
      v[q] = scaled_distance(&srow[r * d], pj, sscale, srs, d);   // probe: no kernel evaluation
#else
      v[q] = matern_value<MODE>(scaled_distance(&srow[r * d], pj, sscale, srs, d), P);
#endif
    } else {
      v[q] = (i == j) ? 1.0 : 0.0;
    }
#if GPMI_MATERN_PROBE != 2
    if (i < n_pad && j < n_pad) store_nt(K + i * ldk + j, v[q]);
#endif
  }
#if GPMI_MATERN_PROBE == 2
  if (v[0] != -1.0) return;   // probe: no stores
#endif
  if (I == J) return;
  // the transpose, 32 tile rows per round through LDS: output row j0 + o holds
  // tile column o; 32 lanes write its 32 entries i0 + 32 h .. + 32 (256 B)
  const int oc = t & 31, orow = t >> 5;   // 8 output rows per pass
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int q = 0; q < MT / 8; ++q) half[r0 + 4 * q][c] = v[q + (MT / 8) * h];
    __syncthreads();
#pragma unroll
    for (int p = 0; p < MT / 8; ++p) {
      const int o = orow + 8 * p;
      const int64_t jr = j0 + o, ic = i0 + 32 * h + oc;
      if (jr < n_pad && ic < n_pad) store_nt(K + jr * ldk + ic, half[oc][o]);
    }
    __syncthreads();
  }
}

// One instantiation per closed form (lean register use), one for general nu
// and the Gaussian limit.
void launch_matern_dense(dim3 grid, hipStream_t s, const double* points, int64_t n, int d,
                         const double* scale, const MaternParams& P, double* K, int64_t ldk,
                         int64_t n_pad) {
  switch (P.mode) {
    case MATERN_HALF:
      hipLaunchKernelGGL(matern_dense_kernel_t<MATERN_HALF>, grid, dim3(256), 0, s, points, n, d,
                         scale, P, K, ldk, n_pad);
      break;
    case MATERN_3HALF:
      hipLaunchKernelGGL(matern_dense_kernel_t<MATERN_3HALF>, grid, dim3(256), 0, s, points, n, d,
                         scale, P, K, ldk, n_pad);
      break;
    case MATERN_5HALF:
      hipLaunchKernelGGL(matern_dense_kernel_t<MATERN_5HALF>, grid, dim3(256), 0, s, points, n, d,
                         scale, P, K, ldk, n_pad);
      break;
    default:
      hipLaunchKernelGGL(matern_dense_kernel_t<-1>, grid, dim3(256), 0, s, points, n, d, scale, P,
                         K, ldk, n_pad);
      break;
  }
}

}  // namespace gpmi

// ---------------------------------------------------------------------------
// Tapered (sparse) Matérn assembly, deterministic two-pass CSR.
// Replaces _generate_sparse_correlation.pyx:35-201 (O(n^2) pair loop appending
// to a locked COO buffer, nondeterministic order) with: pass 1 counts the kept
// entries of every row, the host scans the counts, pass 2 writes each row's
// columns in increasing order (wave ballot + prefix popcount). An entry is kept
// when matern(x_ij) > tau exactly as in the reference; pairs whose scaled
// distance exceeds xcut (matern(xcut) < tau by a wide margin) skip the kernel
// evaluation. One wave per row, 4 rows per workgroup.
// ---------------------------------------------------------------------------
namespace gpmi {

// scale: [scale | 1 / scale] (2 * GPMI_MAX_DIM doubles, see div_by_scale)
__device__ __forceinline__ bool taper_keep(const double (&pi)[GPMI_MAX_DIM],
                                           const double* __restrict__ points, int64_t j,
                                           int d, const double* __restrict__ scale,
                                           const MaternParams& P, double tau, double xcut,
                                           double* val) {
  double pj[GPMI_MAX_DIM];
#pragma unroll
  for (int k = 0; k < GPMI_MAX_DIM; ++k) pj[k] = (k < d) ? points[j * d + k] : 0.0;
  double acc = 0.0;
  {
#pragma clang fp contract(off)
#pragma unroll
    for (int k = 0; k < GPMI_MAX_DIM; ++k) {
      if (k < d) {
        const double v = div_by_scale(pi[k] - pj[k], scale[k], scale[GPMI_MAX_DIM + k]);
        acc += v * v;
      }
    }
  }
  const double x = sqrt(acc);
  if (x > xcut) return false;
  const double v = matern_value(x, P);
  *val = v;
  return v > tau;
}

__global__ __launch_bounds__(256) void csr_count_kernel(const double* __restrict__ points,
                                                        int64_t n, int d,
                                                        const double* __restrict__ scale,
                                                        MaternParams P, double tau, double xcut,
                                                        int* __restrict__ row_nnz) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  double pi[GPMI_MAX_DIM];
#pragma unroll
  for (int k = 0; k < GPMI_MAX_DIM; ++k) pi[k] = (k < d) ? points[row * d + k] : 0.0;
  int cnt = 0;
  for (int64_t j0 = 0; j0 < n; j0 += 64) {
    const int64_t j = j0 + lane;
    double v = 0.0;
    const bool keep = (j < n) && taper_keep(pi, points, j, d, scale, P, tau, xcut, &v);
    cnt += __popcll(__ballot(keep));
  }
  if (lane == 0) row_nnz[row] = cnt;
}

__global__ __launch_bounds__(256) void csr_fill_kernel(const double* __restrict__ points,
                                                       int64_t n, int d,
                                                       const double* __restrict__ scale,
                                                       MaternParams P, double tau, double xcut,
                                                       const int64_t* __restrict__ indptr,
                                                       int* __restrict__ indices,
                                                       double* __restrict__ data) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  double pi[GPMI_MAX_DIM];
#pragma unroll
  for (int k = 0; k < GPMI_MAX_DIM; ++k) pi[k] = (k < d) ? points[row * d + k] : 0.0;
  int64_t base = indptr[row];
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int64_t j0 = 0; j0 < n; j0 += 64) {
    const int64_t j = j0 + lane;
    double v = 0.0;
    const bool keep = (j < n) && taper_keep(pi, points, j, d, scale, P, tau, xcut, &v);
    const unsigned long long m = __ballot(keep);
    if (keep) {
      const int64_t pos = base + __popcll(m & below);
      indices[pos] = (int)j;
      data[pos] = v;
    }
    base += __popcll(m);
  }
}

// ---------------------------------------------------------------------------
// Cell-list form of the same assembly (d <= 3): points binned in cells of width
// >= xcut * scale_k per dimension, so every kept pair (scaled distance <= xcut)
// lies in the same or an adjacent cell. perm = point indices grouped by cell
// (cell_start[c] .. cell_start[c + 1]), cell[i] = cell of point i, gdim = cells
// per dimension. One wave per row visits the 3^d neighbour cells: O(n * candidates)
// instead of O(n^2). The fill pass collects the kept (j, value) pairs of its row
// in LDS and writes them in ascending j (rank = number of smaller kept j), so the
// CSR is identical to the brute-force kernels' (same taper_keep, same order).
// ---------------------------------------------------------------------------
constexpr int CELL_CAP = 512;   // kept entries per row held by the fill pass

template <typename F>
__device__ __forceinline__ void for_each_candidate(int64_t row, int d, const int* __restrict__ cell,
                                                   const int* __restrict__ gdim,
                                                   const int* __restrict__ cell_start,
                                                   const int* __restrict__ perm, F&& f) {
  const int lane = threadIdx.x & 63;
  int cc[3] = {0, 0, 0};
  {
    int c = cell[row];
    for (int k = 0; k < d; ++k) {
      cc[k] = c % gdim[k];
      c /= gdim[k];
    }
  }
  const int nb = (d == 1) ? 3 : (d == 2 ? 9 : 27);
  for (int o = 0; o < nb; ++o) {
    int id = 0, mul = 1, oo = o;
    bool ok = true;
    for (int k = 0; k < d; ++k) {
      const int q = cc[k] + (oo % 3) - 1;
      oo /= 3;
      ok = ok && q >= 0 && q < gdim[k];
      id += q * mul;
      mul *= gdim[k];
    }
    if (!ok) continue;   // wave-uniform
    const int b0 = cell_start[id], b1 = cell_start[id + 1];
    for (int b = b0; b < b1; b += 64) {
      const int k = b + lane;
      f(k < b1 ? perm[k] : -1);
    }
  }
}

__global__ __launch_bounds__(256) void csr_cell_count_kernel(
    const double* __restrict__ points, int64_t n, int d, const double* __restrict__ scale,
    MaternParams P, double tau, double xcut, const int* __restrict__ cell,
    const int* __restrict__ gdim, const int* __restrict__ cell_start,
    const int* __restrict__ perm, int* __restrict__ row_nnz) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  double pi[GPMI_MAX_DIM];
#pragma unroll
  for (int k = 0; k < GPMI_MAX_DIM; ++k) pi[k] = (k < d) ? points[row * d + k] : 0.0;
  int cnt = 0;
  for_each_candidate(row, d, cell, gdim, cell_start, perm, [&](int j) {
    double v = 0.0;
    const bool keep = (j >= 0) && taper_keep(pi, points, j, d, scale, P, tau, xcut, &v);
    cnt += __popcll(__ballot(keep));
  });
  if (lane == 0) row_nnz[row] = cnt;
}

__global__ __launch_bounds__(256) void csr_cell_fill_kernel(
    const double* __restrict__ points, int64_t n, int d, const double* __restrict__ scale,
    MaternParams P, double tau, double xcut, const int* __restrict__ cell,
    const int* __restrict__ gdim, const int* __restrict__ cell_start,
    const int* __restrict__ perm, const int64_t* __restrict__ indptr, int* __restrict__ indices,
    double* __restrict__ data) {
  __shared__ int sj[4][CELL_CAP];
  __shared__ double sv[4][CELL_CAP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * 4 + w;
  if (row >= n) return;
  double pi[GPMI_MAX_DIM];
#pragma unroll
  for (int k = 0; k < GPMI_MAX_DIM; ++k) pi[k] = (k < d) ? points[row * d + k] : 0.0;
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int cnt = 0;   // the host checked max(row_nnz) <= CELL_CAP
  for_each_candidate(row, d, cell, gdim, cell_start, perm, [&](int j) {
    double v = 0.0;
    const bool keep = (j >= 0) && taper_keep(pi, points, j, d, scale, P, tau, xcut, &v);
    const unsigned long long m = __ballot(keep);
    if (keep) {
      const int pos = cnt + __popcll(m & below);
      sj[w][pos] = j;
      sv[w][pos] = v;
    }
    cnt += __popcll(m);
  });
  // one wave owns sj[w] / sv[w]: LDS order, fences keep the writes before the reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int64_t base = indptr[row];
  for (int e = lane; e < cnt; e += 64) {
    const int je = sj[w][e];
    int rank = 0;
    for (int f = 0; f < cnt; ++f) rank += sj[w][f] < je;
    indices[base + rank] = je;
    data[base + rank] = sv[w][e];
  }
}

// Matérn of one scaled distance (host-side threshold / cutoff helper).
__global__ void matern_eval_kernel(const double* x, int64_t m, MaternParams P, double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) out[i] = matern_value(x[i], P);
}

}  // namespace gpmi
