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

namespace gpmi {

// ---------------------------------------------------------------------------
// 1/Gamma(1+mu) and 1/Gamma(1-mu) expansions for the Temme series.
// 1/Gamma(z) = sum_{k>=1} c_k z^k  (Abramowitz & Stegun 6.1.34), so
// 1/Gamma(1+mu) = sum_k c_k mu^(k-1). Then
//   g1 = (1/Gamma(1-mu) - 1/Gamma(1+mu)) / (2 mu) = -(c2 + c4 mu^2 + c6 mu^4 ...)
//   g2 = (1/Gamma(1-mu) + 1/Gamma(1+mu)) / 2     =  c1 + c3 mu^2 + c5 mu^4 ...
// which has no cancellation as mu -> 0.
// ---------------------------------------------------------------------------
__constant__ double kRGammaCoef[26] = {
    1.0000000000000000,  0.5772156649015329,  -0.6558780715202538,
    -0.0420026350340952, 0.1665386113822915,  -0.0421977345555443,
    -0.0096219715278770, 0.0072189432466630,  -0.0011651675918591,
    -0.0002152416741149, 0.0001280502823882,  -0.0000201348547807,
    -0.0000012504934821, 0.0000011330272320,  -0.0000002056338417,
    0.0000000061160950,  0.0000000050020075,  -0.0000000011812746,
    0.0000000001043427,  0.0000000000077823,  -0.0000000000036968,
    0.0000000000005100,  -0.0000000000000206, -0.0000000000000054,
    0.0000000000000014,  0.0000000000000001};

__device__ static void temme_gammas(double mu, double* g1, double* g2,
                                    double* gpl, double* gmi) {
  const double m2 = mu * mu;
  double odd = 0.0, even = 0.0, pw = 1.0;
  // c_{2i+1} mu^{2i} (odd k) and c_{2i+2} mu^{2i} (even k)
  for (int i = 0; i < 13; ++i) {
    odd += kRGammaCoef[2 * i] * pw;
    even += kRGammaCoef[2 * i + 1] * pw;
    pw *= m2;
  }
  *g2 = odd;            // (1/G(1-mu) + 1/G(1+mu))/2
  *g1 = -even;          // (1/G(1-mu) - 1/G(1+mu))/(2mu)
  *gpl = odd + mu * even;   // 1/Gamma(1+mu)
  *gmi = odd - mu * even;   // 1/Gamma(1-mu)
}

// Modified Bessel function of the second kind K_nu(x), x > 0, nu >= 0.
// Temme's series (x < 2) or Steed's continued fraction CF2 (x >= 2) for
// K_mu, K_{mu+1} with |mu| <= 1/2, then forward recurrence in the order.
__device__ double bessel_kv(double nu, double x) {
  const double EPS = 1.0e-16;
  const double PI = 3.141592653589793;
  const int nl = (int)floor(nu + 0.5);
  const double mu = nu - nl;
  const double mu2 = mu * mu;
  const double xi = 1.0 / x;
  const double xi2 = 2.0 * xi;
  double kmu, k1;
  if (x < 2.0) {
    const double x2 = 0.5 * x;
    const double pimu = PI * mu;
    const double fact = (fabs(pimu) < EPS) ? 1.0 : pimu / sin(pimu);
    double d = -log(x2);
    double e = mu * d;
    const double fact2 = (fabs(e) < EPS) ? 1.0 : sinh(e) / e;
    double g1, g2, gpl, gmi;
    temme_gammas(mu, &g1, &g2, &gpl, &gmi);
    double ff = fact * (g1 * cosh(e) + g2 * fact2 * d);
    double sum = ff;
    e = exp(e);
    double p = 0.5 * e / gpl;
    double q = 0.5 / (e * gmi);
    double c = 1.0;
    d = x2 * x2;
    double sum1 = p;
    for (int i = 1; i < 500; ++i) {
      ff = (i * ff + p + q) / (i * (double)i - mu2);
      c *= d / i;
      p /= (i - mu);
      q /= (i + mu);
      const double del = c * ff;
      sum += del;
      sum1 += c * (p - i * ff);
      if (fabs(del) < fabs(sum) * EPS) break;
    }
    kmu = sum;
    k1 = sum1 * xi2;
  } else {
    double b = 2.0 * (1.0 + x);
    double d = 1.0 / b;
    double h = d, delh = d;
    double q1 = 0.0, q2 = 1.0;
    const double a1 = 0.25 - mu2;
    double q = a1, c = a1;
    double a = -a1;
    double s = 1.0 + q * delh;
    for (int i = 1; i < 500; ++i) {
      a -= 2 * i;
      c = -a * c / (i + 1.0);
      const double qnew = (q1 - b * q2) / a;
      q1 = q2;
      q2 = qnew;
      q += c * qnew;
      b += 2.0;
      d = 1.0 / (b + a * d);
      delh = (b * d - 1.0) * delh;
      h += delh;
      const double dels = q * delh;
      s += dels;
      if (fabs(dels / s) < EPS) break;
    }
    h = a1 * h;
    kmu = sqrt(PI / (2.0 * x)) * exp(-x) / s;
    k1 = kmu * (mu + x + 0.5 - h) * xi;
  }
  for (int i = 1; i <= nl; ++i) {
    const double kt = (mu + i) * xi2 * k1 + kmu;
    kmu = k1;
    k1 = kt;
  }
  return kmu;
}

// Matérn correlation of a scaled distance x (_kernels.pyx:73-93).
__device__ __forceinline__ double matern_value(double x, const MaternParams& P) {
#pragma clang fp contract(off)
  if (x == 0.0) return 1.0;
  switch (P.mode) {
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
    case MATERN_GENERAL: {
      const double t = P.sqrt2nu * x;
      return P.prefactor * pow(t, P.nu) * bessel_kv(P.nu, t);
    }
    default:
      return exp(-0.5 * (x * x));
  }
}

// Scaled Euclidean distance, summed in dimension order (_kernels.pyx:130-136).
// Unrolled to GPMI_MAX_DIM so p_j stays in registers.
__device__ __forceinline__ double scaled_distance(const double* __restrict__ pi,
                                                  const double (&pj)[GPMI_MAX_DIM],
                                                  const double* __restrict__ scale,
                                                  int d) {
#pragma clang fp contract(off)
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < GPMI_MAX_DIM; ++k) {
    if (k < d) {
      const double v = (pi[k] - pj[k]) / scale[k];
      acc += v * v;
    }
  }
  return sqrt(acc);
}

// One workgroup = 16 rows x 256 columns of K. Thread t owns column j and keeps
// p_j in registers; row points are broadcast from LDS. Stores are 512-B
// coalesced row segments (8 B/lane). Entries with i >= n or j >= n get the
// identity pad.
__global__ __launch_bounds__(256) void matern_dense_kernel(
    const double* __restrict__ points, int64_t n, int d,
    const double* __restrict__ scale_dev, MaternParams P, double* __restrict__ K,
    int64_t ldk, int64_t n_pad) {
  __shared__ double srow[16 * GPMI_MAX_DIM];
  __shared__ double sscale[GPMI_MAX_DIM];
  const int t = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * 256 + t;
  const int64_t i0 = (int64_t)blockIdx.y * 16;
  if (t < d) sscale[t] = scale_dev[t];
  for (int e = t; e < 16 * d; e += 256) {
    const int64_t i = i0 + e / d;
    srow[e] = (i < n) ? points[i * d + (e % d)] : 0.0;
  }
  __syncthreads();
  double pj[GPMI_MAX_DIM];
#pragma unroll
  for (int k = 0; k < GPMI_MAX_DIM; ++k)
    pj[k] = (k < d && j < n) ? points[j * d + k] : 0.0;
  if (j >= n_pad) return;
  for (int r = 0; r < 16; ++r) {
    const int64_t i = i0 + r;
    if (i >= n_pad) break;
    double v;
    if (i < n && j < n) {
      v = matern_value(scaled_distance(&srow[r * d], pj, sscale, d), P);
    } else {
      v = (i == j) ? 1.0 : 0.0;
    }
    K[i * ldk + j] = v;
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
        const double v = (pi[k] - pj[k]) / scale[k];
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
