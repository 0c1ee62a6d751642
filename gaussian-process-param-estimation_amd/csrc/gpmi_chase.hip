// Eigenvalues of the band form B (bandwidth b = 128, gpmi_band.hip): band ->
// tridiagonal by bulge chasing, then bisection on Sturm counts.
//
// Completes the device form of the reference's eigenvalue operator
// (MixedCorrelation with imate_method='eigenvalue': eigh(K) once,
// mixed_correlation.py:76-79, then trace / traceinv / logdet of K + eta I as
// sums over (lambda_i + eta), :127-133, :172-181, :239-248). Only the
// eigenvalues are needed, so no stage-2 reflector is stored.
//
// chase_task_kernel: one workgroup per task (s, k) of wavefront t = 3 s + k
// (verified order-independent within a wavefront, tools/chase_proto.py). Sweep s
// annihilates column s below the subdiagonal; task k works on the row block
// J_k = [s + 1 + k b, s + 1 + (k + 1) b):
//   reflector H (LAPACK dlarfg) from A[J_0, s] (k = 0) or from the first column
//   c = s + 1 + (k - 1) b of the bulge block F = A[J_k, J_{k-1}] (k >= 1);
//   F <- H F, D = A[J_k, J_k] <- H D H (symmetric rank-2 form on the lower
//   triangle, D staged whole in LDS), E = A[J_{k+1}, J_k] <- E H.
// The matrix is a dense n_pad x n_pad lower-triangle copy of B; every access is
// within 2b of the diagonal.
//
// bisect_kernel: thread i finds the i-th smallest eigenvalue of the symmetric
// tridiagonal (d, e) by bisection on the Sturm count (LDL^T pivots of T - x I,
// pivmin safeguard as LAPACK dstebz), Gershgorin start interval.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gpmi_internal.h"
#include "gpmi_band.h"

namespace gpmi {

constexpr int CB = GPMI_TS;        // band width of B = 128
constexpr int CLD = CB + 1;        // LDS row stride of the staged diagonal block

__device__ __forceinline__ double block_sum(double v, double* red) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void chase_task_kernel(double* __restrict__ A, int64_t lda,
                                                         int n, int t, int s_hi) {
  __shared__ double D[CB * CLD];
  __shared__ double sv[CB];
  __shared__ double sw[CB];
  __shared__ double sp[2][CB];
  __shared__ double red[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int s = s_hi - (int)blockIdx.x;
  const int k = t - 3 * s;
  if (s < 0 || k < 0) return;
  const int r0 = s + 1 + k * CB;
  if (r0 >= n) return;
  const int r1 = min(r0 + CB, n), L = r1 - r0;
  const int col = (k == 0) ? s : s + 1 + (k - 1) * CB;
  // ---- reflector from x = A[r0:r1, col]
  __shared__ double sx0;
  const double xi = (tid < L) ? A[(int64_t)(r0 + tid) * lda + col] : 0.0;
  if (tid == 0) sx0 = xi;
  const double nb2 = block_sum((tid > 0 && tid < L) ? xi * xi : 0.0, red);
  const double xx0 = sx0;
  double tau = 0.0, beta = xx0, scale = 0.0;
  if (nb2 > 0.0) {
    const double nrm = sqrt(xx0 * xx0 + nb2);
    beta = xx0 >= 0.0 ? -nrm : nrm;
    tau = (beta - xx0) / beta;
    scale = 1.0 / (xx0 - beta);
  }
  if (tid < CB) sv[tid] = (tid == 0) ? 1.0 : ((tid < L) ? xi * scale : 0.0);
  __syncthreads();
  // ---- the annihilated column
  if (k == 0) {
    if (tid < L) A[(int64_t)(r0 + tid) * lda + s] = (tid == 0) ? beta : 0.0;
  }
  if (tau == 0.0) return;   // identity reflector: nothing else changes
  // ---- F <- H F, F = A[r0:r1, col:col + CB] (k >= 1)
  if (k >= 1) {
    const int c = tid & 127, h = tid >> 7;
    double acc = 0.0;
    for (int i = h; i < L; i += 2) acc += sv[i] * A[(int64_t)(r0 + i) * lda + col + c];
    sp[h][c] = acc;
    __syncthreads();
    if (tid < CB) sw[tid] = tau * (sp[0][tid] + sp[1][tid]);
    __syncthreads();
    for (int i = h; i < L; i += 2) {
      double* p = A + (int64_t)(r0 + i) * lda + col + c;
      if (c == 0) *p = (i == 0) ? beta : 0.0;
      else *p -= sv[i] * sw[c];
    }
  }
  // ---- D <- H D H on the lower triangle of A[r0:r1, r0:r1], staged symmetric in LDS
  for (int e = tid; e < L * CB; e += 256) {
    const int i = e >> 7, j = e & 127;
    if (j <= i) {
      const double v = A[(int64_t)(r0 + i) * lda + r0 + j];
      D[i * CLD + j] = v;
      D[j * CLD + i] = v;
    }
  }
  __syncthreads();
  {
    // p = tau D v (thread pair per row)
    const int i = tid & 127, h = tid >> 7;
    double acc = 0.0;
    if (i < L)
      for (int j = h; j < L; j += 2) acc += D[i * CLD + j] * sv[j];
    sp[h][i] = acc;
  }
  __syncthreads();
  const double pi = (tid < L) ? tau * (sp[0][tid] + sp[1][tid]) : 0.0;
  const double vp = block_sum((tid < L) ? pi * sv[tid] : 0.0, red);
  if (tid < CB) sw[tid] = (tid < L) ? pi - 0.5 * tau * vp * sv[tid] : 0.0;
  __syncthreads();
  for (int e = tid; e < L * CB; e += 256) {
    const int i = e >> 7, j = e & 127;
    if (j <= i)
      A[(int64_t)(r0 + i) * lda + r0 + j] = D[i * CLD + j] - sv[i] * sw[j] - sw[i] * sv[j];
  }
  // ---- E <- E H, E = A[r1:e1, r0:r1]
  const int e1 = min(r1 + CB, n);
  for (int i = r1 + wv; i < e1; i += 4) {
    double* row = A + (int64_t)i * lda + r0;
    const double a0 = (lane < L) ? row[lane] : 0.0;
    const double a1 = (lane + 64 < L) ? row[lane + 64] : 0.0;
    double q = a0 * sv[lane] + a1 * sv[lane + 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off);
    q *= tau;
    if (lane < L) row[lane] = a0 - q * sv[lane];
    if (lane + 64 < L) row[lane + 64] = a1 - q * sv[lane + 64];
  }
}

// Copy of the band for the chase: B's lower band (0 <= i - j <= 128) of the
// reduced matrix, zero for 128 < i - j <= 2 * 128 + 1 (the bulge envelope; the
// reduced matrix keeps Householder vectors there). Row i per workgroup.
__global__ __launch_bounds__(256) void chase_copy_kernel(const double* __restrict__ Ab,
                                                         double* __restrict__ A, int64_t lda,
                                                         int n) {
  const int i = blockIdx.x;
  const int j0 = max(0, i - 2 * CB - 1);
  for (int j = j0 + threadIdx.x; j <= i; j += 256)
    A[(int64_t)i * lda + j] = (i - j <= CB) ? Ab[(int64_t)i * lda + j] : 0.0;
}

// d[i] = A[i][i], e2[i] = A[i+1][i]^2 (the tridiagonal after the chase)
__global__ __launch_bounds__(256) void tridiag_extract_kernel(const double* __restrict__ A,
                                                              int64_t lda, int n,
                                                              double* __restrict__ d,
                                                              double* __restrict__ e2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  d[i] = A[(int64_t)i * lda + i];
  const double e = (i + 1 < n) ? A[(int64_t)(i + 1) * lda + i] : 0.0;
  e2[i] = e * e;
}

// number of eigenvalues of the tridiagonal below x (Sturm count, dstebz pivmin)
__device__ __forceinline__ int sturm_count(const double* __restrict__ d,
                                           const double* __restrict__ e2, int n, double x,
                                           double pivmin) {
  int cnt = 0;
  double q = d[0] - x;
  if (fabs(q) < pivmin) q = -pivmin;
  cnt += q < 0.0;
  for (int j = 1; j < n; ++j) {
    q = d[j] - x - e2[j - 1] / q;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
  }
  return cnt;
}

// thread i: the i-th smallest eigenvalue, bisection on [lo, hi] to ~2 ulp of
// max(|lo|, |hi|) (the interval width halves each step; at most 96 steps).
__global__ __launch_bounds__(256) void bisect_kernel(const double* __restrict__ d,
                                                     const double* __restrict__ e2, int n,
                                                     double lo0, double hi0, double pivmin,
                                                     double* __restrict__ lam) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double lo = lo0, hi = hi0;
  const double tol = 2.0 * 2.220446049250313e-16 * fmax(fabs(lo0), fabs(hi0)) + pivmin;
  for (int it = 0; it < 96 && hi - lo > tol; ++it) {
    const double mid = 0.5 * (lo + hi);
    if (sturm_count(d, e2, n, mid, pivmin) > i) hi = mid;
    else lo = mid;
  }
  lam[i] = 0.5 * (lo + hi);
}

}  // namespace gpmi
