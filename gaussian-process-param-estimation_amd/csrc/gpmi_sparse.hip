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

// Y[:, 0:s] = (K + eta I) X[:, 0:s]; one wave per row; lanes = (slot, column)
// with sp2 = next pow2 >= s columns and 64 / sp2 nonzero slots.
__global__ __launch_bounds__(256) void csr_spmm_kernel(const int64_t* __restrict__ indptr,
                                                       const int* __restrict__ indices,
                                                       const double* __restrict__ data,
                                                       int64_t n, const double* __restrict__ X,
                                                       int64_t ldx, double* __restrict__ Y,
                                                       int64_t ldy, int s, int sp2, double eta) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const int c = lane & (sp2 - 1);
  const int slot = lane / sp2;
  const int slots = 64 / sp2;
  const int64_t k0 = indptr[row], k1 = indptr[row + 1];
  double acc = 0.0;
  if (c < s)
    for (int64_t k = k0 + slot; k < k1; k += slots) acc += data[k] * X[(int64_t)indices[k] * ldx + c];
  for (int off = sp2; off < 64; off <<= 1) acc += __shfl_xor(acc, off);
  if (slot == 0 && c < s) Y[row * ldy + c] = acc + eta * X[row * ldx + c];
}

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

// out[j][c] = sum_b partial[b][j][c]   (one thread per (j, c), fixed order)
__global__ void col_dot_reduce_kernel(const double* __restrict__ partial, int nblk, int J, int s,
                                      double* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= J * s) return;
  double v = 0.0;
  for (int b = 0; b < nblk; ++b) v += partial[(int64_t)b * J * s + e];
  out[e] = v;
}

// W[i][c] = alpha * W[i][c] - sum_{j<J} A_j[i][c] * H[j][c]   (H on the device)
__global__ __launch_bounds__(256) void col_gs_update_kernel(double* __restrict__ W,
                                                            const double* __restrict__ A,
                                                            int64_t strideA,
                                                            const double* __restrict__ H, int J,
                                                            int64_t n, int s) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * s) return;
  const int c = (int)(e % s);
  double w = W[e];
  for (int j = 0; j < J; ++j) w -= A[j * strideA + e] * H[j * s + c];
  W[e] = w;
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

// Normalised Rademacher probes: V[i][c] = +-1/sqrt(n), bit 63 of
// splitmix64(seed * G + (c + c0) * H + i) (matches oracle/sparse.py).
__global__ __launch_bounds__(256) void rademacher_kernel(double* __restrict__ V, int64_t n, int s,
                                                         unsigned long long seed, int c0,
                                                         double scale) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * s) return;
  const int64_t i = e / s;
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
// partial[blk][e]: e = c' * s + c < s*s -> sum_i B[i][c'] R[i][c]; e = s*s + c -> R_c . R_c.
// Rows are staged through LDS 64 at a time; thread e (and e + 256) owns one output.
__global__ __launch_bounds__(256) void ms_dots_partial_kernel(const double* __restrict__ B,
                                                              const double* __restrict__ R,
                                                              int64_t n, int s,
                                                              double* __restrict__ partial) {
  __shared__ double sB[64 * MS_MAXS], sR[64 * MS_MAXS];
  const int t = threadIdx.x;
  const int ne = s * s + s;
  double acc0 = 0.0, acc1 = 0.0;
  for (int64_t r0 = (int64_t)blockIdx.x * 64; r0 < n; r0 += (int64_t)gridDim.x * 64) {
    const int rows = (int)((n - r0) < 64 ? (n - r0) : 64);
    for (int e = t; e < rows * s; e += 256) {
      sB[e] = B[r0 * s + e];
      sR[e] = R[r0 * s + e];
    }
    __syncthreads();
    for (int h = 0; h < 2; ++h) {
      const int e = t + h * 256;
      if (e < ne) {
        const double* X = e < s * s ? sB : sR;
        const int cx = e < s * s ? e / s : e - s * s;
        const int cy = e < s * s ? e % s : e - s * s;
        double v = 0.0;
        for (int r = 0; r < rows; ++r) v += X[r * s + cx] * sR[r * s + cy];
        if (h == 0) acc0 += v;
        else acc1 += v;
      }
    }
    __syncthreads();
  }
  if (t < ne) partial[(int64_t)blockIdx.x * ne + t] = acc0;
  if (t + 256 < ne) partial[(int64_t)blockIdx.x * ne + t + 256] = acc1;
}

// Scalar step 1 (one thread per column): alpha_c = rr_c / (p_c . A p_c).
__global__ void ms_alpha_kernel(MsState st, const double* __restrict__ pq, int s) {
  const int c = threadIdx.x;
  if (c >= s) return;
  st.a[c] = st.active[c] ? st.rr[c] / pq[c] : 0.0;
}

// r[i][c] -= a[c] q[i][c]
__global__ __launch_bounds__(256) void ms_r_update_kernel(double* __restrict__ R,
                                                          const double* __restrict__ Q,
                                                          const double* __restrict__ a,
                                                          int64_t n, int s) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * s) return;
  R[e] -= a[(int)(e % s)] * Q[e];
}

// Scalar step 2 (thread (j, c), j < S shifts): with BR = B^T r_new and rr_new
// reduced from the partials (fixed order), advance zeta, accumulate G, update
// b^T p and the base beta; a column stops when sqrt(rr) <= rtol ||b||.
__global__ void ms_scalar_kernel(MsState st, const double* __restrict__ partial, int nblk,
                                 const double* __restrict__ dshift, int S, int s, double rtol2,
                                 double* __restrict__ beta_out) {
  __shared__ double br[MS_MAXS * MS_MAXS + MS_MAXS];
  const int ne = s * s + s;
  for (int e = threadIdx.x; e < ne; e += blockDim.x) {
    double v = 0.0;
    for (int b = 0; b < nblk; ++b) v += partial[(int64_t)b * ne + e];
    br[e] = v;
  }
  __syncthreads();
  const int t = threadIdx.x;
  const int j = t / s, c = t % s;
  if (j < S && st.active[c]) {
    const double a = st.a[c], ap = st.a_prev[c], bo = st.beta[c];
    const double z = st.z[j * s + c], zp = st.z_prev[j * s + c];
    const double d = dshift[j];
    const double zn = z * zp * ap / (a * bo * (zp - z) + zp * ap * (1.0 + d * a));
    const double as = a * zn / z;
    const double rrn = br[s * s + c];
    const double bnew = rrn / st.rr[c];
    const double bs = bnew * (zn / z) * (zn / z);
    for (int cp = 0; cp < s; ++cp) {
      const int e = (j * s + cp) * s + c;
      const double bpv = st.bp[e];
      st.g[e] += as * bpv;
      st.bp[e] = zn * br[cp * s + c] + bs * bpv;
    }
    st.z_prev[j * s + c] = z;
    st.z[j * s + c] = zn;
  }
  __syncthreads();
  if (t < s && st.active[t]) {
    const double rrn = br[s * s + t];
    const double bnew = rrn / st.rr[t];
    st.a_prev[t] = st.a[t];
    st.beta[t] = bnew;
    beta_out[t] = bnew;
    st.rr[t] = rrn;
    if (rrn <= rtol2 * st.bn2[t]) st.active[t] = 0;
  }
}

// p[i][c] = r[i][c] + beta[c] p[i][c] for active columns
__global__ __launch_bounds__(256) void ms_p_update_kernel(double* __restrict__ P,
                                                          const double* __restrict__ R,
                                                          const double* __restrict__ beta,
                                                          const int* __restrict__ active,
                                                          int64_t n, int s) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * s) return;
  const int c = (int)(e % s);
  if (active[c]) P[e] = R[e] + beta[c] * P[e];
}

// Initial scalar state from BR0 = B^T b (= b . p_0 for every shift) and ||b||^2.
__global__ void ms_init_kernel(MsState st, const double* __restrict__ partial, int nblk, int S,
                               int s) {
  __shared__ double br[MS_MAXS * MS_MAXS + MS_MAXS];
  const int ne = s * s + s;
  for (int e = threadIdx.x; e < ne; e += blockDim.x) {
    double v = 0.0;
    for (int b = 0; b < nblk; ++b) v += partial[(int64_t)b * ne + e];
    br[e] = v;
  }
  __syncthreads();
  const int t = threadIdx.x;
  const int j = t / s, c = t % s;
  if (j < S) {
    st.z[j * s + c] = 1.0;
    st.z_prev[j * s + c] = 1.0;
    for (int cp = 0; cp < s; ++cp) {
      const int e = (j * s + cp) * s + c;
      st.bp[e] = br[cp * s + c];
      st.g[e] = 0.0;
    }
  }
  if (t < s) {
    st.rr[t] = br[s * s + t];
    st.bn2[t] = br[s * s + t];
    st.a[t] = 0.0;
    st.a_prev[t] = 1.0;
    st.beta[t] = 0.0;
    st.active[t] = br[s * s + t] > 0.0 ? 1 : 0;
  }
}

}  // namespace gpmi
