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

}  // namespace gpmi
