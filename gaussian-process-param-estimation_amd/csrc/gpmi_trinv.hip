// Exact traces of inverse powers of K + eta I from its Cholesky factor:
//   tr(A^-1)      = ||L^-1||_F^2
//   tr(A^-2)      = ||A^-1||_F^2 = ||W W^T||_F^2,   W = L^-T
// Replaces the reference's exact traceinv (MixedCorrelation.traceinv,
// gaussian_proc/_mixed_correlation/mixed_correlation.py:155-215, which calls
// imate.traceinv(..., method='eigenvalue'|'cholesky')) without forming A^-1
// column by column.
//
// Y = L^-1 is built by a right-looking blocked triangular solve of L Y = I,
// stored transposed as W = Y^T (row-major, upper block triangle) so that both
// MFMA operands are always read as [row][k] slabs (the tile_mma of the
// factorization). Per block step k:
//   trinv_diag_kernel   : Y_kj = Linv_kk B_kj,  j <= k     (B_kk = I, so Y_kk = Linv_kk)
//   trinv_update_kernel : B_ij -= L_ik Y_kj,  i > k, j <= k  (first touch at k = j)
// blocked like the factorization: within an outer panel of S block columns only
// the panel's next row is updated before its diagonal step; the rows below get
// one update with K = S * 128 per panel.
// with ||Y_kj||_F^2 per tile written as a partial. For the squared Frobenius
// norm of A^-1 the lower tiles of T = W W^T are accumulated over k-panels
// (gram_panel_kernel) and squared-summed (gram_sumsq_kernel).
// All partials are reduced on the host in a fixed order (deterministic).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gpmi_internal.h"

#include "gpmi_device.h"

namespace gpmi {

namespace {

// sum of acc^2 over the wave tiles, reduced over the work-group through LDS.
__device__ __forceinline__ double block_sumsq(const d4 (&acc)[4][4], double* red) {
  double s = 0.0;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += acc[a][c][r] * acc[a][c][r];
  const int t = threadIdx.x;
  red[t] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h) red[t] += red[t + h];
    __syncthreads();
  }
  return red[0];
}

// Transposed tile store: acc element (row R, col C) -> T[C * ldt + R].
__device__ __forceinline__ void store_transposed(double* T, int64_t ldt, const d4 (&acc)[4][4]) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(int64_t)(wc * 64 + c * 16 + fr) * ldt + wr * 64 + a * 16 + fk + 4 * r] = acc[a][c][r];
}

}  // namespace

// Grid: k + 1 blocks (tile column j = blockIdx.x). W_jk <- (Linv_kk B_kj)^T where
// B_kj^T is held in W_jk (updates of earlier steps); W_kk <- Linv_kk^T.
__global__ __launch_bounds__(256, 2) void trinv_diag_kernel(const double* __restrict__ Linv,
                                                            double* W, int64_t ldw, int k,
                                                            double* partial) {
  __shared__ double smem[4 * STAGE];
  const int j = blockIdx.x, t = threadIdx.x;
  const double* Li = Linv + (int64_t)k * TS * TS;
  double* Wjk = W + (int64_t)j * TS * ldw + (int64_t)k * TS;
  if (j == k) {
    double s = 0.0;
    for (int e = t; e < TS * TS; e += 256) {
      const int r = e >> 7, c = e & 127;
      const double v = Li[r * TS + c];
      Wjk[(int64_t)c * ldw + r] = v;
      s += v * v;
    }
    smem[t] = s;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (t < h) smem[t] += smem[t + h];
      __syncthreads();
    }
    if (t == 0) partial[j] = smem[0];
    return;
  }
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = d4{0.0, 0.0, 0.0, 0.0};
  d4 dummy[2];
  // out[r][c] = sum_q Linv_kk[r][q] B_kj[q][c], B_kj[q][c] = W_jk[c][q]
  tile_mma<false>(Li, TS, Wjk, ldw, TS, smem, smem + 2 * STAGE, acc, nullptr, dummy);
  store_transposed(Wjk, ldw, acc);
  const double s = block_sumsq(acc, smem);
  if (t == 0) partial[j] = s;
}

// Grid: ni * nj blocks; tile (i, j), i = i0 + q / nj, j = q % nj, j < ke:
//   W_ji <- (B_ij - sum_{k in [max(kb, j), ke)} L_ik Y_kj)^T
// (Y_kj = 0 for k < j). B_ij is zero before its first update, which is the
// call whose k-range starts at j (j >= kb). One call per outer panel
// [kb, ke) for the rows below it, one per sub-step for the panel's own rows.
__global__ __launch_bounds__(256, 2) void trinv_update_kernel(const double* __restrict__ L,
                                                              int64_t lda, double* W,
                                                              int64_t ldw, int i0, int nj,
                                                              int kb, int ke) {
  __shared__ double smem[4 * STAGE];
  const int q = xcd_remap(blockIdx.x, gridDim.x);
  const int i = i0 + q / nj, j = q % nj;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  const int ks = j > kb ? j : kb;
  double* Wji = W + (int64_t)j * TS * ldw + (int64_t)i * TS;
  d4 acc[4][4];
  if (j < kb) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[a][c][r] = Wji[(int64_t)(wc * 64 + c * 16 + fr) * ldw + wr * 64 + a * 16 + fk + 4 * r];
  } else {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[a][c] = d4{0.0, 0.0, 0.0, 0.0};
  }
  d4 dummy[2];
  // acc -= sum_p L_i[r][p] Y_.j[p][c] over p in [ks*128, ke*128), Y[p][c] = W_j[c][p]
  tile_mma<false, true>(L + (int64_t)i * TS * lda + (int64_t)ks * TS, lda,
                        W + (int64_t)j * TS * ldw + (int64_t)ks * TS, ldw, (ke - ks) * TS, smem,
                        smem + 2 * STAGE, acc, nullptr, dummy);
  store_transposed(Wji, ldw, acc);
}

// T = W W^T (= A^-1, lower tiles) accumulated panel by panel, like the
// factorization's trailing update: for the k-panel [p0, p0 + kdim), every tile
// (I, J), J <= I < imax = (p0 + kdim) / 128, gets T_IJ += W_Ip W_Jp^T over
// p >= max(p0, I*128) (W_I. is zero left of its diagonal block). All WGs of a
// launch stream the same narrow column panel of W, so the operands stay in
// L2 / MALL, unlike a per-tile sweep over the full K range. Strictly-lower
// T_IJ lives in W's unused lower block triangle, diagonal T_II in Td.
__global__ __launch_bounds__(256, 2) void gram_panel_kernel(double* W, int64_t ldw,
                                                            double* Td, int p0, int kdim,
                                                            int imax) {
  __shared__ double smem[4 * STAGE];
  const int q = xcd_remap(blockIdx.x, gridDim.x);
  int I, J;
  tri_decode(q, imax, &I, &J);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  const int64_t ks = (int64_t)I * TS > p0 ? (int64_t)I * TS : p0;
  const int kd = (int)(p0 + kdim - ks);
  const bool first = ks == (int64_t)I * TS;   // this panel holds T_IJ's first term
  double* C;
  int64_t ldc;
  if (I == J) {
    C = Td + (int64_t)I * TS * TS;
    ldc = TS;
  } else {
    C = W + (int64_t)I * TS * ldw + (int64_t)J * TS;
    ldc = ldw;
  }
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[a][c][r] = first ? 0.0
                             : C[(int64_t)(wr * 64 + a * 16 + fk + 4 * r) * ldc + wc * 64 +
                                 c * 16 + fr];
  d4 dummy[2];
  tile_mma<false>(W + (int64_t)I * TS * ldw + ks, ldw, W + (int64_t)J * TS * ldw + ks, ldw, kd,
                  smem, smem + 2 * STAGE, acc, nullptr, dummy);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(int64_t)(wr * 64 + a * 16 + fk + 4 * r) * ldc + wc * 64 + c * 16 + fr] = acc[a][c][r];
}

// partial[I] = ||T_II||^2 + 2 sum_{J < I} ||T_IJ||^2 (one block per tile row).
__global__ __launch_bounds__(256) void gram_sumsq_kernel(const double* __restrict__ W,
                                                         int64_t ldw,
                                                         const double* __restrict__ Td,
                                                         double* partial) {
  __shared__ double red[256];
  const int I = blockIdx.x, t = threadIdx.x;
  double s = 0.0, d = 0.0;
  const double* row0 = W + (int64_t)I * TS * ldw;
  for (int r = 0; r < TS; ++r)
    for (int c = t; c < I * TS; c += 256) {
      const double v = row0[(int64_t)r * ldw + c];
      s += v * v;
    }
  const double* td = Td + (int64_t)I * TS * TS;
  for (int e = t; e < TS * TS; e += 256) d += td[e] * td[e];
  red[t] = 2.0 * s + d;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h) red[t] += red[t + h];
    __syncthreads();
  }
  if (t == 0) partial[I] = red[0];
}

}  // namespace gpmi
