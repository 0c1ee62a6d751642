// 128 x 128 fp64 MFMA tile products shared by the band-reduction kernels
// (gpmi_band.hip) and the CholeskyQR panel (gpmi_cholqr.hip). One 256-thread
// workgroup per output tile: 4 waves, each a 64 x 64 wave tile of
// v_mfma_f64_16x16x4f64.
#pragma once

#include "gpmi_device.h"
#include "gpmi_band.h"

namespace gpmi {

// ---------------------------------------------------------------------------
// Generic 128 x 128 tile product on fp64 MFMA with either operand layout:
//   KFAST: op(P)[r][k] = P[r * ld + k]   (staged as the swizzled [row][16] slab)
//   KSLOW: op(P)[r][k] = P[k * ld + r]   (staged as [16][SLD], k-major; the
//          fragment reads of lanes 0-15 and 16-31 land 32 banks apart)
// acc (wave tile 64 x 64 at (wr, wc)) (+|-)= op(P1)[0:128, 0:kdim] op(P2)[0:128, 0:kdim]^T.
// Ends with a workgroup barrier (back-to-back calls may reuse smem).
// ---------------------------------------------------------------------------
constexpr int SLD = 144;
constexpr int GSTAGE = 16 * SLD;   // doubles per staged operand (>= STAGE)

template <int L>
__device__ __forceinline__ void gl_op(const double* __restrict__ base, int64_t ld, int k0,
                                      d2 (&r)[4]) {
  if (L == KFAST) {
    gload_slab(base, ld, k0, r);
    return;
  }
  const int t = threadIdx.x, kk = t >> 4, c0 = (t & 15) * 8;
  const double* p = base + (int64_t)(k0 + kk) * ld + c0;
#pragma unroll
  for (int q = 0; q < 4; ++q) r[q] = *reinterpret_cast<const d2*>(p + 2 * q);
}

template <int L>
__device__ __forceinline__ void st_op(double* s, const d2 (&r)[4]) {
  if (L == KFAST) {
    sstore_slab(s, r);
    return;
  }
  const int t = threadIdx.x, kk = t >> 4, c0 = (t & 15) * 8;
#pragma unroll
  for (int q = 0; q < 4; ++q) *reinterpret_cast<d2*>(s + kk * SLD + c0 + 2 * q) = r[q];
}

template <int L>
__device__ __forceinline__ double fr_op(const double* s, int row, int k) {
  return L == KFAST ? s[slab_off(row, k)] : s[k * SLD + row];
}

template <int AL, int BL, bool NEG>
__device__ __forceinline__ void gemm_tile(const double* __restrict__ P1, int64_t ld1,
                                          const double* __restrict__ P2, int64_t ld2, int kdim,
                                          double* smem, d4 (&acc)[4][4]) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  double* sA = smem;
  double* sB = smem + 2 * GSTAGE;
  d2 ra[4], rb[4];
  gl_op<AL>(P1, ld1, 0, ra);
  gl_op<BL>(P2, ld2, 0, rb);
  st_op<AL>(sA, ra);
  st_op<BL>(sB, rb);
  __syncthreads();
  // Drain every global load issued before the loop (a caller's accumulator preload,
  // load_tile) once, here: otherwise the waitcnt pass puts vmcnt waits on the first
  // accumulator uses INSIDE the loop, which (vmcnt counts in order) also drain the
  // next stage's prefetch every iteration (the dense tile_mma does the same).
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
  const int nsteps = kdim / BK;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const double* cA = sA + cur * GSTAGE;
    const double* cB = sB + cur * GSTAGE;
    if (s + 1 < nsteps) {
      gl_op<AL>(P1, ld1, (s + 1) * BK, ra);
      gl_op<BL>(P2, ld2, (s + 1) * BK, rb);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = fr_op<AL>(cA, wr * 64 + i * 16 + fr, kk * 4 + fk);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = fr_op<BL>(cB, wc * 64 + j * 16 + fr, kk * 4 + fk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = NEG ? mfma64_neg(a[i], b[j], acc[i][j]) : mfma64(a[i], b[j], acc[i][j]);
    }
    if (s + 1 < nsteps) {
      st_op<AL>(sA + (cur ^ 1) * GSTAGE, ra);
      st_op<BL>(sB + (cur ^ 1) * GSTAGE, rb);
    }
    __syncthreads();
  }
}

// One 64 x 64 quadrant (qr, qc) of the 128 x 128 product above: the same staging
// (both 128-row slabs, so the operand layouts and swizzles are shared), each wave a
// 32 x 32 piece (wave w: rows qr*64 + (w>>1)*32, columns qc*64 + (w&1)*32). Four
// workgroups then cover one output tile with a quarter of the MFMA chain each: the
// band's serial 128^3 steps (X T, V^T X, T^T M, X - V Zh, the tile-column update)
// are latency-bound single products per tile, ~4x shorter this way.
template <int AL, int BL, bool NEG>
__device__ __forceinline__ void gemm_quad(const double* __restrict__ P1, int64_t ld1,
                                          const double* __restrict__ P2, int64_t ld2, int kdim,
                                          double* smem, d4 (&acc)[2][2], int qr, int qc) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int r0 = qr * 64 + (w >> 1) * 32, c0 = qc * 64 + (w & 1) * 32;
  const int fr = lane & 15, fk = lane >> 4;
  double* sA = smem;
  double* sB = smem + 2 * GSTAGE;
  d2 ra[4], rb[4];
  gl_op<AL>(P1, ld1, 0, ra);
  gl_op<BL>(P2, ld2, 0, rb);
  st_op<AL>(sA, ra);
  st_op<BL>(sB, rb);
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): as gemm_tile
  const int nsteps = kdim / BK;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const double* cA = sA + cur * GSTAGE;
    const double* cB = sB + cur * GSTAGE;
    if (s + 1 < nsteps) {
      gl_op<AL>(P1, ld1, (s + 1) * BK, ra);
      gl_op<BL>(P2, ld2, (s + 1) * BK, rb);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = fr_op<AL>(cA, r0 + i * 16 + fr, kk * 4 + fk);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = fr_op<BL>(cB, c0 + j * 16 + fr, kk * 4 + fk);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = NEG ? mfma64_neg(a[i], b[j], acc[i][j]) : mfma64(a[i], b[j], acc[i][j]);
    }
    if (s + 1 < nsteps) {
      st_op<AL>(sA + (cur ^ 1) * GSTAGE, ra);
      st_op<BL>(sB + (cur ^ 1) * GSTAGE, rb);
    }
    __syncthreads();
  }
}

__device__ __forceinline__ void zero_quad(d4 (&acc)[2][2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
}

// C points at the 128 x 128 tile; the quadrant's wave pieces as in gemm_quad.
__device__ __forceinline__ void load_quad(const double* C, int64_t ldc, d4 (&acc)[2][2], int qr,
                                          int qc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = qr * 64 + (w >> 1) * 32, c0 = qc * 64 + (w & 1) * 32;
  const int fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[a][c][r] = C[(int64_t)(r0 + a * 16 + fk + 4 * r) * ldc + c0 + c * 16 + fr];
}

__device__ __forceinline__ void store_quad(double* C, int64_t ldc, const d4 (&acc)[2][2],
                                           double scale, int qr, int qc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = qr * 64 + (w >> 1) * 32, c0 = qc * 64 + (w & 1) * 32;
  const int fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(int64_t)(r0 + a * 16 + fk + 4 * r) * ldc + c0 + c * 16 + fr] = scale * acc[a][c][r];
}

__device__ __forceinline__ void zero_tile(d4 (&acc)[4][4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
}

// C/D map of v_mfma_f64_16x16x4f64: row = (lane>>4) + 4 r, col = lane & 15.
__device__ __forceinline__ void load_tile(const double* C, int64_t ldc, d4 (&acc)[4][4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[a][c][r] = C[(int64_t)(wr * 64 + a * 16 + fk + 4 * r) * ldc + wc * 64 + c * 16 + fr];
}

__device__ __forceinline__ void store_tile(double* C, int64_t ldc, const d4 (&acc)[4][4],
                                           double scale) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(int64_t)(wr * 64 + a * 16 + fk + 4 * r) * ldc + wc * 64 + c * 16 + fr] =
            scale * acc[a][c][r];
}

}  // namespace gpmi
