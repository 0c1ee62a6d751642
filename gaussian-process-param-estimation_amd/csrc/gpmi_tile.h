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

// gemm_tile<AL, BL, NEG> with both operands' layouts chosen at run time (a_slow /
// b_slow, uniform: KSLOW, else KFAST), leading dimensions 128: every layout is staged
// k-major ([16][SLD], a KFAST operand by a transposing LDS store), so one MFMA loop
// serves all four. For kernels whose products mix layouts (in a rolled loop, or in
// different workgroup roles of one launch): one inlined product instead of one per
// layout pair (two or three in one kernel spilled 92-136 VGPRs). The MFMA sequence
// per output element is gemm_tile's: the same results.
__device__ __forceinline__ void rt_load(const double* __restrict__ P, bool slow, int k0,
                                        d2 (&r)[4]) {
  if (slow) {
    gl_op<KSLOW>(P, TS, k0, r);
    return;
  }
  const int t = threadIdx.x;
  const double* p = P + (int64_t)(t >> 1) * TS + k0 + (t & 1) * 8;
#pragma unroll
  for (int q = 0; q < 4; ++q) r[q] = *reinterpret_cast<const d2*>(p + 2 * q);
}

__device__ __forceinline__ void rt_store(double* s, bool slow, const d2 (&r)[4]) {
  if (slow) {
    st_op<KSLOW>(s, r);
    return;
  }
  const int t = threadIdx.x, row = t >> 1, kc = (t & 1) * 8;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    s[(kc + 2 * q) * SLD + row] = r[q][0];
    s[(kc + 2 * q + 1) * SLD + row] = r[q][1];
  }
}

template <bool NEG>
__device__ __forceinline__ void gemm_tile_rr(const double* __restrict__ P1, bool a_slow,
                                             const double* __restrict__ P2, bool b_slow,
                                             double* smem, d4 (&acc)[4][4]) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  double* sA = smem;
  double* sB = smem + 2 * GSTAGE;
  d2 ra[4], rb[4];
  rt_load(P1, a_slow, 0, ra);
  rt_load(P2, b_slow, 0, rb);
  rt_store(sA, a_slow, ra);
  rt_store(sB, b_slow, rb);
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15), as gemm_tile
  constexpr int nsteps = TS / BK;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const double* cA = sA + cur * GSTAGE;
    const double* cB = sB + cur * GSTAGE;
    if (s + 1 < nsteps) {
      rt_load(P1, a_slow, (s + 1) * BK, ra);
      rt_load(P2, b_slow, (s + 1) * BK, rb);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = cA[(kk * 4 + fk) * SLD + wr * 64 + i * 16 + fr];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = cB[(kk * 4 + fk) * SLD + wc * 64 + j * 16 + fr];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = NEG ? mfma64_neg(a[i], b[j], acc[i][j]) : mfma64(a[i], b[j], acc[i][j]);
    }
    if (s + 1 < nsteps) {
      rt_store(sA + (cur ^ 1) * GSTAGE, a_slow, ra);
      rt_store(sB + (cur ^ 1) * GSTAGE, b_slow, rb);
    }
    __syncthreads();
  }
}

template <bool NEG>
__device__ __forceinline__ void gemm_tile_ra(const double* __restrict__ P1, bool a_slow,
                                             const double* __restrict__ P2, double* smem,
                                             d4 (&acc)[4][4]) {
  gemm_tile_rr<NEG>(P1, a_slow, P2, true, smem, acc);
}

__device__ __forceinline__ void neg_tile(d4 (&acc)[4][4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = -acc[i][j];
}

// One 64 x 64 quadrant (qr, qc) of the 128 x 128 product above, each wave a 32 x 32
// piece (wave w: rows qr*64 + (w>>1)*32, columns qc*64 + (w&1)*32). Four workgroups
// then cover one output tile with a quarter of the MFMA chain each: the band's serial
// 128^3 steps (X T, V^T X, T^T M, X - V Zh, the tile-column update) are latency-bound
// single products per tile. Every operand load is in flight from the start (only the
// quadrant's 64 rows of each operand, in k-chunks of Q2_CK, up to Q2_NR chunks in
// registers at once: all of them at kdim 128), staged k-major ([k][Q2_LP]) into two
// LDS buffers. Against a one-slab-ahead prefetch (the 128 x 128 gemm_tile's staging):
// 140.3 against 141.0 ms for the N = 16384 reduction. The MFMA sequence per output
// element is gemm_tile's (k ascending, 4 per instruction): the same results.
constexpr int Q2_CK = 32;                      // k per chunk
constexpr int Q2_LP = 80;                      // LDS pitch (== 16 mod 32 doubles: the
                                               // fk = 0 / 1 fragment rows 32 banks apart)
constexpr int Q2_NR = 4;                       // chunks in registers at once
constexpr int Q2_SMEM = 2 * 2 * Q2_CK * Q2_LP;   // doubles (80 KB: two per CU)

// chunk c of op(P)'s rows [r0, r0 + 64): 4 d2 per thread
template <int L>
__device__ __forceinline__ void q2_load(const double* __restrict__ P, int64_t ld, int r0, int k0,
                                        d2 (&r)[4]) {
  const int t = threadIdx.x;
  if (L == KSLOW) {   // op(P)[r][k] = P[k * ld + r]: rows contiguous
    const double* p = P + (int64_t)(k0 + (t >> 3)) * ld + r0 + (t & 7) * 8;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = *reinterpret_cast<const d2*>(p + 2 * q);
  } else {            // op(P)[r][k] = P[r * ld + k]: k contiguous
    const double* p = P + (int64_t)(r0 + (t >> 2)) * ld + k0 + (t & 3) * 8;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = *reinterpret_cast<const d2*>(p + 2 * q);
  }
}

template <int L>
__device__ __forceinline__ void q2_store(double* s, const d2 (&r)[4]) {
  const int t = threadIdx.x;
  if (L == KSLOW) {
    double* d = s + (t >> 3) * Q2_LP + (t & 7) * 8;
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<d2*>(d + 2 * q) = r[q];
  } else {
    double* d = s + ((t & 3) * 8) * Q2_LP + (t >> 2);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      d[(2 * q) * Q2_LP] = r[q][0];
      d[(2 * q + 1) * Q2_LP] = r[q][1];
    }
  }
}

template <int AL, int BL, bool NEG, int KDIM>
__device__ __forceinline__ void gemm_quad2(const double* __restrict__ P1, int64_t ld1,
                                           const double* __restrict__ P2, int64_t ld2,
                                           double* smem, d4 (&acc)[2][2], int qr, int qc) {
  constexpr int NC = KDIM / Q2_CK;
  constexpr int NR = NC < Q2_NR ? NC : Q2_NR;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ra0 = (w >> 1) * 32, rb0 = (w & 1) * 32;   // the wave's rows in the halves
  const int fr = lane & 15, fk = lane >> 4;
  d2 ra[NR][4], rb[NR][4];
#pragma unroll
  for (int c = 0; c < NR; ++c) {
    q2_load<AL>(P1, ld1, qr * 64, c * Q2_CK, ra[c]);
    q2_load<BL>(P2, ld2, qc * 64, c * Q2_CK, rb[c]);
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    double* sA = smem + (c & 1) * (2 * Q2_CK * Q2_LP);
    double* sB = sA + Q2_CK * Q2_LP;
    q2_store<AL>(sA, ra[c % NR]);
    q2_store<BL>(sB, rb[c % NR]);
    __syncthreads();
    if (c + NR < NC) {
      q2_load<AL>(P1, ld1, qr * 64, (c + NR) * Q2_CK, ra[c % NR]);
      q2_load<BL>(P2, ld2, qc * 64, (c + NR) * Q2_CK, rb[c % NR]);
    }
#pragma unroll
    for (int kk = 0; kk < Q2_CK / 4; ++kk) {
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = sA[(kk * 4 + fk) * Q2_LP + ra0 + i * 16 + fr];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = sB[(kk * 4 + fk) * Q2_LP + rb0 + j * 16 + fr];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = NEG ? mfma64_neg(a[i], b[j], acc[i][j]) : mfma64(a[i], b[j], acc[i][j]);
    }
  }
  __syncthreads();   // (the caller may reuse smem)
}

__device__ __forceinline__ void zero_quad(d4 (&acc)[2][2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
}

// C points at the 128 x 128 tile; the quadrant's wave pieces as in gemm_quad2.
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
