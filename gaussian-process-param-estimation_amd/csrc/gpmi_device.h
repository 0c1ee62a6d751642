// Device-side helpers shared by the gpmi HIP translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gpmi_internal.h"

namespace gpmi {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int TS = GPMI_TS;      // 128
constexpr int BK = 16;           // k-depth of one LDS stage
constexpr int STAGE = TS * BK;   // doubles per staged operand buffer (128 rows x 16, 16 KB)

// Staged slabs are stored unpadded, [row][16 doubles], with the 16-byte chunk c
// of row r placed at chunk position c ^ ((r >> 1) & 7); the staging
// ds_write_b128 of a row stays one contiguous 128-byte line. The compiler merges
// fragment reads 16 rows apart into ds_read2st64_b64, whose 16-lane groups see
// this layout 2-way conflicted; measured faster than the conflict-free
// k ^ (r & 15) layout (with or without the merge) all the same.
__device__ __forceinline__ int slab_off(int row, int k) {
  return row * BK + 2 * ((k >> 1) ^ ((row >> 1) & 7)) + (k & 1);
}
constexpr int RLD = GPMI_RHS_LD; // 16

// Hand-off words between co-resident workgroups: agent-scope relaxed atomic
// stores / loads (write-through to L2, loads that bypass the non-coherent caches).
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(
      reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
      __HIP_MEMORY_SCOPE_AGENT));
}

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// c - a b: for f64 MFMA the BLGP field is the NEG modifier (bit 0 negates A),
// so the subtraction costs no VALU op.
__device__ __forceinline__ d4 mfma64_neg(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 1);
}


// 128 x 16 slab of rows base[row * ld + p .. p + 15]: each wave-instruction
// reads 32 full 128-B row segments (16 B / lane).
__device__ __forceinline__ void gload_slab(const double* __restrict__ base, int64_t ld,
                                           int p, d2 (&r)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = i * 256 + t;
    const int row = idx >> 3, c2 = idx & 7;
    r[i] = *reinterpret_cast<const d2*>(base + (int64_t)row * ld + p + 2 * c2);
  }
}

__device__ __forceinline__ void sstore_slab(double* s, const d2 (&r)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = i * 256 + t;
    const int row = idx >> 3, c2 = idx & 7;
    *reinterpret_cast<d2*>(s + row * BK + 2 * (c2 ^ ((row >> 1) & 7))) = r[i];
  }
}


// acc (wave tile 64 x 64 at (wr, wc)) += P1[0:128, 0:kdim] * P2[0:128, 0:kdim]^T.
// f64 MFMA 16x16x4 operand maps: A[i = lane&15][k = lane>>4], B[k = lane>>4][j = lane&15].
// WITH_RHS additionally accumulates racc (rows wr*64 + wc*32 + [0,32), 16 cols)
// += P1 * U with U[kdim][16] staged in LDS.
template <bool WITH_RHS, bool NEG = false>
__device__ __forceinline__ void tile_mma(const double* __restrict__ P1, int64_t ld1,
                                         const double* __restrict__ P2, int64_t ld2,
                                         int kdim, double* sA, double* sB,
                                         d4 (&acc)[4][4], const double* sU,
                                         d4 (&racc)[2]) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fk = lane >> 4;
  d2 ra[4], rb[4];
  gload_slab(P1, ld1, 0, ra);
  gload_slab(P2, ld2, 0, rb);
  sstore_slab(sA, ra);
  sstore_slab(sB, rb);
  __syncthreads();
  // Drain every global load issued before the loop (the caller's accumulator
  // preload) here, once. Otherwise the waitcnt pass places vmcnt(3..0) waits
  // on the first accumulator uses INSIDE the loop, which also drain the
  // next-stage prefetch every iteration (vmcnt counts in order).
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
  const int nsteps = kdim / BK;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const double* cA = sA + cur * STAGE;
    const double* cB = sB + cur * STAGE;
    if (s + 1 < nsteps) {
      gload_slab(P1, ld1, (s + 1) * BK, ra);
      gload_slab(P2, ld2, (s + 1) * BK, rb);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = cA[slab_off(wr * 64 + i * 16 + fr, kk * 4 + fk)];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = cB[slab_off(wc * 64 + j * 16 + fr, kk * 4 + fk)];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = NEG ? mfma64_neg(a[i], b[j], acc[i][j]) : mfma64(a[i], b[j], acc[i][j]);
      if (WITH_RHS) {
        const double u = sU[(s * BK + kk * 4 + fk) * RLD + fr];
        const double a0 = wc ? a[2] : a[0];
        const double a1 = wc ? a[3] : a[1];
        racc[0] = mfma64(a0, u, racc[0]);
        racc[1] = mfma64(a1, u, racc[1]);
      }
    }
    if (s + 1 < nsteps) {
      sstore_slab(sA + (cur ^ 1) * STAGE, ra);
      sstore_slab(sB + (cur ^ 1) * STAGE, rb);
    }
    __syncthreads();
  }
}

// Bijective XCD-aware remap (consecutive logical tiles -> one XCD's L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Lower-triangular tile enumeration of a band of w tile columns over t tile
// rows (row-major): rows i < w hold a triangle, rows i >= w hold w tiles.
__device__ __forceinline__ void tri_decode(int q, int w, int* pi, int* pj) {
  const int tri = w * (w + 1) / 2;
  int i, j;
  if (q < tri) {
    i = (int)((sqrt(8.0 * (double)q + 1.0) - 1.0) * 0.5);
    while ((i + 1) * (i + 2) / 2 <= q) ++i;
    while (i * (i + 1) / 2 > q) --i;
    j = q - i * (i + 1) / 2;
  } else {
    const int r = q - tri;
    i = w + r / w;
    j = r % w;
  }
  *pi = i;
  *pj = j;
}

}  // namespace gpmi
