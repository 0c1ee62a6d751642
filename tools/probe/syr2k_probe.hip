// Dev probe (not shipped): the band reduction's trailing SYR2K tile loop in
// isolation, timed per grid size and k depth, to find where the look-ahead
// SYR2K loses MFMA time. build: hipcc --offload-arch=gfx950 -O3 -std=c++17
//   -I../../gaussian-process-param-estimation_amd/csrc syr2k_probe.hip -o syr2k_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <string>
#include "gpmi_tile.h"

using namespace gpmi;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

// the shipped tile (gpmi_band.hip syr2k_tile) with the k depth as a parameter
__device__ __forceinline__ void tile_k(double* A, int64_t lda, const double* U, int64_t ldu, int I,
                                       int J, int kdim, double* smem) {
  double* C = A + (int64_t)I * TS * lda + (int64_t)J * TS;
  d4 acc[4][4];
  load_tile(C, lda, acc);
  gemm_tile<KFAST, KFAST, true>(U + (int64_t)I * TS * ldu, ldu, U + (int64_t)J * TS * ldu + kdim / 2,
                                ldu, kdim, smem, acc);
  store_tile(C, lda, acc, 1.0);
}

__global__ __launch_bounds__(256, 2) void rest_base(double* A, int64_t lda, const double* U,
                                                     int64_t ldu, int mt, int kdim) {
  __shared__ double smem[4 * GSTAGE];
  const int ntiles = (mt - 1) * mt / 2;
  for (int q = blockIdx.x; q < ntiles; q += gridDim.x) {
    int i, j;
    tri_decode(q, mt - 1, &i, &j);
    tile_k(A, lda, U, ldu, i + 1, j + 1, kdim, smem);
  }
}

// rest_base with the second workgroup of each CU (blockIdx >= 256) starting late by
// ~half a tile (s_sleep), so that the two workgroups' tile prologues / epilogues
// (C in and out, first stage) stop coinciding
__global__ __launch_bounds__(256, 2) void rest_stagger(double* A, int64_t lda, const double* U,
                                                       int64_t ldu, int mt, int kdim, int nap) {
  __shared__ double smem[4 * GSTAGE];
  if (blockIdx.x >= 256)
    for (int i = 0; i < nap; ++i) __builtin_amdgcn_s_sleep(127);
  const int ntiles = (mt - 1) * mt / 2;
  for (int q = blockIdx.x; q < ntiles; q += gridDim.x) {
    int i, j;
    tri_decode(q, mt - 1, &i, &j);
    tile_k(A, lda, U, ldu, i + 1, j + 1, kdim, smem);
  }
}

// no C traffic: the same MFMA work with zero accumulators, result not stored
// unless it is NaN (keeps the compiler from dropping it)
__global__ __launch_bounds__(256, 2) void rest_noc(double* A, int64_t lda, const double* U,
                                                    int64_t ldu, int mt, int kdim) {
  __shared__ double smem[4 * GSTAGE];
  const int ntiles = (mt - 1) * mt / 2;
  for (int q = blockIdx.x; q < ntiles; q += gridDim.x) {
    int i, j;
    tri_decode(q, mt - 1, &i, &j);
    d4 acc[4][4];
    zero_tile(acc);
    gemm_tile<KFAST, KFAST, true>(U + (int64_t)(i + 1) * TS * ldu, ldu,
                                  U + (int64_t)(j + 1) * TS * ldu + kdim / 2, ldu, kdim, smem, acc);
    if (acc[0][0][0] != acc[0][0][0]) A[0] = acc[1][1][1];
  }
}


// Software-pipelined persistent tile loop, one wave per SIMD (all 512 registers):
// while tile q runs its 16 k-steps, 4 of the 64 per-lane C values of tile q + grid
// are loaded and 4 of tile q - grid's results are stored per step, and step 15
// stages tile q + grid's first operand slab, so the C traffic is spread over the
// MFMA loop instead of a load and a store phase per tile that every workgroup
// of the launch runs at the same time.
// the previous tile's result values stored by an inline-asm global_store (hipcc
// does not count it, so the wait for this step's operand loads before their LDS
// store is not made conservative by a store pending in the same counter); issued
// BEFORE the step's loads, so vmcnt(N later loads) stays exact
__device__ __forceinline__ void st_asm(double* p, double v) {
  asm volatile("global_store_dwordx2 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int KD, bool SB = false, bool ASM = false>
__global__ __launch_bounds__(256, 1) void rest_pipe(double* __restrict__ A, int64_t lda,
                                                    const double* __restrict__ U, int64_t ldu,
                                                    int mt) {
  __shared__ double smem[4 * GSTAGE];
  constexpr int NS = KD / BK;
  constexpr int PER = (64 + NS - 1) / NS;   // C values per lane per step
  const int ntiles = (mt - 1) * mt / 2;
  int q = blockIdx.x;
  if (q >= ntiles) return;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  double* sA = smem;
  double* sB = smem + 2 * GSTAGE;
  auto tile_ptrs = [&](int qq, double** C, const double** P1, const double** P2) {
    int i, j;
    tri_decode(qq, mt - 1, &i, &j);
    *C = A + (int64_t)(i + 1) * TS * lda + (int64_t)(j + 1) * TS;
    *P1 = U + (int64_t)(i + 1) * TS * ldu;
    *P2 = U + (int64_t)(j + 1) * TS * ldu + KD / 2;
  };
  const int64_t coff = (int64_t)(wr * 64 + fk) * lda + wc * 64 + fr;
  auto cidx = [&](int e) -> int64_t {   // e = a * 16 + c * 4 + r
    return (int64_t)((e >> 4) * 16 + 4 * (e & 3)) * lda + ((e >> 2) & 3) * 16;
  };
  d4 acc[4][4], cn[4][4], po[4][4];
  double* Cq;
  const double *P1, *P2;
  tile_ptrs(q, &Cq, &P1, &P2);
  load_tile(Cq, lda, acc);
  d2 ra[4], rb[4];
  gl_op<KFAST>(P1, ldu, 0, ra);
  gl_op<KFAST>(P2, ldu, 0, rb);
  st_op<KFAST>(sA, ra);
  st_op<KFAST>(sB, rb);
  __syncthreads();
  double* Cp = nullptr;
  bool has_p = false;
  while (true) {
    const int qn = q + gridDim.x;
    const bool has_n = qn < ntiles;
    double* Cn = nullptr;
    const double *N1 = nullptr, *N2 = nullptr;
    if (has_n) tile_ptrs(qn, &Cn, &N1, &N2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int cur = s & 1;
      const double* cA = sA + cur * GSTAGE;
      const double* cB = sB + cur * GSTAGE;
      const bool ld = s + 1 < NS || has_n;
      if (ASM && has_p) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int e = s * PER + u;
          if (e < 64) st_asm(Cp + coff + cidx(e), po[e >> 4][(e >> 2) & 3][e & 3]);
        }
      }
      if (s + 1 < NS) {
        gl_op<KFAST>(P1, ldu, (s + 1) * BK, ra);
        gl_op<KFAST>(P2, ldu, (s + 1) * BK, rb);
      } else if (has_n) {
        gl_op<KFAST>(N1, ldu, 0, ra);
        gl_op<KFAST>(N2, ldu, 0, rb);
      }
      // SB: keep the C traffic after the operand loads in the instruction stream, so
      // the wait for the operands (before their LDS store) does not also wait for it
      if (SB) __builtin_amdgcn_sched_barrier(0);
      if (has_n) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int e = s * PER + u;
          if (e < 64) cn[e >> 4][(e >> 2) & 3][e & 3] = Cn[coff + cidx(e)];
        }
      }
      if (SB) __builtin_amdgcn_sched_barrier(0);
      if (!ASM && has_p) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int e = s * PER + u;
          if (e < 64) Cp[coff + cidx(e)] = po[e >> 4][(e >> 2) & 3][e & 3];
        }
      }
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = fr_op<KFAST>(cA, wr * 64 + i * 16 + fr, kk * 4 + fk);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = fr_op<KFAST>(cB, wc * 64 + j * 16 + fr, kk * 4 + fk);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma64_neg(a[i], b[j], acc[i][j]);
      }
      if (ld) {
        st_op<KFAST>(sA + (cur ^ 1) * GSTAGE, ra);
        st_op<KFAST>(sB + (cur ^ 1) * GSTAGE, rb);
      }
      __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        po[a][c] = acc[a][c];
        acc[a][c] = cn[a][c];
      }
    Cp = Cq;
    has_p = true;
    if (!has_n) break;
    q = qn;
    Cq = Cn;
    P1 = N1;
    P2 = N2;
  }
#pragma unroll
  for (int e = 0; e < 64; ++e) Cp[coff + cidx(e)] = po[e >> 4][(e >> 2) & 3][e & 3];
}

// rest_pipe without any C traffic: the accumulators run on across all of a
// workgroup's tiles (no per-tile load / store) and are stored once at the end; the
// operand staging and the k-loop exactly as rest_pipe
template <int KD>
__global__ __launch_bounds__(256, 1) void rest_pipe_noc(double* __restrict__ A, int64_t lda,
                                                        const double* __restrict__ U, int64_t ldu,
                                                        int mt) {
  __shared__ double smem[4 * GSTAGE];
  constexpr int NS = KD / BK;
  const int ntiles = (mt - 1) * mt / 2;
  int q = blockIdx.x;
  if (q >= ntiles) return;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  double* sA = smem;
  double* sB = smem + 2 * GSTAGE;
  auto tile_ptrs = [&](int qq, const double** P1, const double** P2) {
    int i, j;
    tri_decode(qq, mt - 1, &i, &j);
    *P1 = U + (int64_t)(i + 1) * TS * ldu;
    *P2 = U + (int64_t)(j + 1) * TS * ldu + KD / 2;
  };
  d4 acc[4][4];
  zero_tile(acc);
  const double *P1, *P2;
  tile_ptrs(q, &P1, &P2);
  d2 ra[4], rb[4];
  gl_op<KFAST>(P1, ldu, 0, ra);
  gl_op<KFAST>(P2, ldu, 0, rb);
  st_op<KFAST>(sA, ra);
  st_op<KFAST>(sB, rb);
  __syncthreads();
  while (true) {
    const int qn = q + gridDim.x;
    const bool has_n = qn < ntiles;
    const double *N1 = nullptr, *N2 = nullptr;
    if (has_n) tile_ptrs(qn, &N1, &N2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int cur = s & 1;
      const double* cA = sA + cur * GSTAGE;
      const double* cB = sB + cur * GSTAGE;
      const bool ld = s + 1 < NS || has_n;
      if (s + 1 < NS) {
        gl_op<KFAST>(P1, ldu, (s + 1) * BK, ra);
        gl_op<KFAST>(P2, ldu, (s + 1) * BK, rb);
      } else if (has_n) {
        gl_op<KFAST>(N1, ldu, 0, ra);
        gl_op<KFAST>(N2, ldu, 0, rb);
      }
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = fr_op<KFAST>(cA, wr * 64 + i * 16 + fr, kk * 4 + fk);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = fr_op<KFAST>(cB, wc * 64 + j * 16 + fr, kk * 4 + fk);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma64_neg(a[i], b[j], acc[i][j]);
      }
      if (ld) {
        st_op<KFAST>(sA + (cur ^ 1) * GSTAGE, ra);
        st_op<KFAST>(sB + (cur ^ 1) * GSTAGE, rb);
      }
      __syncthreads();
    }
    if (!has_n) break;
    q = qn;
    P1 = N1;
    P2 = N2;
  }
  store_tile(A + (int64_t)blockIdx.x * TS, lda, acc, 1.0);
}

// rest_pipe with the operand loads issued TWO k-steps ahead (two register sets;
// the LDS double buffer unchanged), paid for by storing each tile's results in one
// burst at its end instead of spreading them over the next tile (no `po` registers).
template <int KD>
__global__ __launch_bounds__(256, 1) void rest_pipe2(double* __restrict__ A, int64_t lda,
                                                     const double* __restrict__ U, int64_t ldu,
                                                     int mt) {
  __shared__ double smem[4 * GSTAGE];
  constexpr int NS = KD / BK;
  static_assert(NS % 2 == 0 && NS >= 2, "stage parity");
  constexpr int PER = (64 + NS - 1) / NS;
  const int ntiles = (mt - 1) * mt / 2;
  int q = blockIdx.x;
  if (q >= ntiles) return;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  double* sA = smem;
  double* sB = smem + 2 * GSTAGE;
  auto tile_ptrs = [&](int qq, double** C, const double** P1, const double** P2) {
    int i, j;
    tri_decode(qq, mt - 1, &i, &j);
    *C = A + (int64_t)(i + 1) * TS * lda + (int64_t)(j + 1) * TS;
    *P1 = U + (int64_t)(i + 1) * TS * ldu;
    *P2 = U + (int64_t)(j + 1) * TS * ldu + KD / 2;
  };
  const int64_t coff = (int64_t)(wr * 64 + fk) * lda + wc * 64 + fr;
  auto cidx = [&](int e) -> int64_t {
    return (int64_t)((e >> 4) * 16 + 4 * (e & 3)) * lda + ((e >> 2) & 3) * 16;
  };
  d4 acc[4][4], cn[4][4];
  double* Cq;
  const double *P1, *P2;
  tile_ptrs(q, &Cq, &P1, &P2);
  load_tile(Cq, lda, acc);
  d2 ra[2][4], rb[2][4];   // register sets by stage parity
  gl_op<KFAST>(P1, ldu, 0, ra[0]);
  gl_op<KFAST>(P2, ldu, 0, rb[0]);
  gl_op<KFAST>(P1, ldu, BK, ra[1]);
  gl_op<KFAST>(P2, ldu, BK, rb[1]);
  st_op<KFAST>(sA, ra[0]);
  st_op<KFAST>(sB, rb[0]);
  __syncthreads();
  while (true) {
    const int qn = q + gridDim.x;
    const bool has_n = qn < ntiles;
    double* Cn = nullptr;
    const double *N1 = nullptr, *N2 = nullptr;
    if (has_n) tile_ptrs(qn, &Cn, &N1, &N2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int cur = s & 1;
      const double* cA = sA + cur * GSTAGE;
      const double* cB = sB + cur * GSTAGE;
      // stage s + 2 into the set stage s used (already in LDS)
      if (s + 2 < NS) {
        gl_op<KFAST>(P1, ldu, (s + 2) * BK, ra[cur]);
        gl_op<KFAST>(P2, ldu, (s + 2) * BK, rb[cur]);
      } else if (has_n) {
        gl_op<KFAST>(N1, ldu, (s + 2 - NS) * BK, ra[cur]);
        gl_op<KFAST>(N2, ldu, (s + 2 - NS) * BK, rb[cur]);
      }
      if (has_n) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int e = s * PER + u;
          if (e < 64) cn[e >> 4][(e >> 2) & 3][e & 3] = Cn[coff + cidx(e)];
        }
      }
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = fr_op<KFAST>(cA, wr * 64 + i * 16 + fr, kk * 4 + fk);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = fr_op<KFAST>(cB, wc * 64 + j * 16 + fr, kk * 4 + fk);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma64_neg(a[i], b[j], acc[i][j]);
      }
      // stage s + 1 (loaded a step ago) into the other LDS buffer
      if (s + 1 < NS || has_n) {
        st_op<KFAST>(sA + (cur ^ 1) * GSTAGE, ra[cur ^ 1]);
        st_op<KFAST>(sB + (cur ^ 1) * GSTAGE, rb[cur ^ 1]);
      }
      __syncthreads();
    }
#pragma unroll
    for (int e = 0; e < 64; ++e) Cq[coff + cidx(e)] = acc[e >> 4][(e >> 2) & 3][e & 3];
    if (!has_n) break;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[a][c] = cn[a][c];
    q = qn;
    Cq = Cn;
    P1 = N1;
    P2 = N2;
  }
}

// The same persistent tile loop with the operand slabs staged by LDS-DMA
// (global_load_lds, 16 B per lane) into a ring of NBUF stages, NBUF - 1 of them in
// flight across the raw barriers (counted vmcnt, never 0 inside a tile): no VGPRs
// for staging, so the C tile's next values can be prefetched into registers. The
// LDS image is lane-linear (row r = 8 chunk + lane / 8, 16-B slot lane % 8); the
// slab swizzle moves to the source address (pair (slot ^ (r >> 1) & 7)), so the
// fragment reads (slab_off) are unchanged.
template <int KD, int NBUF>
__global__ __launch_bounds__(256, 1) void rest_glds(double* __restrict__ A, int64_t lda,
                                                    const double* __restrict__ U, int64_t ldu,
                                                    int mt) {
  __shared__ double lds[NBUF * 2 * STAGE];
  constexpr int NS = KD / BK;
  const int ntiles = (mt - 1) * mt / 2;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  const int nmine = blockIdx.x < ntiles ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  if (nmine == 0) return;
  const int total = nmine * NS;
  auto tile_of = [&](int it, int* I, int* J) {
    int i, j;
    tri_decode(blockIdx.x + it * gridDim.x, mt - 1, &i, &j);
    *I = i + 1;
    *J = j + 1;
  };
  // stage g -> its tile's operands at k0 = (g % NS) * BK into ring slot g % NBUF
  auto issue = [&](int g) {
    int I, J;
    tile_of(g / NS, &I, &J);
    const int k0 = (g % NS) * BK;
    double* dA = lds + (g % NBUF) * 2 * STAGE;
    double* dB = dA + STAGE;
    const double* P1 = U + (int64_t)I * TS * ldu + k0;
    const double* P2 = U + (int64_t)J * TS * ldu + KD / 2 + k0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int chunk = w + 4 * c;
      const int r = 8 * chunk + (lane >> 3), slot = lane & 7;
      const int pair = slot ^ ((r >> 1) & 7);
      __builtin_amdgcn_global_load_lds(P1 + (int64_t)r * ldu + 2 * pair, dA + chunk * 128, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(P2 + (int64_t)r * ldu + 2 * pair, dB + chunk * 128, 16, 0, 0);
    }
  };
  const int64_t coff = (int64_t)(wr * 64 + fk) * lda + wc * 64 + fr;
  d4 acc[4][4];
  zero_tile(acc);
  for (int g = 0; g < NBUF - 1 && g < total; ++g) issue(g);
  for (int g = 0; g < total; ++g) {
    // stage g landed: at most min(NBUF - 2, total - 1 - g) later stages (8 DMAs each) in flight
    const int later = min(NBUF - 2, total - 1 - g);
    if (later >= 2) __builtin_amdgcn_s_waitcnt(0x4F70);        // vmcnt(16)
    else if (later == 1) __builtin_amdgcn_s_waitcnt(0x0F78);   // vmcnt(8)
    else __builtin_amdgcn_s_waitcnt(0x0F70);                   // vmcnt(0)
    __builtin_amdgcn_s_waitcnt(0xC07F);                        // lgkmcnt(0): stage g - 1 read
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (g + NBUF - 1 < total) issue(g + NBUF - 1);
    const double* cA = lds + (g % NBUF) * 2 * STAGE;
    const double* cB = cA + STAGE;
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
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma64_neg(a[i], b[j], acc[i][j]);
    }
    if (g % NS == NS - 1) {
      // the tile's epilogue: C += acc (read-modify-write), acc = 0
      int I, J;
      tile_of(g / NS, &I, &J);
      double* C = A + (int64_t)I * TS * lda + (int64_t)J * TS + coff;
      d4 cv[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) cv[a][c][r] = C[(int64_t)(a * 16 + 4 * r) * lda + c * 16];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            C[(int64_t)(a * 16 + 4 * r) * lda + c * 16] = cv[a][c][r] + acc[a][c][r];
      zero_tile(acc);
    }
  }
}

// SYMM as shipped (gpmi_band.hip symm_kernel), and a timing-only variant that
// reads every tile in the row-major (KFAST) layout: how much the transposed
// (KSLOW, J > I) tiles cost.
template <bool ALLFAST>
__global__ __launch_bounds__(256, 2) void symm_probe(const double* __restrict__ A, int64_t lda,
                                                     const double* __restrict__ U, int64_t ldu,
                                                     int tr0, int mt, int chunk,
                                                     double* __restrict__ Xp) {
  __shared__ double smem[4 * GSTAGE];
  const int il = blockIdx.x, ch = blockIdx.y, nch = gridDim.y;
  const int I = tr0 + il;
  const int jl0 = ch * chunk, jl1 = min(mt, (ch + 1) * chunk);
  const int jsplit = ALLFAST ? jl1 : min(jl1, max(jl0, il + 1));
  d4 acc[4][4];
  zero_tile(acc);
  for (int jl = jl0; jl < jsplit; ++jl) {
    const int J = tr0 + jl;
    gemm_tile<KFAST, KSLOW, false>(A + (int64_t)I * TS * lda + (int64_t)J * TS, lda,
                                   U + (int64_t)J * TS * ldu + TS, ldu, TS, smem, acc);
  }
  for (int jl = jsplit; jl < jl1; ++jl) {
    const int J = tr0 + jl;
    gemm_tile<KSLOW, KSLOW, false>(A + (int64_t)J * TS * lda + (int64_t)I * TS, lda,
                                   U + (int64_t)J * TS * ldu + TS, ldu, TS, smem, acc);
  }
  store_tile(Xp + ((int64_t)il * nch + ch) * TS * TS, TS, acc, 1.0);
}

// KFAST-only tile loop with 8-deep k stages (LDS 32 KB per workgroup: three
// workgroups fit a CU, with <= 168 VGPRs three waves per SIMD), row-group swizzled
// slabs: s[row * 8 + (k ^ 2 ((row >> 2) & 3))].
__device__ __forceinline__ int s8(int row, int k) { return row * 8 + (k ^ (2 * ((row >> 2) & 3))); }
__device__ __forceinline__ void gl8(const double* __restrict__ P, int64_t ld, int k0, d2 (&r)[2]) {
  const int t = threadIdx.x, row = t >> 1, h = (t & 1) * 4;
  const double* p = P + (int64_t)row * ld + k0 + h;
  r[0] = *reinterpret_cast<const d2*>(p);
  r[1] = *reinterpret_cast<const d2*>(p + 2);
}
__device__ __forceinline__ void st8(double* s, const d2 (&r)[2]) {
  const int t = threadIdx.x, row = t >> 1, h = (t & 1) * 4;
  *reinterpret_cast<d2*>(s + s8(row, h)) = r[0];
  *reinterpret_cast<d2*>(s + s8(row, h + 2)) = r[1];
}
template <int OCC>
__global__ __launch_bounds__(256, OCC) void rest_b8(double* __restrict__ A, int64_t lda,
                                                    const double* __restrict__ U, int64_t ldu,
                                                    int mt, int kdim) {
  __shared__ double smem[4 * 1024];
  const int ntiles = (mt - 1) * mt / 2;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1, fr = lane & 15, fk = lane >> 4;
  double* sA = smem;
  double* sB = smem + 2048;
  for (int q = blockIdx.x; q < ntiles; q += gridDim.x) {
    int i, j;
    tri_decode(q, mt - 1, &i, &j);
    double* C = A + (int64_t)(i + 1) * TS * lda + (int64_t)(j + 1) * TS;
    const double* P1 = U + (int64_t)(i + 1) * TS * ldu;
    const double* P2 = U + (int64_t)(j + 1) * TS * ldu + kdim / 2;
    d4 acc[4][4];
    load_tile(C, lda, acc);
    d2 ra[2], rb[2];
    gl8(P1, ldu, 0, ra);
    gl8(P2, ldu, 0, rb);
    st8(sA, ra);
    st8(sB, rb);
    __syncthreads();
    __builtin_amdgcn_s_waitcnt(0x0F70);
    const int nsteps = kdim / 8;
    for (int s = 0; s < nsteps; ++s) {
      const int cur = s & 1;
      const double* cA = sA + cur * 1024;
      const double* cB = sB + cur * 1024;
      if (s + 1 < nsteps) {
        gl8(P1, ldu, (s + 1) * 8, ra);
        gl8(P2, ldu, (s + 1) * 8, rb);
      }
#pragma unroll 1
      for (int kk = 0; kk < 2; ++kk) {
        double a[4], b[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) a[x] = cA[s8(wr * 64 + x * 16 + fr, kk * 4 + fk)];
#pragma unroll
        for (int y = 0; y < 4; ++y) b[y] = cB[s8(wc * 64 + y * 16 + fr, kk * 4 + fk)];
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y) acc[x][y] = mfma64_neg(a[x], b[y], acc[x][y]);
      }
      if (s + 1 < nsteps) {
        st8(sA + (cur ^ 1) * 1024, ra);
        st8(sB + (cur ^ 1) * 1024, rb);
      }
      __syncthreads();
    }
    store_tile(C, lda, acc, 1.0);
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 16384;
  const int nt = n / TS;
  const int64_t ldu = 1024 + 128;
  double *A, *U;
  CK(hipMalloc(&A, sizeof(double) * (size_t)n * n));
  CK(hipMalloc(&U, sizeof(double) * (size_t)n * ldu));
  {
    std::vector<double> h((size_t)n * ldu);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 1e-3 * ((i * 2654435761u) % 1000) / 1000.0;
    CK(hipMemcpy(U, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice));
    CK(hipMemset(A, 0, sizeof(double) * (size_t)n * n));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int mts[] = {nt - 1, nt / 2};
  const int grids[] = {448, 512, 768, 1024, 100000};
  (void)0;
  const int kds[] = {256, 512};
  const bool symm_only = argc > 2 && std::string(argv[2]) == "symm";
  if (argc > 2 && std::string(argv[2]) == "stagger") {
    const int mt = nt - 1, ntiles = (mt - 1) * mt / 2;
    for (int nap : {0, 4, 8, 16, 24, 32})
      for (int kd : {256}) {
        auto launch = [&]() {
          hipLaunchKernelGGL(rest_stagger, dim3(512), dim3(256), 0, 0, A, (int64_t)n, U, ldu, mt, kd, nap);
        };
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < 5; ++r) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        const double fl = 2.0 * TS * TS * (double)kd * ntiles;
        printf("stagger nap=%2d (x 127 x 64 clk) k=%4d  %8.3f ms  %.3f of 78.6\n", nap, kd, ms, fl / ms * 1e-9 / 78.6);
      }
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "noc") {
    // the tile loop with and without its C tile traffic (k per tile 128 .. 1024)
    const int mt = nt - 1, ntiles = (mt - 1) * mt / 2;
    for (int kd : {128, 256, 512, 1024})
      for (int kern = 0; kern < 2; ++kern) {
        auto launch = [&]() {
          if (kern) hipLaunchKernelGGL(rest_noc, dim3(512), dim3(256), 0, 0, A, (int64_t)n, U, ldu, mt, kd);
          else hipLaunchKernelGGL(rest_base, dim3(512), dim3(256), 0, 0, A, (int64_t)n, U, ldu, mt, kd);
        };
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < 5; ++r) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        const double fl = 2.0 * TS * TS * (double)kd * ntiles;
        printf("%s k=%4d  %8.3f ms  %.3f of 78.6\n", kern ? "noC " : "base", kd, ms, fl / ms * 1e-9 / 78.6);
      }
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "glds") {
    // LDS-DMA ring against the register-staged pipeline (k = 256): equal results on
    // the same C, then the rate at the look-ahead grid (224 = 256 - 32 free CUs) and 256
    double *A1, *A2;
    CK(hipMalloc(&A1, sizeof(double) * (size_t)n * n));
    CK(hipMalloc(&A2, sizeof(double) * (size_t)n * n));
    {
      std::vector<double> h((size_t)n * n);
      for (size_t i = 0; i < h.size(); ++i) h[i] = 1e-2 * ((i * 40503u) % 997) / 997.0;
      CK(hipMemcpy(A1, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice));
      CK(hipMemcpy(A2, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice));
    }
    const int mt = nt - 1;
    hipLaunchKernelGGL(rest_pipe<256>, dim3(224), dim3(256), 0, 0, A1, (int64_t)n, U, ldu, mt);
    if (argc > 3 && std::string(argv[3]) == "asm")
      hipLaunchKernelGGL((rest_pipe<256, false, true>), dim3(224), dim3(256), 0, 0, A2, (int64_t)n, U, ldu, mt);
    else if (argc > 3 && std::string(argv[3]) == "pipe2")
      hipLaunchKernelGGL(rest_pipe2<256>, dim3(224), dim3(256), 0, 0, A2, (int64_t)n, U, ldu, mt);
    else
      hipLaunchKernelGGL((rest_glds<256, 4>), dim3(224), dim3(256), 0, 0, A2, (int64_t)n, U, ldu, mt);
    CK(hipDeviceSynchronize());
    {
      std::vector<double> h1((size_t)n * n), h2((size_t)n * n);
      CK(hipMemcpy(h1.data(), A1, sizeof(double) * h1.size(), hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), A2, sizeof(double) * h2.size(), hipMemcpyDeviceToHost));
      double md = 0.0, mx = 0.0;
      for (size_t i = 0; i < h1.size(); ++i) {
        md = fmax(md, fabs(h1[i] - h2[i]));
        mx = fmax(mx, fabs(h1[i]));
      }
      printf("variant vs pipe: max |diff| %.3e (max |C| %.3e)\n", md, mx);
    }
    const int ntiles = (mt - 1) * mt / 2;
    const double fl = 2.0 * TS * TS * 256.0 * ntiles;
    for (int g : {224, 256}) {
      for (int kern = 0; kern < 7; ++kern) {
        auto launch = [&]() {
          if (kern == 4) hipLaunchKernelGGL(rest_pipe_noc<256>, dim3(g), dim3(256), 0, 0, A1, (int64_t)n, U, ldu, mt);
          else if (kern == 5) hipLaunchKernelGGL((rest_pipe<256, true>), dim3(g), dim3(256), 0, 0, A1, (int64_t)n, U, ldu, mt);
          else if (kern == 6) hipLaunchKernelGGL((rest_pipe<256, false, true>), dim3(g), dim3(256), 0, 0, A1, (int64_t)n, U, ldu, mt);
          else if (kern == 3) hipLaunchKernelGGL(rest_pipe2<256>, dim3(g), dim3(256), 0, 0, A1, (int64_t)n, U, ldu, mt);
          else if (kern == 0) hipLaunchKernelGGL(rest_pipe<256>, dim3(g), dim3(256), 0, 0, A1, (int64_t)n, U, ldu, mt);
          else if (kern == 1) hipLaunchKernelGGL((rest_glds<256, 4>), dim3(g), dim3(256), 0, 0, A1, (int64_t)n, U, ldu, mt);
          else hipLaunchKernelGGL((rest_glds<256, 3>), dim3(g), dim3(256), 0, 0, A1, (int64_t)n, U, ldu, mt);
        };
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < 5; ++r) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        printf("%s grid=%d  %8.3f ms  %6.1f TF  %.3f of 78.6 (%.3f per busy CU)\n",
               kern == 0 ? "pipe   " : kern == 1 ? "glds4  " : kern == 2 ? "glds3  " : kern == 3 ? "pipe2  " : kern == 4 ? "pipenoC" : kern == 5 ? "pipeSB " : "pipeASM", g, ms, fl / ms * 1e-9,
               fl / ms * 1e-9 / 78.6, fl / ms * 1e-9 / 78.6 * 256.0 / g);
      }
    }
    return 0;
  }
  if (!symm_only)
  for (int kern : {0, 3, 4, 5})
    for (int mt : mts)
      for (int kd : kds)
        for (int g0 : grids) {
          if (kern == 2 && kd != 256) continue;
          if (kern == 0 && g0 > 512 && g0 < 100000) continue;
          const int ntiles = (mt - 1) * mt / 2;
          const int g = g0 < ntiles ? g0 : ntiles;
          auto launch = [&]() {
            if (kern == 3) hipLaunchKernelGGL(rest_b8<2>, dim3(g), dim3(256), 0, 0, A, (int64_t)n, U, ldu, mt, kd);
            else if (kern == 4) hipLaunchKernelGGL(rest_b8<3>, dim3(g), dim3(256), 0, 0, A, (int64_t)n, U, ldu, mt, kd);
            else if (kern == 5) hipLaunchKernelGGL(rest_b8<4>, dim3(g), dim3(256), 0, 0, A, (int64_t)n, U, ldu, mt, kd);
            else if (kern == 0) hipLaunchKernelGGL(rest_base, dim3(g), dim3(256), 0, 0, A, (int64_t)n, U, ldu, mt, kd);
            else if (kern == 2) hipLaunchKernelGGL(rest_pipe<256>, dim3(g), dim3(256), 0, 0, A, (int64_t)n, U, ldu, mt);
            else hipLaunchKernelGGL(rest_noc, dim3(g), dim3(256), 0, 0, A, (int64_t)n, U, ldu, mt, kd);
          };
          launch();
          CK(hipDeviceSynchronize());
          const int reps = 5;
          CK(hipEventRecord(e0, 0));
          for (int r = 0; r < reps; ++r) launch();
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ms /= reps;
          const double fl = 2.0 * TS * TS * (double)kd * ntiles;
          printf("%s mt=%3d kdim=%4d grid=%6d tiles=%6d  %8.3f ms  %6.1f TF  %.3f of 78.6\n",
                 kern == 3 ? "b8o2" : kern == 4 ? "b8o3" : kern == 5 ? "b8o4" : kern == 2 ? "pipe" : kern ? "noC " : "base", mt, kd, g, ntiles, ms, fl / ms * 1e-9, fl / ms * 1e-9 / 78.6);
        }
  {
    double* Xp;
    CK(hipMalloc(&Xp, sizeof(double) * (size_t)nt * nt * TS * TS));
    // "symm": the split-K chunk sweep at the band's mt values (the shipped kernel only)
    std::vector<int> mtv = symm_only ? std::vector<int>{117, 97, 77, 57} : std::vector<int>{nt - 1, nt / 2};
    std::vector<int> chv = symm_only ? std::vector<int>{4, 6, 8, 9, 10, 12, 13, 16} : std::vector<int>{4, 8, 16, 32};
    for (int mt : mtv)
      for (int chunk : chv)
        for (int af = 0; af < 2; ++af) {
          const int sch = (mt + chunk - 1) / chunk;
          if (!symm_only && sch > 16) continue;
          if (symm_only && af) continue;
          auto launch = [&]() {
            if (af) hipLaunchKernelGGL(symm_probe<true>, dim3(mt, sch), dim3(256), 0, 0, A, (int64_t)n, U, ldu, 1, mt, chunk, Xp);
            else hipLaunchKernelGGL(symm_probe<false>, dim3(mt, sch), dim3(256), 0, 0, A, (int64_t)n, U, ldu, 1, mt, chunk, Xp);
          };
          launch();
          CK(hipDeviceSynchronize());
          CK(hipEventRecord(e0, 0));
          for (int r = 0; r < 5; ++r) launch();
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ms /= 5;
          const double fl = 2.0 * (double)mt * TS * mt * TS * TS;
          printf("symm%s mt=%3d chunk=%2d wgs=%5d  %8.3f ms  %6.1f TF  %.3f\n", af ? "(allfast)" : "         ",
                 mt, chunk, mt * sch, ms, fl / ms * 1e-9, fl / ms * 1e-9 / 78.6);
        }
  }
  return 0;
}
