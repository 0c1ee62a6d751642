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
//   triangle), E = A[J_{k+1}, J_k] <- E H.
// The matrix is a dense n_pad x n_pad lower-triangle copy of B; every access is
// within 2b of the diagonal. The three blocks (F, D, E) are loaded at the start
// (all 16-byte loads of the task in flight together; F parked in LDS), the three
// matrix-vector products taken in one pass, and the blocks written back whole.
//
// bisect_kernel: thread i finds the i-th smallest eigenvalue of the symmetric
// tridiagonal (d, e) by bisection on the Sturm count (LDL^T pivots of T - x I,
// pivmin safeguard as LAPACK dstebz), Gershgorin start interval.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gpmi_internal.h"
#include "gpmi_band.h"
#include "gpmi_device.h"

namespace gpmi {

constexpr int CB = GPMI_TS;        // band width of B = 128

constexpr int CT = 512;             // chase workgroup: 8 waves
constexpr int CPT = CB * CB / 2 / CT;   // 16-byte pairs per thread per 128 x 128 block

__device__ __forceinline__ double block_sum8(double v, double* red) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return ((red[0] + red[1]) + (red[2] + red[3])) + ((red[4] + red[5]) + (red[6] + red[7]));
}

// Rows [0, nr) x columns [0, nc) of a row-major block into registers (pair u of
// thread t: element index e = u * CT + t, row e >> 6, columns 2 (e & 63) + {0,1};
// outside the block: 0). All CPT loads are in flight together.
template <bool LOWER = false>
__device__ __forceinline__ void load_block(const double* __restrict__ src, int64_t lda, int nr,
                                           int nc, d2 (&r)[CPT]) {
#pragma unroll
  for (int u = 0; u < CPT; ++u) {
    const int e = u * CT + threadIdx.x;
    const int i = e >> 6, c2 = 2 * (e & 63);
    const double* p = src + (int64_t)i * lda + c2;
    r[u] = d2{0.0, 0.0};
    if (i < nr && (!LOWER || c2 <= i)) {   // LOWER: pairs starting on or left of the diagonal
      if (c2 + 1 < nc) r[u] = *reinterpret_cast<const d2*>(p);
      else if (c2 < nc) r[u][0] = p[0];
    }
  }
}

// Butterfly reduce-scatter over 8 values: returns in every lane the 64-lane sum of
// value index (lane >> 3) & 7 (10 shuffles for 8 sums, fixed order).
__device__ __forceinline__ double butterfly8(double (&v)[8]) {
  const int lane = threadIdx.x & 63;
#define GPMI_BFLY_STEP(O, NN)                                      \
  {                                                                \
    const bool up = (lane & (O)) != 0;                             \
    _Pragma("unroll") for (int q = 0; q < (NN) / 2; ++q) {         \
      const double keep = up ? v[q + (NN) / 2] : v[q];             \
      const double send = up ? v[q] : v[q + (NN) / 2];             \
      v[q] = keep + __shfl_xor(send, (O));                         \
    }                                                              \
  }
  GPMI_BFLY_STEP(32, 8)
  GPMI_BFLY_STEP(16, 4)
  GPMI_BFLY_STEP(8, 2)
#undef GPMI_BFLY_STEP
  double r = v[0];
  r += __shfl_xor(r, 4);
  r += __shfl_xor(r, 2);
  r += __shfl_xor(r, 1);
  return r;
}

// One chase task with the three products F^T v, D v and E v taken in ONE pass over
// the blocks held in registers (wave w holds rows 8u + w, lane the columns 2 lane,
// 2 lane + 1): row sums by butterfly reductions, column sums as per-wave partials
// in LDS summed in wave order. Only F is parked in LDS (in thread order, to fit the
// register file); 5 barriers per task.
__global__ __launch_bounds__(CT) void chase_task_kernel(double* __restrict__ A, int64_t lda,
                                                        int n, int t, int s_hi) {
  __shared__ double sv[CB];
  __shared__ double cpart[2][8][CB];   // per-wave column partials: F^T v, strict-lower(D)^T v
  __shared__ double srow[2][CB];       // row sums: lower(D) v, E v
  __shared__ double sf[CB], sw[CB], sq[CB];
  __shared__ double red[8];
  __shared__ double sx0;
  __shared__ d2 fbuf[CPT * CT];        // F (k >= 1) in thread order: frees 64 VGPRs
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int s = s_hi - (int)blockIdx.x;
  const int k = t - 3 * s;
  if (s < 0 || k < 0) return;
  const int r0 = s + 1 + k * CB;
  if (r0 >= n) return;
  const int r1 = min(r0 + CB, n), L = r1 - r0;
  const int col = (k == 0) ? s : s + 1 + (k - 1) * CB;
  const int e1 = min(r1 + CB, n), LE = e1 - r1;
  const double xi = (tid < L) ? A[(int64_t)(r0 + tid) * lda + col] : 0.0;
  d2 Dr[CPT], Er[CPT];
  if (k >= 1) {
    d2 Fr[CPT];
    load_block(A + (int64_t)r0 * lda + col, lda, L, CB, Fr);
#pragma unroll
    for (int u = 0; u < CPT; ++u) fbuf[u * CT + tid] = Fr[u];   // own slots: no barrier
  }
  load_block<true>(A + (int64_t)r0 * lda + r0, lda, L, L, Dr);
  if (LE > 0) load_block(A + (int64_t)r1 * lda + r0, lda, LE, L, Er);
  // ---- reflector (LAPACK dlarfg)
  if (tid == 0) sx0 = xi;
  const double nb2 = block_sum8((tid > 0 && tid < L) ? xi * xi : 0.0, red);
  const double xx0 = sx0;
  double tau = 0.0, beta = xx0, scale = 0.0;
  if (nb2 > 0.0) {
    const double nrm = sqrt(xx0 * xx0 + nb2);
    beta = xx0 >= 0.0 ? -nrm : nrm;
    tau = (beta - xx0) / beta;
    scale = 1.0 / (xx0 - beta);
  }
  if (tid < CB) sv[tid] = (tid == 0) ? 1.0 : ((tid < L) ? xi * scale : 0.0);
  if (k == 0 && tid < L) A[(int64_t)(r0 + tid) * lda + s] = (tid == 0) ? beta : 0.0;
  if (tau == 0.0) return;   // identity reflector: nothing else changes
  __syncthreads();
  // ---- one pass: D (lower pairs; the pair starting on the diagonal carries an
  //      unread upper element), E, F
  const int c0 = 2 * lane;
  const double vc0 = sv[c0], vc1 = sv[c0 + 1];
  double dc0 = 0.0, dc1 = 0.0;
  // row sums in two halves of 8 rows (half the live partials): lane holds row
  // u = 8 h + ((lane >> 3) & 7) of each
  double prow[2], qrow[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    double rowv[8];
#pragma unroll
    for (int uu = 0; uu < 8; ++uu) {
      const int u = 8 * h + uu;
      const int i = 8 * u + w;
      const double vi = sv[i];
      const double d0 = (c0 <= i) ? Dr[u][0] : 0.0;
      const double d1 = (c0 + 1 <= i) ? Dr[u][1] : 0.0;
      rowv[uu] = d0 * vc0 + d1 * vc1;
      if (c0 < i) dc0 += d0 * vi;
      if (c0 + 1 < i) dc1 += d1 * vi;
    }
    prow[h] = butterfly8(rowv);
#pragma unroll
    for (int uu = 0; uu < 8; ++uu)
      rowv[uu] = Er[8 * h + uu][0] * vc0 + Er[8 * h + uu][1] * vc1;
    qrow[h] = butterfly8(rowv);
  }
  double fc0 = 0.0, fc1 = 0.0;
  if (k >= 1) {
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const double vi = sv[8 * u + w];
      const d2 f = fbuf[u * CT + tid];
      fc0 += f[0] * vi;
      fc1 += f[1] * vi;
    }
  }
  cpart[0][w][c0] = fc0;
  cpart[0][w][c0 + 1] = fc1;
  cpart[1][w][c0] = dc0;
  cpart[1][w][c0 + 1] = dc1;
  if ((lane & 7) == 0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = 8 * (8 * h + ((lane >> 3) & 7)) + w;
      srow[0][i] = prow[h];
      srow[1][i] = qrow[h];
    }
  }
  __syncthreads();
  double pi = 0.0;
  if (tid < CB) {
    double sd = srow[0][tid], sfv = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      sd += cpart[1][q][tid];
      sfv += cpart[0][q][tid];
    }
    pi = (tid < L) ? tau * sd : 0.0;
    sf[tid] = tau * sfv;
    sq[tid] = tau * srow[1][tid];
  }
  const double vp = block_sum8((tid < L) ? pi * sv[tid] : 0.0, red);
  if (tid < CB) sw[tid] = (tid < L) ? pi - 0.5 * tau * vp * sv[tid] : 0.0;
  __syncthreads();
  // ---- F <- H F: column col becomes (beta, 0 ...)
  if (k >= 1) {
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int e = u * CT + tid;
      const int i = e >> 6, c2 = 2 * (e & 63);
      if (i >= L) continue;
      const d2 f = fbuf[u * CT + tid];
      d2 o;
      o[0] = (c2 == 0) ? (i == 0 ? beta : 0.0) : f[0] - sv[i] * sf[c2];
      o[1] = f[1] - sv[i] * sf[c2 + 1];
      *reinterpret_cast<d2*>(A + (int64_t)(r0 + i) * lda + col + c2) = o;
    }
  }
  // ---- D <- H D H = D - v w^T - w v^T (lower triangle back)
#pragma unroll
  for (int u = 0; u < CPT; ++u) {
    const int e = u * CT + tid;
    const int i = e >> 6, c2 = 2 * (e & 63);
    if (i >= L || c2 >= L || c2 > i) continue;
    d2 o;
    o[0] = Dr[u][0] - sv[i] * sw[c2] - sw[i] * sv[c2];
    o[1] = Dr[u][1] - sv[i] * sw[c2 + 1] - sw[i] * sv[c2 + 1];
    if (c2 + 1 < L) *reinterpret_cast<d2*>(A + (int64_t)(r0 + i) * lda + r0 + c2) = o;
    else A[(int64_t)(r0 + i) * lda + r0 + c2] = o[0];
  }
  // ---- E <- E H = E - q v^T
  if (LE > 0) {
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int e = u * CT + tid;
      const int i = e >> 6, c2 = 2 * (e & 63);
      if (i >= LE || c2 >= L) continue;
      d2 o;
      o[0] = Er[u][0] - sq[i] * sv[c2];
      o[1] = Er[u][1] - sq[i] * sv[c2 + 1];
      if (c2 + 1 < L) *reinterpret_cast<d2*>(A + (int64_t)(r1 + i) * lda + r0 + c2) = o;
      else A[(int64_t)(r1 + i) * lda + r0 + c2] = o[0];
    }
  }
}

// ---------------------------------------------------------------------------
// Split form of the task (default): the F, D and E updates of a task need only its
// reflector, so a small launch forms every task's (v, tau, beta) into a scratch
// slot (and writes the annihilated column s when k = 0), then one workgroup per
// block applies it: three workgroups per task, none exchanging data, each moving a
// third of the task's bytes through its CU. Same arithmetic and order as
// chase_task_kernel, so the result is bit-identical.
// ---------------------------------------------------------------------------
constexpr int SLOT = CB + 2;   // v[128], tau, beta

// Reflector of the first task (s, 0) of sweep s into slot sl; writes the
// annihilated column s. (The reflector of (s, k + 1) comes from the E workgroup of
// (s, k) one wavefront earlier: chase_apply_kernel.)
__global__ __launch_bounds__(CB) void chase_reflect_kernel(double* __restrict__ A, int64_t lda,
                                                           int n, int s,
                                                           double* __restrict__ sl) {
  __shared__ double red[2];
  __shared__ double sx0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int k = 0;
  const int r0 = s + 1;
  if (r0 >= n) return;
  const int L = min(r0 + CB, n) - r0;
  const int col = s;
  const double xi = (tid < L) ? A[(int64_t)(r0 + tid) * lda + col] : 0.0;
  if (tid == 0) sx0 = xi;
  double v = (tid > 0 && tid < L) ? xi * xi : 0.0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  if (lane == 0) red[w] = v;
  __syncthreads();
  const double nb2 = red[0] + red[1];
  const double xx0 = sx0;
  double tau = 0.0, beta = xx0, scale = 0.0;
  if (nb2 > 0.0) {
    const double nrm = sqrt(xx0 * xx0 + nb2);
    beta = xx0 >= 0.0 ? -nrm : nrm;
    tau = (beta - xx0) / beta;
    scale = 1.0 / (xx0 - beta);
  }
  sl[tid] = (tid == 0) ? 1.0 : ((tid < L) ? xi * scale : 0.0);
  if (tid == 0) {
    sl[CB] = tau;
    sl[CB + 1] = beta;
  }
  if (k == 0 && tid < L) A[(int64_t)(r0 + tid) * lda + s] = (tid == 0) ? beta : 0.0;
}

__global__ __launch_bounds__(CT) void chase_apply_kernel(double* __restrict__ A, int64_t lda,
                                                         int n, int t, int s_hi,
                                                         const double* __restrict__ rd,
                                                         double* __restrict__ wr, int ns) {
  __shared__ double sv[CB];
  __shared__ double red2[2];
  __shared__ double cpart[8][CB];
  __shared__ double srow[CB];
  __shared__ double sx[CB];
  __shared__ double red[8];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int slot = (int)blockIdx.x / 3, part = (int)blockIdx.x % 3;   // 0 F, 1 D, 2 E
  const int s = s_hi - slot;
  const int k = t - 3 * s;
  if (s < 0 || k < 0) return;
  const int r0 = s + 1 + k * CB;
  if (r0 >= n) return;
  const int r1 = min(r0 + CB, n), L = r1 - r0;
  const int col = (k == 0) ? s : s + 1 + (k - 1) * CB;
  const int e1 = min(r1 + CB, n), LE = e1 - r1;
  if (part == 0 && k == 0) return;     // no bulge block in the first task of a sweep
  if (part == 2 && LE <= 0) return;
  const double* sl = rd + (int64_t)(s % ns) * SLOT;
  const double tau = sl[CB], beta = sl[CB + 1];
  if (tau == 0.0 && part != 2) return;   // identity reflector (E still forms the next one)
  d2 Br[CPT];
  if (part == 0) load_block(A + (int64_t)r0 * lda + col, lda, L, CB, Br);
  else if (part == 1) load_block<true>(A + (int64_t)r0 * lda + r0, lda, L, L, Br);
  else load_block(A + (int64_t)r1 * lda + r0, lda, LE, L, Br);
  if (tid < CB) sv[tid] = sl[tid];
  __syncthreads();
  const int c0 = 2 * lane;
  const double vc0 = sv[c0], vc1 = sv[c0 + 1];
  if (part == 0) {
    // ---- F <- H F: w = tau F^T v; column col becomes (beta, 0 ...)
    double fc0 = 0.0, fc1 = 0.0;
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const double vi = sv[8 * u + w];
      fc0 += Br[u][0] * vi;
      fc1 += Br[u][1] * vi;
    }
    cpart[w][c0] = fc0;
    cpart[w][c0 + 1] = fc1;
    __syncthreads();
    if (tid < CB) {
      double sfv = 0.0;
#pragma unroll
      for (int q = 0; q < 8; ++q) sfv += cpart[q][tid];
      sx[tid] = tau * sfv;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int e = u * CT + tid;
      const int i = e >> 6, c2 = 2 * (e & 63);
      if (i >= L) continue;
      d2 o;
      o[0] = (c2 == 0) ? (i == 0 ? beta : 0.0) : Br[u][0] - sv[i] * sx[c2];
      o[1] = Br[u][1] - sv[i] * sx[c2 + 1];
      *reinterpret_cast<d2*>(A + (int64_t)(r0 + i) * lda + col + c2) = o;
    }
  } else if (part == 1) {
    // ---- D <- H D H = D - v w^T - w v^T, w = p - tau/2 (v.p) v, p = tau D v
    double dc0 = 0.0, dc1 = 0.0;
    double prow[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double rowv[8];
#pragma unroll
      for (int uu = 0; uu < 8; ++uu) {
        const int u = 8 * h + uu;
        const int i = 8 * u + w;
        const double vi = sv[i];
        const double d0 = (c0 <= i) ? Br[u][0] : 0.0;
        const double d1 = (c0 + 1 <= i) ? Br[u][1] : 0.0;
        rowv[uu] = d0 * vc0 + d1 * vc1;
        if (c0 < i) dc0 += d0 * vi;
        if (c0 + 1 < i) dc1 += d1 * vi;
      }
      prow[h] = butterfly8(rowv);
    }
    cpart[w][c0] = dc0;
    cpart[w][c0 + 1] = dc1;
    if ((lane & 7) == 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h) srow[8 * (8 * h + ((lane >> 3) & 7)) + w] = prow[h];
    }
    __syncthreads();
    double pi = 0.0;
    if (tid < CB) {
      double sd = srow[tid];
#pragma unroll
      for (int q = 0; q < 8; ++q) sd += cpart[q][tid];
      pi = (tid < L) ? tau * sd : 0.0;
    }
    const double vp = block_sum8((tid < L) ? pi * sv[tid] : 0.0, red);
    if (tid < CB) sx[tid] = (tid < L) ? pi - 0.5 * tau * vp * sv[tid] : 0.0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int e = u * CT + tid;
      const int i = e >> 6, c2 = 2 * (e & 63);
      if (i >= L || c2 >= L || c2 > i) continue;
      d2 o;
      o[0] = Br[u][0] - sv[i] * sx[c2] - sx[i] * sv[c2];
      o[1] = Br[u][1] - sv[i] * sx[c2 + 1] - sx[i] * sv[c2 + 1];
      if (c2 + 1 < L) *reinterpret_cast<d2*>(A + (int64_t)(r0 + i) * lda + r0 + c2) = o;
      else A[(int64_t)(r0 + i) * lda + r0 + c2] = o[0];
    }
  } else {
    // ---- E <- E H = E - q v^T, q = tau E v
    if (tau != 0.0) {
    double qrow[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double rowv[8];
#pragma unroll
      for (int uu = 0; uu < 8; ++uu)
        rowv[uu] = Br[8 * h + uu][0] * vc0 + Br[8 * h + uu][1] * vc1;
      qrow[h] = butterfly8(rowv);
    }
    if ((lane & 7) == 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h) srow[8 * (8 * h + ((lane >> 3) & 7)) + w] = qrow[h];
    }
    __syncthreads();
    if (tid < CB) sx[tid] = tau * srow[tid];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int e = u * CT + tid;
      const int i = e >> 6, c2 = 2 * (e & 63);
      if (i >= LE || c2 >= L) continue;
      d2 o;
      o[0] = Br[u][0] - sx[i] * sv[c2];
      o[1] = Br[u][1] - sx[i] * sv[c2 + 1];
      if (c2 + 1 < L) *reinterpret_cast<d2*>(A + (int64_t)(r1 + i) * lda + r0 + c2) = o;
      else A[(int64_t)(r1 + i) * lda + r0 + c2] = o[0];
      Br[u] = o;
    }
    }
    // ---- reflector of task (s, k + 1): its x is E's (updated) first column; the
    //      same arithmetic as chase_reflect_kernel, into this sweep's slot of wr
    __syncthreads();   // sx, srow reuse below
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < CPT; ++u) srow[8 * u + w] = (8 * u + w < LE) ? Br[u][0] : 0.0;
    }
    __syncthreads();
    double xi = 0.0, v2 = 0.0;
    if (tid < CB) {
      xi = srow[tid];
      v2 = (tid > 0 && tid < LE) ? xi * xi : 0.0;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v2 += __shfl_xor(v2, off);
      if (lane == 0) red2[w] = v2;
    }
    __syncthreads();
    if (tid < CB) {
      const double nb2 = red2[0] + red2[1];
      const double xx0 = srow[0];
      double tn = 0.0, bn = xx0, sc = 0.0;
      if (nb2 > 0.0) {
        const double nrm = sqrt(xx0 * xx0 + nb2);
        bn = xx0 >= 0.0 ? -nrm : nrm;
        tn = (bn - xx0) / bn;
        sc = 1.0 / (xx0 - bn);
      }
      double* wl = wr + (int64_t)(s % ns) * SLOT;
      wl[tid] = (tid == 0) ? 1.0 : ((tid < LE) ? xi * sc : 0.0);
      if (tid == 0) {
        wl[CB] = tn;
        wl[CB + 1] = bn;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Systolic form (default): ONE launch, one workgroup per chase position k (the
// row block J_k(s) = [s + 1 + k b, s + 1 + (k + 1) b) of every sweep s), all
// co-resident. Workgroup k keeps its two blocks in registers for the whole chase:
//   D = A[J_k, J_k] (full, exactly symmetric) and E = A[J_{k+1}, J_k],
// so the matrix never goes back to HBM. Per sweep s it
//   1. receives the reflector of task (s, k) from workgroup k - 1 (k = 0 forms it
//      from column s, which it holds);
//   2. applies it: D <- H D H, E <- E H (row sums in one pass over both blocks);
//   3. forms the reflector of task (s, k + 1) from E's first column and posts it
//      to workgroup k + 1, then applies that reflector from the left to E (the
//      bulge block F of task (s, k + 1) is this E, so its owner updates it);
//   4. posts D's first column and E[0][0] to workgroup k - 1: exactly the row and
//      column that workgroup appends when its window slides by one (workgroup 0
//      keeps them: the finished diagonal d[s + 1] and the column of sweep s + 1);
//   5. slides its own window: drops logical row/column 0, appends the message of
//      workgroup k + 1. Indices are circular (physical = (logical + s) mod b), so
//      sliding moves no data.
// Tasks (s, k) run at about (2 s + k) hand-off steps instead of the 3 s + k
// wavefront launches of chase_apply_kernel. Same Householder arithmetic (LAPACK
// dlarfg, H D H in the symmetric rank-2 form); sums are taken in another order, so
// the tridiagonal agrees with the launch form to rounding, not bit for bit.
// Hand-offs (the guide's handoff-1to1 row: data-tagged granules, no flag): every
// double goes as two naturally aligned 8-byte granules {32 data bits, 32-bit tag
// = sweep + 1}, each written by ONE sc1 store; a consumer thread polls its value's
// two granules with sc1 loads until both carry the tag (bounded; a timeout sets
// *err, every workgroup leaves and the host reruns the launch form), then the
// workgroup barrier. Slots are double-buffered by sweep parity: a producer
// reusing slot s & 1 at sweep s + 2 has received data its consumer sent after
// reading sweep s's slot, and the tag tells a fresh slot from a stale one.
// ---------------------------------------------------------------------------
constexpr int CMSG = 136;   // message stride in values: 128 + 1 scalar (padded)

__device__ __forceinline__ void put_granules(unsigned long long* p, double v, unsigned tag) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned long long t = (unsigned long long)tag << 32;
  __hip_atomic_store(p, t | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(p + 1, t | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool get_granules(const unsigned long long* p, unsigned tag, int* err,
                                             unsigned spin_limit, double& v) {
  unsigned spins = 0;
  for (;;) {
    const unsigned long long a =
        __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long b =
        __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(a >> 32) == tag && (unsigned)(b >> 32) == tag) {
      v = __longlong_as_double((long long)(((b & 0xffffffffull) << 32) | (a & 0xffffffffull)));
      return true;
    }
    __builtin_amdgcn_s_sleep(1);
    if (++spins > spin_limit ||
        ((spins & 1023u) == 0 &&
         __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
}

// LAPACK dlarfg on x (x0 first, nb2 = sum of the other squares)
__device__ __forceinline__ void chase_dlarfg(double x0, double nb2, double& tau, double& beta,
                                             double& scale) {
  tau = 0.0;
  beta = x0;
  scale = 0.0;
  if (nb2 > 0.0) {
    const double nrm = sqrt(x0 * x0 + nb2);
    beta = x0 >= 0.0 ? -nrm : nrm;
    tau = (beta - x0) / beta;
    scale = 1.0 / (x0 - beta);
  }
}

// w_i = p_i - (tau / 2)(v.p) v_i, every operation rounded on its own: the row and
// the column side of D's update see bitwise the same w_i (D stays symmetric)
__device__ __forceinline__ double chase_w(double tau, double sp, double hvp, double v) {
#pragma clang fp contract(off)
  return tau * sp - hvp * v;
}

// d - (a b + c e), every operation rounded on its own
__device__ __forceinline__ double chase_dsub(double d, double a, double b, double c, double e) {
#pragma clang fp contract(off)
  return d - (a * b + c * e);
}

constexpr int SCT = CHASE_THREADS;        // systolic chase workgroup (gpmi_band.h)
constexpr int SNW = SCT / 64;             // waves
constexpr int SRW = CB / SNW;             // rows per thread

static_assert(SRW % 8 == 0, "row sums go through 8-row butterflies");

// fixed-order sum of one value per wave
__device__ __forceinline__ double wave_sum_n(const double* r) {
  double a = 0.0;
#pragma unroll
  for (int q = 0; q < SNW; ++q) a += r[q];
  return a;
}

__device__ __forceinline__ double block_sum_n(double v, double* red) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return wave_sum_n(red);
}

// GPMI_CHASE_PROF builds: workgroups 1-4 stamp the wall clock (100 MHz) at 8
// points of sweeps 1000-1015 into the words after *err (tools/eig_timing.py)
#ifdef GPMI_CHASE_PROF
#define CHASE_STAMP(p)                                                                   \
  if (tid == 0 && k >= 1 && k <= 4 && s >= 1000 && s < 1016)                          \
    reinterpret_cast<long long*>(err + 16)[((k - 1) * 16 + (s - 1000)) * 8 + (p)] =      \
        wall_clock64();
#else
#define CHASE_STAMP(p)
#endif

// Cross-lane steps of the systolic kernel on the VALU (DPP, permlane swaps)
// instead of LDS permutes: the row sums sit on the hand-off path.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
constexpr int DPP_QUAD_XOR1 = 0xB1;    // quad_perm [1, 0, 3, 2]
constexpr int DPP_QUAD_MIRROR = 0x1B;  // quad_perm [3, 2, 1, 0]
constexpr int DPP_ROW_MIRROR = 0x140;
constexpr int DPP_ROW_HALF_MIRROR = 0x141;
constexpr int DPP_ROW_ROR8 = 0x128;

// v_permlane{32,16}_swap on both halves of a double pair: afterwards a + b holds, in
// the lanes with that lane bit clear, the pair sums of a, and where it is set, of b
template <int W>
__device__ __forceinline__ double swap_add(double a, double b) {
  const long long A = __double_as_longlong(a), B = __double_as_longlong(b);
  unsigned lo0, lo1, hi0, hi1;
  if constexpr (W == 32) {
    const auto l = __builtin_amdgcn_permlane32_swap((unsigned)A, (unsigned)B, false, false);
    const auto h =
        __builtin_amdgcn_permlane32_swap((unsigned)(A >> 32), (unsigned)(B >> 32), false, false);
    lo0 = l[0]; lo1 = l[1]; hi0 = h[0]; hi1 = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane16_swap((unsigned)A, (unsigned)B, false, false);
    const auto h =
        __builtin_amdgcn_permlane16_swap((unsigned)(A >> 32), (unsigned)(B >> 32), false, false);
    lo0 = l[0]; lo1 = l[1]; hi0 = h[0]; hi1 = h[1];
  }
  const double x = __longlong_as_double((long long)(((unsigned long long)hi0 << 32) | lo0));
  const double y = __longlong_as_double((long long)(((unsigned long long)hi1 << 32) | lo1));
  return x + y;
}

// butterfly8 on the VALU: every lane gets the 64-lane sum of value (lane >> 3) & 7
__device__ __forceinline__ double butterfly8_valu(double (&v)[8]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = swap_add<32>(v[q], v[q + 4]);
#pragma unroll
  for (int q = 0; q < 2; ++q) v[q] = swap_add<16>(v[q], v[q + 2]);
  const bool up = (lane & 8) != 0;
  double r = (up ? v[1] : v[0]) + dpp_d<DPP_ROW_MIRROR>(up ? v[0] : v[1]);
  r += dpp_d<DPP_ROW_HALF_MIRROR>(r);
  r += dpp_d<DPP_QUAD_MIRROR>(r);
  r += dpp_d<DPP_QUAD_XOR1>(r);
  return r;
}

// sum over the lanes (lane & 7) == 0 (others hold 0), in lane 0 (and every lane)
__device__ __forceinline__ double group_lead_sum(double t) {
  t = swap_add<32>(t, t);
  t = swap_add<16>(t, t);
  return t + dpp_d<DPP_ROW_ROR8>(t);
}

__device__ __forceinline__ double readlane_dbl(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__global__ __launch_bounds__(SCT) void chase_systolic_kernel(
    const double* __restrict__ Ab, int64_t lda, int n, unsigned long long* __restrict__ msg_r,
    unsigned long long* __restrict__ msg_c, int* __restrict__ err, unsigned spin_limit,
    double* __restrict__ dout, double* __restrict__ e2out) {
  __shared__ double sv[CB], sv2[CB], sp[CB], sx[CB], scol[CB], serow[CB], snew[CB + 1];
  __shared__ double xk0[CB];
  __shared__ double cpart[SNW][CB];
  __shared__ double red[SNW], redp[SNW], rednb[SNW], redx[SNW];
  __shared__ double sscal[4];
  __shared__ int s_bail;
  constexpr int M = CB - 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c0 = 2 * lane;
  const int k = blockIdx.x;
  const int rb = 1 + k * CB;                      // first row of J_k(0)
  const int s_end = min(n - 3, n - 2 - k * CB);   // last sweep this position works in
  // thread: physical rows SNW u + w (u < SRW), physical columns c0, c0 + 1
  d2 D[SRW], E[SRW];
#pragma unroll
  for (int u = 0; u < SRW; ++u) {
    const int i = SNW * u + w;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = rb + i, c = rb + c0 + j;
      D[u][j] = (r < n && c < n) ? Ab[(int64_t)max(r, c) * lda + min(r, c)] : 0.0;
      const int re = r + CB;   // E = A[J_{k+1}, J_k]: band part only (re - c <= b)
      E[u][j] = (re < n && c < n && re - c <= CB) ? Ab[(int64_t)re * lda + c] : 0.0;
    }
  }
  if (tid == 0) s_bail = 0;
  if (k == 0) {
    // the reflector of sweep 0 from column 0; later sweeps' are formed one sweep
    // ahead (step 4), off the hand-off path
    const double xi = (tid < CB && 1 + tid < n) ? Ab[(int64_t)(1 + tid) * lda] : 0.0;
    if (tid == 0) sscal[1] = xi;
    const double nb2 = block_sum_n((tid > 0 && tid < CB) ? xi * xi : 0.0, red);
    double tau0, beta0, sc0;
    chase_dlarfg(sscal[1], nb2, tau0, beta0, sc0);
    if (tid < CB) sv[tid] = (tid == 0) ? 1.0 : xi * sc0;
    if (tid == 0) {
      sscal[0] = tau0;
      dout[0] = Ab[0];
      e2out[0] = beta0 * beta0;
    }
  }
  __syncthreads();
  for (int s = 0; s <= s_end; ++s) {
    const int off = s & M;
    const int uo = off / SNW, wo = off % SNW, lo = off >> 1, jo = off & 1;
    const bool nxt = s + 1 + (k + 1) * CB < n;   // position k + 1 works in sweep s
    // ---- 1. the reflector of task (s, k) (physical order in sv, tau in sscal[0])
    CHASE_STAMP(0)
    if (k != 0) {
      if (tid <= CB) {
        const unsigned long long* m = msg_r + ((int64_t)k * 2 + (s & 1)) * (2 * CMSG);
        double v = 0.0;
        if (!get_granules(m + 2 * tid, (unsigned)(s + 1), err, spin_limit, v)) s_bail = 1;
        if (tid < CB) sv[(tid + off) & M] = v;
        else sscal[0] = v;
      }
      __syncthreads();
      if (s_bail) return;
    }
    CHASE_STAMP(1)
    const double tau = sscal[0];
    const double vc0 = sv[c0], vc1 = sv[c0 + 1];
    // ---- 2. row sums D v, E v (one pass); v.(D v) per wave; lane lo of every
    //      wave forms E's updated first column x' = E[:, 0] - tau (E v) and keeps
    //      D's first column; one barrier
    constexpr int NH = SRW / 8;   // 8-row halves per thread
    double qrow[NH];
    {
      double prow[NH];
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        double rowv[8];
#pragma unroll
        for (int uu = 0; uu < 8; ++uu)
          rowv[uu] = D[8 * h + uu][0] * vc0 + D[8 * h + uu][1] * vc1;
        prow[h] = butterfly8_valu(rowv);
#pragma unroll
        for (int uu = 0; uu < 8; ++uu)
          rowv[uu] = E[8 * h + uu][0] * vc0 + E[8 * h + uu][1] * vc1;
        qrow[h] = butterfly8_valu(rowv);
      }
      double vpw = 0.0;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const int rr = SNW * (8 * h + ((lane >> 3) & 7)) + w;   // row of this lane's sums
        if ((lane & 7) == 0) {
          vpw += prow[h] * sv[rr];
          sp[rr] = prow[h];
        }
      }
      vpw = group_lead_sum(vpw);
      if (lane == 0) redp[w] = vpw;
    }
    // E's updated first column x' = E[:, 0] - tau (E v) (v_0 = 1; the row sums are
    // wave-uniform by readlane) and D's first column, from lane lo of every wave;
    // the sum of squares over all rows (row off's square is taken out after the
    // barrier)
    if (lane == lo) {
      double part = 0.0;
      if (jo) {
#pragma unroll
        for (int u = 0; u < SRW; ++u) {
          const int r = SNW * u + w;
          const double x = E[u][1] - (tau * readlane_dbl(qrow[u >> 3], 8 * (u & 7))) * vc1;
          sx[r] = x;
          scol[r] = D[u][1];
          part += x * x;
        }
      } else {
#pragma unroll
        for (int u = 0; u < SRW; ++u) {
          const int r = SNW * u + w;
          const double x = E[u][0] - (tau * readlane_dbl(qrow[u >> 3], 8 * (u & 7))) * vc0;
          sx[r] = x;
          scol[r] = D[u][0];
          part += x * x;
        }
      }
      rednb[w] = part;
    }
    __syncthreads();
    CHASE_STAMP(2)
    // ---- 3. post: the reflector of task (s, k + 1) to position k + 1, D's first
    //      column (after H D H) and E[0][0] to position k - 1 (position 0 keeps
    //      them: the finished diagonal and the column of sweep s + 1)
    const double hvp = 0.5 * tau * (tau * wave_sum_n(redp));
    double taun = 0.0, betan = 0.0, scn = 0.0;
    if (nxt) {
      const double x0 = sx[off];
      chase_dlarfg(x0, fmax(wave_sum_n(rednb) - x0 * x0, 0.0), taun, betan, scn);
      unsigned long long* m = msg_r + ((int64_t)(k + 1) * 2 + (s & 1)) * (2 * CMSG);
      if (tid < CB) put_granules(m + 2 * tid, (tid == 0) ? 1.0 : sx[(tid + off) & M] * scn,
                                 (unsigned)(s + 1));
      else if (tid == CB) put_granules(m + 2 * CB, taun, (unsigned)(s + 1));
    }
    const double e00 = nxt ? betan : 0.0;   // E[0][0] after the left update of step 4
    // D[r][0] after H D H (physical column off); the value the update below gives
    auto dcol = [&](int r) {
      if (tau == 0.0) return scol[r];
      const double vr = sv[r], wr = chase_w(tau, sp[r], hvp, vr);
      const double wo_ = chase_w(tau, sp[off], hvp, sv[off]);
      return chase_dsub(scol[r], vr, wo_, wr, sv[off]);
    };
    double xn = 0.0;   // k = 0: this thread's entry of the next sweep's column
    if (k >= 1) {
      const int t2 = tid - 256;
      unsigned long long* m = msg_c + ((int64_t)k * 2 + (s & 1)) * (2 * CMSG);
      if (t2 >= 0 && t2 < CB) put_granules(m + 2 * t2, dcol((t2 + off) & M), (unsigned)(s + 1));
      else if (t2 == CB) put_granules(m + 2 * CB, e00, (unsigned)(s + 1));
    } else {
      if (tid < CB) {
        const double dv = dcol(tid);
        if (tid == off) {
          dout[s + 1] = dv;
        } else {
          xk0[(tid - off - 1) & M] = dv;
          xn = dv;
        }
        if (s == n - 3 && tid == ((off + 1) & M)) {   // last sweep: trailing 2 x 2 block
          e2out[n - 2] = dv * dv;
          e2out[n - 1] = 0.0;
        }
      } else if (tid == CB) {
        xk0[M] = e00;
        xn = e00;
      }
    }
    if (nxt && tid < CB) sv2[tid] = (tid == off) ? 1.0 : sx[tid] * scn;
    CHASE_STAMP(3)
    // ---- 4. D <- H D H, E <- E H (registers), then E <- H' E
    if (tau != 0.0) {
      const double wc0 = chase_w(tau, sp[c0], hvp, vc0), wc1 = chase_w(tau, sp[c0 + 1], hvp, vc1);
#pragma unroll
      for (int u = 0; u < SRW; ++u) {
        const int r = SNW * u + w;
        const double vr = sv[r], wr = chase_w(tau, sp[r], hvp, vr);
        {
          // both products rounded, then summed (commutative): D stays exactly symmetric
#pragma clang fp contract(off)
          D[u][0] = D[u][0] - (vr * wc0 + wr * vc0);
          D[u][1] = D[u][1] - (vr * wc1 + wr * vc1);
        }
        const double qr = tau * readlane_dbl(qrow[u >> 3], 8 * (u & 7));
        E[u][0] = E[u][0] - qr * vc0;
        E[u][1] = E[u][1] - qr * vc1;
      }
    }
    if (k == 0) {
      if (s == n - 3) {
        const int o1 = (off + 1) & M;
        if (w == (o1 % SNW) && lane == (o1 >> 1)) {
#pragma unroll
          for (int u = 0; u < SRW; ++u)
            if (u == o1 / SNW) dout[n - 1] = (o1 & 1) ? D[u][1] : D[u][0];
        }
      }
      // sum of squares of the next column below its first entry
      const int idx = (tid < CB) ? ((tid - off - 1) & M) : M;
      double x2 = (tid <= CB && tid != off && idx >= 1) ? xn * xn : 0.0;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) x2 += __shfl_xor(x2, o);
      if (lane == 0) redx[w] = x2;
    }
    __syncthreads();   // sv2, xk0 / redx
    CHASE_STAMP(4)
    if (nxt && taun != 0.0) {
      double cp0 = 0.0, cp1 = 0.0;
#pragma unroll
      for (int u = 0; u < SRW; ++u) {
        const double vr = sv2[SNW * u + w];
        cp0 += E[u][0] * vr;
        cp1 += E[u][1] * vr;
      }
      cpart[w][c0] = cp0;
      cpart[w][c0 + 1] = cp1;
      __syncthreads();
      double r0s = 0.0, r1s = 0.0;
#pragma unroll
      for (int q = 0; q < SNW; ++q) {
        r0s += cpart[q][c0];
        r1s += cpart[q][c0 + 1];
      }
      r0s *= taun;
      r1s *= taun;
#pragma unroll
      for (int u = 0; u < SRW; ++u) {
        const int r = SNW * u + w;
        const double vr = sv2[r];
        E[u][0] = (c0 == off) ? (r == off ? betan : 0.0) : E[u][0] - vr * r0s;
        E[u][1] = (c0 + 1 == off) ? (r == off ? betan : 0.0) : E[u][1] - vr * r1s;
      }
    }
    if (k == 0 && s < s_end) {
      // the reflector of sweep s + 1 (its column is final now), into sv / sscal[0]
      double tn, bn, scl;
      chase_dlarfg(xk0[0], wave_sum_n(redx), tn, bn, scl);
      if (tid < CB) sv[(tid + off + 1) & M] = (tid == 0) ? 1.0 : xk0[tid] * scl;
      if (tid == 0) {
        sscal[0] = tn;
        e2out[s + 1] = bn * bn;
      }
    }
    // ---- 5. slide the window: physical row / column off becomes logical b - 1
    CHASE_STAMP(5)
    if (w == wo) {
#pragma unroll
      for (int u = 0; u < SRW; ++u)
        if (u == uo) {
          serow[c0] = E[u][0];
          serow[c0 + 1] = E[u][1];
        }
    }
    if (tid <= CB) {
      double v = 0.0;
      if (nxt) {
        const unsigned long long* m = msg_c + ((int64_t)(k + 1) * 2 + (s & 1)) * (2 * CMSG);
        if (!get_granules(m + 2 * tid, (unsigned)(s + 1), err, spin_limit, v)) s_bail = 1;
      }
      if (tid < CB) snew[tid] = v;
      else sscal[3] = v;
    }
    __syncthreads();
    if (s_bail) return;
    CHASE_STAMP(6)
    const double d00 = snew[0], ne00 = sscal[3];
    if (w == wo) {   // row off: D's from E's old first row, E's (0 ... 0, ne00)
#pragma unroll
      for (int u = 0; u < SRW; ++u)
        if (u == uo) {
          D[u][0] = (c0 == off) ? d00 : serow[c0];
          D[u][1] = (c0 + 1 == off) ? d00 : serow[c0 + 1];
          E[u][0] = (c0 == off) ? ne00 : 0.0;
          E[u][1] = (c0 + 1 == off) ? ne00 : 0.0;
        }
    }
    if (lane == lo) {   // column off below / above row off
#pragma unroll
      for (int u = 0; u < SRW; ++u) {
        const int r = SNW * u + w;
        if (r != off) {
          const double dn = serow[r], en = snew[((r - off - 1) & M) + 1];
          if (jo) {
            D[u][1] = dn;
            E[u][1] = en;
          } else {
            D[u][0] = dn;
            E[u][0] = en;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Split systolic chase (default where 2K workgroups fit): every chase position
// has a D workgroup (D_k) and an E workgroup (E_k), so each sweep's products
// pass (D v, E v) runs on two CUs at once and the per-sweep loop
// E(k) -> D(k+1) / E(k+1) -> E(k) carries one block's products per hop instead
// of two. Messages (tagged granules, slots by sweep parity):
//   R[k]    reflector (s, k) + tau: from E(k-1), for k = 0 from D(0); read by E(k), D(k)
//   Dcol[k] D(k)'s first column after H D H: read by E(k-1) (its new last column)
//           and D(k-1) (entry 0: its new diagonal entry)
//   Erow[k] E(k)'s first row after both updates (physical order): read by D(k)
//   E00[k]  E(k)[0][0] = beta': read by E(k-1), for k = 0 by D(0) (the last entry
//           of the next sweep's column)
// (host prototype of the protocol: tools/chase_systolic_proto.py, chase_split)
// ---------------------------------------------------------------------------
// fixed-order sums over the NW waves of a workgroup (templated on NW)
template <int NW>
__device__ __forceinline__ double wave_sum_t(const double* r) {
  double a = 0.0;
#pragma unroll
  for (int q = 0; q < NW; ++q) a += r[q];
  return a;
}
template <int NW>
__device__ __forceinline__ double block_sum_t(double v, double* red) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return wave_sum_t<NW>(red);
}

template <int T>
__device__ __forceinline__ void chase_split_body(
    const double* __restrict__ Ab, int64_t lda, int n, unsigned long long* __restrict__ msg,
    int K, int* __restrict__ err, unsigned spin_limit, double* __restrict__ dout,
    double* __restrict__ e2out) {
  constexpr int NW = T / 64, RW = CB / NW;
  static_assert(RW % 8 == 0, "row sums go through 8-row butterflies");
  __shared__ double sv[CB], sv2[CB], sp[CB], sx[CB], serow[CB], snew[CB + 1];
  __shared__ double xk0[CB];
  __shared__ double cpart[NW][CB];
  __shared__ double red[NW], redp[NW], rednb[NW];
  __shared__ double sscal[4];
  __shared__ int s_bail;
  constexpr int M = CB - 1;
  constexpr size_t SLOTS = 2 * (size_t)(2 * CMSG);   // per position: 2 parities x granules
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c0 = 2 * lane;
  const bool isD = blockIdx.x >= (unsigned)K;
#ifdef GPMI_CHASE_PROF
  // positions 2 and 3, both roles: rows q = 2 (k - 2) + isD of the stamp table
#define SPLIT_STAMP(p)                                                                   \
  if (tid == 0 && (k == 2 || k == 3) && s >= 1000 && s < 1016)                          \
    reinterpret_cast<long long*>(err + 16)[((2 * (k - 2) + (isD ? 1 : 0)) * 16 + (s - 1000)) * 8 + \
                                          (p)] = wall_clock64();
#else
#define SPLIT_STAMP(p)
#endif
  const int k = isD ? (int)blockIdx.x - K : (int)blockIdx.x;
  unsigned long long* mR = msg;                                  // [K + 1] positions
  unsigned long long* mDcol = mR + (size_t)(K + 1) * SLOTS;
  unsigned long long* mErow = mDcol + (size_t)(K + 1) * SLOTS;
  unsigned long long* mE00 = mErow + (size_t)(K + 1) * SLOTS;
  auto slot = [&](unsigned long long* base, int pos, int s) {
    return base + (size_t)pos * SLOTS + (size_t)(s & 1) * (2 * CMSG);
  };
  const int rb = 1 + k * CB;
  const int s_end = min(n - 3, n - 2 - k * CB);
  d2 Bk[RW];   // this workgroup's block: D_k or E_k
#pragma unroll
  for (int u = 0; u < RW; ++u) {
    const int i = NW * u + w;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = rb + i, c = rb + c0 + j;
      if (isD) {
        Bk[u][j] = (r < n && c < n) ? Ab[(int64_t)max(r, c) * lda + min(r, c)] : 0.0;
      } else {
        const int re = r + CB;
        Bk[u][j] = (re < n && c < n && re - c <= CB) ? Ab[(int64_t)re * lda + c] : 0.0;
      }
    }
  }
  if (tid == 0) s_bail = 0;
  if (isD && k == 0) {
    if (tid < CB) xk0[tid] = (1 + tid < n) ? Ab[(int64_t)(1 + tid) * lda] : 0.0;
    if (tid == 0) dout[0] = Ab[0];
  }
  __syncthreads();
  for (int s = 0; s <= s_end; ++s) {
    const int off = s & M;
    const int uo = off / NW, wo = off % NW, lo = off >> 1, jo = off & 1;
    const bool nxt = s + 1 + (k + 1) * CB < n;
    const unsigned tag = (unsigned)(s + 1);
    SPLIT_STAMP(0)
    // ---- 1. the reflector of task (s, k) into sv, tau into sscal[0]
    if (isD && k == 0) {
      const double xi = (tid < CB) ? xk0[tid] : 0.0;
      const double x0 = xk0[0];
      const double nb2 = block_sum_t<NW>((tid > 0 && tid < CB) ? xi * xi : 0.0, red);
      double tau0, beta0, sc0;
      chase_dlarfg(x0, nb2, tau0, beta0, sc0);
      const double vi = (tid == 0) ? 1.0 : xi * sc0;
      if (tid < CB) {
        sv[(tid + off) & M] = vi;
        put_granules(slot(mR, 0, s) + 2 * tid, vi, tag);
      } else if (tid == CB) {
        put_granules(slot(mR, 0, s) + 2 * CB, tau0, tag);
        sscal[0] = tau0;
      }
      if (tid == 0) e2out[s] = beta0 * beta0;
    } else {
      if (tid <= CB) {
        double v = 0.0;
        if (!get_granules(slot(mR, k, s) + 2 * tid, tag, err, spin_limit, v)) s_bail = 1;
        if (tid < CB) sv[(tid + off) & M] = v;
        else sscal[0] = v;
      }
    }
    __syncthreads();
    if (s_bail) return;
    SPLIT_STAMP(1)
    const double tau = sscal[0];
    const double vc0 = sv[c0], vc1 = sv[c0 + 1];
    // ---- 2. row sums B v (one block) and, for D, v.(D v) per wave
    constexpr int NH = RW / 8;
    double qrow[NH];
    {
      double vpw = 0.0;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        double rowv[8];
#pragma unroll
        for (int uu = 0; uu < 8; ++uu)
          rowv[uu] = Bk[8 * h + uu][0] * vc0 + Bk[8 * h + uu][1] * vc1;
        qrow[h] = butterfly8_valu(rowv);
        const int rr = NW * (8 * h + ((lane >> 3) & 7)) + w;
        if ((lane & 7) == 0) {
          vpw += qrow[h] * sv[rr];
          sp[rr] = qrow[h];
        }
      }
      if (isD) {
        vpw = group_lead_sum(vpw);
        if (lane == 0) redp[w] = vpw;
      }
    }
    if (!isD && lane == lo) {   // E's updated first column x' and its sum of squares
      double part = 0.0;
      if (jo) {
#pragma unroll
        for (int u = 0; u < RW; ++u) {
          const double x = Bk[u][1] - (tau * readlane_dbl(qrow[u >> 3], 8 * (u & 7))) * vc1;
          sx[NW * u + w] = x;
          part += x * x;
        }
      } else {
#pragma unroll
        for (int u = 0; u < RW; ++u) {
          const double x = Bk[u][0] - (tau * readlane_dbl(qrow[u >> 3], 8 * (u & 7))) * vc0;
          sx[NW * u + w] = x;
          part += x * x;
        }
      }
      rednb[w] = part;
    }
    if (isD && lane == lo) {    // D's first column before the update
#pragma unroll
      for (int u = 0; u < RW; ++u) sx[NW * u + w] = jo ? Bk[u][1] : Bk[u][0];
    }
    __syncthreads();
    SPLIT_STAMP(2)
    if (isD) {
      // ---- 3D. post D's first column after H D H; position 0 keeps it
      const double hvp = 0.5 * tau * (tau * wave_sum_t<NW>(redp));
      auto dcol = [&](int r) {
        if (tau == 0.0) return sx[r];
        const double vr = sv[r], wr = chase_w(tau, sp[r], hvp, vr);
        const double wo_ = chase_w(tau, sp[off], hvp, sv[off]);
        return chase_dsub(sx[r], vr, wo_, wr, sv[off]);
      };
      if (k >= 1) {
        if (tid < CB) put_granules(slot(mDcol, k, s) + 2 * tid, dcol((tid + off) & M), tag);
      } else if (tid < CB) {
        const double dv = dcol(tid);
        if (tid == off) dout[s + 1] = dv;
        else xk0[(tid - off - 1) & M] = dv;
        if (s == n - 3 && tid == ((off + 1) & M)) {
          e2out[n - 2] = dv * dv;
          e2out[n - 1] = 0.0;
        }
      }
      SPLIT_STAMP(3)
      // ---- 4D. D <- H D H
      if (tau != 0.0) {
        const double wc0 = chase_w(tau, sp[c0], hvp, vc0), wc1 = chase_w(tau, sp[c0 + 1], hvp, vc1);
#pragma unroll
        for (int u = 0; u < RW; ++u) {
          const int r = NW * u + w;
          const double vr = sv[r], wr = chase_w(tau, sp[r], hvp, vr);
          Bk[u][0] = chase_dsub(Bk[u][0], vr, wc0, wr, vc0);
          Bk[u][1] = chase_dsub(Bk[u][1], vr, wc1, wr, vc1);
        }
      }
      if (k == 0 && s == n - 3) {
        const int o1 = (off + 1) & M;
        if (w == (o1 % NW) && lane == (o1 >> 1)) {
#pragma unroll
          for (int u = 0; u < RW; ++u)
            if (u == o1 / NW) dout[n - 1] = (o1 & 1) ? Bk[u][1] : Bk[u][0];
        }
      }
      SPLIT_STAMP(4)
      SPLIT_STAMP(5)
      // ---- 5D. slide: E(k)'s first row (and for position 0 the next column's
      //      last entry), D(k+1)'s diagonal entry
      if (tid < CB) {
        double v = 0.0;
        if (!get_granules(slot(mErow, k, s) + 2 * tid, tag, err, spin_limit, v)) s_bail = 1;
        serow[tid] = v;
      } else if (tid == CB) {
        double v = 0.0;
        if (nxt && !get_granules(slot(mDcol, k + 1, s), tag, err, spin_limit, v)) s_bail = 1;
        sscal[3] = v;
      } else if (tid == CB + 1 && k == 0) {
        double v = 0.0;
        if (!get_granules(slot(mE00, 0, s), tag, err, spin_limit, v)) s_bail = 1;
        xk0[M] = v;
      }
      __syncthreads();
      if (s_bail) return;
      SPLIT_STAMP(6)
      const double d00 = sscal[3];
      if (lane == lo) {   // column off (every row; (off, off) is rewritten below)
        if (jo) {
#pragma unroll
          for (int u = 0; u < RW; ++u) Bk[u][1] = serow[NW * u + w];
        } else {
#pragma unroll
          for (int u = 0; u < RW; ++u) Bk[u][0] = serow[NW * u + w];
        }
      }
      if (w == wo) {
#pragma unroll
        for (int u = 0; u < RW; ++u)
          if (u == uo) {
            Bk[u][0] = (c0 == off) ? d00 : serow[c0];
            Bk[u][1] = (c0 + 1 == off) ? d00 : serow[c0 + 1];
          }
      }
    } else {
      // ---- 3E. the reflector of task (s, k + 1): post it and beta' (E00)
      double taun = 0.0, betan = 0.0, scn = 0.0;
      if (nxt) {
        const double x0 = sx[off];
        chase_dlarfg(x0, fmax(wave_sum_t<NW>(rednb) - x0 * x0, 0.0), taun, betan, scn);
        if (tid < CB) {
          sv2[tid] = (tid == off) ? 1.0 : sx[tid] * scn;
          put_granules(slot(mR, k + 1, s) + 2 * tid,
                       (tid == 0) ? 1.0 : sx[(tid + off) & M] * scn, tag);
        } else if (tid == CB) {
          put_granules(slot(mR, k + 1, s) + 2 * CB, taun, tag);
        }
      }
      if (tid == 256) put_granules(slot(mE00, k, s), nxt ? betan : 0.0, tag);
      SPLIT_STAMP(3)
      // ---- 4E. E <- E H, then E <- H' E (column off -> (beta', 0 ...))
      if (tau != 0.0) {
#pragma unroll
        for (int u = 0; u < RW; ++u) {
          const double qr = tau * readlane_dbl(qrow[u >> 3], 8 * (u & 7));
          Bk[u][0] = Bk[u][0] - qr * vc0;
          Bk[u][1] = Bk[u][1] - qr * vc1;
        }
      }
      __syncthreads();   // sv2
      SPLIT_STAMP(4)
      if (nxt && taun != 0.0) {
        double cp0 = 0.0, cp1 = 0.0;
#pragma unroll
        for (int u = 0; u < RW; ++u) {
          const double vr = sv2[NW * u + w];
          cp0 += Bk[u][0] * vr;
          cp1 += Bk[u][1] * vr;
        }
        cpart[w][c0] = cp0;
        cpart[w][c0 + 1] = cp1;
        __syncthreads();
        double r0s = 0.0, r1s = 0.0;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          r0s += cpart[q][c0];
          r1s += cpart[q][c0 + 1];
        }
        r0s *= taun;
        r1s *= taun;
#pragma unroll
        for (int u = 0; u < RW; ++u) {
          const int r = NW * u + w;
          const double vr = sv2[r];
          Bk[u][0] = (c0 == off) ? (r == off ? betan : 0.0) : Bk[u][0] - vr * r0s;
          Bk[u][1] = (c0 + 1 == off) ? (r == off ? betan : 0.0) : Bk[u][1] - vr * r1s;
          if (u == uo && w == wo) {   // row off is final: D(k) may slide
            put_granules(slot(mErow, k, s) + 2 * c0, Bk[u][0], tag);
            put_granules(slot(mErow, k, s) + 2 * (c0 + 1), Bk[u][1], tag);
          }
        }
      } else if (w == wo) {
#pragma unroll
        for (int u = 0; u < RW; ++u)
          if (u == uo) {
            put_granules(slot(mErow, k, s) + 2 * c0, Bk[u][0], tag);
            put_granules(slot(mErow, k, s) + 2 * (c0 + 1), Bk[u][1], tag);
          }
      }
      SPLIT_STAMP(5)
      // ---- 5E. slide with D(k+1)'s first column (stored by physical row: entry
      //      i >= 1 becomes row (i + off) mod b of column off) and E(k+1)'s beta'
      if (tid <= CB) {
        double v = 0.0;
        if (nxt) {
          unsigned long long* src = tid < CB ? slot(mDcol, k + 1, s) + 2 * tid
                                             : slot(mE00, k + 1, s);
          if (!get_granules(src, tag, err, spin_limit, v)) s_bail = 1;
        }
        if (tid == CB) sscal[3] = v;
        else if (tid > 0) snew[(tid + off) & M] = v;
      }
      __syncthreads();
      if (s_bail) return;
      SPLIT_STAMP(6)
      const double ne00 = sscal[3];
      // column off (every row; (off, off) is rewritten by the row below), then row off
      if (lane == lo) {
        if (jo) {
#pragma unroll
          for (int u = 0; u < RW; ++u) Bk[u][1] = snew[NW * u + w];
        } else {
#pragma unroll
          for (int u = 0; u < RW; ++u) Bk[u][0] = snew[NW * u + w];
        }
      }
      if (w == wo) {
#pragma unroll
        for (int u = 0; u < RW; ++u)
          if (u == uo) {
            Bk[u][0] = (c0 == off) ? ne00 : 0.0;
            Bk[u][1] = (c0 + 1 == off) ? ne00 : 0.0;
          }
      }
    }
  }
}


__global__ __launch_bounds__(CHASE_SPLIT_THREADS) void chase_split_kernel(
    const double* __restrict__ Ab, int64_t lda, int n, unsigned long long* __restrict__ msg,
    int K, int* __restrict__ err, unsigned spin_limit, double* __restrict__ dout,
    double* __restrict__ e2out) {
  chase_split_body<CHASE_SPLIT_THREADS>(Ab, lda, n, msg, K, err, spin_limit, dout, e2out);
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

// Multisection: BG lanes per eigenvalue evaluate the Sturm count at BG interior
// points of its interval at once; the interval shrinks (BG + 1)x per round (a
// bit over 4 bits) instead of 2x, so ~13 sequential counts replace ~52, and
// 16 x n lanes keep the SIMDs busy where n threads left most of them idle.
// The count streams d and e2 in blocks of 8 loaded ahead of the dependent
// pivot chain.
constexpr int BG = BISECT_LANES;

__device__ __forceinline__ int sturm_count_blk(const double* __restrict__ d,
                                               const double* __restrict__ e2, int n, double x,
                                               double pivmin) {
  int cnt = 0;
  double q = d[0] - x;
  if (fabs(q) < pivmin) q = -pivmin;
  cnt += q < 0.0;
  int j = 1;
  for (; j + 8 <= n; j += 8) {
    double dd[8], ee[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      dd[t] = d[j + t];
      ee[t] = e2[j + t - 1];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
#ifdef GPMI_BISECT_FASTDIV
      // e2 / q as e2 * (1 / q): v_rcp_f64 and two Newton steps (a few ulp; the
      // count is the number of negative pivots, insensitive at that level)
      double r = __builtin_amdgcn_rcp(q);
      r = fma(fma(-q, r, 1.0), r, r);
      r = fma(fma(-q, r, 1.0), r, r);
      q = dd[t] - x - ee[t] * r;
#else
      q = dd[t] - x - ee[t] / q;
#endif
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
    }
  }
  for (; j < n; ++j) {
    q = d[j] - x - e2[j - 1] / q;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
  }
  return cnt;
}

__global__ __launch_bounds__(256) void bisect_multi_kernel(const double* __restrict__ d,
                                                           const double* __restrict__ e2, int n,
                                                           double lo0, double hi0, double pivmin,
                                                           double* __restrict__ lam) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int i = t / BG, j = t % BG;
  if (i >= n) return;   // whole groups leave together (BG divides 64)
  double lo = lo0, hi = hi0;
  const double tol = 2.0 * 2.220446049250313e-16 * fmax(fabs(lo0), fabs(hi0)) + pivmin;
  for (int it = 0; it < 64 && hi - lo > tol; ++it) {
    const double wdt = hi - lo;
    const double x = lo + wdt * (double)(j + 1) / (double)(BG + 1);
    const int cnt = sturm_count_blk(d, e2, n, x, pivmin);
    const unsigned long long m = __ballot(cnt > i);
    const unsigned long long gm = (m >> (lane & ~(BG - 1))) & ((2ull << (BG - 1)) - 1ull);
    const int js = gm ? __builtin_ctzll(gm) : BG;   // first point whose count exceeds i
    const double nlo = (js == 0) ? lo : lo + wdt * (double)js / (double)(BG + 1);
    const double nhi = (js == BG) ? hi : lo + wdt * (double)(js + 1) / (double)(BG + 1);
    lo = nlo;
    hi = nhi;
  }
  if (j == 0) lam[i] = 0.5 * (lo + hi);
}

}  // namespace gpmi
