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
