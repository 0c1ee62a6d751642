// C-ABI (include/gpmi.h) and host orchestration of the gpmi kernels.
//
// One gpmi_op = one device-resident correlation matrix K (padded to n_pad, a
// multiple of 128, identity in the pad) plus workspace for max_batch
// concurrent factorizations of K + eta_b I. All work of an op runs in order on
// the op's own HIP stream; the host blocks only when it reads results back.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <array>
#include <map>
#include <vector>

#include "gpmi_internal.h"
#include "gpmi_band.h"
#include "../../include/gpmi.h"

using namespace gpmi;

namespace {

thread_local char g_err[512] = "";

int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess)                                                          \
      return set_err(-(int)e_, "%s failed: %s", #expr, hipGetErrorString(e_));     \
  } while (0)

#define LAUNCH_CHECK(name)                                                         \
  do {                                                                             \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ != hipSuccess)                                                          \
      return set_err(-(int)e_, "launch of %s failed: %s", name,                    \
                     hipGetErrorString(e_));                                       \
  } while (0)

constexpr int TS = GPMI_TS;
constexpr int RLD = GPMI_RHS_LD;
constexpr int OUT_LD = 1 + RLD * RLD;

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

struct gpmi_op {
  int device = 0;
  int64_t n = 0, n_pad = 0;
  int nt = 0;
  int max_batch = 1;
  int outer = 16;                      // outer panel width in 128-column tiles
  hipStream_t stream = nullptr;
  hipStream_t stream3 = nullptr;       // second batch group (groups == 2)
  int groups = 0;                      // 2: the batch runs as two halves on two streams;
                                       // 0: auto (2 for batches of 2..32, 1 above)
  hipEvent_t ev_g = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  bool dry = false;                    // schedule dry run: collect SYRK shapes only
  std::vector<std::pair<int, int>> shapes;
  double* K = nullptr;       // [n_pad][n_pad]
  double* A = nullptr;       // [max_batch][n_pad][n_pad]
  double* R = nullptr;       // [max_batch][n_pad][16]
  double* X = nullptr;       // [max_batch][n_pad][16]
  double* U = nullptr;       // [max_batch][128][16]
  double* Linv = nullptr;    // [max_batch][nt][128][128]
  double* logdiag = nullptr; // [max_batch][nt]
  double* gram = nullptr;    // [max_batch][nt][256]
  double* out = nullptr;     // [max_batch][OUT_LD]
  double* etas = nullptr;    // [max_batch]
  double* rhs_src = nullptr; // [n_pad][16]
  double* scratch = nullptr; // [n_pad][16] (matvec input)
  double* scratch2 = nullptr;// [n_pad][16] (matvec output)
  double* tracebuf = nullptr;// [n_pad][2]
  double* W = nullptr;       // [n_pad][n_pad] L^-T workspace (traceinv, allocated lazily)
  double* tpart = nullptr;   // [nt * (nt + 1) / 2 + nt * nt] traceinv partials
  double* Td = nullptr;      // [nt][128][128] diagonal tiles of A^-1 (traceinv exponent 2)
  int* info = nullptr;       // [max_batch]
  // grouped syrk tile orders, one per trailing-update shape (w, t) of the schedule
  uint32_t* order = nullptr;
  int order_nt = -1, order_outer = -1, group = 8;
  std::map<std::pair<int, int>, int64_t> order_off;
  int nrhs = 0;
  bool has_K = false;
  // factor cache: batch slot 0 holds the factor of K + cached_eta I
  bool cache_valid = false;
  double cached_eta = 0.0;
  uint64_t factor_gen = 0;             // bumped by every factorization
  // traceinv cache (valid for factor generation tinv_gen)
  uint64_t tinv_gen = ~0ull;
  int tinv_have = 0;                   // bit 0: tr(A^-1), bit 1: tr(A^-2)
  double tinv[2] = {0.0, 0.0};
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev;
  hipEvent_t ev_begin = nullptr, ev_end = nullptr;
  double last_syrk_ms = 0.0, last_syrk_flops = 0.0, last_total_ms = 0.0;
  int last_syrk_launches = 0;
  std::vector<std::pair<int, double>> syrk_log;  // (event index, flops)
  std::vector<std::array<int, 3>> syrk_shape;    // (w, t, kdim) per logged launch
  double last_syrk_busy_ms = 0.0;                // union of syrk launch intervals

  BatchPtrs ptrs() const {
    BatchPtrs p;
    p.A = A;
    p.sA = n_pad * n_pad;
    p.R = R;
    p.sR = n_pad * RLD;
    p.U = U;
    p.sU = (int64_t)TS * RLD;
    p.Linv = Linv;
    p.sL = (int64_t)nt * TS * TS;
    p.logdiag = logdiag;
    p.sLD = nt;
    p.gram = gram;
    p.sG = (int64_t)nt * 256;
    p.info = info;
    return p;
  }
};

namespace {

// Lower-triangular tiles of a band (w tile columns over t tile rows) in row
// groups of G rows, column-major inside a group, packed (i << 16) | j. The
// 32 CUs x 2 workgroups in flight on one XCD then cover ~G rows x (64/G)
// columns, so each operand slab is re-read from that XCD's L2, not from the
// Infinity Cache / HBM.
void grouped_order(int w, int t, int G, std::vector<uint32_t>* out) {
  for (int r0 = 0; r0 < t; r0 += G) {
    const int r1 = std::min(t, r0 + G);
    const int jmax = std::min(r1 - 1, w - 1);
    for (int j = 0; j <= jmax; ++j)
      for (int i = std::max(r0, j); i < r1; ++i) out->push_back(((uint32_t)i << 16) | j);
  }
}

int launch_syrk(gpmi_op* op, hipStream_t st, int b0, int nb, int tc0, int w, int t, int p0,
                int kdim, bool from_k = false) {
  // b0: first batch member of the launch (a batch group's offset)
  const int tri = w * (w + 1) / 2;
  const int tiles = tri + (t - w) * w;
  if (tiles <= 0 || nb <= 0) return 0;
  if (op->dry) {
    op->shapes.push_back({w, t});
    return 0;
  }
  int evi = -1;
  if (op->timing) {
    evi = (int)op->syrk_log.size() * 2;
    if ((int)op->ev.size() < evi + 2) {
      for (int k = 0; k < 64; ++k) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, timing_event_flags()));
        op->ev.push_back(e);
      }
    }
    HIP_TRY(hipEventRecord(op->ev[evi], st));
  }
  const uint32_t* order = nullptr;
  if (op->order && w > 1) {
    auto it = op->order_off.find({w, t});
    if (it != op->order_off.end()) order = op->order + it->second;
  }
  hipLaunchKernelGGL(syrk_kernel, dim3(tiles, nb), dim3(256), 0, st,
                     op->A + (int64_t)b0 * op->n_pad * op->n_pad, (int64_t)op->n_pad,
                     op->n_pad * op->n_pad, tc0, w, t, p0, kdim, order,
                     from_k ? op->K : nullptr, op->etas + b0, (int64_t)op->n);
  LAUNCH_CHECK("syrk_kernel");
  if (op->timing) {
    HIP_TRY(hipEventRecord(op->ev[evi + 1], st));
    // algorithmic flops: lower triangle only (diagonal tiles count 128*129/2 entries)
    const double offd = (double)(tiles - std::min(tiles, w)) * TS * TS;
    const double diag = (double)std::min(tiles, w) * TS * (TS + 1) / 2.0;
    const double fl = 2.0 * (offd + diag) * kdim * nb;
    op->syrk_log.push_back({evi, fl});
    op->syrk_shape.push_back({w, t, kdim});
  }
  return 0;
}

// Recursive panel factorization of tile columns [c0, c0 + W) (all contributions
// of columns < c0 already applied): factor the left half, update the right half
// from it (a band SYRK with kdim = half width), factor the right half. A single
// column is the diagonal-block kernel (Cholesky, inverse, fused forward solve,
// logdet / Gram partials) followed by the panel kernel (L_ik and r_i updates).
int factor_panel(gpmi_op* op, const BatchPtrs& P, int b0, int nb, hipStream_t st, int c0,
                 int W) {
  const int nt = op->nt;
  if (W == 1) {
    if (op->dry) return 0;
    hipLaunchKernelGGL(diag_block_kernel, dim3(nb), dim3(256), 0, st, P, (int64_t)op->n_pad,
                       c0, nt);
    LAUNCH_CHECK("diag_block_kernel");
    if (c0 + 1 < nt) {
      hipLaunchKernelGGL(panel_kernel, dim3(nt - c0 - 1, nb), dim3(256), 0, st, P,
                         (int64_t)op->n_pad, c0);
      LAUNCH_CHECK("panel_kernel");
    }
    return 0;
  }
  const int h = W / 2;
  int rc = factor_panel(op, P, b0, nb, st, c0, h);
  if (rc) return rc;
  rc = launch_syrk(op, st, b0, nb, c0 + h, W - h, nt - c0 - h, c0 * TS, h * TS);
  if (rc) return rc;
  return factor_panel(op, P, b0, nb, st, c0 + h, W - h);
}


// The blocked factorization schedule over outer panels P_k of `outer` tile
// columns, in order on one stream: factor P_k (recursive panel factorization), then
// one trailing SYRK over all columns right of it (kdim = 128 * outer). (Round 5
// removed the look-ahead form, the panel chain of P_{k+1} on a second high-priority
// stream beside the bulk update of P_k: at the batch-64 headline 1441.8 against
// 1442.9 ms per 64-eta step, and within +-1 % at 8 and 16 eta in round 3: the batched
// SYRK keeps every CU busy, so the chain beside it gains nothing.)
// P points at batch member b0 (a batch group); `main` replaces op->stream.
int schedule(gpmi_op* op, const BatchPtrs& P, int b0, int nb, hipStream_t main = nullptr) {
  const int nt = op->nt, O = op->outer;
  hipStream_t A = main ? main : op->stream;
  for (int c0 = 0; c0 < nt; c0 += O) {
    const int W = std::min(O, nt - c0);
    int rc = factor_panel(op, P, b0, nb, A, c0, W);
    if (rc) return rc;
    const int c1 = c0 + W;
    if (c1 >= nt) break;
    // the first trailing update reads its C tiles from K (run_factor copies only
    // the first outer panel's tile columns into the members)
    rc = launch_syrk(op, A, b0, nb, c1, nt - c1, nt - c1, c0 * TS, W * TS, c0 == 0);
    if (rc) return rc;
  }
  return 0;
}

// Trailing-update shapes (w, t) the schedule launches, from a dry run.
int ensure_order(gpmi_op* op) {
  if (op->group <= 0) return 0;
  if (op->order && op->order_nt == op->nt && op->order_outer == op->outer &&
      true)
    return 0;
  if (op->order) HIP_TRY(hipFree(op->order));
  op->order = nullptr;
  op->order_off.clear();
  op->dry = true;
  op->shapes.clear();
  BatchPtrs P = op->ptrs();
  int rc = schedule(op, P, 0, 1);
  op->dry = false;
  if (rc) return rc;
  std::vector<uint32_t> h;
  for (auto& wt : op->shapes) {
    if (wt.first < 2 || op->order_off.count(wt)) continue;
    op->order_off[wt] = (int64_t)h.size();
    grouped_order(wt.first, wt.second, op->group, &h);
  }
  if (h.empty()) h.push_back(0);
  HIP_TRY(hipMalloc(&op->order, sizeof(uint32_t) * h.size()));
  HIP_TRY(hipMemcpy(op->order, h.data(), sizeof(uint32_t) * h.size(), hipMemcpyHostToDevice));
  op->order_nt = op->nt;
  op->order_outer = op->outer;
  return 0;
}

BatchPtrs shifted(const BatchPtrs& P, int b0) {
  BatchPtrs q = P;
  q.A += b0 * P.sA;
  q.R += b0 * P.sR;
  q.U += b0 * P.sU;
  q.Linv += b0 * P.sL;
  q.logdiag += b0 * P.sLD;
  q.gram += b0 * P.sG;
  q.info += b0;
  return q;
}

// Factor K + eta_b I for b < nb, with the fused forward substitution of the
// RHS block (copied from rhs_src). Results stay on the device.
int run_factor(gpmi_op* op, const double* etas_host, int nb, const double* rhs_dev) {
  if (!op->has_K) return set_err(-1000, "operator has no matrix (load or assemble first)");
  if (nb < 1 || nb > op->max_batch)
    return set_err(-1001, "batch %d outside [1, %d]", nb, op->max_batch);
  DeviceGuard g(op->device);
  hipStream_t s = op->stream;
  const int nt = op->nt;
  const int64_t lda = op->n_pad;
  BatchPtrs P = op->ptrs();
  {
    int rc = ensure_order(op);
    if (rc) return rc;
  }
  op->syrk_log.clear();
  op->syrk_shape.clear();
  op->cache_valid = false;
  ++op->factor_gen;
  if (op->timing) {
    if (!op->ev_begin) {
      HIP_TRY(hipEventCreateWithFlags(&op->ev_begin, timing_event_flags()));
      HIP_TRY(hipEventCreateWithFlags(&op->ev_end, timing_event_flags()));
    }
    HIP_TRY(hipEventRecord(op->ev_begin, s));
  }
  HIP_TRY(hipMemcpyAsync(op->etas, etas_host, sizeof(double) * nb, hipMemcpyHostToDevice, s));
  // K + eta_b I into the members' tile columns of the first outer panel only; the
  // rest is formed by the first trailing SYRK from K (schedule)
  const int wc = std::min(op->outer, nt);
  hipLaunchKernelGGL(shift_copy_kernel, dim3(wc * (wc + 1) / 2 + (nt - wc) * wc), dim3(256), 0,
                     s, op->K, lda, op->A, lda, P.sA, op->etas, nb, op->n, wc);
  LAUNCH_CHECK("shift_copy_kernel");
  for (int b = 0; b < nb; ++b)
    HIP_TRY(hipMemcpyAsync(op->R + b * P.sR, rhs_dev, sizeof(double) * P.sR,
                           hipMemcpyDeviceToDevice, s));
  HIP_TRY(hipMemsetAsync(op->info, 0, sizeof(int) * nb, s));
  int rc = 0;
  // auto: a small batch (the per-rank block of a strong-scaled curve) keeps more CUs
  // busy with its halves overlapped (batch 8: +2.3 %); a large one is all SYRK
  // already (batch 64: +0.2 %) and keeps one stream (clean per-launch timing)
  const int groups = op->groups ? op->groups : (nb <= 32 ? 2 : 1);
  if (groups == 2 && nb >= 2) {
    // two independent halves of the batch on two streams: one half's
    // latency-bound diagonal-block / panel kernels run beside the other's SYRK.
    // Only batched callers (nb >= 2) get here, and the one batched caller,
    // gpmi_op_loglik_batch, releases stream3 after its synchronisation
    // (the single-eta factor calls never create it)
    const int h = nb / 2;
    if (!op->stream3) {
      HIP_TRY(hipStreamCreateWithFlags(&op->stream3, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&op->ev_g, sync_event_flags()));
    }
    HIP_TRY(hipEventRecord(op->ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(op->stream3, op->ev_fork, 0));
    if ((rc = schedule(op, P, 0, h, s))) return rc;
    if ((rc = schedule(op, shifted(P, h), h, nb - h, op->stream3))) return rc;
    HIP_TRY(hipEventRecord(op->ev_g, op->stream3));
    HIP_TRY(hipStreamWaitEvent(s, op->ev_g, 0));
  } else {
    rc = schedule(op, P, 0, nb);
  }
  if (rc) return rc;
  hipLaunchKernelGGL(finalize_kernel, dim3(nb), dim3(256), 0, s, P, nt, op->out, OUT_LD);
  LAUNCH_CHECK("finalize_kernel");
  if (op->timing) HIP_TRY(hipEventRecord(op->ev_end, s));
  return 0;
}

int collect_timing(gpmi_op* op) {
  if (!op->timing) return 0;
  HIP_TRY(hipEventSynchronize(op->ev_end));
  double tot = 0.0, fl = 0.0;
  std::vector<std::pair<double, double>> iv;
  for (auto& pr : op->syrk_log) {
    float ms = 0.f, t0 = 0.f, t1 = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, op->ev[pr.first], op->ev[pr.first + 1]));
    HIP_TRY(hipEventElapsedTime(&t0, op->ev_begin, op->ev[pr.first]));
    HIP_TRY(hipEventElapsedTime(&t1, op->ev_begin, op->ev[pr.first + 1]));
    iv.push_back({t0, t1});
    tot += ms;
    fl += pr.second;
  }
  if (std::getenv("GPMI_SYRK_TRACE")) {
    // dev aid: SYRK time by class (bulk trailing update w == t vs band w < t) and kdim
    std::map<std::pair<int, int>, std::array<double, 3>> cls;
    for (size_t i = 0; i < op->syrk_log.size(); ++i) {
      const auto& sh = op->syrk_shape[i];
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, op->ev[op->syrk_log[i].first],
                                  op->ev[op->syrk_log[i].first + 1]));
      auto& c = cls[{sh[0] == sh[1] ? 1 : 0, sh[2]}];
      c[0] += 1;
      c[1] += ms;
      c[2] += op->syrk_log[i].second;
    }
    for (auto& kv : cls)
      fprintf(stderr, "[gpmi syrk] %s kdim=%4d launches=%3.0f ms=%8.3f TF/s=%6.2f\n",
              kv.first.first ? "bulk" : "band", kv.first.second, kv.second[0], kv.second[1],
              kv.second[2] / (kv.second[1] * 1e-3) / 1e12);
  }
  std::sort(iv.begin(), iv.end());
  double busy = 0.0, cs = -1.0, ce = -1.0;
  for (auto& x : iv) {
    if (x.first > ce) {
      if (ce > cs) busy += ce - cs;
      cs = x.first;
      ce = x.second;
    } else if (x.second > ce) {
      ce = x.second;
    }
  }
  if (ce > cs) busy += ce - cs;
  float all = 0.f;
  HIP_TRY(hipEventElapsedTime(&all, op->ev_begin, op->ev_end));
  op->last_syrk_ms = tot;
  op->last_syrk_busy_ms = busy;
  op->last_syrk_flops = fl;
  op->last_syrk_launches = (int)op->syrk_log.size();
  op->last_total_ms = all;
  return 0;
}

int upload_rhs(gpmi_op* op, double* dst, const double* rhs, int64_t ld, int nrhs, int col0) {
  // pack columns [col0, col0 + nrhs) of an [n][ld] host block into [n_pad][16]
  std::vector<double> h((size_t)op->n_pad * RLD, 0.0);
  for (int64_t i = 0; i < op->n; ++i)
    for (int c = 0; c < nrhs; ++c) h[(size_t)i * RLD + c] = rhs[i * ld + col0 + c];
  HIP_TRY(hipMemcpyAsync(dst, h.data(), sizeof(double) * h.size(),
                         hipMemcpyHostToDevice, op->stream));
  HIP_TRY(hipStreamSynchronize(op->stream));
  return 0;
}

int ensure_factor(gpmi_op* op, double eta, const double* rhs_dev, bool* fresh) {
  *fresh = false;
  if (op->cache_valid && op->cached_eta == eta) return 0;
  int rc = run_factor(op, &eta, 1, rhs_dev);
  if (rc) return rc;
  op->cache_valid = true;
  op->cached_eta = eta;
  *fresh = true;
  return 0;
}

}  // namespace

namespace gpmi {
int matern_params_host(double nu, MaternParams* P);
int set_error(int code, const char* msg) { return set_err(code, "%s", msg); }
int op_view(const gpmi_op* op, OpView* v) {
  if (!op) return set_err(-1006, "null handle");
  v->device = op->device;
  v->n = op->n;
  v->n_pad = op->n_pad;
  v->K = op->K;
  v->has_K = op->has_K;
  return 0;
}
}  // namespace gpmi

namespace {
// K[i][i] = 1 for the pad rows n <= i < n_pad (at most 127 of them).
__global__ void pad_identity_kernel(double* K, int64_t ldk, int64_t n) {
  const int64_t i = n + threadIdx.x;
  if (i < ldk) K[i * ldk + i] = 1.0;
}
}  // namespace

extern "C" {

int gpmi_version(void) { return 100; }

int gpmi_last_error(char* buf, size_t len) {
  if (!buf || !len) return 0;
  strncpy(buf, g_err, len - 1);
  buf[len - 1] = 0;
  return 0;
}

int gpmi_device_count(int* count) {
  HIP_TRY(hipGetDeviceCount(count));
  return 0;
}

thread_local double g_assembly_ms = 0.0;   // last matern_dense_kernel launch (HIP events)

static int matern_params(double nu, MaternParams* P) {
  if (!(nu > 0.0)) return set_err(-1002, "nu must be positive (got %g)", nu);
  P->nu = nu;
  P->sqrt2nu = std::sqrt(2.0 * nu);
  P->mu = nu < 2.0 ? nu : nu - std::floor(nu) + 1.0;
  P->lp0 = (1.0 - P->mu) * std::log(2.0) - std::lgamma(P->mu);
  P->lp1 = -P->mu * std::log(2.0) - std::lgamma(P->mu + 1.0);
  if (nu == 0.5) P->mode = MATERN_HALF;
  else if (nu == 1.5) P->mode = MATERN_3HALF;
  else if (nu == 2.5) P->mode = MATERN_5HALF;
  else if (nu < 100) P->mode = MATERN_GENERAL;
  else P->mode = MATERN_GAUSS;
  return 0;
}

int gpmi_last_assembly_ms(double* ms) {
  if (!ms) return set_err(-1004, "null output");
  *ms = g_assembly_ms;
  return 0;
}

int gpmi_matern_values(int device, const double* x, int64_t m, double nu, double* out) {
  if (m <= 0) return 0;
  MaternParams P;
  int rc = matern_params(nu, &P);
  if (rc) return rc;
  DeviceGuard g(device);
  double *dx = nullptr, *dv = nullptr;
  HIP_TRY(hipMalloc(&dx, sizeof(double) * m));
  HIP_TRY(hipMalloc(&dv, sizeof(double) * m));
  HIP_TRY(hipMemcpy(dx, x, sizeof(double) * m, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(matern_eval_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, 0, dx,
                     m, P, dv);
  LAUNCH_CHECK("matern_eval_kernel");
  HIP_TRY(hipMemcpy(out, dv, sizeof(double) * m, hipMemcpyDeviceToHost));
  HIP_TRY(hipFree(dx));
  HIP_TRY(hipFree(dv));
  return 0;
}

static int assemble(int device, hipStream_t s, const double* points, int64_t n, int d,
                    const double* scale, double nu, double* Kdev, int64_t ldk,
                    int64_t n_pad) {
  if (d < 1 || d > GPMI_MAX_DIM)
    return set_err(-1003, "dimension %d outside [1, %d]", d, GPMI_MAX_DIM);
  MaternParams P;
  int rc = matern_params(nu, &P);
  if (rc) return rc;
  DeviceGuard g(device);
  double *dp = nullptr, *ds = nullptr;
  HIP_TRY(hipMalloc(&dp, sizeof(double) * std::max<int64_t>(1, n * d)));
  HIP_TRY(hipMalloc(&ds, sizeof(double) * d));
  HIP_TRY(hipMemcpyAsync(dp, points, sizeof(double) * n * d, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(ds, scale, sizeof(double) * d, hipMemcpyHostToDevice, s));
  // lower-triangular 64 x 64 tiles, each mirrored (gpmi_matern.hip)
  const int64_t T = (n_pad + 63) / 64;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  HIP_TRY(hipEventRecord(e0, s));
  launch_matern_dense(dim3((unsigned)(T * (T + 1) / 2)), s, dp, n, d, ds, P, Kdev, ldk, n_pad);
  LAUNCH_CHECK("matern_dense_kernel");
  HIP_TRY(hipEventRecord(e1, s));
  HIP_TRY(hipStreamSynchronize(s));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  g_assembly_ms = ms;
  HIP_TRY(hipEventDestroy(e0));
  HIP_TRY(hipEventDestroy(e1));
  HIP_TRY(hipFree(dp));
  HIP_TRY(hipFree(ds));
  return 0;
}

int gpmi_matern_dense(int device, const double* points, int64_t n, int d,
                      const double* scale, double nu, double* K_out, int64_t ldk) {
  if (n <= 0) return 0;
  DeviceGuard g(device);
  double* dK = nullptr;
  HIP_TRY(hipMalloc(&dK, sizeof(double) * n * n));
  int rc = assemble(device, nullptr, points, n, d, scale, nu, dK, n, n);
  if (rc) {
    (void)hipFree(dK);
    return rc;
  }
  HIP_TRY(hipMemcpy2D(K_out, sizeof(double) * ldk, dK, sizeof(double) * n, sizeof(double) * n,
                      n, hipMemcpyDeviceToHost));
  HIP_TRY(hipFree(dK));
  return 0;
}

int gpmi_op_create(int device, int64_t n, int max_batch, gpmi_op** out) {
  if (!out) return set_err(-1004, "null output handle");
  if (n <= 0) return set_err(-1005, "matrix size must be positive");
  if (max_batch < 1) max_batch = 1;
  DeviceGuard g(device);
  gpmi_op* op = new gpmi_op();
  op->device = device;
  op->n = n;
  op->n_pad = (n + TS - 1) / TS * TS;
  op->nt = (int)(op->n_pad / TS);
  op->max_batch = max_batch;
  if (const char* g = std::getenv("GPMI_GROUPS")) op->groups = std::atoi(g);
  const int64_t np = op->n_pad;
  auto fail = [&](hipError_t e, const char* what) {
    gpmi_op_destroy(op);
    return set_err(-(int)e, "allocation of %s failed: %s", what, hipGetErrorString(e));
  };
  hipError_t e;
  if ((e = hipStreamCreateWithFlags(&op->stream, hipStreamNonBlocking)) != hipSuccess)
    return fail(e, "stream");
  // (one stream; op->stream3 only for the two-halves batch form: HIP streams beyond
  // the process's hardware queues (GPU_MAX_HW_QUEUES = 4) share queues and slow other
  // objects' multi-stream work, a band reduction beside a dense operator holding three
  // streams: 161 -> 181 ms)
  if ((e = hipEventCreateWithFlags(&op->ev_fork, sync_event_flags())) != hipSuccess)
    return fail(e, "event");
  if ((e = hipEventCreateWithFlags(&op->ev_join, sync_event_flags())) != hipSuccess)
    return fail(e, "event");
#define ALLOC(ptr, count)                                                           \
  if ((e = hipMalloc(&op->ptr, sizeof(*op->ptr) * (size_t)(count))) != hipSuccess)  \
    return fail(e, #ptr);
  ALLOC(K, np * np);
  ALLOC(A, (size_t)max_batch * np * np);
  ALLOC(R, (size_t)max_batch * np * RLD);
  ALLOC(X, (size_t)max_batch * np * RLD);
  ALLOC(U, (size_t)max_batch * TS * RLD);
  ALLOC(Linv, (size_t)max_batch * op->nt * TS * TS);
  ALLOC(logdiag, (size_t)max_batch * op->nt);
  ALLOC(gram, (size_t)max_batch * op->nt * 256);
  ALLOC(out, (size_t)max_batch * OUT_LD);
  ALLOC(etas, max_batch);
  ALLOC(rhs_src, np * RLD);
  ALLOC(scratch, np * RLD);
  ALLOC(scratch2, np * RLD);
  ALLOC(tracebuf, np * 2);
  ALLOC(info, max_batch);
#undef ALLOC
  if ((e = hipMemsetAsync(op->rhs_src, 0, sizeof(double) * np * RLD, op->stream)) != hipSuccess)
    return fail(e, "rhs memset");
  if ((e = hipStreamSynchronize(op->stream)) != hipSuccess) return fail(e, "sync");
  *out = op;
  return 0;
}

int gpmi_op_destroy(gpmi_op* op) {
  if (!op) return 0;
  DeviceGuard g(op->device);
  if (op->stream) (void)hipStreamSynchronize(op->stream);
  if (op->stream3) (void)hipStreamSynchronize(op->stream3);
  double* bufs[] = {op->K, op->A, op->R, op->X, op->U, op->Linv, op->logdiag, op->gram,
                    op->out, op->etas, op->rhs_src, op->scratch, op->scratch2, op->tracebuf,
                    op->W, op->tpart, op->Td};
  for (double* p : bufs)
    if (p) (void)hipFree(p);
  if (op->info) (void)hipFree(op->info);
  if (op->order) (void)hipFree(op->order);
  for (auto e : op->ev) (void)hipEventDestroy(e);
  if (op->ev_begin) (void)hipEventDestroy(op->ev_begin);
  if (op->ev_end) (void)hipEventDestroy(op->ev_end);
  if (op->ev_fork) (void)hipEventDestroy(op->ev_fork);
  if (op->ev_join) (void)hipEventDestroy(op->ev_join);
  if (op->stream3) (void)hipStreamDestroy(op->stream3);
  if (op->ev_g) (void)hipEventDestroy(op->ev_g);
  if (op->stream) (void)hipStreamDestroy(op->stream);
  delete op;
  return 0;
}

int gpmi_op_size(const gpmi_op* op, int64_t* n, int64_t* n_pad) {
  if (!op) return set_err(-1006, "null handle");
  if (n) *n = op->n;
  if (n_pad) *n_pad = op->n_pad;
  return 0;
}

int gpmi_op_load_matrix(gpmi_op* op, const double* K_host, int64_t ldk) {
  if (!op) return set_err(-1006, "null handle");
  DeviceGuard g(op->device);
  const int64_t np = op->n_pad, n = op->n;
  // identity pad, then the n x n block
  std::vector<double> pad_rows;
  HIP_TRY(hipMemsetAsync(op->K, 0, sizeof(double) * np * np, op->stream));
  HIP_TRY(hipMemcpy2DAsync(op->K, sizeof(double) * np, K_host, sizeof(double) * ldk,
                           sizeof(double) * n, n, hipMemcpyHostToDevice, op->stream));
  if (np > n) {
    std::vector<double> one(1, 1.0);
    for (int64_t i = n; i < np; ++i)
      HIP_TRY(hipMemcpyAsync(op->K + i * np + i, one.data(), sizeof(double),
                             hipMemcpyHostToDevice, op->stream));
  }
  HIP_TRY(hipStreamSynchronize(op->stream));
  op->has_K = true;
  op->cache_valid = false;
  return 0;
}

int gpmi_op_load_sparse(gpmi_op* op, const gpmi_sp* sp) {
  if (!op || !sp) return set_err(-1006, "null handle");
  int64_t n_sp = 0;
  if (int rc = gpmi_sp_info(sp, &n_sp, nullptr)) return rc;
  if (n_sp != op->n) return set_err(-1005, "sparse operator has n = %lld, dense has %lld",
                                    (long long)n_sp, (long long)op->n);
  DeviceGuard g(op->device);
  const int64_t np = op->n_pad;
  HIP_TRY(hipMemsetAsync(op->K, 0, sizeof(double) * np * np, op->stream));
  if (int rc = gpmi::sp_scatter_dense(sp, op->device, op->K, np, op->stream)) return rc;
  if (np > op->n) {
    hipLaunchKernelGGL(pad_identity_kernel, dim3(1), dim3(128), 0, op->stream, op->K, np, op->n);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(op->stream));
  op->has_K = true;
  op->cache_valid = false;
  return 0;
}

int gpmi_op_assemble_matern(gpmi_op* op, const double* points, int d, const double* scale,
                            double nu) {
  if (!op) return set_err(-1006, "null handle");
  int rc = assemble(op->device, op->stream, points, op->n, d, scale, nu, op->K, op->n_pad,
                    op->n_pad);
  if (rc) return rc;
  op->has_K = true;
  op->cache_valid = false;
  return 0;
}

int gpmi_op_get_matrix(gpmi_op* op, double* K_out, int64_t ldk) {
  if (!op) return set_err(-1006, "null handle");
  DeviceGuard g(op->device);
  HIP_TRY(hipMemcpy2DAsync(K_out, sizeof(double) * ldk, op->K, sizeof(double) * op->n_pad,
                           sizeof(double) * op->n, op->n, hipMemcpyDeviceToHost, op->stream));
  HIP_TRY(hipStreamSynchronize(op->stream));
  return 0;
}

int gpmi_op_set_rhs(gpmi_op* op, const double* rhs, int64_t ld, int nrhs) {
  if (!op) return set_err(-1006, "null handle");
  if (nrhs < 0 || nrhs > RLD) return set_err(-1007, "nrhs %d outside [0, %d]", nrhs, RLD);
  DeviceGuard g(op->device);
  int rc = upload_rhs(op, op->rhs_src, rhs, ld, nrhs, 0);
  if (rc) return rc;
  op->nrhs = nrhs;
  return 0;
}

int gpmi_op_loglik_batch(gpmi_op* op, const double* etas, int neta, double* logdet,
                         double* gram, int* info) {
  if (!op) return set_err(-1006, "null handle");
  DeviceGuard g(op->device);
  int rc = run_factor(op, etas, neta, op->rhs_src);
  if (rc) return rc;
  std::vector<double> hout((size_t)neta * OUT_LD);
  std::vector<int> hinfo(neta);
  HIP_TRY(hipMemcpyAsync(hout.data(), op->out, sizeof(double) * hout.size(),
                         hipMemcpyDeviceToHost, op->stream));
  HIP_TRY(hipMemcpyAsync(hinfo.data(), op->info, sizeof(int) * neta, hipMemcpyDeviceToHost,
                         op->stream));
  HIP_TRY(hipStreamSynchronize(op->stream));
  // the batch-halves stream is joined and idle: release it, so that it does not hold
  // one of the process's hardware queues while other objects run (a band reduction
  // after a batch-8 call here: 181 ms with it alive, 162 ms without)
  if (op->stream3) {
    HIP_TRY(hipStreamDestroy(op->stream3));
    op->stream3 = nullptr;
  }
  rc = collect_timing(op);
  if (rc) return rc;
  const int m = op->nrhs;
  int status = 0;
  for (int e = 0; e < neta; ++e) {
    if (logdet) logdet[e] = hout[(size_t)e * OUT_LD];
    if (gram)
      for (int a = 0; a < m; ++a)
        for (int c = 0; c < m; ++c)
          gram[((size_t)e * m + a) * m + c] = hout[(size_t)e * OUT_LD + 1 + a * RLD + c];
    if (info) info[e] = hinfo[e];
    if (hinfo[e] && !status) status = hinfo[e];
  }
  op->cache_valid = (neta >= 1 && hinfo[0] == 0);
  op->cached_eta = etas[0];
  if (status) set_err(status, "matrix K + eta I is not positive definite (pivot %d)", status);
  return 0;
}

int gpmi_op_logdet(gpmi_op* op, double eta, double* logdet) {
  if (!op) return set_err(-1006, "null handle");
  DeviceGuard g(op->device);
  bool fresh;
  int rc = ensure_factor(op, eta, op->rhs_src, &fresh);
  if (rc) return rc;
  double ld = 0.0;
  int inf = 0;
  HIP_TRY(hipMemcpyAsync(&ld, op->out, sizeof(double), hipMemcpyDeviceToHost, op->stream));
  HIP_TRY(hipMemcpyAsync(&inf, op->info, sizeof(int), hipMemcpyDeviceToHost, op->stream));
  HIP_TRY(hipStreamSynchronize(op->stream));
  if (inf) {
    op->cache_valid = false;
    return set_err(inf, "matrix K + eta I is not positive definite (pivot %d)", inf);
  }
  *logdet = ld;
  return 0;
}

int gpmi_op_solve(gpmi_op* op, double eta, const double* rhs, int64_t ld, int nrhs,
                  double* sol, int64_t ldsol) {
  if (!op) return set_err(-1006, "null handle");
  DeviceGuard g(op->device);
  const int nt = op->nt;
  const int64_t lda = op->n_pad;
  BatchPtrs P = op->ptrs();
  std::vector<double> h((size_t)op->n_pad * RLD);
  for (int c0 = 0; c0 < nrhs; c0 += RLD) {
    const int nc = std::min(RLD, nrhs - c0);
    int rc = upload_rhs(op, op->scratch, rhs, ld, nc, c0);
    if (rc) return rc;
    bool fresh;
    rc = ensure_factor(op, eta, op->scratch, &fresh);
    if (rc) return rc;
    int inf = 0;
    HIP_TRY(hipMemcpyAsync(&inf, op->info, sizeof(int), hipMemcpyDeviceToHost, op->stream));
    HIP_TRY(hipStreamSynchronize(op->stream));
    if (inf) {
      op->cache_valid = false;
      return set_err(inf, "matrix K + eta I is not positive definite (pivot %d)", inf);
    }
    if (!fresh) {
      // cached factor: forward substitution of the new RHS block
      HIP_TRY(hipMemcpyAsync(op->R, op->scratch, sizeof(double) * P.sR,
                             hipMemcpyDeviceToDevice, op->stream));
      for (int kb = 0; kb < nt; ++kb) {
        hipLaunchKernelGGL(fwd_step_kernel, dim3(nt - kb, 1), dim3(256), 0, op->stream, P, lda,
                           kb);
        LAUNCH_CHECK("fwd_step_kernel");
      }
    }
    for (int kb = nt - 1; kb >= 0; --kb) {
      hipLaunchKernelGGL(bwd_step_kernel, dim3(std::max(kb, 1), 1), dim3(256), 0, op->stream, P,
                         lda, kb, op->X, P.sR);
      LAUNCH_CHECK("bwd_step_kernel");
    }
    HIP_TRY(hipMemcpyAsync(h.data(), op->X, sizeof(double) * h.size(), hipMemcpyDeviceToHost,
                           op->stream));
    HIP_TRY(hipStreamSynchronize(op->stream));
    for (int64_t i = 0; i < op->n; ++i)
      for (int c = 0; c < nc; ++c) sol[i * ldsol + c0 + c] = h[(size_t)i * RLD + c];
  }
  return 0;
}

int gpmi_op_matvec(gpmi_op* op, const double* x, int64_t ld, int ncol, double* y,
                   int64_t ldy) {
  if (!op) return set_err(-1006, "null handle");
  if (!op->has_K) return set_err(-1000, "operator has no matrix");
  DeviceGuard g(op->device);
  std::vector<double> h((size_t)op->n_pad * RLD, 0.0);
  for (int c0 = 0; c0 < ncol; c0 += RLD) {
    const int nc = std::min(RLD, ncol - c0);
    std::fill(h.begin(), h.end(), 0.0);
    for (int64_t i = 0; i < op->n; ++i)
      for (int c = 0; c < nc; ++c) h[(size_t)i * RLD + c] = x[i * ld + c0 + c];
    HIP_TRY(hipMemcpyAsync(op->scratch, h.data(), sizeof(double) * h.size(),
                           hipMemcpyHostToDevice, op->stream));
    hipLaunchKernelGGL(gemv_sym_kernel, dim3((unsigned)((op->n + 3) / 4)), dim3(256), 0,
                       op->stream, op->K, op->n_pad, op->n, op->scratch, (int64_t)RLD, nc,
                       op->scratch2, 0.0, 1);
    LAUNCH_CHECK("gemv_sym_kernel");
    HIP_TRY(hipMemcpyAsync(h.data(), op->scratch2, sizeof(double) * h.size(),
                           hipMemcpyDeviceToHost, op->stream));
    HIP_TRY(hipStreamSynchronize(op->stream));
    for (int64_t i = 0; i < op->n; ++i)
      for (int c = 0; c < nc; ++c) y[i * ldy + c0 + c] = h[(size_t)i * RLD + c];
  }
  return 0;
}

int gpmi_op_trace(gpmi_op* op, double* trace_k, double* trace_k2) {
  if (!op) return set_err(-1006, "null handle");
  if (!op->has_K) return set_err(-1000, "operator has no matrix");
  DeviceGuard g(op->device);
  hipLaunchKernelGGL(trace_kernel, dim3((unsigned)op->n), dim3(256), 0, op->stream, op->K,
                     op->n_pad, op->n, op->tracebuf);
  LAUNCH_CHECK("trace_kernel");
  std::vector<double> h((size_t)op->n * 2);
  HIP_TRY(hipMemcpyAsync(h.data(), op->tracebuf, sizeof(double) * h.size(),
                         hipMemcpyDeviceToHost, op->stream));
  HIP_TRY(hipStreamSynchronize(op->stream));
  double a = 0.0, f = 0.0;
  for (int64_t i = 0; i < op->n; ++i) {
    a += h[2 * i];
    f += h[2 * i + 1];
  }
  if (trace_k) *trace_k = a;
  if (trace_k2) *trace_k2 = f;
  return 0;
}

int gpmi_op_traceinv(gpmi_op* op, double eta, int exponent, double* value) {
  if (!op) return set_err(-1006, "null handle");
  if (!value) return set_err(-1004, "null output");
  if (exponent < 1 || exponent > 2)
    return set_err(-1010, "traceinv exponent %d outside [1, 2]", exponent);
  DeviceGuard g(op->device);
  bool fresh;
  int rc = ensure_factor(op, eta, op->rhs_src, &fresh);
  if (rc) return rc;
  int inf = 0;
  HIP_TRY(hipMemcpyAsync(&inf, op->info, sizeof(int), hipMemcpyDeviceToHost, op->stream));
  HIP_TRY(hipStreamSynchronize(op->stream));
  if (inf) {
    op->cache_valid = false;
    return set_err(inf, "matrix K + eta I is not positive definite (pivot %d)", inf);
  }
  if (op->tinv_gen != op->factor_gen) {
    op->tinv_gen = op->factor_gen;
    op->tinv_have = 0;
  }
  const int bit = 1 << (exponent - 1);
  if (!(op->tinv_have & bit)) {
    const int nt = op->nt;
    const int64_t np = op->n_pad;
    const int ntri = nt * (nt + 1) / 2;
    if (!op->W) {
      HIP_TRY(hipMalloc(&op->W, sizeof(double) * (size_t)np * np));
      HIP_TRY(hipMalloc(&op->tpart, sizeof(double) * (size_t)(ntri + nt * nt)));
      HIP_TRY(hipMalloc(&op->Td, sizeof(double) * (size_t)nt * TS * TS));
    }
    hipStream_t s = op->stream;
    double* p1 = op->tpart + ntri;   // [nt][nt]: ||Y_kj||^2 at [k * nt + j]
    if (!(op->tinv_have & 1)) {
      // W = L^-T from the cached factor in slot 0 (needed by both exponents)
      for (int kb = 0; kb < nt; kb += op->outer) {
        const int ke = std::min(nt, kb + op->outer);
        for (int k = kb; k < ke; ++k) {
          if (k > kb) {
            hipLaunchKernelGGL(trinv_update_kernel, dim3(k), dim3(256), 0, s, op->A, np, op->W,
                               np, k, k, kb, k);
            LAUNCH_CHECK("trinv_update_kernel");
          }
          hipLaunchKernelGGL(trinv_diag_kernel, dim3(k + 1), dim3(256), 0, s, op->Linv, op->W,
                             np, k, p1 + (int64_t)k * nt);
          LAUNCH_CHECK("trinv_diag_kernel");
        }
        if (ke < nt) {
          hipLaunchKernelGGL(trinv_update_kernel, dim3((nt - ke) * ke), dim3(256), 0, s, op->A,
                             np, op->W, np, ke, ke, kb, ke);
          LAUNCH_CHECK("trinv_update_kernel");
        }
      }
      std::vector<double> h((size_t)nt * nt);
      HIP_TRY(hipMemcpyAsync(h.data(), p1, sizeof(double) * h.size(), hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      double acc = 0.0;
      for (int k = 0; k < nt; ++k)
        for (int j = 0; j <= k; ++j) acc += h[(size_t)k * nt + j];
      // the identity pad contributes n_pad - n
      op->tinv[0] = acc - (double)(np - op->n);
      op->tinv_have |= 1;
    }
    if (exponent == 2) {
      // T = W W^T over k-panels of 4 tiles; panel [p0, p0 + kd) updates tile rows I < imax
      for (int p0 = 0; p0 < (int)np; p0 += 4 * TS) {
        const int kd = std::min<int>(4 * TS, (int)np - p0);
        const int imax = (p0 + kd) / TS;
        hipLaunchKernelGGL(gram_panel_kernel, dim3(imax * (imax + 1) / 2), dim3(256), 0, s,
                           op->W, np, op->Td, p0, kd, imax);
        LAUNCH_CHECK("gram_panel_kernel");
      }
      hipLaunchKernelGGL(gram_sumsq_kernel, dim3(nt), dim3(256), 0, s, op->W, np, op->Td,
                         op->tpart);
      LAUNCH_CHECK("gram_sumsq_kernel");
      std::vector<double> h((size_t)nt);
      HIP_TRY(hipMemcpyAsync(h.data(), op->tpart, sizeof(double) * h.size(),
                             hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      double acc = 0.0;
      for (int q = 0; q < nt; ++q) acc += h[q];
      op->tinv[1] = acc - (double)(np - op->n);
      op->tinv_have |= 2;
    }
  }
  *value = op->tinv[exponent - 1];
  return 0;
}

int gpmi_op_set_timing(gpmi_op* op, int enable) {
  if (!op) return set_err(-1006, "null handle");
  op->timing = enable != 0;
  return 0;
}

int gpmi_op_last_timing(gpmi_op* op, double* syrk_ms, int* syrk_launches, double* syrk_flops,
                        double* total_ms, double* syrk_busy_ms) {
  if (!op) return set_err(-1006, "null handle");
  if (syrk_busy_ms) *syrk_busy_ms = op->last_syrk_busy_ms;
  if (syrk_ms) *syrk_ms = op->last_syrk_ms;
  if (syrk_launches) *syrk_launches = op->last_syrk_launches;
  if (syrk_flops) *syrk_flops = op->last_syrk_flops;
  if (total_ms) *total_ms = op->last_total_ms;
  return 0;
}


int gpmi_op_set_outer(gpmi_op* op, int s) {
  if (!op) return set_err(-1006, "null handle");
  if (s < 1 || s > 32) return set_err(-1008, "outer panel width %d outside [1, 32]", s);
  op->outer = s;
  return 0;
}

}  // extern "C"

namespace gpmi {
int matern_params_host(double nu, MaternParams* P) { return matern_params(nu, P); }
}  // namespace gpmi
