// C-ABI of the band path (include/gpmi.h, gpmi_band_*): reduction of an
// operator's K to symmetric band form (bandwidth 128) on the device, Q^T applied
// to a resident RHS block, and batched banded-Cholesky likelihood terms for any
// number of eta values (kernels: gpmi_band.hip).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gpmi_internal.h"
#include "gpmi_band.h"
#include "../../include/gpmi.h"

using namespace gpmi;

namespace gpmi {
int set_error(int code, const char* msg);   // gpmi_api.hip
int op_view(const gpmi_op* op, OpView* v);  // gpmi_api.hip
}  // namespace gpmi

namespace {

#define BD_TRY(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) {                                                            \
      char b_[400];                                                                    \
      snprintf(b_, sizeof(b_), "%s failed: %s", #expr, hipGetErrorString(e_));        \
      return set_error(-(int)e_, b_);                                                  \
    }                                                                                  \
  } while (0)

#define BD_LAUNCH(name)                                                                \
  do {                                                                                 \
    hipError_t e_ = hipGetLastError();                                                 \
    if (e_ != hipSuccess) {                                                            \
      char b_[400];                                                                    \
      snprintf(b_, sizeof(b_), "launch of %s failed: %s", name, hipGetErrorString(e_)); \
      return set_error(-(int)e_, b_);                                                  \
    }                                                                                  \
  } while (0)

constexpr int TS = GPMI_TS;
constexpr int RLD = GPMI_RHS_LD;
constexpr int OUT_LD = 1 + RLD * RLD;

struct Guard {
  int prev = -1;
  explicit Guard(int d) {
    (void)hipGetDevice(&prev);
    if (prev != d) (void)hipSetDevice(d);
  }
  ~Guard() {
    int c = -1;
    (void)hipGetDevice(&c);
    if (prev >= 0 && c != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

constexpr int RGROUP = 8;   // tile rows per group of the look-ahead SYR2K's tile order

struct gpmi_band {
  int device = 0;
  int64_t n = 0, n_pad = 0;
  int nt = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr;
  double* Ab = nullptr;      // [n_pad][n_pad]: band (diagonal tiles, triu of subdiagonal
                             // tiles) + Householder vectors below the band
  double* U = nullptr;       // [n_pad][384] = [W | V | W] of the current panel
  double* X = nullptr;       // [n_pad][128] (rows relative to the panel's trailing block)
  double* X2 = nullptr;      // [n_pad][128] X T (quadrant steps: out of place)
  double* Xp = nullptr;      // symm split-K partials
  double* part = nullptr;    // [2][HH_MAXG][HH_PART_LD] column partials
  double* pivrow = nullptr;  // [2][128]
  double* tau = nullptr;     // [nt][128]
  double* Tm = nullptr;      // [nt][128][128] compact-WY T per panel
  double* tnp = nullptr;     // tn partials [nch][128][128]
  double* tnp2 = nullptr;    // tn partials of V^T V (side stream) [nch][128][128]
  hipStream_t side = nullptr;          // V^T V and T of a panel, beside its SYMM
  // look-ahead: the next panel's QR (high-priority stream) beside the rest of the
  // SYR2K: a CholeskyQR panel beside syr2k_pipe_kernel on all but LA_FREE CUs, a
  // Householder panel beside syr2k_rest_kernel on la_grid workgroups
  int lookahead = 1, la_grid = 128, ncu = 256;
  hipStream_t s_pan = nullptr;
  hipEvent_t ev_col = nullptr, ev_pan = nullptr;
  hipEvent_t ev_v = nullptr, ev_t = nullptr, ev_q = nullptr;
  double* VtV = nullptr;     // [128][128]
  double* M = nullptr;       // [128][128]
  double* Zh = nullptr;      // [128][128]
  double* Y = nullptr;       // [n_pad][16] = Q^T R
  double* qtp = nullptr;     // [HH_MAXG][128][16]
  double* qa = nullptr;      // [128][16]
  double* qb = nullptr;      // [128][16]
  double* etas = nullptr;    // [cap]
  double* out = nullptr;     // [cap][OUT_LD]
  int* info = nullptr;       // [cap]
  unsigned* ctr = nullptr;   // hh_panel hand-off counter: 8 shards, 64 B apart (512 bytes)
  int* err = nullptr;        // hh_panel timeout flag
  // hh_panel_kernel needs all G workgroups co-resident: used only for G <= panel_maxg
  // (CU count x resident workgroups per CU, at most HH_PANEL_MAXG); a timed-out
  // hand-off makes band_reduce redo the reduction with hh_col_kernel launches
  int panel_maxg = HH_PANEL_MAXG;
  unsigned spin_limit = 1u << 24;
  int panel_fallbacks = 0;
  // CholeskyQR panel (gpmi_cholqr.hip; default, GPMI_BAND_PANEL=hh selects the
  // Householder panel): Q [n_pad][128], Gram partials, the three Cholesky factors
  // and inverses, the reconstruction's U^-T, V1, signs, scratch, failure flag
  int panel_mode = 0;        // 0 CholeskyQR, 1 Householder (single launch)
  int cq_fallbacks = 0;      // reductions redone with Householder panels
  double* Qb = nullptr;
  double* cqpart = nullptr;
  double* cqG = nullptr;
  // per panel (cq_top_kernel forms every panel's R after the reduction):
  double* cqL = nullptr;     // [nt][3][128][128] exact factors (first-order passes: by top)
  double* cqLinv = nullptr;  // [nt][3][128][128] applied inverses
  double* cqS = nullptr;     // [nt][128] reconstruction signs
  double* cqscr = nullptr;   // [nt][128][128]
  int* cqflag = nullptr;     // [nt][8]: [0..2] first-order flag per pass, [3] CholeskyQR
                             // succeeded, [4] failed (the guarded Householder panel ran),
                             // [6] the look-ahead SYR2K's tile tickets
  int la_free = LA_FREE, la_free_late = LA_FREE_LATE, la_late_mt = LA_LATE_MT;   // GPMI_LA_*
  bool poison = false;          // GPMI_BAND_POISON=1: Ab set to NaN before a K-first copy
  int cq_panel_fallbacks = 0;   // panels factored by the guarded Householder panel, or
                                // (past its single-launch size) by per-column launches
  int cq_host_checks = 0;       // panels past the single-launch size whose flag the host read
  // grouped tile orders of the look-ahead SYR2K, one per (w x w)-triangle, w < nt
  // (RGROUP tile rows per group; measured within +-0.5 % of the plain triangle order)
  uint32_t* rorder = nullptr;
  std::vector<int64_t> rorder_off;
  // block cyclic reduction of B + eta I (gpmi_bcr.hip; GPMI_BAND_BCR): per eta
  // capacity bcap, half = ceil(nt / 2) blocks per level
  int bcr_mode = 2;          // 0 sequential band_chol_kernel, 1 cyclic reduction, 2 auto:
                             // cyclic reduction up to 64 eta per call (measured at N = 16384:
                             // 1 eta 9.97 -> 1.30 ms, 8 eta 10.05 -> 1.85, 64 eta 9.9 -> 8.8;
                             // the sequential kernel's time is flat up to the CU count)
  int bcap = 0;
  double* bcrD[2] = {nullptr, nullptr};   // [bcap][half][128][128]
  double* bcrF[2] = {nullptr, nullptr};
  double* bcrY[2] = {nullptr, nullptr};   // [bcap][half][128][16]
  double* bcrL = nullptr;    // [bcap][nt][128][128]     every level's Linv, by original block
  double* bcrW = nullptr;    // [bcap][nt][2][128][128]  every level's W_l, W_r, likewise
  double* bcrZ = nullptr;    // [bcap][nt][128][16]
  double* bcrX = nullptr;    // [bcap][nt][128][16]      derivative terms: X, then Z'
  double* bcrZp = nullptr;
  double* bcrG2 = nullptr;   // [bcap][nt][16][16]
  double* bcrG3 = nullptr;
  double* bcrG = nullptr;    // [bcap][nt][16][16]
  double* bcrLd = nullptr;   // [bcap][nt]
  int* bcrFail = nullptr;    // [bcap][nt]
  double* bcrF0 = nullptr;   // [nt - 1][128][128]
  // selected inversion down the reduction tree (traceinv without eigenvalues)
  double* sinvZd = nullptr;  // [scap][nt][128][128]     diagonal blocks of (B + eta I)^-1
  double* sinvZo = nullptr;  // [scap][nt][2][128][128]  Z_lp, Z_rp of every eliminated block
  double* sinvX = nullptr;   // [scap][nt][2][128][128]  X_l, X_r
  double* sinvTr = nullptr;  // [scap][nt] per-block traces, then [scap] sums
  int scap = 0;
  double sinv_ms = 0.0;
  // eta-tangents of the cyclic-reduction factor and of the selected inversion
  // (traceinv of exponent 2, gpmi_bcr.hip bcr_d*): per eta of a chunk of at most
  // BAND_TAN_MAX (tcap), strides per eta as the primal blocks
  double* tanL = nullptr;    // [tcap][nt][128][128]     dLinv
  double* tanW = nullptr;    // [tcap][nt][2][128][128]  dW_l, dW_r
  double* tanX = nullptr;    // [tcap][nt][2][128][128]  dX_l, dX_r (bcr_dfac's scratch first)
  double* tanZd = nullptr;   // [tcap][nt][128][128]
  double* tanZo = nullptr;   // [tcap][nt][2][128][128]
  double* tanD[2] = {nullptr, nullptr};   // [tcap][half][128][128]
  double* tanF[2] = {nullptr, nullptr};
  double* tanTr = nullptr;   // [tcap][nt] per-block -tr dZ_pp, then [tcap] sums
  int tcap = 0;
  double* cqMinv = nullptr;  // C = U^-T M3 of the current panel
  // T of a CholeskyQR panel from its reconstruction (cq_t_kernel) on the side stream
  // (not a stream of its own: the process's streams share GPU_MAX_HW_QUEUES hardware
  // queues, and two streams on one queue serialise): U S and V1^-1 per panel;
  // t_from_q[j]: panel j's T comes from there (the side stream's V^T V / tbuild_kernel
  // then run only if the panel fell back)
  double* cqUS = nullptr;    // [nt][128][128]
  double* cqW = nullptr;     // [nt][128][128]
  hipEvent_t ev_rc = nullptr;
  std::vector<char> t_from_q;
  std::vector<char> v_in_u;   // v_in_u[j]: panel j's reflectors are in U already
  double cq_fo[3] = {0.0, 1e-4, 3e-8};   // first-order thresholds on ||G - I||_F
  int cap = 0;
  int nrhs = 0;
  double reduce_ms = 0.0, rhs_ms = 0.0, loglik_ms = 0.0, der_ms = 0.0;
  // eta-derivative terms (allocated on first use): per eta of a chunk, the
  // banded factor blocks, the solution block and the two higher Grams
  double* fac = nullptr;     // [dcap][nt][2][128][128]
  double* ysol = nullptr;    // [dcap][n_pad][16]
  double* der = nullptr;     // [dcap][2][16][16]
  int dcap = 0;
  // eigenvalues (bulge chase + bisection), computed on request
  double* Ac = nullptr;      // [n_pad][n_pad] chase copy of the band (lower)
  double* td = nullptr;      // [n] diagonal, then [n] squared subdiagonal, then [n] eigenvalues
  double eig_ms = 0.0;
  // systolic chase (chase_systolic_kernel): one workgroup per position, all
  // co-resident; used when chase_maxg (CU count x resident workgroups per CU)
  // covers the positions, else (and after a timed-out hand-off) the launch form
  unsigned long long* cmsg = nullptr;  // reflector, column slots [2][K + 1][2][2 CHASE_MSG], err
  int chase_maxg = 0;
  int split_maxg = 0;        // the same for chase_split_kernel (2K workgroups)
  unsigned chase_spin = 1u << 24;
  int chase_systolic = 0;    // the last eigenvalues(): 2 split, 1 one-per-position, 0 launches
  int chase_fallbacks = 0;   // systolic attempts that timed out and reran the launch form
};

namespace {

int band_free(gpmi_band* b) {
  double* bufs[] = {b->Ab, b->U, b->X, b->X2, b->Xp, b->part, b->pivrow, b->tau, b->Tm, b->tnp, b->tnp2,
                    b->VtV, b->M, b->Zh, b->Y, b->qtp, b->qa, b->qb, b->etas, b->out, b->Ac, b->td,
                    b->fac, b->ysol, b->der, b->Qb, b->cqpart, b->cqG, b->cqL, b->cqLinv,
                    b->cqMinv, b->cqS, b->cqscr, b->cqUS, b->cqW,
                    b->bcrD[0], b->bcrD[1], b->bcrF[0], b->bcrF[1], b->bcrY[0], b->bcrY[1],
                    b->bcrL, b->bcrW, b->bcrZ, b->bcrG, b->bcrLd, b->bcrF0, b->bcrX,
                    b->bcrZp, b->bcrG2, b->bcrG3, b->sinvZd, b->sinvZo, b->sinvX,
                    b->sinvTr, b->tanL, b->tanW, b->tanX, b->tanZd, b->tanZo, b->tanD[0],
                    b->tanD[1], b->tanF[0], b->tanF[1], b->tanTr};
  if (b->bcrFail) (void)hipFree(b->bcrFail);
  if (b->cqflag) (void)hipFree(b->cqflag);
  if (b->rorder) (void)hipFree(b->rorder);
  for (double* p : bufs)
    if (p) (void)hipFree(p);
  if (b->info) (void)hipFree(b->info);
  if (b->ctr) (void)hipFree(b->ctr);
  if (b->err) (void)hipFree(b->err);
  if (b->cmsg) (void)hipFree(b->cmsg);
  if (b->ev0) (void)hipEventDestroy(b->ev0);
  if (b->ev1) (void)hipEventDestroy(b->ev1);
  if (b->ev2) (void)hipEventDestroy(b->ev2);
  if (b->ev3) (void)hipEventDestroy(b->ev3);
  if (b->stream) (void)hipStreamDestroy(b->stream);
  if (b->side) (void)hipStreamDestroy(b->side);
  if (b->s_pan) (void)hipStreamDestroy(b->s_pan);
  for (hipEvent_t e : {b->ev_col, b->ev_pan, b->ev_rc})
    if (e) (void)hipEventDestroy(e);
  if (b->ev_q) (void)hipEventDestroy(b->ev_q);
  if (b->ev_v) (void)hipEventDestroy(b->ev_v);
  if (b->ev_t) (void)hipEventDestroy(b->ev_t);
  delete b;
  return 0;
}

// The systolic chase (one launch): d, e2 of the tridiagonal. Returns 0 when done,
// 1 when the positions cannot all be co-resident, 2 after a timed-out hand-off.
int chase_systolic_run(gpmi_band* b, hipStream_t s, double* d, double* e2, bool split) {
  const int n = (int)b->n;
  const int K = (n - 1 + TS - 1) / TS;
  if (split ? 2 * K > b->split_maxg : K > b->chase_maxg) return 1;
  // per message slot: CHASE_MSG values as two tagged 8-byte granules each
  // four message kinds (the one-per-position kernel uses two) x (K + 1) positions
  const size_t slots = (size_t)(K + 1) * 2 * 2 * CHASE_MSG;
  if (!b->cmsg) {
    BD_TRY(hipMalloc(&b->cmsg, sizeof(unsigned long long) * 4 * slots + 64 + 8192));
  }
  int* err = reinterpret_cast<int*>(b->cmsg + 4 * slots);
  BD_TRY(hipMemsetAsync(b->cmsg, 0, sizeof(unsigned long long) * 4 * slots + 64 + 8192, s));
  if (split) {
    hipLaunchKernelGGL(chase_split_kernel, dim3(2 * K), dim3(CHASE_SPLIT_THREADS), 0, s, b->Ab,
                       (int64_t)b->n_pad, n, b->cmsg, K, err, b->chase_spin, d, e2);
    BD_LAUNCH("chase_split_kernel");
  } else {
    hipLaunchKernelGGL(chase_systolic_kernel, dim3(K), dim3(CHASE_THREADS), 0, s, b->Ab,
                       (int64_t)b->n_pad, n, b->cmsg, b->cmsg + slots, err, b->chase_spin, d, e2);
    BD_LAUNCH("chase_systolic_kernel");
  }
  int herr = 0;
  BD_TRY(hipMemcpyAsync(&herr, err, sizeof(int), hipMemcpyDeviceToHost, s));
  BD_TRY(hipStreamSynchronize(s));
#ifdef GPMI_CHASE_PROF
  {
    std::vector<long long> st(4 * 16 * 8);
    BD_TRY(hipMemcpy(st.data(), err + 16, sizeof(long long) * st.size(), hipMemcpyDeviceToHost));
    for (int q = 0; q < 4; ++q)
      for (int i = 0; i < 16; ++i) {
        const long long* t = st.data() + (q * 16 + i) * 8;
        const long long* tn = (i + 1 < 16) ? t + 8 : nullptr;
        fprintf(stderr, "[chase prof] k=%d s=%d dt(10ns): recvR %lld prod %lld post %lld upd %lld "
                "F %lld recvC %lld shift %lld\n", q + 1, 1000 + i, t[1] - t[0], t[2] - t[1],
                t[3] - t[2], t[4] - t[3], t[5] - t[4], t[6] - t[5], tn ? tn[0] - t[6] : 0LL);
      }
  }
#endif
  return herr ? 2 : 0;
}

// Y <- Q_j^T Y for panel j (Y = b->Y, rows from 128 (j + 1)) on stream st.
int qt_panel(gpmi_band* b, int j, hipStream_t st) {
  const int64_t np = b->n_pad;
  const int64_t r0 = (int64_t)(j + 1) * TS, c0 = (int64_t)j * TS;
  const int m = (int)(np - r0);
  const int G = (m + QT_ROWS - 1) / QT_ROWS;
  const double* P = b->Ab + r0 * np + c0;
  double* Yr = b->Y + r0 * RLD;
  hipLaunchKernelGGL(qt_partial_kernel, dim3(G), dim3(256), 0, st, P, np, m, Yr, b->qtp);
  BD_LAUNCH("qt_partial_kernel");
  hipLaunchKernelGGL(qt_reduce_kernel, dim3(TS * RLD / 256), dim3(256), 0, st, b->qtp, G, b->qa);
  BD_LAUNCH("qt_reduce_kernel");
  hipLaunchKernelGGL(qt_tb_kernel, dim3(1), dim3(256), 0, st, b->qa, b->Tm + (int64_t)j * TS * TS,
                     b->qb);
  BD_LAUNCH("qt_tb_kernel");
  hipLaunchKernelGGL(qt_apply_kernel, dim3(G), dim3(256), 0, st, P, np, m, Yr, b->qb);
  BD_LAUNCH("qt_apply_kernel");
  return 0;
}

// CholeskyQR panel j (gpmi_cholqr.hip): shifted CholeskyQR3 of the m x 128 panel,
// then Householder reconstruction into V (the panel below its top block), tau and
// S R (the top block). A failure sets the panel's flag [4] before anything is written
// to the panel, and the guarded Householder panel factors it instead.
int cq_guard(gpmi_band* b, int j, hipStream_t st);

// guard: launch the guarded Householder panel right behind the chain (false: the
// caller launches it, cq_guard, where every CU is free again)
int cq_panel(gpmi_band* b, int j, hipStream_t st, bool guard = true) {
  const int64_t np = b->n_pad;
  const int64_t r0 = (int64_t)(j + 1) * TS, c0 = (int64_t)j * TS;
  const int m = (int)(np - r0);
  const int mt = m / TS;
  double* P = b->Ab + r0 * np + c0;
  const double coef = 11.0 * ((double)m * TS + (double)TS * (TS + 1)) * 1.1102230246251565e-16;
  const int64_t pt = (int64_t)j * 3 * TS * TS;   // this panel's factor slots
  int* fl = b->cqflag + 8 * j;
  // Gram partials of P (64-row tiles), then per pass: reduce -> factor -> apply
  // (+ the next Gram)
  const int rt = m / 64;
  hipLaunchKernelGGL(cq_gram_kernel, dim3(rt), dim3(256), CQ_DYN_LDS, st, P, np, b->cqpart);
  BD_LAUNCH("cq_gram_kernel");
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(cq_reduce_kernel, dim3(CQ_GPK / 64), dim3(256), 0, st, b->cqpart, rt,
                       b->cqG);
    BD_LAUNCH("cq_reduce_kernel");
    double* L = b->cqL + pt + (int64_t)pass * TS * TS;
    double* Li = b->cqLinv + pt + (int64_t)pass * TS * TS;
    hipLaunchKernelGGL(cq_chol_kernel, dim3(1), dim3(256), 0, st, b->cqG, pass, coef,
                       b->cq_fo[pass], L, Li, fl, fl + 4, b->ctr);
    BD_LAUNCH("cq_chol_kernel");
    const double* src = pass == 0 ? P : b->Qb;
    hipLaunchKernelGGL(cq_apply_kernel, dim3(rt), dim3(256), CQ_DYN_LDS, st, src,
                       pass == 0 ? np : (int64_t)TS, b->Qb, (int64_t)TS, Li, b->cqpart,
                       nullptr);
    BD_LAUNCH("cq_apply_kernel");
  }
  hipLaunchKernelGGL(cq_reduce_kernel, dim3(CQ_GPK / 64), dim3(256), 0, st, b->cqpart, rt,
                     b->cqG);
  BD_LAUNCH("cq_reduce_kernel");
  // third factor, reconstruction: V1 into P, tau, S, C = U^-T M3
  hipLaunchKernelGGL(cq_recon_kernel, dim3(1), dim3(256), 0, st, b->Qb, b->cqG, b->cq_fo[2], P,
                     np, b->cqS + (int64_t)j * TS, b->tau + (int64_t)j * TS,
                     b->cqL + pt + 2 * TS * TS, b->cqLinv + pt + 2 * TS * TS, b->cqMinv, fl,
                     fl + 4, b->cqUS + (int64_t)j * TS * TS);
  BD_LAUNCH("cq_recon_kernel");
  // T = -U S V1^-T on the side stream beside the rest of the chain (exits when the
  // panel failed); the side stream's later work for this panel is behind it
  BD_TRY(hipEventRecord(b->ev_rc, st));
  BD_TRY(hipStreamWaitEvent(b->side, b->ev_rc, 0));
  hipLaunchKernelGGL(cq_t_kernel, dim3(1), dim3(256), 0, b->side, P, np,
                     b->cqUS + (int64_t)j * TS * TS, b->cqW + (int64_t)j * TS * TS,
                     b->Tm + (int64_t)j * TS * TS, fl + 4);
  BD_LAUNCH("cq_t_kernel");
  b->t_from_q[j] = 1;
  // V2 = Q2 C^T below the top block
  if (mt > 1) {
    hipLaunchKernelGGL(cq_apply_kernel, dim3(rt - 2), dim3(256), CQ_DYN_LDS, st, b->Qb + TS * TS,
                       (int64_t)TS, P + TS * np, np, b->cqMinv, nullptr, fl + 4);
    BD_LAUNCH("cq_apply_kernel");
  }
  return guard ? cq_guard(b, j, st) : 0;
}

// A failed CholeskyQR panel j (flag fl[4], P untouched) by the Householder panel in
// one launch, guarded on the device (it exits at once when the flag is clear); past
// that launch's size (G > panel_maxg workgroups cannot all be co-resident) the host
// reads the flag after the chain and, only for a failed panel, runs the per-column
// Householder launches on the same stream: that panel alone falls back, the
// reduction goes on (one host round trip per such panel). The guarded launch needs
// its G workgroups co-resident, so it runs where no SYR2K holds CUs.
int cq_guard(gpmi_band* b, int j, hipStream_t st) {
  const int64_t np = b->n_pad;
  const int64_t r0 = (int64_t)(j + 1) * TS, c0 = (int64_t)j * TS;
  const int m = (int)(np - r0);
  double* P = b->Ab + r0 * np + c0;
  int* fl = b->cqflag + 8 * j;
  const int G = (m + HH_ROWS - 1) / HH_ROWS;
  if (G <= b->panel_maxg) {
    // (it also copies the panel's reflectors into U, vcopy_kernel's work)
    hipLaunchKernelGGL(hh_panel_kernel, dim3(G), dim3(HH_THREADS), HH_PANEL_LDS, st, P, np, m,
                       b->part, b->pivrow, b->ctr, b->tau + (int64_t)j * TS, b->err,
                       b->spin_limit, fl + 4, b->U + r0 * BAND_ULD, (int64_t)BAND_ULD);
    BD_LAUNCH("hh_panel_kernel");
    b->v_in_u[j] = 1;
  } else {
    int failed = 0;
    BD_TRY(hipMemcpyAsync(&failed, fl + 4, sizeof(int), hipMemcpyDeviceToHost, st));
    BD_TRY(hipStreamSynchronize(st));
    ++b->cq_host_checks;
    if (failed) {
      for (int c = -1; c < TS; ++c) {
        hipLaunchKernelGGL(hh_col_kernel, dim3(G), dim3(HH_THREADS), 0, st, P, np, m, c, b->part,
                           b->pivrow, b->tau + (int64_t)j * TS);
        BD_LAUNCH("hh_col_kernel");
      }
    }
  }
  return 0;
}

// Panel j (columns [128 j, +128), rows from 128 (j + 1)) on st. mode 0: CholeskyQR;
// 1: Householder, one launch per panel where its workgroups fit; 2: Householder,
// one launch per column.
int panel_qr(gpmi_band* b, int j, hipStream_t st, int mode, bool* guard_deferred = nullptr) {
  const int64_t np = b->n_pad;
  const int64_t r0 = (int64_t)(j + 1) * TS, c0 = (int64_t)j * TS;
  if (guard_deferred) *guard_deferred = false;
  // a last panel with fewer than 128 real rows (ragged n: the rest is the zero
  // pad) has rank < 128, which CholeskyQR cannot orthonormalise: Householder
  if (mode == 0 && b->n - r0 >= TS) {
    if (guard_deferred) *guard_deferred = true;
    return cq_panel(b, j, st, guard_deferred == nullptr);
  }
  if (mode == 0) mode = 1;
  const int m = (int)(np - r0);
  const int G = (m + HH_ROWS - 1) / HH_ROWS;
  double* P = b->Ab + r0 * np + c0;
  double* tau = b->tau + (int64_t)j * TS;
  if (mode == 1 && G <= b->panel_maxg) {
    // one launch per panel (rows in registers, in-launch reductions)
    BD_TRY(hipMemsetAsync(b->ctr, 0, 512, st));
    hipLaunchKernelGGL(hh_panel_kernel, dim3(G), dim3(HH_THREADS), HH_PANEL_LDS, st, P, np, m,
                       b->part, b->pivrow, b->ctr, tau, b->err, b->spin_limit, nullptr, nullptr,
                       (int64_t)0);
    BD_LAUNCH("hh_panel_kernel");
  } else {
    for (int c = -1; c < TS; ++c) {
      hipLaunchKernelGGL(hh_col_kernel, dim3(G), dim3(HH_THREADS), 0, st, P, np, m, c, b->part,
                         b->pivrow, tau);
      BD_LAUNCH("hh_col_kernel");
    }
  }
  return 0;
}

// RHS [n][ld] (nrhs columns) -> the padded [n_pad][16] host layout of Y.
std::vector<double> pack_rhs(const gpmi_band* b, const double* rhs, int64_t ld, int nrhs) {
  std::vector<double> h((size_t)b->n_pad * RLD, 0.0);
  for (int64_t i = 0; i < b->n; ++i)
    for (int c = 0; c < nrhs; ++c) h[(size_t)i * RLD + c] = rhs[i * ld + c];
  return h;
}

// Dense -> band: panels j = 0 .. nt-2 of 128 columns (see gpmi_band.hip).
// With yh (the packed RHS), Y = Q^T R is applied panel by panel on the side
// stream as soon as each panel's T exists, beside the rest of the reduction.
// mode: the panel algorithm (panel_qr); mode 2 runs without look-ahead.
int band_reduce_pass(gpmi_band* b, const double* K, const std::vector<double>* yh, int mode) {
  hipStream_t s = b->stream;
  const int64_t np = b->n_pad;
  const int nt = b->nt;
  BD_TRY(hipMemsetAsync(b->err, 0, 16, s));
  if (mode == 0) BD_TRY(hipMemsetAsync(b->cqflag, 0, sizeof(int) * 8 * nt, s));
  BD_TRY(hipEventRecord(b->ev0, s));
  const auto host_t0 = std::chrono::steady_clock::now();
  if (yh) {
    BD_TRY(hipMemcpyAsync(b->Y, yh->data(), sizeof(double) * yh->size(), hipMemcpyHostToDevice,
                          b->side));
  }
  std::fill(b->t_from_q.begin(), b->t_from_q.end(), 0);
  std::fill(b->v_in_u.begin(), b->v_in_u.end(), 0);
  const bool la = mode != 2 && b->lookahead && b->s_pan;
  // The pipelined CholeskyQR form copies only tile column 0 of K into the working matrix:
  // the first panel's SYMM reads A22 from K, and its update (the tile column and the
  // pipelined SYR2K) reads its C tiles from K and writes them to Ab, which holds the
  // lower triangle from then on (the upper one is never read). 2 GB -> 16 MB at N = 16384
  // (the copy took 0.8 ms). Every other form copies all of K.
  const bool k_first = mode == 0 && la && nt > 2;
  if (k_first && b->poison)   // (tests: NaN wherever the reduction would read unwritten Ab)
    BD_TRY(hipMemsetAsync(b->Ab, 0xff, sizeof(double) * np * np, s));
  if (k_first)
    BD_TRY(hipMemcpy2DAsync(b->Ab, sizeof(double) * np, K, sizeof(double) * np,
                            sizeof(double) * TS, np, hipMemcpyDeviceToDevice, s));
  else
    BD_TRY(hipMemcpyAsync(b->Ab, K, sizeof(double) * np * np, hipMemcpyDeviceToDevice, s));
  bool ahead = false;   // panel j already factored by the previous look-ahead
  for (int j = 0; j + 1 < nt; ++j) {
    const int64_t r0 = (int64_t)(j + 1) * TS, c0 = (int64_t)j * TS;
    const int m = (int)(np - r0), mt = nt - j - 1;
    double* P = b->Ab + r0 * np + c0;
    double* tau = b->tau + (int64_t)j * TS;
    double* T = b->Tm + (int64_t)j * TS * TS;
    if (!ahead) {
      int rc = panel_qr(b, j, s, mode);
      if (rc) return rc;
    }
    ahead = false;
    double* Ur = b->U + r0 * BAND_ULD;
    if (!b->v_in_u[j]) {   // (the guarded Householder panel copied them already)
      hipLaunchKernelGGL(vcopy_kernel, dim3((unsigned)((int64_t)m * TS / 256)), dim3(256), 0, s,
                         P, np, m, Ur, (int64_t)BAND_ULD);
      BD_LAUNCH("vcopy_kernel");
    }
    const int nch = (m + TN_CH - 1) / TN_CH;
    // T from V^T V on the side stream, beside the SYMM (which needs only V)
    BD_TRY(hipEventRecord(b->ev_v, s));
    BD_TRY(hipStreamWaitEvent(b->side, b->ev_v, 0));
    if (b->t_from_q[j]) {
      // a CholeskyQR panel's T came from cq_t_kernel; only if it fell back does this
      // one-workgroup launch form it (it exits at once otherwise)
      hipLaunchKernelGGL(t_fallback_kernel, dim3(1), dim3(256), 0, b->side, Ur + TS,
                         (int64_t)BAND_ULD, m, tau, b->VtV, T, b->cqflag + 8 * j + 4);
      BD_LAUNCH("t_fallback_kernel");
    } else {
      hipLaunchKernelGGL(tn_partial_kernel, dim3(nch), dim3(256), 0, b->side, Ur + TS,
                         (int64_t)BAND_ULD, Ur + TS, (int64_t)BAND_ULD, m, b->tnp2, nullptr);
      BD_LAUNCH("tn_partial_kernel");
      hipLaunchKernelGGL(tn_reduce_kernel, dim3(TS * TS / 64), dim3(256), 0, b->side, b->tnp2,
                         nch, b->VtV, 1.0, nullptr);
      BD_LAUNCH("tn_reduce_kernel");
      hipLaunchKernelGGL(tbuild_kernel, dim3(1), dim3(256), 0, b->side, b->VtV, tau, T, nullptr);
      BD_LAUNCH("tbuild_kernel");
    }
    b->t_from_q[j] = 0;
    BD_TRY(hipEventRecord(b->ev_t, b->side));
    if (yh) {
      // Q_j^T on the side stream right after T_j (a stream of its own measured the
      // same, and a fourth stream of the reduction costs more elsewhere: DESIGN 5)
      int rc = qt_panel(b, j, b->side);
      if (rc) return rc;
    }
    const int chunk = symm_chunk(mt, 2 * b->ncu);
    const int sch = (mt + chunk - 1) / chunk;
    const double* ksrc = (k_first && j == 0) ? K : nullptr;   // panel 0: C and A22 from K
    hipLaunchKernelGGL(symm_kernel, dim3(mt, sch), dim3(256), 0, s, ksrc ? ksrc : b->Ab, np,
                       b->U, (int64_t)BAND_ULD, j + 1, mt, chunk, b->Xp);
    BD_LAUNCH("symm_kernel");
    hipLaunchKernelGGL(psum_kernel, dim3(TS * TS / 512, mt), dim3(256), 0, s, b->Xp, sch, b->X);
    BD_LAUNCH("psum_kernel");
    BD_TRY(hipStreamWaitEvent(s, b->ev_t, 0));
    // the serial 128^3 steps on quadrant workgroups (gemm_quad2, gpmi_tile.h; one
    // launch summing the split-K partials and forming X T per half tile instead:
    // slower, 139.0 against 138.2 ms, its 34-234 workgroups each read 1/2 of a row
    // tile's partials)
    hipLaunchKernelGGL(xt_q_kernel, dim3(mt, 4), dim3(256), 0, s, b->X, T, b->X2);
    BD_LAUNCH("xt_q_kernel");
    hipLaunchKernelGGL(tn_partial_q_kernel, dim3(nch, 4), dim3(256), 0, s, Ur + TS,
                       (int64_t)BAND_ULD, b->X2, (int64_t)TS, m, b->tnp);
    BD_LAUNCH("tn_partial_q_kernel");
    hipLaunchKernelGGL(tn_reduce_kernel, dim3(TS * TS / 64), dim3(256), 0, s, b->tnp, nch, b->M,
                       1.0, nullptr);
    BD_LAUNCH("tn_reduce_kernel");
    hipLaunchKernelGGL(z_q_kernel, dim3(4), dim3(256), 0, s, T, b->M, b->Zh);
    BD_LAUNCH("z_q_kernel");
    hipLaunchKernelGGL(w_q_kernel, dim3(mt, 4), dim3(256), 0, s, b->X2, Ur, (int64_t)BAND_ULD,
                       b->Zh);
    BD_LAUNCH("w_q_kernel");
    const int next_g = (int)((np - r0 - TS + HH_ROWS - 1) / HH_ROWS);   // panel j + 1's grid
    if (la && j + 2 < nt && (mode == 0 || next_g <= b->panel_maxg)) {
      // tile column 0 of the update (panel j + 1's columns) first; then that
      // panel's QR beside the rest of the update on a grid capped to la_grid
      // workgroups, so that the panel's workgroups find free CUs
      hipLaunchKernelGGL(syr2k_col_q_kernel, dim3(mt, 4), dim3(256), 0, s, b->Ab, np, b->U,
                         (int64_t)BAND_ULD, j + 1, ksrc);
      BD_LAUNCH("syr2k_col_q_kernel");
      BD_TRY(hipEventRecord(b->ev_col, s));
      BD_TRY(hipStreamWaitEvent(b->s_pan, b->ev_col, 0));
      const bool pipe = mode == 0;
      const int rest = (mt - 1) * mt / 2;
      const int la_free = mt < b->la_late_mt ? b->la_free_late : b->la_free;
      const int nmain = std::min(rest, std::max(1, b->ncu - la_free));
      int* tcnt = pipe ? b->cqflag + 8 * j + 6 : nullptr;
      // The rest of the update on s_pan, panel j + 1's QR on s right behind the tile
      // column it needs (round 5: the chain used to run on s_pan between two cross-stream
      // waits, ~12 us before it and ~10 us after it on every chain-bound late panel)
      if (pipe) {
        // one SYR2K workgroup per CU on all but la_free CUs, which the chain (its
        // single-workgroup kernels need a whole CU) has to itself
        hipLaunchKernelGGL(syr2k_pipe_kernel, dim3(nmain), dim3(256), 0, b->s_pan, b->Ab, np,
                           b->U, (int64_t)BAND_ULD, j + 1, mt, tcnt, nmain, 0, ksrc);
        BD_LAUNCH("syr2k_pipe_kernel");
      } else {
        // the Householder panel (its workgroups must be co-resident) beside a capped
        // grid; la_grid 0: leave exactly the panel's workgroup count of CUs free
        // (measured: slower than a fixed 128-workgroup cap at N = 16384, 302 vs 262 ms)
        const int cap = b->la_grid > 0 ? b->la_grid : std::max(64, b->ncu - next_g);
        hipLaunchKernelGGL(syr2k_rest_kernel, dim3(std::min(rest, cap)), dim3(256), 0, b->s_pan,
                           b->Ab, np, b->U, (int64_t)BAND_ULD, j + 1,
                           mt, b->rorder ? b->rorder + b->rorder_off[mt - 1] : nullptr);
        BD_LAUNCH("syr2k_rest_kernel");
      }
      BD_TRY(hipEventRecord(b->ev_pan, b->s_pan));
      bool guard = false;
      int rc = panel_qr(b, j + 1, s, mode, pipe ? &guard : nullptr);
      if (rc) return rc;
      if (tcnt && rest > nmain) {
        // the chain's CUs join the update once the chain ends (tickets of tcnt;
        // 139.2 against 141.0 ms at N = 16384; launched only from panels whose
        // update outlasts the chain: no difference)
        hipLaunchKernelGGL(syr2k_pipe_kernel, dim3(std::min(la_free, rest - nmain)), dim3(256),
                           0, s, b->Ab, np, b->U, (int64_t)BAND_ULD, j + 1, mt, tcnt, nmain, 1,
                           ksrc);
        BD_LAUNCH("syr2k_pipe_kernel");
      }
      BD_TRY(hipStreamWaitEvent(s, b->ev_pan, 0));
      if (guard) {
        // the guarded Householder panel behind the SYR2K (its workgroups must be
        // co-resident: every CU is free again here)
        rc = cq_guard(b, j + 1, s);
        if (rc) return rc;
      }
      ahead = true;
    } else {
      const int tiles = mt * (mt + 1) / 2;
      hipLaunchKernelGGL(syr2k_kernel, dim3(tiles), dim3(256), 0, s, b->Ab, np, b->U,
                         (int64_t)BAND_ULD, j + 1, mt);
      BD_LAUNCH("syr2k_kernel");
    }
  }
  if (yh) {
    BD_TRY(hipEventRecord(b->ev_q, b->side));
    BD_TRY(hipStreamWaitEvent(s, b->ev_q, 0));
  }
  if (mode == 0 && nt > 1) {
    // R (the band's subdiagonal blocks) of every CholeskyQR panel
    hipLaunchKernelGGL(cq_top_kernel, dim3(nt - 1), dim3(256), 0, s, b->cqL, b->cqLinv, b->cqflag,
                       b->cqS, b->cqscr, b->Ab, np);
    BD_LAUNCH("cq_top_kernel");
  }
  BD_TRY(hipEventRecord(b->ev1, s));
  // host time to enqueue the whole reduction (GPMI_BAND_TRACE: against its device time,
  // printed below; a device span not far above it would mean the host's launches bound it)
  const double host_enqueue_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - host_t0).count();
  int herr = 0;
  std::vector<int> hflag(mode == 0 ? 8 * nt : 0);
  BD_TRY(hipMemcpyAsync(&herr, b->err, sizeof(int), hipMemcpyDeviceToHost, s));
  if (mode == 0)
    BD_TRY(hipMemcpyAsync(hflag.data(), b->cqflag, sizeof(int) * hflag.size(),
                          hipMemcpyDeviceToHost, s));
  BD_TRY(hipEventSynchronize(b->ev1));
  BD_TRY(hipStreamSynchronize(s));
  if (herr) return set_error(-1201, "band reduction: panel hand-off timed out (workgroups not co-resident?)");
  if (mode == 0) {
    // failed CholeskyQR panels, each refactored in place during the pass (cq_panel)
    for (int j = 0; j + 1 < nt; ++j)
      if (hflag[8 * j + 4]) ++b->cq_panel_fallbacks;
  }
  float ms = 0.f;
  BD_TRY(hipEventElapsedTime(&ms, b->ev0, b->ev1));
  b->reduce_ms = ms;
  if (std::getenv("GPMI_BAND_TRACE"))
    fprintf(stderr, "[gpmi band] reduction %.3f ms on the device, enqueued in %.3f ms\n", ms,
            host_enqueue_ms);
  return 0;
}

// The reduction with the single-launch panel QR; if a hand-off times out (its
// workgroups were not all resident, e.g. the GPU is shared or partitioned), the
// whole reduction is redone from K with the per-column panel launches.
// CholeskyQR panels first (unless GPMI_BAND_PANEL=hh); if one of them reports a
// breakdown (a numerically rank-deficient panel) the reduction is redone with
// Householder panels.
int band_reduce(gpmi_band* b, const double* K, const std::vector<double>* yh = nullptr) {
  int rc;
  if (b->panel_mode == 0) {
    // a failed CholeskyQR panel is refactored in place (cq_panel); only a timed-out
    // guarded Householder panel (its workgroups not co-resident on a shared GPU)
    // sends the reduction back, straight to the per-column launches
    rc = band_reduce_pass(b, K, yh, 0);
    if (rc != -1201) return rc;
    ++b->cq_fallbacks;
    ++b->panel_fallbacks;
    return band_reduce_pass(b, K, yh, 2);
  }
  rc = band_reduce_pass(b, K, yh, 1);
  if (rc != -1201) return rc;
  ++b->panel_fallbacks;
  return band_reduce_pass(b, K, yh, 2);
}

int ensure_cap(gpmi_band* b, int neta) {
  if (b->cap >= neta) return 0;
  if (b->etas) BD_TRY(hipFree(b->etas));
  if (b->out) BD_TRY(hipFree(b->out));
  if (b->info) BD_TRY(hipFree(b->info));
  b->etas = b->out = nullptr;
  b->info = nullptr;
  b->cap = 0;
  const int cap = std::max(neta, 64);
  BD_TRY(hipMalloc(&b->etas, sizeof(double) * cap));
  BD_TRY(hipMalloc(&b->out, sizeof(double) * cap * OUT_LD));
  BD_TRY(hipMalloc(&b->info, sizeof(int) * cap));
  b->cap = cap;
  return 0;
}

}  // namespace

extern "C" {

int gpmi_band_create(gpmi_op* op, gpmi_band** out) {
  if (!out) return set_error(-1004, "null output handle");
  OpView v;
  int rc = op_view(op, &v);
  if (rc) return rc;
  if (!v.has_K) return set_error(-1000, "operator has no matrix (load or assemble first)");
  if (v.n_pad > BAND_MAX_NPAD) return set_error(-1200, "band path supports n <= 32768");
  Guard g(v.device);
  gpmi_band* b = new gpmi_band();
  b->device = v.device;
  b->n = v.n;
  b->n_pad = v.n_pad;
  b->nt = (int)(v.n_pad / TS);
  const int64_t np = b->n_pad;
  const int nt = b->nt;
  int ncu_alloc = 0;   // (b->ncu is read below; the Xp size needs it here)
  if (hipDeviceGetAttribute(&ncu_alloc, hipDeviceAttributeMultiprocessorCount, v.device) !=
      hipSuccess)
    ncu_alloc = 256;
  int64_t xp_tiles = 1;   // the largest mt x split-K chunks over the panels
  for (int mt = 1; mt < nt; ++mt) {
    const int ch = symm_chunk(mt, 2 * ncu_alloc);
    xp_tiles = std::max<int64_t>(xp_tiles, (int64_t)mt * ((mt + ch - 1) / ch));
  }
  const int nch = (int)std::max<int64_t>(1, (np + TN_CH - 1) / TN_CH);
  hipError_t e;
  auto fail = [&](hipError_t err, const char* what) {
    band_free(b);
    char msg[200];
    snprintf(msg, sizeof(msg), "allocation of %s failed: %s", what, hipGetErrorString(err));
    return set_error(-(int)err, msg);
  };
  if ((e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking)) != hipSuccess)
    return fail(e, "stream");
  if ((e = hipEventCreate(&b->ev0)) != hipSuccess) return fail(e, "event");
  if ((e = hipEventCreate(&b->ev1)) != hipSuccess) return fail(e, "event");
  if ((e = hipEventCreate(&b->ev2)) != hipSuccess) return fail(e, "event");
  if ((e = hipEventCreate(&b->ev3)) != hipSuccess) return fail(e, "event");
  if ((e = hipStreamCreateWithFlags(&b->side, hipStreamNonBlocking)) != hipSuccess)
    return fail(e, "side stream");
  if (const char* la = std::getenv("GPMI_BAND_LA")) b->lookahead = std::atoi(la);
  if (const char* po = std::getenv("GPMI_BAND_POISON")) b->poison = std::atoi(po) != 0;
  if (const char* v = std::getenv("GPMI_LA_FREE")) b->la_free = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("GPMI_LA_FREE_LATE")) b->la_free_late = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("GPMI_LA_LATE_MT")) b->la_late_mt = std::atoi(v);
  if (const char* pm = std::getenv("GPMI_BAND_PANEL")) b->panel_mode = std::strcmp(pm, "hh") == 0;
  if (const char* bm = std::getenv("GPMI_BAND_BCR")) b->bcr_mode = std::max(0, std::min(2, std::atoi(bm)));
  // GPMI_CQ_FO=0: every CholeskyQR pass by an exact Cholesky (no first-order passes)
  if (const char* fo = std::getenv("GPMI_CQ_FO"))
    if (std::atoi(fo) == 0) b->cq_fo[1] = b->cq_fo[2] = 0.0;

  if ((e = hipDeviceGetAttribute(&b->ncu, hipDeviceAttributeMultiprocessorCount, v.device)) !=
      hipSuccess)
    return fail(e, "CU count");
  if (b->lookahead) {
    // s_pan at the high dispatch priority. Alone, the priorities do not matter (135.5
    // ms all normal, 135.9-136.3 with one stream high); in a process that holds other
    // operators' streams (the bench line: the dense operator's) a high-priority stream
    // gets a hardware queue of its own, while normal-priority streams beyond the
    // process's GPU_MAX_HW_QUEUES (4) share queues and serialise: the bench line's
    // reduction took 165.4 ms with all three at normal priority, 137 with this one high
    int lo = 0, hi = 0;
    if ((e = hipDeviceGetStreamPriorityRange(&lo, &hi)) != hipSuccess) return fail(e, "prio");
    if ((e = hipStreamCreateWithPriority(&b->s_pan, hipStreamNonBlocking, hi)) != hipSuccess)
      return fail(e, "panel stream");
    for (hipEvent_t* ev : {&b->ev_col, &b->ev_pan})
      if ((e = hipEventCreateWithFlags(ev, sync_event_flags())) != hipSuccess)
        return fail(e, "event");
  }
  if ((e = hipEventCreateWithFlags(&b->ev_q, sync_event_flags())) != hipSuccess)
    return fail(e, "event");
  if ((e = hipEventCreateWithFlags(&b->ev_v, sync_event_flags())) != hipSuccess ||
      (e = hipEventCreateWithFlags(&b->ev_t, sync_event_flags())) != hipSuccess)
    return fail(e, "event");
#define BALLOC(ptr, count)                                                          \
  if ((e = hipMalloc(&b->ptr, sizeof(double) * (size_t)(count))) != hipSuccess)     \
    return fail(e, #ptr);
  BALLOC(Ab, np * np);
  BALLOC(U, np * BAND_ULD);
  BALLOC(X, np * TS);
  BALLOC(X2, np * TS);
  BALLOC(Xp, (size_t)xp_tiles * TS * TS);
  BALLOC(part, 2 * HH_MAXG * HH_PART_LD);
  BALLOC(pivrow, 2 * TS);
  BALLOC(tau, (size_t)nt * TS);
  BALLOC(Tm, (size_t)nt * TS * TS);
  BALLOC(tnp, (size_t)nch * TS * TS);
  BALLOC(tnp2, (size_t)nch * TS * TS);
  BALLOC(VtV, TS * TS);
  BALLOC(M, TS * TS);
  BALLOC(Zh, TS * TS);
  BALLOC(Y, np * RLD);
  BALLOC(qtp, (size_t)(np / QT_ROWS + 1) * TS * RLD);
  BALLOC(qa, TS * RLD);
  BALLOC(qb, TS * RLD);
  BALLOC(Qb, np * TS);
  BALLOC(cqpart, (size_t)(np / 64) * CQ_GPK);
  BALLOC(cqG, TS * TS);
  BALLOC(cqL, (size_t)nt * 3 * TS * TS);
  BALLOC(cqLinv, (size_t)nt * 3 * TS * TS);
  BALLOC(cqMinv, TS * TS);
  BALLOC(cqUS, (int64_t)nt * TS * TS);
  BALLOC(cqW, (int64_t)nt * TS * TS);
  if ((e = hipEventCreateWithFlags(&b->ev_rc, sync_event_flags())) != hipSuccess)
    return fail(e, "event");
  b->t_from_q.assign((size_t)nt, 0);
  b->v_in_u.assign((size_t)nt, 0);
  BALLOC(cqS, (size_t)nt * TS);
  BALLOC(cqscr, (size_t)nt * TS * TS);
#undef BALLOC
  if ((e = hipMalloc(&b->cqflag, sizeof(int) * 8 * nt)) != hipSuccess) return fail(e, "cqflag");
  if (nt > 2) {
    // row groups of RGROUP tile rows, column-major inside a group (packed (i << 16) | j)
    std::vector<uint32_t> h;
    b->rorder_off.assign(nt, 0);
    for (int w = 1; w < nt; ++w) {
      b->rorder_off[w] = (int64_t)h.size();
      for (int r0 = 0; r0 < w; r0 += RGROUP) {
        const int r1 = std::min(w, r0 + RGROUP);
        for (int j = 0; j < r1; ++j)
          for (int i = std::max(r0, j); i < r1; ++i) h.push_back(((uint32_t)i << 16) | (uint32_t)j);
      }
    }
    if ((e = hipMalloc(&b->rorder, sizeof(uint32_t) * h.size())) != hipSuccess)
      return fail(e, "rorder");
    if ((e = hipMemcpy(b->rorder, h.data(), sizeof(uint32_t) * h.size(), hipMemcpyHostToDevice)) !=
        hipSuccess)
      return fail(e, "rorder copy");
  }
  if ((e = hipMalloc(&b->ctr, 512)) != hipSuccess) return fail(e, "ctr");
  if ((e = hipMalloc(&b->err, 16)) != hipSuccess) return fail(e, "err");
  if ((e = hipMemsetAsync(b->err, 0, 16, b->stream)) != hipSuccess) return fail(e, "err memset");
  for (const void* f : {reinterpret_cast<const void*>(&cq_gram_kernel),
                        reinterpret_cast<const void*>(&cq_apply_kernel)})
    if ((e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, CQ_DYN_LDS)) !=
        hipSuccess)
      return fail(e, "CholeskyQR LDS attribute");
  // per device (this one is current): cheap, so set on every create
  if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(&hh_panel_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, HH_PANEL_LDS)) !=
      hipSuccess)
    return fail(e, "hh_panel LDS attribute");
  {
    int per_cu = 0;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
             &per_cu, reinterpret_cast<const void*>(&hh_panel_kernel), HH_THREADS,
             HH_PANEL_LDS)) != hipSuccess)
      return fail(e, "hh_panel occupancy");
    b->panel_maxg = std::min(HH_PANEL_MAXG, std::max(0, per_cu) * b->ncu);
  }
  {
    int per_cu = 0;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
             &per_cu, reinterpret_cast<const void*>(&chase_systolic_kernel), CHASE_THREADS, 0)) !=
        hipSuccess)
      return fail(e, "chase occupancy");
    b->chase_maxg = std::max(0, per_cu) * b->ncu;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
             &per_cu, reinterpret_cast<const void*>(&chase_split_kernel), CHASE_SPLIT_THREADS,
             0)) !=
        hipSuccess)
      return fail(e, "chase split occupancy");
    b->split_maxg = std::max(0, per_cu) * b->ncu;
  }
  // test hook: GPMI_CHASE_SPIN_LIMIT=0 times the systolic chase out at its first wait
  if (const char* sl = std::getenv("GPMI_CHASE_SPIN_LIMIT"))
    b->chase_spin = (unsigned)std::strtoul(sl, nullptr, 10);
  // test hook: GPMI_HH_SPIN_LIMIT=0 makes the first unsuccessful poll a timeout
  if (const char* sl = std::getenv("GPMI_HH_SPIN_LIMIT"))
    b->spin_limit = (unsigned)std::strtoul(sl, nullptr, 10);
  if ((e = hipMemsetAsync(b->U, 0, sizeof(double) * np * BAND_ULD, b->stream)) != hipSuccess)
    return fail(e, "U memset");
  if ((e = hipMemsetAsync(b->Y, 0, sizeof(double) * np * RLD, b->stream)) != hipSuccess)
    return fail(e, "Y memset");
  rc = band_reduce(b, v.K);
  if (rc) {
    band_free(b);
    return rc;
  }
  *out = b;
  return 0;
}

int gpmi_band_refresh(gpmi_band* b, gpmi_op* op) {
  if (!b) return set_error(-1006, "null handle");
  OpView v;
  int rc = op_view(op, &v);
  if (rc) return rc;
  if (!v.has_K) return set_error(-1000, "operator has no matrix (load or assemble first)");
  if (v.n != b->n || v.device != b->device)
    return set_error(-1202, "operator size or device differs from the band's");
  Guard g(b->device);
  b->nrhs = 0;
  return band_reduce(b, v.K);
}

int gpmi_band_refresh_rhs(gpmi_band* b, gpmi_op* op, const double* rhs, int64_t ld, int nrhs) {
  if (!b) return set_error(-1006, "null handle");
  if (nrhs < 0 || nrhs > RLD) return set_error(-1007, "nrhs outside [0, 16]");
  OpView v;
  int rc = op_view(op, &v);
  if (rc) return rc;
  if (!v.has_K) return set_error(-1000, "operator has no matrix (load or assemble first)");
  if (v.n != b->n || v.device != b->device)
    return set_error(-1202, "operator size or device differs from the band's");
  Guard g(b->device);
  b->nrhs = 0;
  const std::vector<double> h = pack_rhs(b, rhs, ld, nrhs);
  rc = band_reduce(b, v.K, &h);
  if (rc) return rc;
  b->nrhs = nrhs;
  b->rhs_ms = 0.0;   // overlapped with the reduction
  return 0;
}

int gpmi_band_destroy(gpmi_band* b) {
  if (!b) return 0;
  Guard g(b->device);
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  return band_free(b);
}

int gpmi_band_set_rhs(gpmi_band* b, const double* rhs, int64_t ld, int nrhs) {
  if (!b) return set_error(-1006, "null handle");
  if (nrhs < 0 || nrhs > RLD) return set_error(-1007, "nrhs outside [0, 16]");
  Guard g(b->device);
  hipStream_t s = b->stream;
  const int64_t np = b->n_pad;
  (void)np;
  const std::vector<double> h = pack_rhs(b, rhs, ld, nrhs);
  BD_TRY(hipEventRecord(b->ev0, s));
  BD_TRY(hipMemcpyAsync(b->Y, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice, s));
  for (int j = 0; j + 1 < b->nt; ++j) {
    int rc = qt_panel(b, j, s);
    if (rc) return rc;
  }
  BD_TRY(hipEventRecord(b->ev1, s));
  BD_TRY(hipEventSynchronize(b->ev1));
  float ms = 0.f;
  BD_TRY(hipEventElapsedTime(&ms, b->ev0, b->ev1));
  b->rhs_ms = ms;
  b->nrhs = nrhs;
  return 0;
}

// Tangent buffers for neta <= BAND_TAN_MAX etas (band_loglik_bcr / band_sinv_bcr
// with tan).
int ensure_tan(gpmi_band* b, int neta) {
  if (b->tcap >= neta) return 0;
  for (double** q : {&b->tanL, &b->tanW, &b->tanX, &b->tanZd, &b->tanZo, &b->tanD[0],
                     &b->tanD[1], &b->tanF[0], &b->tanF[1], &b->tanTr})
    if (*q) {
      BD_TRY(hipFree(*q));
      *q = nullptr;
    }
  b->tcap = 0;
  const int nt = b->nt, half = (nt + 1) / 2;
  const size_t blk = (size_t)TS * TS;
  BD_TRY(hipMalloc(&b->tanL, sizeof(double) * neta * nt * blk));
  BD_TRY(hipMalloc(&b->tanW, sizeof(double) * neta * nt * 2 * blk));
  BD_TRY(hipMalloc(&b->tanX, sizeof(double) * neta * nt * 2 * blk));
  BD_TRY(hipMalloc(&b->tanZd, sizeof(double) * neta * nt * blk));
  BD_TRY(hipMalloc(&b->tanZo, sizeof(double) * neta * nt * 2 * blk));
  for (int q = 0; q < 2; ++q) {
    BD_TRY(hipMalloc(&b->tanD[q], sizeof(double) * neta * half * blk));
    BD_TRY(hipMalloc(&b->tanF[q], sizeof(double) * neta * half * blk));
  }
  BD_TRY(hipMalloc(&b->tanTr, sizeof(double) * neta * (nt + 1)));
  b->tcap = neta;
  return 0;
}

// The likelihood terms of neta eta (b->etas on the device) by block cyclic
// reduction (gpmi_bcr.hip) into b->out / b->info, on stream s. With tan (neta <=
// b->tcap), also every eliminated block's dLinv and dW (bcr_dfac / bcr_dw / bcr_dupd)
// for band_sinv_bcr's exponent-2 trace.
int band_loglik_bcr(gpmi_band* b, int neta, hipStream_t s, bool tan = false) {
  const int nt = b->nt;
  const int64_t np = b->n_pad;
  const int half = (nt + 1) / 2;
  if (b->bcap < neta) {
    double** bufs[] = {&b->bcrD[0], &b->bcrD[1], &b->bcrF[0], &b->bcrF[1], &b->bcrY[0],
                       &b->bcrY[1], &b->bcrL, &b->bcrW, &b->bcrZ, &b->bcrG, &b->bcrLd,
                       &b->bcrX, &b->bcrZp, &b->bcrG2, &b->bcrG3};
    for (double** q : bufs)
      if (*q) {
        BD_TRY(hipFree(*q));
        *q = nullptr;
      }
    if (b->bcrFail) BD_TRY(hipFree(b->bcrFail));
    b->bcrFail = nullptr;
    b->bcap = 0;
    const size_t blk = (size_t)TS * TS, yb = (size_t)TS * RLD;
    for (int q = 0; q < 2; ++q) {
      BD_TRY(hipMalloc(&b->bcrD[q], sizeof(double) * neta * half * blk));
      BD_TRY(hipMalloc(&b->bcrF[q], sizeof(double) * neta * half * blk));
      BD_TRY(hipMalloc(&b->bcrY[q], sizeof(double) * neta * half * yb));
    }
    BD_TRY(hipMalloc(&b->bcrL, sizeof(double) * neta * nt * blk));
    BD_TRY(hipMalloc(&b->bcrW, sizeof(double) * neta * nt * 2 * blk));
    BD_TRY(hipMalloc(&b->bcrZ, sizeof(double) * neta * nt * yb));
    BD_TRY(hipMalloc(&b->bcrX, sizeof(double) * neta * nt * yb));
    BD_TRY(hipMalloc(&b->bcrZp, sizeof(double) * neta * nt * yb));
    BD_TRY(hipMalloc(&b->bcrG, sizeof(double) * neta * nt * RLD * RLD));
    BD_TRY(hipMalloc(&b->bcrG2, sizeof(double) * neta * nt * RLD * RLD));
    BD_TRY(hipMalloc(&b->bcrG3, sizeof(double) * neta * nt * RLD * RLD));
    BD_TRY(hipMalloc(&b->bcrLd, sizeof(double) * neta * nt));
    BD_TRY(hipMalloc(&b->bcrFail, sizeof(int) * neta * nt));
    b->bcap = neta;
  }
  if (!b->bcrF0 && nt > 1) BD_TRY(hipMalloc(&b->bcrF0, sizeof(double) * (nt - 1) * TS * TS));
  const int64_t sH = (int64_t)half * TS * TS, sHY = (int64_t)half * TS * RLD;
  const int64_t sZ = (int64_t)nt * TS * RLD, sL = (int64_t)nt * TS * TS, sW = 2 * sL;
  if (nt > 1) {
    hipLaunchKernelGGL(bcr_f0_kernel, dim3(nt - 1), dim3(256), 0, s, b->Ab, np, b->bcrF0);
    BD_LAUNCH("bcr_f0_kernel");
  }
  const double* Din = nullptr;
  const double* Yin = b->Y;
  const double* Fin = b->bcrF0;
  const double* dDin = nullptr;   // tangents of the level's D, F (level 0: I, 0)
  const double* dFin = nullptr;
  int64_t sD = 0, sY = 0, sF = 0;
  int m = nt, lvl = 0, cur = 0;
  bool dupd_pending = false;   // the last bcr_dupd_kernel (side stream) not yet waited for
  while (m > 1) {
    const int nodd = m / 2, neven = (m + 1) / 2;
    hipLaunchKernelGGL(bcr_chol_kernel, dim3(nodd, neta), dim3(256), 0, s, b->Ab, np, b->etas,
                       lvl, 1, Din, sD, Yin, sY, b->bcrL, sL, 1, b->bcrZ, sZ, b->bcrLd, b->bcrG,
                       b->bcrFail, nt, b->n);
    BD_LAUNCH("bcr_chol_kernel");
    // W (and with tangents the level's dLinv beside it), then D', F', Y' (and dW),
    // then dD', dF' on the side stream beside the next level's Cholesky (the dLinv of
    // the next bcr_w_kernel launch waits for them)
    if (dupd_pending) BD_TRY(hipStreamWaitEvent(s, b->ev_t, 0));
    dupd_pending = false;
    hipLaunchKernelGGL(bcr_w_kernel, dim3(2 * nodd + (tan ? nodd : 0), neta), dim3(256), 0, s,
                       b->bcrL, sL, Fin, sF, b->bcrW, sW, m, lvl, dDin, sH, b->tanX, b->tanL);
    BD_LAUNCH("bcr_w_kernel");
    hipLaunchKernelGGL(bcr_upd_kernel, dim3(3 * neven + (tan ? 2 * nodd : 0), neta), dim3(256), 0,
                       s, b->Ab, np, b->etas, lvl, Din, sD, Yin, sY, b->bcrW, sW, b->bcrZ, sZ,
                       b->bcrD[cur], b->bcrF[cur], b->bcrY[cur], sH, sHY, m, b->bcrL, b->tanL, sL,
                       Fin, sF, dFin, sH, b->tanW);
    BD_LAUNCH("bcr_upd_kernel");
    if (tan) {
      BD_TRY(hipEventRecord(b->ev_v, s));
      BD_TRY(hipStreamWaitEvent(b->side, b->ev_v, 0));
      hipLaunchKernelGGL(bcr_dupd_kernel, dim3(2 * neven, neta), dim3(256), 0, b->side, b->bcrW,
                         b->tanW, sW, dDin, sH, b->tanD[cur], b->tanF[cur], sH, m, lvl);
      BD_LAUNCH("bcr_dupd_kernel");
      BD_TRY(hipEventRecord(b->ev_t, b->side));
      dupd_pending = true;
      dDin = b->tanD[cur];
      dFin = b->tanF[cur];
    }
    Din = b->bcrD[cur];
    Yin = b->bcrY[cur];
    Fin = b->bcrF[cur];
    sD = sH;
    sY = sHY;
    sF = sH;
    cur ^= 1;
    m = neven;
    ++lvl;
  }
  hipLaunchKernelGGL(bcr_chol_kernel, dim3(1, neta), dim3(256), 0, s, b->Ab, np, b->etas, lvl, 0,
                     Din, sD, Yin, sY, b->bcrL, sL, 1, b->bcrZ, sZ, b->bcrLd, b->bcrG, b->bcrFail,
                     nt, b->n);
  BD_LAUNCH("bcr_chol_kernel");
  if (tan) {   // the last level's dLinv (bcr_w_kernel with m = 1: its dfac role only)
    if (dupd_pending) BD_TRY(hipStreamWaitEvent(s, b->ev_t, 0));
    hipLaunchKernelGGL(bcr_w_kernel, dim3(1, neta), dim3(256), 0, s, b->bcrL, sL, nullptr, 0,
                       nullptr, sW, 1, lvl, dDin, sH, b->tanX, b->tanL);
    BD_LAUNCH("bcr_w_kernel");
  }
  hipLaunchKernelGGL(bcr_final_kernel, dim3(neta), dim3(256), 0, s, b->bcrLd, b->bcrG, b->bcrFail,
                     nt, b->out, OUT_LD, b->info);
  BD_LAUNCH("bcr_final_kernel");
  return 0;
}

// Derivative terms by cyclic reduction (after band_loglik_bcr, whose levels stay
// stored): X = (B + eta I)^-1 Y by back substitution from the last level down, then
// the forward elimination of X; G2, G3 into b->der (gpmi_bcr.hip).
int band_der_solves(gpmi_band* b, int neta, hipStream_t s) {
  const int nt = b->nt;
  const int half = (nt + 1) / 2;
  const int64_t sHY = (int64_t)half * TS * RLD;
  const int64_t sZ = (int64_t)nt * TS * RLD, sL = (int64_t)nt * TS * TS, sW = 2 * sL;
  std::vector<int> ms;   // blocks per level, the last level has one
  for (int m = nt; m > 1; m = (m + 1) / 2) ms.push_back(m);
  const int L = (int)ms.size();
  hipLaunchKernelGGL(bcr_back_kernel, dim3(1, neta), dim3(256), 0, s, b->bcrL, sL, b->bcrW, sW,
                     b->bcrZ, sZ, b->bcrX, b->bcrG2, nt, L, 0, 1);
  BD_LAUNCH("bcr_back_kernel");
  for (int l = L - 1; l >= 0; --l) {
    hipLaunchKernelGGL(bcr_back_kernel, dim3(ms[l] / 2, neta), dim3(256), 0, s, b->bcrL, sL,
                       b->bcrW, sW, b->bcrZ, sZ, b->bcrX, b->bcrG2, nt, l, 1, ms[l]);
    BD_LAUNCH("bcr_back_kernel");
  }
  const double* Yin = b->bcrX;
  int64_t sY = sZ;
  int cur = 0;
  for (int l = 0; l < L; ++l) {
    hipLaunchKernelGGL(bcr_rhs_odd_kernel, dim3(ms[l] / 2, neta), dim3(256), 0, s, b->bcrL, sL,
                       Yin, sY, b->bcrZp, sZ, b->bcrG3, nt, l, 1);
    BD_LAUNCH("bcr_rhs_odd_kernel");
    hipLaunchKernelGGL(bcr_rhs_even_kernel, dim3((ms[l] + 1) / 2, neta), dim3(256), 0, s, b->bcrW,
                       sW, b->bcrZp, sZ, Yin, sY, b->bcrY[cur], sHY, l, ms[l]);
    BD_LAUNCH("bcr_rhs_even_kernel");
    Yin = b->bcrY[cur];
    sY = sHY;
    cur ^= 1;
  }
  hipLaunchKernelGGL(bcr_rhs_odd_kernel, dim3(1, neta), dim3(256), 0, s, b->bcrL, sL, Yin, sY,
                     b->bcrZp, sZ, b->bcrG3, nt, L, 0);
  BD_LAUNCH("bcr_rhs_odd_kernel");
  hipLaunchKernelGGL(bcr_der_final_kernel, dim3(neta), dim3(256), 0, s, b->bcrG2, b->bcrG3, nt,
                     b->der);
  BD_LAUNCH("bcr_der_final_kernel");
  return 0;
}

int band_der_bcr(gpmi_band* b, int neta, hipStream_t s) {
  int rc = band_loglik_bcr(b, neta, s);
  if (rc) return rc;
  return band_der_solves(b, neta, s);
}

// tr((B + eta_e I)^-1) for the neta etas whose cyclic-reduction factor band_loglik_bcr
// left in bcrL / bcrW: selected inversion down the tree, top-down (gpmi_bcr.hip
// bcr_sinv_*), into sinvTr[nt * neta + e] (device). With tan (the factor's tangents
// computed by band_loglik_bcr(.., tan)) also tr((B + eta_e I)^-2) into
// tanTr[nt * neta + e] (bcr_dsinv_*).
int band_sinv_bcr(gpmi_band* b, int neta, hipStream_t s, bool tan = false) {
  const int nt = b->nt;
  const size_t blk = (size_t)TS * TS;
  if (b->scap < neta) {
    for (double** q : {&b->sinvZd, &b->sinvZo, &b->sinvX, &b->sinvTr})
      if (*q) {
        BD_TRY(hipFree(*q));
        *q = nullptr;
      }
    b->scap = 0;
    BD_TRY(hipMalloc(&b->sinvZd, sizeof(double) * neta * nt * blk));
    BD_TRY(hipMalloc(&b->sinvZo, sizeof(double) * neta * nt * 2 * blk));
    BD_TRY(hipMalloc(&b->sinvX, sizeof(double) * neta * nt * 2 * blk));
    BD_TRY(hipMalloc(&b->sinvTr, sizeof(double) * neta * (nt + 1)));
    b->scap = neta;
  }
  const int64_t sL = (int64_t)nt * blk, sW = 2 * sL, sZd = sL, sZo = 2 * sL, sX = 2 * sL;
  std::vector<int> ms;   // blocks per level; the last level has one
  for (int m = nt; m > 1; m = (m + 1) / 2) ms.push_back(m);
  const int L = (int)ms.size();
  const int nt_ = tan ? 1 : 0;
  // every block's X_l, X_r, Linv^T Linv (and tangents), the root's trace
  hipLaunchKernelGGL(bcr_sinv_pre_kernel, dim3(nt * (3 + 3 * nt_), neta), dim3(256), 0, s,
                     b->bcrL, b->tanL, sL, b->bcrW, b->tanW, sW, b->sinvX, b->tanX, sX, b->sinvZd,
                     b->tanZd, sZd, b->sinvTr, b->tanTr, nt, L, b->n, nt_);
  BD_LAUNCH("bcr_sinv_pre_kernel");
  for (int l = L - 1; l >= 0; --l) {
    const int nodd = ms[l] / 2;
    hipLaunchKernelGGL(bcr_sinv_off_kernel, dim3((2 + 2 * nt_) * nodd, neta), dim3(256), 0, s,
                       b->sinvZd, b->tanZd, sZd, b->sinvZo, b->tanZo, sZo, b->sinvX, b->tanX, sX,
                       ms[l], l, nt_);
    BD_LAUNCH("bcr_sinv_off_kernel");
    hipLaunchKernelGGL(bcr_sinv_diag_kernel, dim3((1 + nt_) * nodd, neta), dim3(256), 0, s,
                       b->sinvX, b->tanX, sX, b->sinvZo, b->tanZo, sZo, b->sinvZd, b->tanZd, sZd,
                       b->sinvTr, b->tanTr, nt, b->n, ms[l], l, nt_);
    BD_LAUNCH("bcr_sinv_diag_kernel");
  }
  hipLaunchKernelGGL(bcr_sinv_final_kernel, dim3((neta + 63) / 64), dim3(64), 0, s, b->sinvTr, nt,
                     b->sinvTr + (size_t)nt * neta, neta);
  BD_LAUNCH("bcr_sinv_final_kernel");
  if (tan) {
    hipLaunchKernelGGL(bcr_sinv_final_kernel, dim3((neta + 63) / 64), dim3(64), 0, s, b->tanTr,
                       nt, b->tanTr + (size_t)nt * neta, neta);
    BD_LAUNCH("bcr_sinv_final_kernel");
  }
  return 0;
}

int gpmi_band_loglik(gpmi_band* b, const double* etas, int neta, double* logdet, double* gram,
                     int* info) {
  if (!b) return set_error(-1006, "null handle");
  if (neta <= 0) return 0;
  Guard g(b->device);
  int rc = ensure_cap(b, neta);
  if (rc) return rc;
  hipStream_t s = b->stream;
  BD_TRY(hipMemcpyAsync(b->etas, etas, sizeof(double) * neta, hipMemcpyHostToDevice, s));
  BD_TRY(hipEventRecord(b->ev0, s));
  if (b->bcr_mode == 1 || (b->bcr_mode == 2 && neta <= 64)) {
    rc = band_loglik_bcr(b, neta, s);
    if (rc) return rc;
  } else {
    hipLaunchKernelGGL(band_chol_kernel, dim3(neta), dim3(256), 0, s, b->Ab, b->n_pad, b->nt,
                       b->n, b->Y, b->etas, b->out, OUT_LD, b->info, nullptr, nullptr);
    BD_LAUNCH("band_chol_kernel");
  }
  BD_TRY(hipEventRecord(b->ev1, s));
  std::vector<double> hout((size_t)neta * OUT_LD);
  std::vector<int> hinfo(neta);
  BD_TRY(hipMemcpyAsync(hout.data(), b->out, sizeof(double) * hout.size(), hipMemcpyDeviceToHost,
                        s));
  BD_TRY(hipMemcpyAsync(hinfo.data(), b->info, sizeof(int) * neta, hipMemcpyDeviceToHost, s));
  BD_TRY(hipStreamSynchronize(s));
  float ms = 0.f;
  BD_TRY(hipEventElapsedTime(&ms, b->ev0, b->ev1));
  b->loglik_ms = ms;
  const int m = b->nrhs;
  for (int e = 0; e < neta; ++e) {
    if (logdet) logdet[e] = hout[(size_t)e * OUT_LD];
    if (gram)
      for (int a = 0; a < m; ++a)
        for (int c = 0; c < m; ++c)
          gram[((size_t)e * m + a) * m + c] = hout[(size_t)e * OUT_LD + 1 + a * RLD + c];
    if (info) info[e] = hinfo[e];
  }
  return 0;
}

int gpmi_band_der_terms(gpmi_band* b, const double* etas, int neta, double* logdet,
                        double* g1, double* g2, double* g3, int* info) {
  return gpmi_band_der_terms_ex(b, etas, neta, logdet, g1, g2, g3, nullptr, info);
}

int gpmi_band_der_terms_ex(gpmi_band* b, const double* etas, int neta, double* logdet,
                           double* g1, double* g2, double* g3, double* tr1, int* info) {
  return gpmi_band_der_terms_ex2(b, etas, neta, logdet, g1, g2, g3, tr1, nullptr, info);
}

int gpmi_band_der_terms_ex2(gpmi_band* b, const double* etas, int neta, double* logdet,
                            double* g1, double* g2, double* g3, double* tr1, double* tr2,
                            int* info) {
  if (!b) return set_error(-1006, "null handle");
  if (neta <= 0) return 0;
  if (neta > GPMI_BAND_DER_MAX)
    return set_error(-1203, "gpmi_band_der_terms: at most GPMI_BAND_DER_MAX etas per call");
  if (tr2 && neta > GPMI_BAND_TAN_MAX) {
    // the tangent store is sized per chunk: chunks of GPMI_BAND_TAN_MAX etas
    const size_t mm = (size_t)b->nrhs * b->nrhs;
    for (int c = 0; c < neta; c += GPMI_BAND_TAN_MAX) {
      const int k = std::min(GPMI_BAND_TAN_MAX, neta - c);
      int rc = gpmi_band_der_terms_ex2(b, etas + c, k, logdet ? logdet + c : nullptr,
                                       g1 ? g1 + c * mm : nullptr, g2 ? g2 + c * mm : nullptr,
                                       g3 ? g3 + c * mm : nullptr, tr1 ? tr1 + c : nullptr,
                                       tr2 + c, info ? info + c : nullptr);
      if (rc) return rc;
    }
    return 0;
  }
  std::vector<double> tr1_scratch;
  if (tr2 && !tr1) {
    tr1_scratch.resize(neta);
    tr1 = tr1_scratch.data();
  }
  Guard g(b->device);
  int rc = ensure_cap(b, neta);
  if (rc) return rc;
  const int64_t np = b->n_pad;
  const int nt = b->nt;
  if (b->dcap < neta) {
    if (b->fac) BD_TRY(hipFree(b->fac));
    if (b->ysol) BD_TRY(hipFree(b->ysol));
    if (b->der) BD_TRY(hipFree(b->der));
    b->fac = b->ysol = b->der = nullptr;
    b->dcap = 0;
    BD_TRY(hipMalloc(&b->fac, sizeof(double) * neta * nt * 2 * TS * TS));
    BD_TRY(hipMalloc(&b->ysol, sizeof(double) * neta * np * RLD));
    BD_TRY(hipMalloc(&b->der, sizeof(double) * neta * 2 * RLD * RLD));
    b->dcap = neta;
  }
  if (tr2 && (rc = ensure_tan(b, neta))) return rc;
  hipStream_t s = b->stream;
  BD_TRY(hipMemcpyAsync(b->etas, etas, sizeof(double) * neta, hipMemcpyHostToDevice, s));
  BD_TRY(hipEventRecord(b->ev0, s));
  // tr1 needs the cyclic-reduction factor (the tree it inverts along); the selected
  // inversion (side stream) and the G2 / G3 solves (s) both read only the factor, so
  // they run side by side
  if (tr1) {
    if ((rc = band_loglik_bcr(b, neta, s, tr2 != nullptr))) return rc;
    BD_TRY(hipEventRecord(b->ev_q, s));
    BD_TRY(hipStreamWaitEvent(b->side, b->ev_q, 0));
    BD_TRY(hipEventRecord(b->ev2, b->side));
    if ((rc = band_sinv_bcr(b, neta, b->side, tr2 != nullptr))) return rc;
    BD_TRY(hipEventRecord(b->ev3, b->side));
    if ((rc = band_der_solves(b, neta, s))) return rc;
    BD_TRY(hipStreamWaitEvent(s, b->ev3, 0));
  } else if (b->bcr_mode == 1 || (b->bcr_mode == 2 && neta <= 64)) {
    rc = band_der_bcr(b, neta, s);
    if (rc) return rc;
  } else {
    hipLaunchKernelGGL(band_chol_kernel, dim3(neta), dim3(256), 0, s, b->Ab, np, nt, b->n, b->Y,
                       b->etas, b->out, OUT_LD, b->info, b->fac, b->ysol);
    BD_LAUNCH("band_chol_kernel");
    hipLaunchKernelGGL(band_der_kernel, dim3(neta), dim3(256), 0, s, b->fac, nt, b->ysol,
                       b->der);
    BD_LAUNCH("band_der_kernel");
  }
  std::vector<double> htr, htr2;
  if (tr1) {
    htr.resize(neta);
    BD_TRY(hipMemcpyAsync(htr.data(), b->sinvTr + (size_t)nt * neta, sizeof(double) * neta,
                          hipMemcpyDeviceToHost, s));
    if (tr2) {
      htr2.resize(neta);
      BD_TRY(hipMemcpyAsync(htr2.data(), b->tanTr + (size_t)nt * neta, sizeof(double) * neta,
                            hipMemcpyDeviceToHost, s));
    }
  }
  BD_TRY(hipEventRecord(b->ev1, s));
  std::vector<double> hout((size_t)neta * OUT_LD), hder((size_t)neta * 2 * RLD * RLD);
  std::vector<int> hinfo(neta);
  BD_TRY(hipMemcpyAsync(hout.data(), b->out, sizeof(double) * hout.size(), hipMemcpyDeviceToHost,
                        s));
  BD_TRY(hipMemcpyAsync(hder.data(), b->der, sizeof(double) * hder.size(), hipMemcpyDeviceToHost,
                        s));
  BD_TRY(hipMemcpyAsync(hinfo.data(), b->info, sizeof(int) * neta, hipMemcpyDeviceToHost, s));
  BD_TRY(hipStreamSynchronize(s));
  float ms = 0.f;
  BD_TRY(hipEventElapsedTime(&ms, b->ev0, b->ev1));
  b->der_ms = ms;
  if (tr1) {
    float ms2 = 0.f;
    BD_TRY(hipEventElapsedTime(&ms2, b->ev2, b->ev3));
    b->sinv_ms = ms2;
    for (int e = 0; e < neta; ++e) tr1[e] = htr[e];
    if (tr2)
      for (int e = 0; e < neta; ++e) tr2[e] = htr2[e];
  }
  const int m = b->nrhs;
  for (int e = 0; e < neta; ++e) {
    if (logdet) logdet[e] = hout[(size_t)e * OUT_LD];
    for (int a = 0; a < m; ++a)
      for (int c = 0; c < m; ++c) {
        const size_t o = ((size_t)e * m + a) * m + c;
        if (g1) g1[o] = hout[(size_t)e * OUT_LD + 1 + a * RLD + c];
        if (g2) g2[o] = hder[(size_t)e * 2 * RLD * RLD + a * RLD + c];
        if (g3) g3[o] = hder[(size_t)e * 2 * RLD * RLD + RLD * RLD + a * RLD + c];
      }
    if (info) info[e] = hinfo[e];
  }
  return 0;
}

int gpmi_band_traceinv(gpmi_band* b, const double* etas, int neta, double* tr, int* info) {
  return gpmi_band_traceinv2(b, etas, neta, tr, nullptr, info);
}

int gpmi_band_traceinv2(gpmi_band* b, const double* etas, int neta, double* tr1, double* tr2,
                        int* info) {
  if (!b) return set_error(-1006, "null handle");
  if (neta <= 0) return 0;
  if (neta > GPMI_BAND_DER_MAX)
    return set_error(-1203, "gpmi_band_traceinv: at most GPMI_BAND_DER_MAX etas per call");
  if (!tr1) return set_error(-1006, "gpmi_band_traceinv2: tr1 is required");
  if (tr2 && neta > GPMI_BAND_TAN_MAX) {
    for (int c = 0; c < neta; c += GPMI_BAND_TAN_MAX) {
      const int k = std::min(GPMI_BAND_TAN_MAX, neta - c);
      int rc = gpmi_band_traceinv2(b, etas + c, k, tr1 + c, tr2 + c, info ? info + c : nullptr);
      if (rc) return rc;
    }
    return 0;
  }
  Guard g(b->device);
  int rc = ensure_cap(b, neta);
  if (rc) return rc;
  const bool tan = tr2 != nullptr;
  if (tan && (rc = ensure_tan(b, neta))) return rc;
  hipStream_t s = b->stream;
  BD_TRY(hipMemcpyAsync(b->etas, etas, sizeof(double) * neta, hipMemcpyHostToDevice, s));
  BD_TRY(hipEventRecord(b->ev0, s));
  if ((rc = band_loglik_bcr(b, neta, s, tan))) return rc;
  BD_TRY(hipEventRecord(b->ev2, s));
  if ((rc = band_sinv_bcr(b, neta, s, tan))) return rc;
  BD_TRY(hipEventRecord(b->ev1, s));
  std::vector<double> htr(neta), htr2(tan ? neta : 0);
  std::vector<int> hinfo(neta);
  BD_TRY(hipMemcpyAsync(htr.data(), b->sinvTr + (size_t)b->nt * neta, sizeof(double) * neta,
                        hipMemcpyDeviceToHost, s));
  if (tan)
    BD_TRY(hipMemcpyAsync(htr2.data(), b->tanTr + (size_t)b->nt * neta, sizeof(double) * neta,
                          hipMemcpyDeviceToHost, s));
  BD_TRY(hipMemcpyAsync(hinfo.data(), b->info, sizeof(int) * neta, hipMemcpyDeviceToHost, s));
  BD_TRY(hipStreamSynchronize(s));
  float ms = 0.f;
  BD_TRY(hipEventElapsedTime(&ms, b->ev2, b->ev1));
  b->sinv_ms = ms;
  for (int e = 0; e < neta; ++e) {
    tr1[e] = htr[e];
    if (tan) tr2[e] = htr2[e];
    if (info) info[e] = hinfo[e];
  }
  return 0;
}

int gpmi_band_sinv_ms(gpmi_band* b, double* ms) {
  if (!b || !ms) return set_error(-1006, "null handle");
  *ms = b->sinv_ms;
  return 0;
}

int gpmi_band_eigenvalues(gpmi_band* b, double* lam) {
  if (!b) return set_error(-1006, "null handle");
  Guard g(b->device);
  hipStream_t s = b->stream;
  const int64_t np = b->n_pad;
  const int n = (int)b->n;
  if (!b->td) {
    // td: [n] diagonal, [n] squared subdiagonal, [n] eigenvalues, then the launch
    // form's reflector slots (two wavefront parities x ((n - 2) / 128 + 3) slots of 130)
    BD_TRY(hipMalloc(&b->td, sizeof(double) * (3 * np + 2 * ((np - 2) / TS + 3) * (TS + 2))));
  }
  double* d = b->td;
  double* e2 = b->td + np;
  double* dl = b->td + 2 * np;
  BD_TRY(hipEventRecord(b->ev0, s));
  // GPMI_CHASE_MODE: systolic (default; one launch), split (reflector + per-block
  // launches per wavefront t = 3 s + k), task (one workgroup per task per wavefront)
  // GPMI_CHASE_MODE: unset = the systolic chase with a D and an E workgroup per
  // position if its 2K workgroups fit, else one workgroup per position (K), else the
  // launch form; "systolic" = one workgroup per position; "split" / "task" = the
  // launch forms
  const char* mode_env = std::getenv("GPMI_CHASE_MODE");
  const int chase_mode = !mode_env ? 0 : std::strcmp(mode_env, "split") == 0 ? 1
                                     : std::strcmp(mode_env, "task") == 0    ? 2
                                     : std::strcmp(mode_env, "systolic") == 0 ? 3 : 0;
  bool done = false;
  b->chase_systolic = 0;
  if ((chase_mode == 0 || chase_mode == 3) && n > 2) {
    int rc = 1;
    if (chase_mode == 0) {
      rc = chase_systolic_run(b, s, d, e2, true);
      if (rc < 0) return rc;
      if (rc == 2) ++b->chase_fallbacks;
      if (rc == 0) b->chase_systolic = 2;
    }
    if (rc != 0) {
      rc = chase_systolic_run(b, s, d, e2, false);
      if (rc < 0) return rc;
      if (rc == 2) ++b->chase_fallbacks;
      if (rc == 0) b->chase_systolic = 1;
    }
    done = rc == 0;
  }
  if (!done) {
  if (!b->Ac) BD_TRY(hipMalloc(&b->Ac, sizeof(double) * np * np));
  hipLaunchKernelGGL(chase_copy_kernel, dim3(n), dim3(256), 0, s, b->Ab, b->Ac, np, n);
  BD_LAUNCH("chase_copy_kernel");
  const bool chase_split = chase_mode != 2;
  const int kmax = (n - 2) / TS + 1;
  const int tmax = 3 * std::max(0, n - 3) + kmax;
  for (int t = 0; t <= tmax && n > 2; ++t) {
    const int s_hi = std::min(t / 3, n - 3);
    const int s_lo = std::max(0, (t - kmax + 2) / 3);
    if (s_hi < s_lo) continue;
    if (chase_split) {
      // reflector slots by sweep (s % ns), double-buffered by wavefront parity: the
      // E workgroup of (s, k) writes the reflector of (s, k + 1) for wavefront t + 1;
      // a sweep's first task (t = 3 s) gets its own small launch
      const int ns = kmax + 2;
      double* scr = b->td + 3 * np;
      double* rd = scr + (int64_t)(t & 1) * ns * (TS + 2);
      double* wr = scr + (int64_t)((t + 1) & 1) * ns * (TS + 2);
      if (t % 3 == 0 && t / 3 >= s_lo && t / 3 <= s_hi) {
        const int s0 = t / 3;
        hipLaunchKernelGGL(chase_reflect_kernel, dim3(1), dim3(TS), 0, s, b->Ac, np, n, s0,
                           rd + (int64_t)(s0 % ns) * (TS + 2));
        BD_LAUNCH("chase_reflect_kernel");
      }
      hipLaunchKernelGGL(chase_apply_kernel, dim3(3 * (s_hi - s_lo + 1)), dim3(512), 0, s, b->Ac,
                         np, n, t, s_hi, rd, wr, ns);
      BD_LAUNCH("chase_apply_kernel");
    } else {
      hipLaunchKernelGGL(chase_task_kernel, dim3(s_hi - s_lo + 1), dim3(512), 0, s, b->Ac, np, n,
                         t, s_hi);
      BD_LAUNCH("chase_task_kernel");
    }
  }
  hipLaunchKernelGGL(tridiag_extract_kernel, dim3((n + 255) / 256), dim3(256), 0, s, b->Ac, np, n,
                     d, e2);
  BD_LAUNCH("tridiag_extract_kernel");
  }
  std::vector<double> hd(n), he2(n);
  BD_TRY(hipMemcpyAsync(hd.data(), d, sizeof(double) * n, hipMemcpyDeviceToHost, s));
  BD_TRY(hipMemcpyAsync(he2.data(), e2, sizeof(double) * n, hipMemcpyDeviceToHost, s));
  BD_TRY(hipStreamSynchronize(s));
  // Gershgorin interval and the dstebz pivot floor
  double lo = hd[0], hi = hd[0], emax = 0.0;
  for (int i = 0; i < n; ++i) {
    const double el = i > 0 ? std::sqrt(he2[i - 1]) : 0.0;
    const double er = i + 1 < n ? std::sqrt(he2[i]) : 0.0;
    lo = std::min(lo, hd[i] - el - er);
    hi = std::max(hi, hd[i] + el + er);
    emax = std::max(emax, he2[i]);
  }
  const double span = std::max(hi - lo, std::fabs(hi)) * 1e-15 + 1e-300;
  lo -= span;
  hi += span;
  const double pivmin = 2.2250738585072014e-308 * std::max(1.0, emax);
  // GPMI_BISECT=1: one thread per eigenvalue (plain bisection) instead of multisection
  const char* bis = std::getenv("GPMI_BISECT");
  if (bis && std::atoi(bis) == 1) {
    hipLaunchKernelGGL(bisect_kernel, dim3((n + 255) / 256), dim3(256), 0, s, d, e2, n, lo, hi,
                       pivmin, dl);
    BD_LAUNCH("bisect_kernel");
  } else {
    const int64_t lanes = (int64_t)n * BISECT_LANES;
    hipLaunchKernelGGL(bisect_multi_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s,
                       d, e2, n, lo, hi, pivmin, dl);
    BD_LAUNCH("bisect_multi_kernel");
  }
  BD_TRY(hipMemcpyAsync(lam, dl, sizeof(double) * n, hipMemcpyDeviceToHost, s));
  BD_TRY(hipEventRecord(b->ev1, s));
  BD_TRY(hipStreamSynchronize(s));
  float ms = 0.f;
  BD_TRY(hipEventElapsedTime(&ms, b->ev0, b->ev1));
  b->eig_ms = ms;
  return 0;
}

int gpmi_band_get(gpmi_band* b, double* B_out, int64_t ld) {
  if (!b) return set_error(-1006, "null handle");
  Guard g(b->device);
  const int64_t np = b->n_pad, n = b->n;
  std::vector<double> h((size_t)np * np);
  BD_TRY(hipMemcpyAsync(h.data(), b->Ab, sizeof(double) * h.size(), hipMemcpyDeviceToHost,
                        b->stream));
  BD_TRY(hipStreamSynchronize(b->stream));
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < n; ++j) {
      const int64_t hi = std::max(i, j), lo = std::min(i, j);
      B_out[i * ld + j] = (hi - lo <= TS) ? h[(size_t)hi * np + lo] : 0.0;
    }
  return 0;
}

int gpmi_band_last_timing(gpmi_band* b, double* reduce_ms, double* rhs_ms, double* loglik_ms) {
  if (!b) return set_error(-1006, "null handle");
  if (std::getenv("GPMI_BAND_TRACE")) fprintf(stderr, "[gpmi band] eigenvalues %.3f ms\n", b->eig_ms);
  if (reduce_ms) *reduce_ms = b->reduce_ms;
  if (rhs_ms) *rhs_ms = b->rhs_ms;
  if (loglik_ms) *loglik_ms = b->loglik_ms;
  return 0;
}

int gpmi_band_chase_info(gpmi_band* b, int* systolic, int* fallbacks, int* maxg) {
  if (!b) return set_error(-1006, "null handle");
  if (systolic) *systolic = b->chase_systolic;
  if (fallbacks) *fallbacks = b->chase_fallbacks;
  if (maxg) *maxg = b->chase_maxg;
  return 0;
}

int gpmi_band_cq_stats(gpmi_band* b, int* panel_mode, int* cq_fallbacks,
                       int* cq_panel_fallbacks) {
  if (!b) return set_error(-1006, "null handle");
  if (panel_mode) *panel_mode = b->panel_mode;
  if (cq_fallbacks) *cq_fallbacks = b->cq_fallbacks;
  if (cq_panel_fallbacks) *cq_panel_fallbacks = b->cq_panel_fallbacks;
  return 0;
}

int gpmi_band_stats(gpmi_band* b, int* panel_fallbacks, int* panel_maxg) {
  if (!b) return set_error(-1006, "null handle");
  if (panel_fallbacks) *panel_fallbacks = b->panel_fallbacks;
  if (panel_maxg) *panel_maxg = b->panel_maxg;
  return 0;
}

int gpmi_band_der_ms(gpmi_band* b, double* der_ms) {
  if (!b) return set_error(-1006, "null handle");
  if (der_ms) *der_ms = b->der_ms;
  return 0;
}

}  // extern "C"
