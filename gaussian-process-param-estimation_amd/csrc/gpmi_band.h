// Band path (gpmi_band.hip, gpmi_band_api.hip): constants and kernel declarations.
#pragma once

#include "gpmi_internal.h"

namespace gpmi {

enum { KFAST = 0, KSLOW = 1 };

constexpr int HH_WAVES = 8;        // hh_col workgroup: 8 waves x 16 rows = 128 panel rows
constexpr int HH_THREADS = 64 * HH_WAVES;
constexpr int HH_RPW = 16;
constexpr int HH_ROWS = HH_WAVES * HH_RPW;
constexpr int HH_MAXG = 256;       // max hh_col workgroups (n_pad <= 32768)
constexpr int HH_PANEL_MAXG = 128;  // hh_panel (single-launch) workgroups: m <= 16384
constexpr int HH_PANEL_LDS = 96 * 1024;  // dynamic LDS: one hh_panel workgroup per CU
constexpr int HH_PART_LD = 136;    // partial record: S_j (j < 128), sum x^2 at [128]
constexpr int QT_ROWS = 64;        // rows per qt_partial / qt_apply workgroup
constexpr int TN_CH = 128;         // rows per tn_partial chunk
constexpr int SY_CH = 16;          // tile columns per symm split-K chunk (at most)
// symm split-K chunk for an mt-tile trailing block on `slots` resident workgroups (two
// per CU): the mt x ceil(mt / chunk) workgroups run in ceil(W / slots) rounds of chunk
// 128^3 products each, so the chunk minimising rounds x chunk (+ the partial sums'
// reads, ~1/620 of a product each) ends the grid in full rounds: at mt = 117, chunk 9
// (1521 workgroups, 2.97 rounds of 512) instead of mt^2 / 1024 = 13 (1053, 2.06 rounds
// run as 3: the third nearly empty, 1.06 ms against ~0.73).
inline int symm_chunk(int mt, int slots) {
  int best = 1;
  long long bc = -1;
  for (int ch = 1; ch <= SY_CH; ++ch) {
    const long long w = (long long)mt * ((mt + ch - 1) / ch);
    const long long c = (w + slots - 1) / slots * ch * 620 + w;
    if (bc < 0 || c <= bc) {
      bc = c;
      best = ch;
    }
  }
  return best;
}
constexpr int BAND_ULD = 384;      // U = [W | V | W]
// CUs the pipelined look-ahead SYR2K (one workgroup per CU) leaves to the next panel's
// CholeskyQR chain, whose single-workgroup kernels need a whole CU (N = 16384:
// 16 171 ms, 24-28 172-173, 32 153, 36 153, 40 154, 48 155, 64 158; the capped
// two-per-CU SYR2K 160). A filler launch gives them back to the update once the
// chain ends; with it: 24 164, 32 139.2-139.6, 40 140.4, 48 140.4, 64 140.1 ms.
constexpr int LA_FREE = 32;
// The last panels (trailing tile count mt < LA_LATE_MT) are chain-bound: their SYR2K
// is short and the chain's many-workgroup kernels (cq_gram / cq_apply, m / 64
// workgroups) finish sooner on more CUs. Free CUs for mt < T (32 above; N = 16384,
// one box): 64 for T = 60 137.0 ms, 96 137.7, 128 137.6; 64 for T = 40 138.1, T = 80
// 137.3; against 138.7-139.0 with 32 throughout (and 64 for mt >= 50: 140.0).
constexpr int LA_FREE_LATE = 64;
constexpr int LA_LATE_MT = 60;
constexpr int BAND_MAX_NPAD = HH_MAXG * HH_ROWS;

__global__ void hh_col_kernel(double* P, int64_t lda, int m, int c, double* part, double* pivrow,
                              double* tau);
__global__ void hh_panel_kernel(double* P, int64_t lda, int m, double* part, double* pivrow,
                                unsigned* counter, double* tau, int* err, unsigned spin_limit,
                                const int* guard, double* Uv, int64_t ldu);
__global__ void vcopy_kernel(const double* P, int64_t lda, int m, double* U, int64_t ldu);
__global__ void tn_partial_kernel(const double* P1, int64_t ld1, const double* P2, int64_t ld2,
                                  int m, double* part, const int* only_if);
__global__ void tn_reduce_kernel(const double* part, int nch, double* out, double scale,
                                 const int* only_if);
__global__ void tbuild_kernel(const double* VtV, const double* tau, double* T, const int* only_if);
__global__ void t_fallback_kernel(const double* V, int64_t ldv, int m, const double* tau,
                                  double* VtV, double* T, const int* only_if);
__global__ void symm_kernel(const double* A, int64_t lda, const double* U, int64_t ldu, int tr0,
                            int mt, int chunk, double* Xp);
__global__ void psum_kernel(const double* Xp, int nch, double* X);
__global__ void xt_q_kernel(const double* X, const double* T, double* X2);
__global__ void tn_partial_q_kernel(const double* P1, int64_t ld1, const double* P2, int64_t ld2,
                                    int m, double* part);
__global__ void z_q_kernel(const double* T, const double* M, double* Zh);
__global__ void w_q_kernel(const double* X, double* U, int64_t ldu, const double* Zh);
__global__ void syr2k_col_q_kernel(double* A, int64_t lda, const double* U, int64_t ldu, int tr0,
                                   const double* Ksrc);
__global__ void syr2k_kernel(double* A, int64_t lda, const double* U, int64_t ldu, int tr0,
                             int mt);
__global__ void syr2k_rest_kernel(double* A, int64_t lda, const double* U, int64_t ldu, int tr0,
                                  int mt, const uint32_t* order);
__global__ void syr2k_pipe_kernel(double* A, int64_t lda, const double* U, int64_t ldu, int tr0,
                                  int mt, int* cnt, int nmain, int filler, const double* Ksrc);
__global__ void bcr_f0_kernel(const double* Ab, int64_t lda, double* F0);
__global__ void bcr_chol_kernel(const double* Ab, int64_t lda, const double* etas, int lvl,
                                int first, const double* Din, int64_t sD, const double* Yin,
                                int64_t sY, double* Lout, int64_t sL, int lout, double* Zall,
                                int64_t sZ, double* logd, double* gpart, int* failv, int nt,
                                int64_t n);
__global__ void bcr_w_kernel(const double* Lin, int64_t sL, const double* Fin, int64_t sF,
                             double* W, int64_t sW, int m, int lvl, const double* dDin,
                             int64_t sdD, double* scr, double* dL);
__global__ void bcr_upd_kernel(const double* Ab, int64_t lda, const double* etas, int lvl,
                               const double* Din, int64_t sD, const double* Yin, int64_t sY,
                               const double* W, int64_t sW, const double* Zall, int64_t sZ,
                               double* Dout, double* Fout, double* Yout, int64_t sO, int64_t sOY,
                               int m, const double* L, const double* dL, int64_t sL,
                               const double* Fin, int64_t sF, const double* dFin, int64_t sdF,
                               double* dW);
__global__ void bcr_sinv_pre_kernel(const double* L, const double* dL, int64_t sL, const double* W,
                                    const double* dW, int64_t sW, double* X, double* dX,
                                    int64_t sX, double* Zd, double* dZd, int64_t sZd,
                                    double* trpart, double* dtrpart, int nt, int nlev, int64_t n,
                                    int ntan);
__global__ void bcr_sinv_off_kernel(const double* Zd, const double* dZd, int64_t sZd, double* Zo,
                                    double* dZo, int64_t sZo, const double* X, const double* dX,
                                    int64_t sX, int m, int lvl, int ntan);
__global__ void bcr_sinv_diag_kernel(const double* X, const double* dX, int64_t sX,
                                     const double* Zo, const double* dZo, int64_t sZo, double* Zd,
                                     double* dZd, int64_t sZd, double* trpart, double* dtrpart,
                                     int nt, int64_t n, int m, int lvl, int ntan);
__global__ void bcr_back_kernel(const double* L, int64_t sL, const double* W, int64_t sW,
                                const double* Zall, int64_t sZ, double* Xall, double* g2part,
                                int nt, int lvl, int first, int m);
__global__ void bcr_rhs_odd_kernel(const double* L, int64_t sL, const double* Yin, int64_t sY,
                                   double* Zp, int64_t sZ, double* g3part, int nt, int lvl,
                                   int first);
__global__ void bcr_rhs_even_kernel(const double* W, int64_t sW, const double* Zp, int64_t sZ,
                                    const double* Yin, int64_t sY, double* Yout, int64_t sOY,
                                    int lvl, int m);
__global__ void bcr_der_final_kernel(const double* g2part, const double* g3part, int nt,
                                     double* der);
__global__ void bcr_sinv_final_kernel(const double* trpart, int nt, double* tr, int neta);
__global__ void bcr_dupd_kernel(const double* W, const double* dW, int64_t sW, const double* dDin,
                                int64_t sdD, double* dDout, double* dFout, int64_t sO, int m,
                                int lvl);
__global__ void bcr_final_kernel(const double* logd, const double* gpart, const int* failv, int nt,
                                 double* out, int out_ld, int* info);
__global__ void qt_partial_kernel(const double* P, int64_t lda, int m, const double* Y,
                                  double* part);
__global__ void qt_reduce_kernel(const double* part, int G, double* a);
__global__ void qt_tb_kernel(const double* a, const double* T, double* b);
__global__ void qt_apply_kernel(const double* P, int64_t lda, int m, double* Y, const double* b);
__global__ void band_chol_kernel(const double* B, int64_t lda, int nt, int64_t n, const double* Y,
                                 const double* etas, double* out, int out_ld, int* info,
                                 double* fac, double* ysol);
__global__ void cq_chol_kernel(const double* G, int pass, double coef, double tau_fo, double* Lout,
                               double* Linv, int* fo, int* fail, unsigned* ctr);
__global__ void cq_gram_kernel(const double* Src, int64_t lds, double* part);
__global__ void cq_reduce_kernel(const double* part, int np, double* G);
constexpr int CQ_GPK = 36 * 256;   // doubles per packed CholeskyQR Gram partial
__global__ void cq_apply_kernel(const double* Src, int64_t lds, double* Dst, int64_t ldd,
                                const double* M, double* part, const int* skip);
__global__ void cq_recon_kernel(const double* Q2, const double* G3, double tau_fo, double* P,
                                int64_t lda, double* S, double* tau, double* Lx3, double* Linv3,
                                double* C, int* fo, int* fail, double* US);
__global__ void cq_t_kernel(const double* P, int64_t lda, const double* US, double* W, double* T,
                            const int* fail);
constexpr int CQ_DYN_LDS = 64 * (GPMI_TS + 4) * 8;   // cq_gram / cq_apply dynamic LDS (bytes)
__global__ void cq_top_kernel(double* Lx, const double* Linv, const int* flags, const double* S,
                              double* scr, double* Ab, int64_t lda);
__global__ void band_der_kernel(const double* fac, int nt, double* ysol, double* der);

__global__ void chase_copy_kernel(const double* Ab, double* A, int64_t lda, int n);
constexpr int CHASE_MSG = 136;   // = CMSG (gpmi_chase.hip): values per hand-off slot
constexpr int CHASE_THREADS = 512;   // = SCT (gpmi_chase.hip): systolic chase workgroup
#ifndef GPMI_CHASE_SPLIT_THREADS
#define GPMI_CHASE_SPLIT_THREADS 512
#endif
constexpr int CHASE_SPLIT_THREADS = GPMI_CHASE_SPLIT_THREADS;   // split chase workgroup
__global__ void chase_split_kernel(const double* Ab, int64_t lda, int n, unsigned long long* msg,
                                   int K, int* err, unsigned spin_limit, double* dout,
                                   double* e2out);
__global__ void chase_systolic_kernel(const double* Ab, int64_t lda, int n,
                                      unsigned long long* msg_r, unsigned long long* msg_c,
                                      int* err, unsigned spin_limit, double* dout, double* e2out);
__global__ void chase_task_kernel(double* A, int64_t lda, int n, int t, int s_hi);
__global__ void chase_reflect_kernel(double* A, int64_t lda, int n, int s, double* sl);
__global__ void chase_apply_kernel(double* A, int64_t lda, int n, int t, int s_hi,
                                   const double* rd, double* wr, int ns);
__global__ void tridiag_extract_kernel(const double* A, int64_t lda, int n, double* d, double* e2);
__global__ void bisect_kernel(const double* d, const double* e2, int n, double lo0, double hi0,
                              double pivmin, double* lam);
__global__ void bisect_multi_kernel(const double* d, const double* e2, int n, double lo0,
                                    double hi0, double pivmin, double* lam);
#ifndef GPMI_BISECT_LANES
#define GPMI_BISECT_LANES 16
#endif
constexpr int BISECT_LANES = GPMI_BISECT_LANES;   // lanes per eigenvalue (multisection)

// Read-only view of an operator for the band path (gpmi_api.hip).
struct OpView {
  int device;
  int64_t n, n_pad;
  const double* K;
  bool has_K;
};

}  // namespace gpmi
