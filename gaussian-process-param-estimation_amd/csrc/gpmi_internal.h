// Internal declarations shared by the gpmi HIP translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#define GPMI_MAX_DIM 8     // max point dimension handled by the assembly kernel
#define GPMI_TS 128        // tile / diagonal-block size of the blocked Cholesky
#define GPMI_RHS_LD 16     // leading dimension (max columns) of a resident RHS block

struct gpmi_sp;   // include/gpmi.h

namespace gpmi {

// Flags of the events that only order one device's streams (never read by the host):
// no timing, and no system-scope fence on record (the default release writes back and
// invalidates caches for host visibility, which a consumer kernel on the same device
// does not need). GPMI_EV_SYSFENCE=1 restores the system-scope fence (A/B).
inline unsigned sync_event_flags() {
  static const unsigned f = [] {
    const char* e = getenv("GPMI_EV_SYSFENCE");
    return (unsigned)hipEventDisableTiming |
           ((e && e[0] == '1') ? 0u : (unsigned)hipEventDisableSystemFence);
  }();
  return f;
}
// Timing events (elapsed time only; the host never reads memory behind them): timing
// kept, the system-scope fence dropped the same way.
inline unsigned timing_event_flags() {
  return sync_event_flags() & ~(unsigned)hipEventDisableTiming;
}

enum MaternMode { MATERN_HALF = 0, MATERN_3HALF = 1, MATERN_5HALF = 2,
                  MATERN_GENERAL = 3, MATERN_GAUSS = 4 };

struct MaternParams {
  int mode;
  double nu;
  double sqrt2nu;     // sqrt(2 nu)
  double mu;          // general nu >= 2: starting order nu - floor(nu) + 1 in [1, 2)
  double lp0, lp1;    // log(2^(1-a) / Gamma(a)) at a = mu, mu + 1 (a = nu when nu < 2)
};

// Dense Matérn assembly: lower-triangular 64 x 64 tiles (grid = T (T + 1) / 2,
// T = ceil(n_pad / 64)), each mirrored (gpmi_matern.hip).
void launch_matern_dense(dim3 grid, hipStream_t s, const double* points, int64_t n, int d,
                         const double* scale, const MaternParams& P, double* K, int64_t ldk,
                         int64_t n_pad);

// Batched factorization kernels (gpmi_chol.hip). All matrices are row-major
// n_pad x n_pad with leading dimension lda; batch member b lives at base + b*stride.
struct BatchPtrs {
  double* A;        int64_t sA;       // working matrices K + eta_b I -> L
  double* R;        int64_t sR;       // RHS blocks [n_pad][16] -> L^-1 R
  double* U;        int64_t sU;       // per-step u_k = A_kk^-1 r_k  [128][16]
  double* Linv;     int64_t sL;       // inverses of the diagonal blocks [nt][128][128]
  double* logdiag;  int64_t sLD;      // per diagonal block: 2 sum log L_ii  [nt]
  double* gram;     int64_t sG;       // per diagonal block Gram partials [nt][16][16]
  int* info;                          // first non-positive pivot (1-based), per member
};

__global__ void shift_copy_kernel(const double* K, int64_t ldk, double* A, int64_t lda,
                                  int64_t sA, const double* etas, int nb, int64_t n,
                                  int wc);
__global__ void diag_block_kernel(BatchPtrs P, int64_t lda, int kb, int nt);
__global__ void panel_kernel(BatchPtrs P, int64_t lda, int kb);
__global__ void syrk_kernel(double* A, int64_t lda, int64_t sA, int tc0, int w, int t,
                            int p0, int kdim, const uint32_t* order, const double* Ksrc,
                            const double* etas, int64_t n);
__global__ void finalize_kernel(BatchPtrs P, int nt, double* out, int out_ld);
__global__ void bwd_step_kernel(BatchPtrs P, int64_t lda, int kb, double* X, int64_t sX);
__global__ void fwd_step_kernel(BatchPtrs P, int64_t lda, int kb);
__global__ void gemv_sym_kernel(const double* K, int64_t ldk, int64_t n,
                                const double* x, int64_t ldx, int ncol, double* y,
                                double eta, int exponent);
__global__ void trace_kernel(const double* K, int64_t ldk, int64_t n, double* out);
__global__ void trinv_diag_kernel(const double* Linv, double* W, int64_t ldw, int k,
                                  double* partial);
__global__ void trinv_update_kernel(const double* L, int64_t lda, double* W, int64_t ldw, int i0,
                                    int nj, int kb, int ke);
__global__ void gram_panel_kernel(double* W, int64_t ldw, double* Td, int p0, int kdim,
                                  int imax);
__global__ void gram_sumsq_kernel(const double* W, int64_t ldw, const double* Td,
                                  double* partial);
__global__ void matern_eval_kernel(const double* x, int64_t m, MaternParams P, double* out);

// Multi-shift CG Gram state (gpmi_sparse.hip, gpmi_sparse_api.hip); device pointers.
constexpr int MS_MAXS = 16;   // RHS columns per multi-shift block
#ifndef GPMI_LZ_JC
#define GPMI_LZ_JC 16
#endif
constexpr int LZ_JC = GPMI_LZ_JC;   // basis vectors per lz_dots_kernel launch (DCGS2 Lanczos)

// A multi-shift CG batch's end state, written by the batch's last ms_tail_kernel
// (block 0) straight into host-mapped pinned memory: the host reads it after an
// event behind that kernel (no copy launches; round 4 copied the three fields with
// three hipMemcpyAsync blits, ~75 us per batch with their gaps).
// The Chronopoulos-Gear multi-shift CG (ms_cg2_update_kernel): the seed scalars,
// double-buffered by iteration parity (every block of iteration k reads cur, block 0
// writes nxt), and the shift state only block 0 touches.
struct MsScal {
  double* rr;      // [s] gamma_{k-1} = r_{k-1} . r_{k-1} (cur at iteration k)
  double* a;       // [s] alpha_{k-1}
  double* a_prev;  // [s] alpha_{k-2}
  double* beta;    // [s] beta_{k-2}
  int* active;     // [s] the column took step k-1
};
struct MsShift {
  double* bn2;     // [s] ||b_c||^2
  double* z;       // [S][s] zeta_j
  double* z_prev;  // [S][s]
  double* bp;      // [S][s'][s] b_c' . p_{j,c}
  double* g;       // [S][s'][s] accumulated G_j[c'][c]
  int* flags;      // [1] p^T (K + eta_0 I) p <= 0 in an active column
  int* it_stop;    // [1] the first iteration with no active column (-1: none yet)
};
constexpr int MS_UB = 512;      // vector blocks of ms_cg2_update_kernel (256 / 1024: cfg 5
                                // 12.37 / 12.12 against 11.91 ms per step)
constexpr int MS_DOT_BLK = 256; // blocks of ms_dots2_kernel (SpMM kinds without the epilogue)

// One active-column compaction of the multi-shift CG as ONE launch (round 6): up to
// MS_CJOBS column gathers src[r][s][L] -> dst[r][a][L] by the map, the stopped columns'
// Grams scattered into their final slots (gfin[jc][s0], by original column), and the
// compacted block's active flags set. Everything by value: no host copy, no sync.
constexpr int MS_CJOBS = 12;
struct MsCompactJob {
  const double* src;
  double* dst;
  int64_t rows;
  int L;
  int pad;
};
struct MsCompactArgs {
  MsCompactJob job[MS_CJOBS];
  int njob, s, a, nd, s0, pad;
  int map[MS_MAXS];         // the kept columns (old block index), in order
  int drop[MS_MAXS];        // the dropped columns (old block index)
  int drop_orig[MS_MAXS];   // their original column
  const double* g;          // [SN][s] the old block's Grams
  double* gfin;             // [SN][s0]
  int64_t SN;               // S * nbd
  const int* act_src;       // [s] the old block's active flags at the compaction
  int* act;                 // [a] the compacted block's (a kept column may have stopped
                            //     since the slot the map came from was written)
};

struct MsPin {
  int act[MS_MAXS];
  int flag;
  int pad;
  double rr[MS_MAXS];
  double bn2[MS_MAXS];   // ||b_c||^2, written by ms_init_kernel into both slots
};

// Scatter a sparse operator's CSR (original point order) into a zeroed dense
// [n][ldk] matrix on the same device (gpmi_sparse_api.hip).
int sp_scatter_dense(const ::gpmi_sp* sp, int device, double* K, int64_t ldk,
                     hipStream_t st);

}  // namespace gpmi
