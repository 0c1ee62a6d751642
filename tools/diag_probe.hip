// Phase timing of diag_block_kernel (diagnostic build with GPMI_DIAG_STAMPS).
// Build (from tools/): hipcc --offload-arch=gfx950 -O3 -DGPMI_DIAG_STAMPS -DGPMI_CHOL_STAMPS=1
//        -I../gaussian-process-param-estimation_amd/csrc -I../include diag_probe.hip -o probe/diag_probe
// (lds_chol_block's per-block phases print from the kernel, 10 ns units)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "gpmi_diag.hip"



#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

int main() {
  const int nb = 8, TS = 128, lda = 128;
  std::vector<double> hA((size_t)nb * TS * TS);
  for (int b = 0; b < nb; ++b)
    for (int i = 0; i < TS; ++i)
      for (int j = 0; j < TS; ++j)
        hA[(size_t)b * TS * TS + i * TS + j] = std::exp(-std::fabs(i - j) * 0.05) + (i == j ? 0.5 : 0.0);
  double *A, *R, *U, *Linv, *ld, *gram; int* info;
  CK(hipMalloc(&A, hA.size() * 8)); CK(hipMalloc(&R, nb * TS * 16 * 8)); CK(hipMalloc(&U, nb * TS * 16 * 8));
  CK(hipMalloc(&Linv, nb * TS * TS * 8)); CK(hipMalloc(&ld, nb * 8)); CK(hipMalloc(&gram, nb * 256 * 8));
  CK(hipMalloc(&info, nb * 4)); CK(hipMemset(info, 0, nb * 4)); CK(hipMemset(R, 0, nb * TS * 16 * 8));
  CK(hipMemcpy(A, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
  gpmi::BatchPtrs P{A, (int64_t)TS * TS, R, (int64_t)TS * 16, U, (int64_t)TS * 16, Linv, (int64_t)TS * TS, ld, 1, gram, 256, info};
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipMemcpy(A, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(gpmi::diag_block_kernel, dim3(nb), dim3(256), 0, 0, P, (int64_t)lda, 0, 1);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long st[64];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(gpmi::g_diag_stamps), sizeof(st)));
    printf("rep %d: %.1f us (s_memtime cycles) load %llu chol %llu | Lwrite %llu inv+rhs-load %llu "
           "Linvwrite %llu rhs %llu total %llu\n", rep, ms * 1e3, st[1] - st[0], st[26] - st[1],
           st[26] - st[26], st[27] - st[26], st[28] - st[27], st[29] - st[28], st[29] - st[0]);
  }
  double hld[8]; CK(hipMemcpy(hld, ld, 64, hipMemcpyDeviceToHost));
  printf("logdet block0 %.12f\n", hld[0]);
  return 0;
}
