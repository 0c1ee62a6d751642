// Dev microbenchmark: the achievable fp64 MFMA rate on this MI355X
// (v_mfma_f64_16x16x4f64 back-to-back, 16 independent accumulators per wave,
// every CU busy), to price the syrk roofline against a measured ceiling next to
// the 78.6 TFLOP/s spec figure. Build:
//   hipcc --offload-arch=gfx950 -O3 tools/fp64_peak.hip -o tools/fp64_peak
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void peak_kernel(double* out, int iters, double seed) {
  d4 acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  // 8 x 16 MFMAs per trip, so the loop-carried accumulator copies the compiler
  // adds at the back edge are amortized
  for (int it = 0; it < iters; it += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0.0;
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  double* out;
  const int waves_per_simd[] = {1, 2, 4};
  for (int wps : waves_per_simd) {
    const int nblk = ncu * wps;   // 256 threads = 4 waves = one per SIMD
    hipMalloc(&out, (size_t)nblk * 256 * sizeof(double));
    const int iters = 4000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    peak_kernel<<<nblk, 256>>>(out, 10, 1.0);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) peak_kernel<<<nblk, 256>>>(out, iters, 1.0 + r);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)reps * nblk * 4 * (double)iters * 16 * 2048.0;
    printf("{\"kernel\": \"fp64_mfma_16x16x4_peak\", \"cus\": %d, \"waves_per_simd\": %d, "
           "\"tflops\": %.2f, \"ms\": %.3f}\n", ncu, wps, flops / (ms * 1e-3) / 1e12, ms);
    hipFree(out);
  }
  return 0;
}
