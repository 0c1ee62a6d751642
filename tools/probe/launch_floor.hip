// Probe: what one dependent kernel launch costs on one stream (the band reduction's
// serial steps and CholeskyQR chain are chains of small kernels). Times K back-to-back
// launches with HIP events for: an empty kernel (1 and 256 workgroups), a kernel whose
// 256 workgroups each store one 16-B value, and the same stores with each kernel reading
// the previous one's output (a true data dependence). Also K launches captured in a
// HIP graph and replayed. Prints microseconds per launch.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_floor tools/probe/launch_floor.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__global__ void empty_kernel() {}

__global__ void store_kernel(double* out) {
  if (threadIdx.x == 0) out[blockIdx.x * 2] = 1.0;
}

__global__ void chain_kernel(const double* in, double* out) {
  if (threadIdx.x == 0) out[blockIdx.x * 2] = in[blockIdx.x * 2] + 1.0;
}

template <typename F>
static double time_launches(hipStream_t s, int k, F launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 50; ++i) launch(i);
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(a, s));
  for (int i = 0; i < k; ++i) launch(i);
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 1e3 * ms / k;
}

int main(int argc, char** argv) {
  const int k = argc > 1 ? atoi(argv[1]) : 2000;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  double *x, *y;
  CK(hipMalloc(&x, 256 * 2 * sizeof(double)));
  CK(hipMalloc(&y, 256 * 2 * sizeof(double)));
  CK(hipMemset(x, 0, 256 * 2 * sizeof(double)));
  CK(hipMemset(y, 0, 256 * 2 * sizeof(double)));
  printf("empty 1 WG        %.2f us/launch\n", time_launches(s, k, [&](int) {
           hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(256), 0, s);
         }));
  printf("empty 256 WG      %.2f us/launch\n", time_launches(s, k, [&](int) {
           hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s);
         }));
  printf("store 256 WG      %.2f us/launch\n", time_launches(s, k, [&](int) {
           hipLaunchKernelGGL(store_kernel, dim3(256), dim3(256), 0, s, x);
         }));
  printf("chain 256 WG      %.2f us/launch\n", time_launches(s, k, [&](int i) {
           if (i & 1) hipLaunchKernelGGL(chain_kernel, dim3(256), dim3(256), 0, s, y, x);
           else hipLaunchKernelGGL(chain_kernel, dim3(256), dim3(256), 0, s, x, y);
         }));
  // the chain captured once as a graph of 100 launches, replayed
  const int per = 100;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < per; ++i) {
    if (i & 1) hipLaunchKernelGGL(chain_kernel, dim3(256), dim3(256), 0, s, y, x);
    else hipLaunchKernelGGL(chain_kernel, dim3(256), dim3(256), 0, s, x, y);
  }
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  const double us = time_launches(s, k / per, [&](int) { CK(hipGraphLaunch(ge, s)); });
  printf("chain 256 WG graph %.2f us/launch\n", us / per);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipStreamDestroy(s));
  return 0;
}
