// Device-side helpers shared by the gpmi HIP translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gpmi_internal.h"

namespace gpmi {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int TS = GPMI_TS;      // 128
constexpr int BK = 16;           // k-depth of one LDS stage
constexpr int LDSK = 18;         // padded row stride (doubles) of a staged [row][k] slab
constexpr int STAGE = TS * LDSK; // doubles per staged operand buffer
constexpr int RLD = GPMI_RHS_LD; // 16

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

}  // namespace gpmi
