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
constexpr int STAGE = TS * BK;   // doubles per staged operand buffer (128 rows x 16, 16 KB)

// Staged slabs are stored unpadded, [row][16 doubles], with the 16-byte chunk c
// of row r placed at chunk position c ^ ((r >> 1) & 7). MFMA fragment reads
// (16 consecutive rows at one k) then hit 32 distinct banks per 32-lane group,
// and the staging ds_write_b128 of a row stays one contiguous 128-byte line.
__device__ __forceinline__ int slab_off(int row, int k) {
  return row * BK + 2 * ((k >> 1) ^ ((row >> 1) & 7)) + (k & 1);
}
constexpr int RLD = GPMI_RHS_LD; // 16

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

}  // namespace gpmi
