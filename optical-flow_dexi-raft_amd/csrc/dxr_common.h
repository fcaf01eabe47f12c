// Internal helpers shared by the HIP translation units of libdexiraft_corr.so.
// Not part of the public ABI (that is include/dexiraft_corr.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dexiraft_corr.h"

namespace dxr {

// Thread-local record of the last failed HIP launch (dxr_last_hip_error()).
void set_last_hip_error(hipError_t e);

// Check the launch that was just issued; map a HIP error to DXR_EHIP.
inline int launch_status() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_last_hip_error(e);
    return DXR_EHIP;
  }
  return DXR_OK;
}

// Pyramid geometry: level sizes follow F.avg_pool2d(2, stride=2) floor mode.
struct Levels {
  int n;
  int h[8];
  int w[8];
  int64_t off[8];  // element offset of each level in the pyramid buffer
  int64_t numel;
};

inline bool make_levels(int64_t B, int64_t H, int64_t W, int num_levels, Levels* L) {
  if (B < 0 || H < 1 || W < 1 || num_levels < 1 || num_levels > 8) return false;
  const int64_t N = H * W;
  int64_t off = 0, h = H, w = W;
  L->n = num_levels;
  for (int l = 0; l < num_levels; ++l) {
    if (l > 0) { h /= 2; w /= 2; }
    if (h < 1 || w < 1) return false;
    L->h[l] = (int)h;
    L->w[l] = (int)w;
    L->off[l] = off;
    off += B * N * h * w;
  }
  L->numel = off;
  return true;
}

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// Round-to-nearest-even f32 -> bf16 that keeps NaN a NaN.
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

}  // namespace dxr
