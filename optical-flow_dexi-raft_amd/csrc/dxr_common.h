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

// ---------------------------------------------------------------------------
// Pyramid layout ("paged" correlation volume).
//
// Level sizes follow F.avg_pool2d(2, stride=2) floor mode: H_l = floor(H_{l-1}/2).
// Storage is tiled so that each build workgroup owns one contiguous block:
// a PAGE = (QB query pixels) x (one TH x TW tile of image-2 cells).  Levels 0..3
// use QB = 128 and a level-0 tile of 8 x 16 cells, pooled to 4x8, 2x4, 1x2 at
// levels 1..3 (so one page's pooled cells come from the same workgroup).  Pages
// are padded: queries to a multiple of 128, image-2 to whole tiles.  Levels >= 4
// are plain row-major images (QB = 1, one tile = the whole level).  The element
// index of (pair b, query q, cell y, x) at a level is
//   ((((b*QT + q/QB)*TY + y/TH)*TX + x/TW)*QB + q%QB)*(TH*TW) + (y%TH)*TW + x%TW
// ---------------------------------------------------------------------------
constexpr int PAGE_Q = 128;    // queries per page (levels 0..3)
constexpr int PAGE_H = 8;      // level-0 tile rows
constexpr int PAGE_W = 16;     // level-0 tile cols
constexpr int TILED_LEVELS = 4;

struct LevelLayout {
  int h, w;          // true level size (floor-mode pooling)
  int th, tw;        // tile rows / cols at this level
  int ty, tx;        // tiles per image along y / x
  int qb, qt;        // queries per page, query blocks per pair
  long long off;     // element offset of the level in the pyramid buffer
};

struct Levels {
  int n;
  int h[8];
  int w[8];
  int64_t off[8];  // element offset of each level in the pyramid buffer
  int64_t numel;
  LevelLayout lay[8];
};

inline bool make_levels(int64_t B, int64_t H, int64_t W, int num_levels, Levels* L) {
  if (B < 0 || H < 1 || W < 1 || num_levels < 1 || num_levels > 8) return false;
  if (H * W > (1LL << 30)) return false;
  const int64_t N = H * W;
  const int64_t qt = (N + PAGE_Q - 1) / PAGE_Q;
  const int64_t ty = (H + PAGE_H - 1) / PAGE_H, tx = (W + PAGE_W - 1) / PAGE_W;
  int64_t off = 0, h = H, w = W;
  L->n = num_levels;
  for (int l = 0; l < num_levels; ++l) {
    if (l > 0) { h /= 2; w /= 2; }
    if (h < 1 || w < 1) return false;
    LevelLayout& y = L->lay[l];
    y.h = (int)h;
    y.w = (int)w;
    y.off = off;
    if (l < TILED_LEVELS) {
      y.th = PAGE_H >> l; y.tw = PAGE_W >> l;
      y.ty = (int)ty; y.tx = (int)tx;
      y.qb = PAGE_Q; y.qt = (int)qt;
      off += B * qt * PAGE_Q * ty * tx * (int64_t)y.th * y.tw;
    } else {
      y.th = (int)h; y.tw = (int)w; y.ty = 1; y.tx = 1; y.qb = 1; y.qt = (int)N;
      off += B * N * h * w;
    }
    L->h[l] = (int)h;
    L->w[l] = (int)w;
    L->off[l] = y.off;
  }
  L->numel = off;
  return true;
}

// Element index of (pair b, query q, cell y, x) inside one level (see above).
__host__ __device__ __forceinline__ long long cell_index(const LevelLayout& y, int b, int q, int cy,
                                                        int cx) {
  const long long page = (((long long)b * y.qt + q / y.qb) * y.ty + cy / y.th) * y.tx + cx / y.tw;
  return y.off + (page * y.qb + q % y.qb) * (y.th * y.tw) + (cy % y.th) * y.tw + cx % y.tw;
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

// Exact hi/mid/lo split of 8 floats into three 8 x bf16 MFMA operands
// (x = hi + mid + lo; hi and mid round to nearest, lo keeps the residual's top
// 16 bits).  Used by the bf16 kernels and the three-way bf16 fallback of the f32-class kernels.
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  typedef float f2_t __attribute__((ext_vector_type(2)));
  const f2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf2_t));
}

__device__ __forceinline__ void split8(const float (&x)[8], uint4& h, uint4& m, uint4& l) {
  uint32_t hh[4], mm[4], ll[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a = x[2 * e], b = x[2 * e + 1];
    uint32_t hp = cvt_pk_bf16(a, b);
    // a finite value that rounds past bf16's largest finite (|x| > ~3.39e38)
    // keeps its truncation as hi, so the pair stays finite and exact
    if (__builtin_isinf(__uint_as_float(hp << 16)) && !__builtin_isinf(a))
      hp = (hp & 0xffff0000u) | (__float_as_uint(a) >> 16);
    if (__builtin_isinf(__uint_as_float(hp & 0xffff0000u)) && !__builtin_isinf(b))
      hp = (hp & 0xffffu) | (__float_as_uint(b) & 0xffff0000u);
    // an infinite hi (an infinite input) keeps mid = lo = 0 (inf - inf would
    // turn +-inf products into NaN)
    const float ha = __uint_as_float(hp << 16), hb = __uint_as_float(hp & 0xffff0000u);
    const float ra = __builtin_isinf(ha) ? 0.f : a - ha, rb = __builtin_isinf(hb) ? 0.f : b - hb;
    const uint32_t mp = cvt_pk_bf16(ra, rb);
    const float la = ra - __uint_as_float(mp << 16), lb = rb - __uint_as_float(mp & 0xffff0000u);
    hh[e] = hp;
    mm[e] = mp;
    ll[e] = __builtin_amdgcn_perm(__float_as_uint(lb), __float_as_uint(la), 0x07060302u);
  }
  h = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  m = make_uint4(mm[0], mm[1], mm[2], mm[3]);
  l = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

}  // namespace dxr
