// Stage (a)+(b): all-pairs correlation volume fused with its avg-pool pyramid.
//
// Replaces core/corr.py:52-60 (CorrBlock.corr: matmul(f1^T, f2) / sqrt(D)) and
// core/corr.py:21-27 (CorrBlock.__init__: reshape + 3x F.avg_pool2d(2, stride 2)).
// The reference materialises the level-0 volume, divides it in a second pass and
// re-reads each level to pool the next; here every level is written once, from
// registers, in the epilogue of the MFMA tile that produced it.
//
// GEMM view (per pair b): C[i, j] = sum_d f1[d, i] * f2[d, j], i = query pixel
// (M = H*W), j = target pixel (N = H*W, taken as 2-D spatial tiles of image 2),
// K = D.  MFMA orientation is transposed (rows = targets, cols = queries) so that
// an accumulator lane owns ONE query and a 2-row x 16-col patch of targets:
//   v_mfma_f32_32x32x2_f32 D layout: col = lane & 31, row = (reg&3) + 8*(reg>>2)
//   + 4*(lane>>5).  Target row-index j maps to spatial (row = (j>>2)&1,
//   col = (j&3) + 4*(j>>3)), so lane half h holds spatial row h and register r
//   holds spatial column r of that row.
// A wave owns 32 queries x an 8x16 target tile (4 MFMA tiles: rows 2t, 2t+1),
// so 2x2, 4x4 and 8x8 pooling all finish inside the wave: in-lane adds plus one
// exchange between lane halves (lane ^ 32).  Floor-mode pooling falls out of the
// per-level bounds checks (a pooled cell is written only if it exists at that
// level).
#include <cmath>
#include <cstdlib>

#include "dxr_common.h"

namespace {

constexpr int TH = 8;            // target tile rows   (image-2 rows)
constexpr int TW = 16;           // target tile cols
constexpr int NTGT = TH * TW;    // 128 targets per workgroup

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct BuildGeom {
  int D, H, W, N;       // N = H * W
  int levels;           // fused levels (1..4)
  int tiles_w;          // ceil(W / TW)
  float divisor;        // sqrt(D) in the reference
  float recip;          // 1/divisor when that is exact (power of two), else 0
  int lh[4], lw[4];     // level sizes
  long long loff[4];    // element offset of each level
};

// Global -> register staging of one BK slice of the query panel (A: [BK][BM])
// and the target tile (B: [BK][TH][TW]).  VEC: W % 4 == 0, so every float4 is
// fully inside or fully outside the map.
template <bool VEC, int WAVES, int BK>
struct Stage {
  static constexpr int NT = 64 * WAVES;
  static constexpr int BM = 32 * WAVES;
  static constexpr int NA = VEC ? BK * BM / 4 / NT : BK * BM / NT;    // per-thread units
  static constexpr int NB = VEC ? BK * NTGT / 4 / NT : BK * NTGT / NT;
  static_assert(NA >= 1 && NB >= 1, "tile too small for the thread count");
  float a[VEC ? 4 * NA : NA];
  float b[VEC ? 4 * NB : NB];

  __device__ __forceinline__ void load(const float* __restrict__ f1b,
                                       const float* __restrict__ f2b, int k0,
                                       int q0, int th0, int tw0,
                                       const BuildGeom& g, int tid) {
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      const int idx = tid + NT * s;
      if constexpr (VEC) {
        const int k = idx / (BM / 4), c = (idx % (BM / 4)) * 4;
        const int kk = k0 + k, q = q0 + c;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (kk < g.D && q < g.N)
          v = *reinterpret_cast<const float4*>(f1b + (long long)kk * g.N + q);
        a[4 * s + 0] = v.x; a[4 * s + 1] = v.y; a[4 * s + 2] = v.z; a[4 * s + 3] = v.w;
      } else {
        const int k = idx / BM, c = idx % BM;
        const int kk = k0 + k, q = q0 + c;
        a[s] = (kk < g.D && q < g.N) ? f1b[(long long)kk * g.N + q] : 0.f;
      }
    }
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      const int idx = tid + NT * s;
      if constexpr (VEC) {
        const int k = idx >> 5, r = (idx >> 2) & 7, c = (idx & 3) * 4;
        const int kk = k0 + k, hh = th0 + r, ww = tw0 + c;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (kk < g.D && hh < g.H && ww < g.W)
          v = *reinterpret_cast<const float4*>(f2b + (long long)kk * g.N + hh * g.W + ww);
        b[4 * s + 0] = v.x; b[4 * s + 1] = v.y; b[4 * s + 2] = v.z; b[4 * s + 3] = v.w;
      } else {
        const int k = idx >> 7, r = (idx >> 4) & 7, c = idx & 15;
        const int kk = k0 + k, hh = th0 + r, ww = tw0 + c;
        b[s] = (kk < g.D && hh < g.H && ww < g.W) ? f2b[(long long)kk * g.N + hh * g.W + ww]
                                                  : 0.f;
      }
    }
  }

  __device__ __forceinline__ void store(float* As, float* Bs, int tid) {
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      const int idx = tid + NT * s;
      if constexpr (VEC) {
        const int k = idx / (BM / 4), c = (idx % (BM / 4)) * 4;
        *reinterpret_cast<float4*>(As + k * BM + c) =
            make_float4(a[4 * s], a[4 * s + 1], a[4 * s + 2], a[4 * s + 3]);
      } else {
        As[idx] = a[s];
      }
    }
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      const int idx = tid + NT * s;
      if constexpr (VEC) {
        *reinterpret_cast<float4*>(Bs + idx * 4) =
            make_float4(b[4 * s], b[4 * s + 1], b[4 * s + 2], b[4 * s + 3]);
      } else {
        Bs[idx] = b[s];
      }
    }
  }
};

// Store n (<= 4) consecutive floats of a row; vec4 when aligned & complete.
__device__ __forceinline__ void store4(float* dst, const float* v, int nvalid, bool vec) {
  if (vec && nvalid >= 4) {
    *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (e < nvalid) dst[e] = v[e];
  }
}

template <bool VEC, int WAVES, int BK>
__global__ __launch_bounds__(64 * WAVES) void corr_build_f32_kernel(
    const float* __restrict__ f1, const float* __restrict__ f2,
    float* __restrict__ pyr, BuildGeom g) {
  constexpr int BM = 32 * WAVES;
  constexpr int KP = BK / 2;                        // MFMA k-pairs per stage
  __shared__ float lds[2 * BK * (BM + NTGT)];       // [buf][A: BK*BM | B: BK*NTGT]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int th0 = (blockIdx.x / g.tiles_w) * TH;
  const int tw0 = (blockIdx.x % g.tiles_w) * TW;
  const int q0 = blockIdx.y * BM;
  const int b = blockIdx.z;
  const long long fstride = (long long)g.D * g.N;
  const float* f1b = f1 + b * fstride;
  const float* f2b = f2 + b * fstride;

  // Per-lane LDS read offsets (constant over K).
  const int j = lane & 31;
  const int tgt_off = (((j >> 2) & 1) * TW) + (j & 3) + 4 * (j >> 3);
  const int qry_off = wave * 32 + j;
  const int khalf = lane >> 5;

  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  auto As = [&](int buf) { return lds + buf * BK * (BM + NTGT); };
  auto Bs = [&](int buf) { return lds + buf * BK * (BM + NTGT) + BK * BM; };

  Stage<VEC, WAVES, BK> st;
  const int nk = (g.D + BK - 1) / BK;
  st.load(f1b, f2b, 0, q0, th0, tw0, g, tid);
  st.store(As(0), Bs(0), tid);
  __syncthreads();

  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) st.load(f1b, f2b, (ks + 1) * BK, q0, th0, tw0, g, tid);
    const float* a_s = As(buf);
    const float* b_s = Bs(buf);
    // Operand fragments are read one k-pair ahead of the MFMAs that use them,
    // so the LDS latency hides under four 64-cycle MFMAs.
    float bq[2], at[2][4];
    bq[0] = a_s[khalf * BM + qry_off];
#pragma unroll
    for (int t = 0; t < 4; ++t) at[0][t] = b_s[khalf * NTGT + 2 * t * TW + tgt_off];
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      const int cur = kp & 1, nxt = cur ^ 1;
      if (kp + 1 < KP) {
        const int k = 2 * (kp + 1) + khalf;
        bq[nxt] = a_s[k * BM + qry_off];
#pragma unroll
        for (int t = 0; t < 4; ++t) at[nxt][t] = b_s[k * NTGT + 2 * t * TW + tgt_off];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(at[cur][t], bq[cur], acc[t], 0, 0, 0);
    }
    if (ks + 1 < nk) st.store(As(buf ^ 1), Bs(buf ^ 1), tid);
    __syncthreads();
  }

  // ---------------- epilogue: scale, level 0, fused pooling ----------------
  const int h = lane >> 5;                 // spatial row within each 2-row MFMA tile
  const int qi = q0 + wave * 32 + j;       // this lane's query pixel
  // Lanes l and l^32 share the query, so they leave together and the
  // lane-half exchange below never reads an exited lane.
  if (qi >= g.N) return;
  const long long qimg = (long long)b * g.N + qi;

  // x / sqrt(D): a multiply is bit-identical when 1/sqrt(D) is exact (D = 4^k).
  if (g.recip != 0.f) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] *= g.recip;
  } else {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = acc[t][r] / g.divisor;
  }

  // Level 0: lane writes 16 contiguous columns of row th0 + 2t + h.
  {
    float* img = pyr + g.loff[0] + qimg * g.N;
    const int nv = g.W - tw0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int row = th0 + 2 * t + h;
      if (row < g.H) {
        float* dst = img + (long long)row * g.W + tw0;
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          float v[4] = {acc[t][4 * c4], acc[t][4 * c4 + 1], acc[t][4 * c4 + 2], acc[t][4 * c4 + 3]};
          store4(dst + 4 * c4, v, nv - 4 * c4, VEC);
        }
      }
    }
  }
  if (g.levels < 2) return;

  // Level 1 (2x2): rows 2t / 2t+1 live in lane halves 0 / 1.  Both halves compute
  // identical values in the reference's window order ((v00+v01)+v10)+v11.
  float l1[4][8];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const float o0 = acc[t][2 * m], o1 = acc[t][2 * m + 1];
      const float p0 = __shfl_xor(o0, 32), p1 = __shfl_xor(o1, 32);
      const float t0 = h ? p0 : o0, t1 = h ? p1 : o1;
      const float b0 = h ? o0 : p0, b1 = h ? o1 : p1;
      l1[t][m] = (((t0 + t1) + b0) + b1) * 0.25f;
    }
  }
  {
    const int lh = g.lh[1], lw = g.lw[1];
    float* img = pyr + g.loff[1] + qimg * ((long long)lh * lw);
    const int c0 = tw0 / 2 + 4 * h;
    const bool vec = VEC && (lw % 4 == 0);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int row = th0 / 2 + t;
      if (row < lh && c0 < lw) {
        float v[4] = {l1[t][4 * h], l1[t][4 * h + 1], l1[t][4 * h + 2], l1[t][4 * h + 3]};
        store4(img + (long long)row * lw + c0, v, lw - c0, vec);
      }
    }
  }
  if (g.levels < 3) return;

  // Level 2 (4x4 of level 0 = 2x2 of level 1), fully in-lane.
  float l2[2][4];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int n = 0; n < 4; ++n)
      l2[u][n] = (((l1[2 * u][2 * n] + l1[2 * u][2 * n + 1]) + l1[2 * u + 1][2 * n]) +
                  l1[2 * u + 1][2 * n + 1]) * 0.25f;
  {
    const int lh = g.lh[2], lw = g.lw[2];
    float* img = pyr + g.loff[2] + qimg * ((long long)lh * lw);
    const int row = th0 / 4 + h, c0 = tw0 / 4;
    const bool vec = VEC && (lw % 4 == 0);
    if (row < lh && c0 < lw) {
      float v[4] = {l2[h][0], l2[h][1], l2[h][2], l2[h][3]};
      store4(img + (long long)row * lw + c0, v, lw - c0, vec);
    }
  }
  if (g.levels < 4) return;

  // Level 3 (8x8 of level 0): two cells per wave-tile; half h writes cell h.
  {
    float l3[2];
#pragma unroll
    for (int v = 0; v < 2; ++v)
      l3[v] = (((l2[0][2 * v] + l2[0][2 * v + 1]) + l2[1][2 * v]) + l2[1][2 * v + 1]) * 0.25f;
    const int lh = g.lh[3], lw = g.lw[3];
    float* img = pyr + g.loff[3] + qimg * ((long long)lh * lw);
    const int row = th0 / 8, col = tw0 / 8 + h;
    if (row < lh && col < lw) img[(long long)row * lw + col] = l3[h];
  }
}

// Generic floor-mode 2x2 average pool over [planes, H, W] (levels >= 4, and the
// fmap pyramid of AlternateCorrBlock).  Window order matches F.avg_pool2d.
__global__ __launch_bounds__(256) void avg_pool2x2_kernel(const float* __restrict__ in,
                                                          float* __restrict__ out,
                                                          long long planes, int H, int W) {
  const int Ho = H / 2, Wo = W / 2;
  const long long total = planes * Ho * Wo;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(idx % Wo);
    const long long r = idx / Wo;
    const int y = (int)(r % Ho);
    const long long p = r / Ho;
    const float* s = in + (p * H + 2 * y) * W + 2 * x;
    out[idx] = (((s[0] + s[1]) + s[W]) + s[W + 1]) * 0.25f;
  }
}

int launch_avg_pool(const float* in, float* out, long long planes, int H, int W,
                    hipStream_t stream) {
  const long long total = planes * (long long)(H / 2) * (W / 2);
  if (total == 0) return DXR_OK;
  long long blocks = (total + 255) / 256;
  if (blocks > 2048 * 8) blocks = 2048 * 8;
  hipLaunchKernelGGL(avg_pool2x2_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     in, out, planes, H, W);
  return dxr::launch_status();
}

// Tile variants (queries per workgroup = 32 * WAVES, K step BK).  Selected by
// DXR_BUILD_VARIANT for same-process A/B timing; 0 is the tuned default.
template <bool VEC, int WAVES, int BK>
int launch_build_cfg(const float* f1, const float* f2, float* pyr, const BuildGeom& g,
                     int tiles_t, int B, hipStream_t stream) {
  constexpr int BM = 32 * WAVES;
  const dim3 grid((unsigned)tiles_t, (unsigned)((g.N + BM - 1) / BM), (unsigned)B);
  if (grid.y > 65535) return DXR_EINVAL;
  hipLaunchKernelGGL((corr_build_f32_kernel<VEC, WAVES, BK>), grid, dim3(64 * WAVES), 0, stream,
                     f1, f2, pyr, g);
  return dxr::launch_status();
}

int build_variant() {
  const char* v = std::getenv("DXR_BUILD_VARIANT");
  return v ? std::atoi(v) : 0;
}

int launch_build_f32(bool vec, int variant, const float* f1, const float* f2, float* pyr,
                     const BuildGeom& g, int tiles_t, int B, hipStream_t stream) {
  if (!vec) return launch_build_cfg<false, 4, 16>(f1, f2, pyr, g, tiles_t, B, stream);
  switch (variant) {
    case 1: return launch_build_cfg<true, 4, 32>(f1, f2, pyr, g, tiles_t, B, stream);
    case 2: return launch_build_cfg<true, 8, 16>(f1, f2, pyr, g, tiles_t, B, stream);
    case 3: return launch_build_cfg<true, 8, 32>(f1, f2, pyr, g, tiles_t, B, stream);
    default: return launch_build_cfg<true, 4, 16>(f1, f2, pyr, g, tiles_t, B, stream);
  }
}

}  // namespace

extern "C" int dxr_avg_pool2x2(const float* in, float* out, int64_t planes, int64_t H,
                               int64_t W, hipStream_t stream) {
  if (planes < 0 || H < 1 || W < 1 || H > (1 << 30) || W > (1 << 30)) return DXR_EINVAL;
  if (planes == 0 || H < 2 || W < 2) return DXR_OK;
  if (!in || !out) return DXR_EINVAL;
  return launch_avg_pool(in, out, planes, (int)H, (int)W, stream);
}

extern "C" int dxr_corr_pyramid_build(const void* fmap1, const void* fmap2, int in_dtype,
                                      int64_t B, int64_t D, int64_t H, int64_t W,
                                      int num_levels, float divisor, void* pyramid,
                                      int pyr_dtype, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L)) return DXR_EINVAL;
  if (D < 1 || !(divisor == divisor) || divisor == 0.f) return DXR_EINVAL;
  if (H * W > (1LL << 30) || D > (1 << 20)) return DXR_EINVAL;
  if (B > 65535) return DXR_EINVAL;
  if (B == 0) return DXR_OK;
  if (!fmap1 || !fmap2 || !pyramid) return DXR_EINVAL;
  if (in_dtype != DXR_F32 || pyr_dtype != DXR_F32) return DXR_EUNSUPPORTED;

  BuildGeom g;
  g.D = (int)D; g.H = (int)H; g.W = (int)W; g.N = (int)(H * W);
  g.levels = num_levels < 4 ? num_levels : 4;
  g.tiles_w = (int)((W + TW - 1) / TW);
  g.divisor = divisor;
  int e2 = 0;
  g.recip = (std::frexp(divisor, &e2) == 0.5f) ? 1.f / divisor : 0.f;  // exact iff 2^k
  for (int l = 0; l < 4; ++l) {
    g.lh[l] = l < L.n ? L.h[l] : 1;
    g.lw[l] = l < L.n ? L.w[l] : 1;
    g.loff[l] = l < L.n ? L.off[l] : 0;
  }
  float* pyr = static_cast<float*>(pyramid);
  const float* f1 = static_cast<const float*>(fmap1);
  const float* f2 = static_cast<const float*>(fmap2);
  const bool vec = (W % 4) == 0 && ((uintptr_t)f1 % 16) == 0 && ((uintptr_t)f2 % 16) == 0 &&
                   ((uintptr_t)pyr % 16) == 0;
  const int tiles_t = (int)((H + TH - 1) / TH) * g.tiles_w;
  int st = launch_build_f32(vec, build_variant(), f1, f2, pyr, g, tiles_t, (int)B, stream);
  if (st != DXR_OK) return st;

  // Levels beyond the fused four: plain pooling passes, level l from level l-1.
  for (int l = 4; l < L.n; ++l) {
    st = launch_avg_pool(pyr + L.off[l - 1], pyr + L.off[l], B * H * W, L.h[l - 1], L.w[l - 1],
                         stream);
    if (st != DXR_OK) return st;
  }
  return DXR_OK;
}
