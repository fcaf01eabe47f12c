// Stage (a)+(b): all-pairs correlation volume fused with its avg-pool pyramid.
//
// Replaces core/corr.py:52-60 (CorrBlock.corr: matmul(f1^T, f2) / sqrt(D)) and
// core/corr.py:21-27 (CorrBlock.__init__: reshape + 3x F.avg_pool2d(2, stride 2)).
// The reference materialises the level-0 volume, divides it in a second pass and
// re-reads each level to pool the next; here every level is written once, from
// registers, in the epilogue of the MFMA tile that produced it.
//
// GEMM view (per pair b): C[i, j] = sum_d f1[d, i] * f2[d, j], i = query pixel
// (M = H*W), j = target pixel (N = H*W, taken as 8 x 16 spatial tiles of image 2),
// K = D.  MFMA orientation is transposed (rows = targets, cols = queries) so that
// an accumulator lane owns ONE query and a 2-row x 16-col patch of targets:
//   v_mfma_f32_32x32x2_f32 D layout: col = lane & 31, row = (reg&3) + 8*(reg>>2)
//   + 4*(lane>>5).  Target row-index j maps to spatial (row = (j>>2)&1,
//   col = (j&3) + 4*(j>>3)), so lane half h holds spatial row h and register r
//   holds spatial column r of that row.
// A wave owns 32 queries x an 8x16 target tile (4 MFMA tiles: rows 2t, 2t+1),
// so 2x2, 4x4 and 8x8 pooling all finish inside the wave: in-lane adds plus one
// exchange between lane halves (lane ^ 32).
//
// Output: the paged pyramid layout of dxr_common.h.  A workgroup computes exactly
// one page per level (128 queries x one tile), stored contiguously, so the
// epilogue streams 1 KiB-contiguous wave stores: level-0/1 values go through a
// per-wave LDS transpose, level-2/3 values are already contiguous per wave.
// (Scattered per-query row stores — 64 lines per wave store — cost more than the
// MFMA loop itself: measured 346 vs 220 us at Sintel shape.)
#include <algorithm>
#include <cmath>
#include <type_traits>

#include "dxr_common.h"

namespace {

constexpr int TH = dxr::PAGE_H;  // target tile rows   (image-2 rows)
constexpr int TW = dxr::PAGE_W;  // target tile cols
constexpr int NTGT = TH * TW;    // 128 targets per workgroup
constexpr int WAVES = 4;         // waves split the 128 queries of a page
constexpr int BM = 32 * WAVES;   // = dxr::PAGE_Q
constexpr int NT = 64 * WAVES;
constexpr int P0 = NTGT + 4;     // LDS pitch (floats) of a staged level-0 query row
constexpr int P1 = 32 + 4;       // LDS pitch of a staged level-1 query block
static_assert(BM == dxr::PAGE_Q, "one workgroup = one page");

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct BuildGeom {
  int D, H, W, N;       // N = H * W
  int levels;           // fused levels (1..4)
  int tiles_w, tiles_h; // tiles per image (TX, TY)
  int qt;               // query blocks (pages along queries) per pair
  int strip;            // target tiles per strip of the XCD-banded page order
  float divisor;        // sqrt(D) in the reference
  float recip;          // 1/divisor when that is exact (power of two), else 0
  int lh[4], lw[4];     // level sizes
  long long loff[4];    // element offset of each level
  int nmain;            // DMA build: workgroups [0, nmain) take whole units, the
                        // rest quarter units of the tail (dma_tail_split)
};

// Page coordinates of this workgroup.  3-D grid (tiles, query blocks, pairs), or
// with REMAP a 1-D grid laid out for the per-XCD L2s: workgroup w runs on XCD
// w % 8 (round-robin dispatch; used for speed only), the bijective remap of
// cdna_hip_programming.md §5 gives each XCD a contiguous range of a linear
// order, and that order walks strips of STRIP target tiles query-block-major,
// so the ~128 workgroups an XCD holds at once share ~8 target panels and ~16
// query panels (~3 MB of f32 operands: its L2) instead of every target panel.
struct PageCoord {
  int txi, tyi, qblk, b;
  long long page;
};

constexpr int STRIP = 8;          // default strip width (BuildGeom::strip)

// Position wl of the linear (strip-walking) order -> page coordinates.  QB:
// query blocks per workgroup (the order walks groups of QB blocks; qblk is the
// group's first block, page its first page).
template <int QB>
__device__ __forceinline__ PageCoord unit_coord(const BuildGeom& g, long long wl) {
  PageCoord c;
  const int T = g.tiles_w * g.tiles_h;
  const int qtq = (g.qt + QB - 1) / QB;
  const long long per_pair = (long long)qtq * T;
  {
    c.b = (int)(wl / per_pair);
    long long rem = wl - c.b * per_pair;
    const int S = g.strip;
    const int nfull = T / S;
    int tile;
    if (rem < (long long)nfull * qtq * S) {
      const int st = (int)(rem / ((long long)qtq * S));
      const int in = (int)(rem - (long long)st * qtq * S);
      c.qblk = in / S * QB;
      tile = st * S + in % S;
    } else {
      const int nl = T - nfull * S;
      const int in = (int)(rem - (long long)nfull * qtq * S);
      c.qblk = in / nl * QB;
      tile = nfull * S + in % nl;
    }
    c.txi = tile % g.tiles_w;
    c.tyi = tile / g.tiles_w;
  }
  c.page = (((long long)c.b * g.qt + c.qblk) * g.tiles_h + c.tyi) * g.tiles_w + c.txi;
  return c;
}

template <bool REMAP, int QB = 1>
__device__ __forceinline__ PageCoord page_coord(const BuildGeom& g) {
  if constexpr (REMAP) {
    const long long nwg = (long long)min((unsigned)g.nmain, gridDim.x);
    const long long w = blockIdx.x;
    const long long q8 = nwg / 8, r8 = nwg % 8, xcd = w % 8;
    const long long wl = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + w / 8;
    return unit_coord<QB>(g, wl);
  } else {
    PageCoord c;
    c.txi = blockIdx.x % g.tiles_w;
    c.tyi = blockIdx.x / g.tiles_w;
    c.qblk = blockIdx.y * QB;
    c.b = blockIdx.z;
    c.page = (((long long)c.b * g.qt + c.qblk) * g.tiles_h + c.tyi) * g.tiles_w + c.txi;
    return c;
  }
}

// Global -> register staging of one BK slice of the query panel (A: [BK][BM])
// and the target tile (B: [BK][TH][TW]).  VEC: W % 4 == 0, so every float4 is
// fully inside or fully outside the map; outside elements stage as zero.
// NHWC (scalar form only): channels-last fmaps [H*W][D].
template <bool VEC, int BK, bool NHWC = false>
struct Stage {
  static_assert(!(VEC && NHWC), "channels-last staging is scalar");
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
        a[s] = (kk < g.D && q < g.N)
                   ? f1b[NHWC ? (long long)q * g.D + kk : (long long)kk * g.N + q] : 0.f;
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
        const long long p = (long long)hh * g.W + ww;
        b[s] = (kk < g.D && hh < g.H && ww < g.W) ? f2b[NHWC ? p * g.D + kk : kk * g.N + p]
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

__device__ __forceinline__ float4 f4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}

// f32 -> output element.  bf16: the hardware conversion (v_cvt_pk_bf16_f32, RNE,
// NaN stays NaN) — the software RNE of dxr::f32_to_bf16 cost ~6 VALU per value
// and left the bf16 build VALU-bound (round 4 PMC: 1,850 VALU per wave against
// 64 MFMAs at KITTI B=8).
template <typename OT>
__device__ __forceinline__ OT to_out(float v) {
  if constexpr (sizeof(OT) == 2) return (OT)(dxr::cvt_pk_bf16(v, 0.f) & 0xffffu);
  else return v;
}
// Two values as one packed word (first in the low half).
template <typename OT>
__device__ __forceinline__ uint32_t to_out2(float a, float b) {
  static_assert(sizeof(OT) == 2, "packed pairs are bf16");
  return dxr::cvt_pk_bf16(a, b);
}

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

// Paged epilogue (levels 0..3 of one page), shared by the f32 and bf16 builds.
// acc holds this wave's 32 queries x 8x16 targets, already divided by sqrt(D).
// Each level's page holds 128 queries x (TH x TW >> l) cells, query-major; this
// wave owns queries 32w .. 32w+31.  Padding queries/cells are written too (zeros
// or pools of zeros) and never read.  Every pooled value is computed from the
// f32 values of the level above, in the reference's window order
// ((v00+v01)+v10)+v11 (F.avg_pool2d), then rounded to OT once.
// `wave`: which 32 queries of the page this wave holds (and its private LDS
// staging region).
// EX: bit 0 syncs only the wave around its private staging region instead of
// the workgroup; bit 1 streams the pyramid with non-temporal stores; bit 2 with
// write-through (sc1) buffer stores.
template <int EX>
__device__ __forceinline__ void epi_sync() {
  if constexpr ((EX & 1) != 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}
// EX bit 2: buffer stores from a workgroup-uniform base `ub` (a level's page)
// with the sc1 cache-policy bit (write-through).
template <int EX, typename V, typename T>
__device__ __forceinline__ void epi_put(T* ub, T* p, const V v) {
  constexpr int AUX = 16;
  if constexpr ((EX & 4) != 0) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(ub, (short)0, 0x7fffffff, 0x00020000);
    const unsigned off = (unsigned)((p - ub) * (long long)sizeof(T));
    if constexpr (sizeof(V) == 16)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), r, off, 0, AUX);
    else if constexpr (sizeof(V) == 8)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, v), r, off, 0, AUX);
    else if constexpr (sizeof(V) == 4)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, AUX);
    else
      __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, v), r, off, 0, AUX);
  } else if constexpr ((EX & 2) != 0 && sizeof(V) >= 8) {
    __builtin_nontemporal_store(v, reinterpret_cast<V*>(p));
  } else {
    *reinterpret_cast<V*>(p) = v;
  }
}
// Store 8 consecutive values (two float4 read from LDS) as OT: 16 B of bf16 or
// 2 x 16 B of f32.
template <typename OT, int EX = 0>
__device__ __forceinline__ void store8(OT* ub, OT* dst, const float* src) {
  const float4 a = f4(src), c = f4(src + 4);
  if constexpr (sizeof(OT) == 2) {
    u32x4v u;
    u.x = to_out2<OT>(a.x, a.y);
    u.y = to_out2<OT>(a.z, a.w);
    u.z = to_out2<OT>(c.x, c.y);
    u.w = to_out2<OT>(c.z, c.w);
    epi_put<EX>(ub, dst, u);
  } else {
    epi_put<EX>(ub, dst, f32x4v{a.x, a.y, a.z, a.w});
    epi_put<EX>(ub, dst + 4, f32x4v{c.x, c.y, c.z, c.w});
  }
}

template <typename OT, int EX = 0>
__device__ __forceinline__ float paged_epilogue(f32x16 (&acc)[4], float* lds, OT* __restrict__ pyr,
                                                const BuildGeom& g, long long page, int wave,
                                                int lane) {
  const int j = lane & 31, h = lane >> 5;
  float* wl = lds + wave * 16 * P0;   // this wave's private LDS region

  // Level 0: 16 queries per round staged as [q][8][16] f32 rows, then streamed
  // as 1 KiB wave stores.
  OT* const pb0 = pyr + g.loff[0] + page * (BM * NTGT);   // page bases (workgroup-uniform)
  OT* pg0 = pb0 + (long long)wave * 32 * NTGT;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if ((j >> 4) == r) {
      float* row = wl + (j & 15) * P0 + h * TW;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4)
          st4(row + 2 * t * TW + 4 * c4, acc[t][4 * c4], acc[t][4 * c4 + 1],
              acc[t][4 * c4 + 2], acc[t][4 * c4 + 3]);
    }
    epi_sync<EX>();
    if constexpr (sizeof(OT) == 4) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int qq = 2 * k + (lane >> 5);
        const int off = (lane & 31) * 4;
        { const float4 x = f4(wl + qq * P0 + off);
          epi_put<EX>(pb0, pg0 + (r * 16 + qq) * NTGT + off, f32x4v{x.x, x.y, x.z, x.w}); }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int qq = 4 * k + (lane >> 4);
        const int off = (lane & 15) * 8;
        store8<OT, EX>(pb0, pg0 + (r * 16 + qq) * NTGT + off, wl + qq * P0 + off);
      }
    }
    epi_sync<EX>();
  }
  if (g.levels < 2) return 0.f;

  // Levels 1 and 2 (round 5): lane half h pools the level-1 cells 4h .. 4h+3 of
  // every level-1 row t.  acc[t][c] holds level-0 row 2t + h, col c; one
  // v_permlane32_swap of the pair (col k, col 8 + k) leaves every lane with
  // rows 2t AND 2t + 1 of col 8h + k (x: row 2t, y: row 2t + 1), so each cell is
  // pooled in-lane in the reference's window order ((v00 + v01) + v10) + v11.
  // Per row t: 8 swaps + 16 VALU (round 4: both halves pooled all 8 cells from
  // self-swapped copies, 64 VALU + 4 selects).  acc is consumed (level 0 is out).
  // Level 2 follows in-lane for cols 2h, 2h + 1 (l2[u][i]: level-2 row u, col 2h + i).
  float l2[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float l1[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int t = 2 * u + s;
      float x[8], y[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[t][k]),
                                                        __float_as_uint(acc[t][8 + k]), false, false);
        x[k] = __uint_as_float(p[0]);
        y[k] = __uint_as_float(p[1]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        l1[s][i] = (((x[2 * i] + x[2 * i + 1]) + y[2 * i]) + y[2 * i + 1]) * 0.25f;
      st4(wl + j * P1 + t * 8 + 4 * h, l1[s][0], l1[s][1], l1[s][2], l1[s][3]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
      l2[u][i] = (((l1[0][2 * i] + l1[0][2 * i + 1]) + l1[1][2 * i]) + l1[1][2 * i + 1]) * 0.25f;
  }
  epi_sync<EX>();
  {
    OT* const pb1 = pyr + g.loff[1] + page * (BM * NTGT / 4);
    OT* pg1 = pb1 + (long long)wave * 32 * (NTGT / 4);
    if constexpr (sizeof(OT) == 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int qq = 8 * k + (lane >> 3);
        const int off = (lane & 7) * 4;
        { const float4 x = f4(wl + qq * P1 + off);
        epi_put<EX>(pb1, pg1 + qq * 32 + off, f32x4v{x.x, x.y, x.z, x.w}); }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int qq = 16 * k + (lane >> 2);
        const int off = (lane & 3) * 8;
        store8<OT, EX>(pb1, pg1 + qq * 32 + off, wl + qq * P1 + off);
      }
    }
  }
  if (g.levels < 3) return 0.f;   // no barriers below this point

  // Level 3 (8x8 of level 0) is in-lane too: lane half h pools cell h.
  const float l3 = (((l2[0][0] + l2[0][1]) + l2[1][0]) + l2[1][1]) * 0.25f;

  // Level 2: [q][2][4] per page; lane (j, h) writes row h (a 1 KiB wave run).
  // Swapping (row 0, row 1) of each of the half's two cols gives lane half h
  // row h whole: x = cols 0-1, y = cols 2-3.
  {
    OT* const pb2 = pyr + g.loff[2] + page * (BM * NTGT / 16);
    OT* pg2 = pb2 + (long long)wave * 32 * 8 + j * 8 + 4 * h;
    float r[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(l2[0][i]),
                                                      __float_as_uint(l2[1][i]), false, false);
      r[i] = __uint_as_float(p[0]);
      r[2 + i] = __uint_as_float(p[1]);
    }
    if constexpr (sizeof(OT) == 4) {
      epi_put<EX>(pb2, pg2, f32x4v{r[0], r[1], r[2], r[3]});
    } else {
      u32x2v w;
      w.x = to_out2<OT>(r[0], r[1]);
      w.y = to_out2<OT>(r[2], r[3]);
      epi_put<EX>(pb2, pg2, w);
    }
  }
  if (g.levels < 4) return 0.f;

  // Level 3: lane (j, h) writes cell h.
  OT* const pb3 = pyr + g.loff[3] + page * (BM * 2);
  OT* pg3 = pb3 + (long long)wave * 32 * 2;
  epi_put<EX>(pb3, pg3 + j * 2 + h, to_out<OT>(l3));
  // the lane pair (j, 0), (j, 1) pools every f32 value of query j into its two
  // level-3 cells: a non-finite value anywhere in the wave's acc shows here
  return l3;
}

// PAGED: write the paged pyramid (levels 1..4 fused).  !PAGED: write level 0
// only, row-major [B*N][H][W] (CorrBlock.corr's [B,H,W,1,H,W] volume).
template <int BK>
constexpr int build_lds_floats() {
  return 2 * BK * (BM + NTGT) > WAVES * 16 * P0 ? 2 * BK * (BM + NTGT) : WAVES * 16 * P0;
}

// One page (128 queries x one 8x16 target tile of pair b): K loop + epilogue.
// `page` is the flat page index ((b*QT + qblk)*TY + tyi)*TX + txi, which is also
// the page's position in every paged level.
// x / sqrt(D) as the reference (core/corr.py:60): DIV = false multiplies by the
// exact reciprocal (sqrt(D) a power of two, e.g. D = 256 -> 1/16: bit-identical);
// DIV = true performs the IEEE division (compiled only where it is needed, as
// its expansion costs registers).
template <bool DIV>
__device__ __forceinline__ void scale_acc(f32x16 (&acc)[4], const BuildGeom& g) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if constexpr (DIV) acc[t][r] = acc[t][r] / g.divisor;
      else acc[t][r] *= g.recip;
    }
}

// `tid`: the thread's index among the page's NT threads (its workgroup may hold
// several such groups, each with its own `lds` region, running in step).
template <bool VEC, int BK, bool PAGED, typename OT, bool DIV, bool NHWC = false>
__device__ __forceinline__ void build_page_f32(const float* __restrict__ f1,
                                               const float* __restrict__ f2,
                                               OT* __restrict__ pyr, const BuildGeom& g,
                                               float* lds, long long page, int tid) {
  constexpr int KP = BK / 2;                        // MFMA k-pairs per stage

  const int lane = tid & 63;
  const int wave = tid >> 6;
  // Page coordinates in 32-bit arithmetic (pages < 2^31; 64-bit division expands
  // to a long emulation loop on the GPU).
  const int tpi = g.tiles_w * g.tiles_h;
  const int pg = (int)page;
  const int pimg = pg / tpi, pin = pg - pimg * tpi;
  const int tyi = pin / g.tiles_w, txi = pin - tyi * g.tiles_w;
  const int b = pimg / g.qt, qblk = pimg - b * g.qt;
  const int th0 = tyi * TH, tw0 = txi * TW;
  const int q0 = qblk * BM;
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

  const int nk = (g.D + BK - 1) / BK;
  auto mfma_stage = [&](int buf) {
    const float* a_s = As(buf);
    const float* b_s = Bs(buf);
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
      const int k = 2 * kp + khalf;
      const float bq = a_s[k * BM + qry_off];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(b_s[k * NTGT + 2 * t * TW + tgt_off], bq,
                                                      acc[t], 0, 0, 0);
    }
  };
  {
    Stage<VEC, BK, NHWC> st;
    st.load(f1b, f2b, 0, q0, th0, tw0, g, tid);
    st.store(As(0), Bs(0), tid);
    __syncthreads();
    for (int ks = 0; ks < nk; ++ks) {
      const int buf = ks & 1;
      if (ks + 1 < nk) st.load(f1b, f2b, (ks + 1) * BK, q0, th0, tw0, g, tid);
      mfma_stage(buf);
      if (ks + 1 < nk) st.store(As(buf ^ 1), Bs(buf ^ 1), tid);
      __syncthreads();
    }
  }

  // ---------------- epilogue: scale, level 0, fused pooling ----------------
  const int h = lane >> 5;                 // spatial row within each 2-row MFMA tile
  scale_acc<DIV>(acc, g);

  if constexpr (!PAGED) {
    static_assert(sizeof(OT) == 4, "row-major volume is float32");
    const int qi = q0 + wave * 32 + j;
    if (qi >= g.N) return;
    float* img = pyr + ((long long)b * g.N + qi) * g.N;
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
    return;
  } else {
    paged_epilogue<OT>(acc, lds, pyr, g, page, wave, lane);
  }
}

// Exact-f32 build (v_mfma_f32_32x32x2_f32): the fallback when the split build's
// layout conditions fail (D % 16 != 0, odd W), the kernel of CorrBlock.corr, and
// the f32 reference the split build is tested against (DXR_BUILD_EXACT_F32).
// One page per workgroup (grid = TX*TY x QT x B).  MINW = waves per SIMD the
// register allocation must allow (0 = compiler's choice).
template <bool VEC, int BK, bool PAGED, typename OT, int MINW, bool DIV>
__global__ __launch_bounds__(NT, MINW) void corr_build_f32_kernel(const float* __restrict__ f1,
                                                            const float* __restrict__ f2,
                                                            OT* __restrict__ pyr, BuildGeom g) {
  __shared__ float lds[build_lds_floats<BK>()];
  const long long page =
      ((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  build_page_f32<VEC, BK, PAGED, OT, DIV>(f1, f2, pyr, g, lds, page, (int)threadIdx.x);
}

// ---------------------------------------------------------------------------
// bf16 build: v_mfma_f32_32x32x16_bf16, f32 accumulation, same tile, same
// transposed orientation and the same paged epilogue.  Operand tiles are staged
// in their natural [k][n] order (fmaps are NCHW: a k-row of a panel is
// contiguous) — the target tile with its 32-column groups permuted into MFMA-row
// order — and fragments are read with ds_read_b64_tr_b16, which hands each lane
// one column (4 consecutive k) of a 4 x 16 block: two reads = one 8-element
// operand (lane l: A[row l&31][k 8*(l>>5)+e]).  Row pitch 320 B makes those
// reads conflict-free (rows 16 banks apart, the two 16-lane groups of a half 8
// banks apart).
// ---------------------------------------------------------------------------
typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

constexpr int BKH = 32;            // K per stage (two 16-deep MFMA steps)
constexpr int PH = BM + 32;        // LDS row pitch in bf16 elements (320 B)
static_assert(NTGT + 32 == PH, "A and B images share the pitch");
constexpr int STAGE_H = 2 * BKH * PH;  // bf16 elements per stage (A image + B image)

__device__ __forceinline__ s4v tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4v*)(p));
}

// LDS column of target (tile row r in 0..7, tile col c in 0..15): MFMA tile
// t = r/2, MFMA row j = (c & 3) + 4*(r & 1) + 8*(c >> 2) (inverse of tgt mapping).
__device__ __forceinline__ int tgt_col(int r, int c) {
  return (r >> 1) * 32 + (c & 3) + 4 * (r & 1) + 8 * (c >> 2);
}

template <bool VEC, typename OT, bool DIV, int MINW, bool REMAP = false>
__global__ __launch_bounds__(NT, MINW) void corr_build_bf16_kernel(const uint16_t* __restrict__ f1,
                                                             const uint16_t* __restrict__ f2,
                                                             OT* __restrict__ pyr, BuildGeom g) {
  constexpr int LDS_E = WAVES * 16 * P0 * 4;          // epilogue bytes
  constexpr int LDS_K = 2 * STAGE_H * 2;              // two stages, bytes
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_K > LDS_E ? LDS_K : LDS_E];
  uint16_t* lh = reinterpret_cast<uint16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const PageCoord pc = page_coord<REMAP>(g);
  const int txi = pc.txi, tyi = pc.tyi;
  const int th0 = tyi * TH, tw0 = txi * TW;
  const int q0 = pc.qblk * BM;
  const int b = pc.b;
  const long long fstride = (long long)g.D * g.N;
  const uint16_t* f1b = f1 + b * fstride;
  const uint16_t* f2b = f2 + b * fstride;

  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // Staging units: VEC = 4 bf16 (8 B) per unit, 4 units per thread per image,
  // read with buffer loads (per-lane byte offsets fixed over the K loop, the
  // stage's k offset in an SGPR; units past the query count, off the image or
  // past D fall outside the resource and read zeros).  Host side guarantees
  // D * N * 2 < 2^31 for VEC.
  uint2 ra[4], rb[4];
  uint16_t sa[16], sb[16];
  uint32_t voa[4], vob[4];
  __amdgpu_buffer_rsrc_t rsa, rsb;
  if constexpr (VEC) {
    rsa = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(f1b), (short)0, g.D * g.N * 2,
                                            0x00020000);
    rsb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(f2b), (short)0, g.D * g.N * 2,
                                            0x00020000);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int idx = tid + NT * s;
      const int k = idx >> 5;
      const int q = q0 + (idx & 31) * 4;
      voa[s] = q < g.N ? (uint32_t)(k * g.N + q) * 2u : 0x80000000u;
      const int r = (idx >> 2) & 7, c = (idx & 3) * 4, hh = th0 + r, ww = tw0 + c;
      vob[s] = (hh < g.H && ww < g.W) ? (uint32_t)(k * g.N + hh * g.W + ww) * 2u : 0x80000000u;
    }
  }
  auto load = [&](int k0) {
    if constexpr (VEC) {
      const int so = k0 * g.N * 2;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        ra[s] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rsa, voa[s], so, 0));
        rb[s] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rsb, vob[s], so, 0));
      }
    } else {
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int idx = tid + NT * s;
        const int k = idx >> 7, kk = k0 + k;
        {
          const int q = q0 + (idx & 127);
          sa[s] = (kk < g.D && q < g.N) ? f1b[(long long)kk * g.N + q] : (uint16_t)0;
        }
        {
          const int r = (idx >> 4) & 7, c = idx & 15, hh = th0 + r, ww = tw0 + c;
          sb[s] = (kk < g.D && hh < g.H && ww < g.W) ? f2b[(long long)kk * g.N + hh * g.W + ww]
                                                     : (uint16_t)0;
        }
      }
    }
  };
  auto store = [&](int buf) {
    uint16_t* A = lh + buf * STAGE_H;
    uint16_t* Bt = A + BKH * PH;
    if constexpr (VEC) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int idx = tid + NT * s;
        const int k = idx >> 5;
        *reinterpret_cast<uint2*>(A + k * PH + (idx & 31) * 4) = ra[s];
        const int r = (idx >> 2) & 7, c = (idx & 3) * 4;
        *reinterpret_cast<uint2*>(Bt + k * PH + tgt_col(r, c)) = rb[s];
      }
    } else {
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int idx = tid + NT * s;
        const int k = idx >> 7;
        A[k * PH + (idx & 127)] = sa[s];
        Bt[k * PH + tgt_col((idx >> 4) & 7, idx & 15)] = sb[s];
      }
    }
  };

  // Per-lane transposed-read geometry: lane 4q+p of each 16-lane group addresses
  // row q, columns 4p..4p+3 of its block; the block's columns are this lane
  // group's 16 MFMA rows/cols, its rows the lane half's 8 k values (2 reads).
  const int li = lane & 15;
  const int rd_off = (li >> 2) * PH + 4 * (li & 3) + 16 * ((lane >> 4) & 1) + 8 * (lane >> 5) * PH;

  const int nk = (g.D + BKH - 1) / BKH;
  load(0);
  store(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) load((ks + 1) * BKH);
    const uint16_t* A = lh + buf * STAGE_H;
    const uint16_t* Bt = A + BKH * PH;
#pragma unroll
    for (int kk = 0; kk < BKH; kk += 16) {
      const uint16_t* pa = A + kk * PH + rd_off + wave * 32;
      const s8v qv = __builtin_shufflevector(tr_read(pa), tr_read(pa + 4 * PH), 0, 1, 2, 3, 4, 5,
                                             6, 7);
      const bf8v qf = __builtin_bit_cast(bf8v, qv);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint16_t* pb = Bt + kk * PH + rd_off + t * 32;
        const s8v tv = __builtin_shufflevector(tr_read(pb), tr_read(pb + 4 * PH), 0, 1, 2, 3, 4,
                                               5, 6, 7);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8v, tv), qf, acc[t],
                                                         0, 0, 0);
      }
    }
    if (ks + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  scale_acc<DIV>(acc, g);
  paged_epilogue<OT, 0>(acc, reinterpret_cast<float*>(smem), pyr, g, pc.page, wave, lane);
}

// ---------------------------------------------------------------------------
// bf16 build, two query blocks per workgroup (8 waves: waves 0-3 hold queries
// q0..q0+127, waves 4-7 the next 128, all of them the same 8x16 target tile).
// The target tile is staged once for 256 queries, so a page costs 96 KB of
// operand reads from L2 instead of 128 KB (KITTI B=8: the r02 ablations put the
// 3.65 GB of operand re-reads at ~196 of 625 us).  Same MFMA tile per wave,
// same products in the same order, same epilogue: bit-identical pages.
// The epilogue syncs per wave (each wave stages through its own LDS region),
// so a half whose query block is past the end (odd block count) just returns.
// r02, KITTI B=8: 556 us per build against 619 for one query block per
// workgroup (both with their r02 epilogues; K loop alone 295 vs 391 us).
// ---------------------------------------------------------------------------
constexpr int STAGE_Q2 = 3 * BKH * PH;  // A0, A1, target images (bf16 elements)
// NHWC (channels-last bf16 fmaps): the three images are
// stored row-major, one row per query / target (MFMA row order) holding the
// stage's 32 k, at an 80-byte pitch: a ds_read_b128 hands lane l row l & 31,
// k 8 (l >> 5) .. +7 — the operand the two transposed reads of the NCHW form
// assemble — and its 16-lane groups hit 16 distinct 16-byte bank slots
// (row stride 5 slots).  Same operands, same products: bit-identical pages.
constexpr int PQN = BKH + 8;             // NHWC row pitch (bf16 elements)
static_assert(BM * PQN == BKH * PH, "an NHWC image is the size of an NCHW one");

template <typename OT, bool DIV, int MINW, bool NHWC = false>
__global__ __launch_bounds__(2 * NT, MINW) void corr_build_bf16_q2_kernel(
    const uint16_t* __restrict__ f1, const uint16_t* __restrict__ f2, OT* __restrict__ pyr,
    BuildGeom g) {
  constexpr int LDS_E = 2 * WAVES * 16 * P0 * 4;   // epilogue bytes (8 waves)
  constexpr int LDS_K = 2 * STAGE_Q2 * 2;          // two stages, bytes
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_K > LDS_E ? LDS_K : LDS_E];
  uint16_t* lh = reinterpret_cast<uint16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = wave >> 2, w4 = wave & 3;
  const PageCoord pc = page_coord<true, 2>(g);
  const int th0 = pc.tyi * TH, tw0 = pc.txi * TW;
  const int q0 = pc.qblk * BM;                      // first of the two blocks
  const long long fstride = (long long)g.D * g.N;
  const uint16_t* f1b = f1 + pc.b * fstride;
  const uint16_t* f2b = f2 + pc.b * fstride;

  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // NCHW staging units of 4 bf16 (8 B): thread unit s covers idx = tid + 512 s;
  // s = 0,1 -> image A0, 2,3 -> A1, 4,5 -> targets; u = idx & 1023 within the
  // image: k = u >> 5, 4 consecutive queries / target cols.
  // NHWC units of 8 bf16 (16 B, 8 consecutive k of one pixel): unit s covers
  // idx = tid + 512 s, image idx >> 9 (A0, A1, targets), u = idx & 511: row
  // u >> 2, k 8 (u & 3) .. +7.
  // Buffer loads, out-of-range units read zeros.  Host side guarantees
  // D * N * 2 < 2^31 (and D % 32 == 0 for NHWC).
  constexpr int NU = NHWC ? 3 : 6;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(f1b), (short)0, g.D * g.N * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(f2b), (short)0, g.D * g.N * 2, 0x00020000);
  uint32_t vo[NU];
  int lo[NU];
#pragma unroll
  for (int s = 0; s < NU; ++s) {
    if constexpr (NHWC) {
      const int idx = tid + 2 * NT * s, img = idx >> 9, u = idx & 511;
      const int row = u >> 2, kq = u & 3;
      if (img < 2) {
        const int q = q0 + img * BM + row;
        vo[s] = q < g.N ? (uint32_t)(q * g.D + 8 * kq) * 2u : 0x80000000u;
        lo[s] = (img * BM + row) * PQN + 8 * kq;
      } else {
        const int r = row >> 4, c = row & 15, hh = th0 + r, ww = tw0 + c;
        vo[s] = (hh < g.H && ww < g.W) ? (uint32_t)((hh * g.W + ww) * g.D + 8 * kq) * 2u
                                       : 0x80000000u;
        lo[s] = (2 * BM + tgt_col(r, c)) * PQN + 8 * kq;
      }
    } else {
      const int u = (tid + 2 * NT * s) & 1023, img = s >> 1;
      const int k = u >> 5;
      if (img < 2) {
        const int q = q0 + img * BM + (u & 31) * 4;
        vo[s] = q < g.N ? (uint32_t)(k * g.N + q) * 2u : 0x80000000u;
        lo[s] = img * BKH * PH + k * PH + (u & 31) * 4;
      } else {
        const int r = (u >> 2) & 7, c = (u & 3) * 4, hh = th0 + r, ww = tw0 + c;
        vo[s] = (hh < g.H && ww < g.W) ? (uint32_t)(k * g.N + hh * g.W + ww) * 2u : 0x80000000u;
        lo[s] = 2 * BKH * PH + k * PH + tgt_col(r, c);
      }
    }
  }
  using Unit = std::conditional_t<NHWC, uint4, uint2>;
  Unit rr[NU];
  auto load = [&](int k0) {
    const int so = NHWC ? k0 * 2 : k0 * g.N * 2;
#pragma unroll
    for (int s = 0; s < NU; ++s) {
      const __amdgpu_buffer_rsrc_t r = (s < (NHWC ? 2 : 4)) ? rsa : rsb;
      if constexpr (NHWC)
        rr[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, vo[s], so, 0));
      else
        rr[s] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, vo[s], so, 0));
    }
  };
  auto store = [&](int buf) {
    uint16_t* S = lh + buf * STAGE_Q2;
#pragma unroll
    for (int s = 0; s < NU; ++s) *reinterpret_cast<Unit*>(S + lo[s]) = rr[s];
  };

  const int li = lane & 15;
  const int rd_off = NHWC ? (lane & 31) * PQN + 8 * (lane >> 5)
                          : (li >> 2) * PH + 4 * (li & 3) + 16 * ((lane >> 4) & 1) +
                                8 * (lane >> 5) * PH;
  auto frag = [&](const uint16_t* p) -> bf8v {
    if constexpr (NHWC) {
      return *reinterpret_cast<const bf8v*>(p);
    } else {
      return __builtin_bit_cast(bf8v, __builtin_shufflevector(tr_read(p), tr_read(p + 4 * PH), 0,
                                                              1, 2, 3, 4, 5, 6, 7));
    }
  };
  constexpr int KSTEP = NHWC ? 1 : PH;          // LDS elements per k
  constexpr int RSTEP = NHWC ? 32 * PQN : 32;   // LDS elements per 32 MFMA rows
  constexpr int IMG = BKH * PH;                 // LDS elements per image (both layouts)
  const int nk = (g.D + BKH - 1) / BKH;
  load(0);
  store(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) load((ks + 1) * BKH);
    const uint16_t* A = lh + buf * STAGE_Q2 + half * IMG;
    const uint16_t* Bt = lh + buf * STAGE_Q2 + 2 * IMG;
#pragma unroll
    for (int kk = 0; kk < BKH; kk += 16) {
      const bf8v qf = frag(A + kk * KSTEP + rd_off + w4 * RSTEP);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf8v tv = frag(Bt + kk * KSTEP + rd_off + t * RSTEP);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tv, qf, acc[t], 0, 0, 0);
      }
    }
    if (ks + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  if (pc.qblk + half >= g.qt) return;   // past the last query block: no page
  scale_acc<DIV>(acc, g);
  const long long page = pc.page + (long long)half * g.tiles_h * g.tiles_w;
  // wave-local staging syncs and non-temporal pyramid stores (KITTI B=8: 556 vs
  // 606 us; the 1.13 GB pyramid outgrows the caches anyway; write-through sc1
  // stores are slower here: step 1,258 -> 1,345 us)
  constexpr int EX = 3;
  paged_epilogue<OT, EX>(acc, reinterpret_cast<float*>(smem) + half * WAVES * 16 * P0, pyr, g, page,
                         w4, lane);
}

// ---------------------------------------------------------------------------
// f32 build on bf16 MFMA by exact 3-way operand split ("split" build).
// Every f32 operand x is split as x = hi + mid + lo with hi, mid, lo bf16 and the
// sum EXACT: hi = RNE_bf16(x), mid = RNE_bf16(x - hi), lo = x - hi - mid (the
// residuals are multiples of ulp(x) spanning <= 16 and <= 8 significant bits, so
// both subtractions and lo are exact; |x| in the normal f32 range).  A product
// x*y is then the sum of nine exact bf16 x bf16 products; the six kept here (hh,
// hm, mh, hl, lh, mm) leave out |mid*lo| + |lo*mid| + |lo*lo| <= 2^-25 |x y|,
// below f32 rounding of the product itself.  Round-to-nearest splitting makes
// the residuals sign-symmetric, so the dropped terms carry no bias (a truncating
// split leaves them all with the sign of x*y: a -3e-8 relative shrink of every
// sum, visible in the 49.5 M-cell checksums of the Sintel volume).  They are
// accumulated in f32 by v_mfma_f32_32x32x16_bf16 — 6 x 32 cycles per 16 k
// against 8 x 64 for v_mfma_f32_32x32x2_f32.  The result has f32-class error
// (tests compare it with the f64 oracle at the same tolerance as the f32 MFMA
// build, and its checksums with the reference's).
//
// Operands: the wave's 32 queries are loaded straight from global memory into
// MFMA B-operand order (lane l: query l&31, k 8(l>>5)..+7) and split in
// registers — no other wave reads them, so they skip LDS; the 8x16 target tile
// (shared by the four waves) is split once per workgroup into three bf16 LDS
// planes in the transposed-read layout of the bf16 build, double-buffered.
// ---------------------------------------------------------------------------
constexpr int BKS = 16;                 // K per stage
constexpr int PLANE_S = BKS * PH;       // bf16 elements per split plane

struct Split3 {
  uint32_t h, m, l;  // bf16x2 words (first element in the low half)
};

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// v_cvt_pk_bf16_f32: round-to-nearest-even of two floats into one bf16x2 word.
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// bf16x2 word of the high halves of two f32 bit patterns (element a low).
__device__ __forceinline__ uint32_t pack_hi(uint32_t a, uint32_t b) {
  return __builtin_amdgcn_perm(b, a, 0x07060302u);
}

// Exact 3-way split of two floats (see above), packed for the MFMA operands.
__device__ __forceinline__ Split3 split3(float a, float b) {
  const uint32_t h = cvt_pk_bf16(a, b);
  // an infinite hi keeps mid = lo = 0 (inf - inf would make them NaN: x*y must stay +-inf)
  const float ha = __uint_as_float(h << 16), hb = __uint_as_float(h & 0xffff0000u);
  const float ra = __builtin_isinf(ha) ? 0.f : a - ha, rb = __builtin_isinf(hb) ? 0.f : b - hb;
  const uint32_t m = cvt_pk_bf16(ra, rb);
  const float la = ra - __uint_as_float(m << 16), lb = rb - __uint_as_float(m & 0xffff0000u);
  return {h, m, pack_hi(__float_as_uint(la), __float_as_uint(lb))};
}

// f16 pair split (H2 form of the split build): x = hi + 2^-11 lo with
// hi = RNE_f16(x) and lo = RNE_f16((x - hi) * 2^11).  x - hi is exact in f32 and
// the scaling is exact, so the representation error is lo's rounding:
// <= 2^-22 |x| (hi normal) or <= 2^-36 absolute (|x| < 2^-14, lo subnormal).
// x*y = hi*hi + 2^-11 (hi*lo + lo*hi) + 2^-22 lo*lo; the last term (<= 2^-22 |x y|,
// sign-symmetric under RNE) is dropped.  f16 x f16 products are exact in f32.
// Valid while |x| < 65520 (hi finite): the kernel detects the overflow from its
// own accumulators and re-runs the page on the 3-way bf16 split.
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 h8v __attribute__((ext_vector_type(8)));

struct Split2 {
  uint32_t h, l;  // f16x2 words (first element in the low half)
};

__device__ __forceinline__ uint32_t cvt_pk_f16(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2_t));
}

// The residual is formed and rounded by mixed-precision FMAs:
// lo = RNE_f16(fma(hi, -2048, 2048 x)).  2048 x and 2048 hi are exact and so is
// their difference (= 2048 (x - hi)), so the single rounding is the RNE of
// (x - hi) * 2^11; hi stays an f16 operand (v_fma_mix*_f16), no conversion back.
__device__ __forceinline__ Split2 split2h_mix(float a, float b) {
  const uint32_t h = cvt_pk_f16(a, b);
  const f16x2_t hv = __builtin_bit_cast(f16x2_t, h);
  f16x2_t lv;
  lv[0] = (_Float16)__builtin_fmaf((float)hv[0], -2048.f, a * 2048.f);
  lv[1] = (_Float16)__builtin_fmaf((float)hv[1], -2048.f, b * 2048.f);
  return {h, __builtin_bit_cast(uint32_t, lv)};
}

// Raw buffer access (gfx9 resource word 3: 0x00020000), byte offsets.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* base, int elems) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, elems * 4,
                                           0x00020000);
}
__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ float2 bload2(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
  return make_float2(v.x, v.y);
}
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t voff, int soff) {
  const f32x4v v = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
  return make_float4(v.x, v.y, v.z, v.w);
}

// BV: target staging width in floats — 4 (float4 units; W % 4 == 0) or 2
// (float2 units; W even, e.g. Chairs' 62-wide fmaps).
// NHWC: channels-last fmaps [B, H, W, D]: every operand
// unit is 4 consecutive k of one pixel, so the query operand is two 16-byte
// loads per lane and the target tile is staged target-major ([target][k] planes,
// read with ds_read_b128) instead of k-major; same products, same order, same
// bits as the NCHW build.
// H2: the f16 pair split (3 products) with the 3-way bf16 split as the
// per-page overflow fallback; !H2: the 3-way bf16 split only.
template <typename OT, bool DIV, int MINW, int BV = 4, bool NHWC = false, bool H2 = false>
__global__ __launch_bounds__(NT, MINW) void corr_build_split_kernel(const float* __restrict__ f1,
                                                                    const float* __restrict__ f2,
                                                                    OT* __restrict__ pyr,
                                                                    BuildGeom g) {
  constexpr int LDS_E = WAVES * 16 * P0 * 4;                         // epilogue bytes
  constexpr int LDS_K = 2 * 3 * (NHWC ? NTGT * 24 : PLANE_S) * 2;     // two stages, bytes
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_K > LDS_E ? LDS_K : LDS_E];
  __shared__ int redo;  // H2: some accumulator of the page is not finite
  uint16_t* lh = reinterpret_cast<uint16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (H2 && tid == 0) redo = 0;
  const PageCoord pc = page_coord<false>(g);
  const int txi = pc.txi, tyi = pc.tyi;
  const int th0 = tyi * TH, tw0 = txi * TW;
  const int q0 = pc.qblk * BM;
  const int b = pc.b;
  const long long fstride = (long long)g.D * g.N;
  const float* f1b = f1 + b * fstride;
  const float* f2b = f2 + b * fstride;

  f32x16 acc[4], acc2[4];  // acc2: H2 cross terms (hi*lo + lo*hi, scaled 2^11)
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = acc2[t][r] = 0.f;

  // Operands are read with buffer loads: one resource per fmap of this pair,
  // per-lane 32-bit byte offsets fixed for the whole K loop, and the stage's k
  // offset in an SGPR — no per-stage vector address arithmetic (64-bit address
  // adds and exec-masked loads were half of the loop's VALU cycles, r02 PMC).
  // Off-image target units get an offset past the resource: the range check
  // returns zeros.  Host side guarantees D * N * 4 < 2^31.
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(f1b, g.D * g.N);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(f2b, g.D * g.N);
  // Query operand: lane -> (query q0 + 32 wave + (lane & 31), k rows 8 (lane >> 5) + e).
  // Padding queries read a clamped, valid address (their outputs are page padding).
  const int qa = min(q0 + wave * 32 + (lane & 31), g.N - 1);
  const uint32_t va = NHWC ? (uint32_t)(qa * g.D + 8 * (lane >> 5)) * 4u
                           : (uint32_t)(qa + 8 * (lane >> 5) * g.N) * 4u;
  // Target staging: NBS units of BV floats per thread per stage.  NCHW: unit
  // idx -> (k, tile row, col / BV), BV consecutive targets of one k row; NHWC:
  // unit idx -> (target, k / 4), 4 consecutive k of one target.
  static_assert(!NHWC || BV == 4, "NHWC units are 4 consecutive channels");
  constexpr int UPR = TW / BV;               // units per tile row
  constexpr int NBS = BKS * NTGT / BV / NT;  // units per thread
  int bk[NBS], bcol[NBS];
  uint32_t vb[NBS];
#pragma unroll
  for (int s = 0; s < NBS; ++s) {
    const int idx = tid + NT * s;
    int r, c;
    if constexpr (NHWC) {
      const int p = idx >> 2;
      r = p >> 4;
      c = p & 15;
      bk[s] = 4 * (idx & 3);
      vb[s] = (uint32_t)(((th0 + r) * g.W + tw0 + c) * g.D + bk[s]) * 4u;
    } else {
      r = (idx / UPR) & 7;
      c = (idx % UPR) * BV;
      bk[s] = idx / (8 * UPR);
      vb[s] = (uint32_t)(bk[s] * g.N + (th0 + r) * g.W + tw0 + c) * 4u;
    }
    bcol[s] = tgt_col(r, c);
    if (!(th0 + r < g.H && tw0 + c < g.W)) vb[s] = 0x80000000u;
  }

  float an[8];
  float4 bn[NBS];
  auto load = [&](int k0) {
    if constexpr (NHWC) {
      const float4 u = bload4(ra, va, k0 * 4), v = bload4(ra, va, k0 * 4 + 16);
      an[0] = u.x; an[1] = u.y; an[2] = u.z; an[3] = u.w;
      an[4] = v.x; an[5] = v.y; an[6] = v.z; an[7] = v.w;
#pragma unroll
      for (int s = 0; s < NBS; ++s) bn[s] = bload4(rb, vb[s], k0 * 4);
      return;
    }
    const int rowb = g.N * 4;
#pragma unroll
    for (int e = 0; e < 8; ++e) an[e] = bload1(ra, va, (k0 + e) * rowb);
#pragma unroll
    for (int s = 0; s < NBS; ++s) {
      if constexpr (BV == 4) {
        bn[s] = bload4(rb, vb[s], k0 * rowb);
      } else {
        const float2 v = bload2(rb, vb[s], k0 * rowb);
        bn[s] = make_float4(v.x, v.y, 0.f, 0.f);
      }
    }
  };
  s8v ah, am, al;   // split query operand of the current stage (H2: ah, al)
  using S3 = std::integral_constant<bool, false>;
  using S2 = std::integral_constant<bool, true>;
  // Operand split by mixed-precision FMAs (split2h_mix: 44 instead of 68 VALU per
  // k step, bit-identical to split2h; Sintel step 225.4 -> 223.6 us).
  auto split_a = [&](auto mode) {
    uint32_t h[4], m[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if constexpr (decltype(mode)::value) {
        const Split2 x = split2h_mix(an[2 * e], an[2 * e + 1]);
        h[e] = x.h;
        m[e] = 0;
        l[e] = x.l;
      } else {
        const Split3 x = split3(an[2 * e], an[2 * e + 1]);
        h[e] = x.h;
        m[e] = x.m;
        l[e] = x.l;
      }
    }
    ah = __builtin_bit_cast(s8v, make_uint4(h[0], h[1], h[2], h[3]));
    am = __builtin_bit_cast(s8v, make_uint4(m[0], m[1], m[2], m[3]));
    al = __builtin_bit_cast(s8v, make_uint4(l[0], l[1], l[2], l[3]));
  };
  // NHWC target planes: [target (MFMA row order)][16 k] bf16 at a 48-byte
  // pitch, which keeps the ds_read_b128 lane groups bank-conflict free.
  constexpr int PN = 24;                      // NHWC plane row pitch (bf16)
  constexpr int PLANE_N = NTGT * PN;          // bf16 elements per NHWC plane
  constexpr int PLANE = NHWC ? PLANE_N : PLANE_S;
  // Target planes of a stage: hi, mid, lo (bf16) or hi, lo (H2: f16).
  auto store_b = [&](int buf, auto mode) {
    uint16_t* P = lh + buf * 3 * PLANE;
#pragma unroll
    for (int s = 0; s < NBS; ++s) {
      const int o = NHWC ? bcol[s] * PN + bk[s] : bk[s] * PH + bcol[s];
      if constexpr (decltype(mode)::value) {
        const Split2 x = split2h_mix(bn[s].x, bn[s].y);
        if constexpr (BV == 4) {
          const Split2 z = split2h_mix(bn[s].z, bn[s].w);
          *reinterpret_cast<uint2*>(P + o) = make_uint2(x.h, z.h);
          *reinterpret_cast<uint2*>(P + PLANE + o) = make_uint2(x.l, z.l);
        } else {
          *reinterpret_cast<uint32_t*>(P + o) = x.h;
          *reinterpret_cast<uint32_t*>(P + PLANE + o) = x.l;
        }
      } else {
        const Split3 x = split3(bn[s].x, bn[s].y);
        if constexpr (BV == 4) {
          const Split3 z = split3(bn[s].z, bn[s].w);
          *reinterpret_cast<uint2*>(P + o) = make_uint2(x.h, z.h);
          *reinterpret_cast<uint2*>(P + PLANE + o) = make_uint2(x.m, z.m);
          *reinterpret_cast<uint2*>(P + 2 * PLANE + o) = make_uint2(x.l, z.l);
        } else {
          *reinterpret_cast<uint32_t*>(P + o) = x.h;
          *reinterpret_cast<uint32_t*>(P + PLANE + o) = x.m;
          *reinterpret_cast<uint32_t*>(P + 2 * PLANE + o) = x.l;
        }
      }
    }
  };

  const int li = lane & 15;
  const int rd_off = NHWC ? (lane & 31) * PN + 8 * (lane >> 5)
                          : (li >> 2) * PH + 4 * (li & 3) + 16 * ((lane >> 4) & 1) +
                                8 * (lane >> 5) * PH;
  auto frag = [&](const uint16_t* p) {
    if constexpr (NHWC) {
      return *reinterpret_cast<const bf8v*>(p);
    } else {
      return __builtin_bit_cast(bf8v, __builtin_shufflevector(tr_read(p), tr_read(p + 4 * PH), 0,
                                                              1, 2, 3, 4, 5, 6, 7));
    }
  };
  const int tstride = NHWC ? 32 * PN : 32;    // MFMA tile t's first row / column

  const int nk = g.D / BKS;
  // The K loop, on the 3-way bf16 split (six products into acc) or on the f16
  // pair split (hi*hi into acc, the two cross products into acc2).
  auto kloop = [&](auto mode) {
    constexpr bool M2 = decltype(mode)::value;
    load(0);
    store_b(0, mode);
    split_a(mode);
    __syncthreads();
    for (int ks = 0; ks < nk; ++ks) {
      const int buf = ks & 1;
      if (ks + 1 < nk) load((ks + 1) * BKS);
      const uint16_t* P = lh + buf * 3 * PLANE + rd_off;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if constexpr (M2) {
          const h8v th = __builtin_bit_cast(h8v, frag(P + t * tstride)),
                    tl = __builtin_bit_cast(h8v, frag(P + PLANE + t * tstride));
          const h8v qh = __builtin_bit_cast(h8v, ah), ql = __builtin_bit_cast(h8v, al);
          acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, qh, acc2[t], 0, 0, 0);
          acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ql, acc2[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, qh, acc[t], 0, 0, 0);
        } else {
          const bf8v qh = __builtin_bit_cast(bf8v, ah), qm = __builtin_bit_cast(bf8v, am),
                     ql = __builtin_bit_cast(bf8v, al);
          const bf8v th = frag(P + t * tstride), tm = frag(P + PLANE + t * tstride),
                     tl = frag(P + 2 * PLANE + t * tstride);
          // small terms first
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tm, qm, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tl, qh, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, ql, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tm, qh, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, qm, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, qh, acc[t], 0, 0, 0);
        }
      }
      if (ks + 1 < nk) {
        store_b(buf ^ 1, mode);
        split_a(mode);
      }
      __syncthreads();
    }
  };

  if constexpr (H2) {
    kloop(S2{});
    // Combine (one rounding) and vote: a non-finite sum means an operand of the
    // page overflowed f16 (|x| >= 65520) or was itself inf/NaN; the page is then
    // recomputed on the 3-way bf16 split, which covers the whole f32 range and
    // propagates inf/NaN operands as the f32 product would.
    bool bad = false;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[t][r] = __builtin_fmaf(acc2[t][r], 0x1p-11f, acc[t][r]);
        bad |= !(__builtin_fabsf(acc[t][r]) <= 3.40282347e38f);
      }
    if (bad) redo = 1;
    __syncthreads();
    if (redo) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
      kloop(S3{});
    }
  } else {
    kloop(S3{});
  }

  scale_acc<DIV>(acc, g);
  // Wave-local syncs around the per-wave staging (r02: -2 % per Sintel step).
  // Pyramid stores are write-through (sc1, round 2): no dirty lines pile up in
  // the XCDs' L2s for the K loops' operand reads to evict around, and none are
  // left for the kernel boundary to write back (Sintel B=1 step 232 -> 211 us
  // with the lookups' sc1 stores; build alone 125 -> 115).
  constexpr int EX = 1 | 4;
  paged_epilogue<OT, EX>(acc, reinterpret_cast<float*>(smem), pyr, g, pc.page, wave, lane);
}

// ---------------------------------------------------------------------------
// Round 3: the f32 build as a pure f16 GEMM on pre-split operands.
//
// (1) split_pairs_kernel, once per build: every pixel's f32 channel vector is
//     scaled by a power of two 2^s (s = 14 - e for max_k |x| = f 2^e, f in
//     [0.5, 1), so |x 2^s| < 2^14) and split into an f16 pair
//     x 2^s = hi + lo (hi = RNE_f16(x 2^s), lo = RNE_f16(x 2^s - hi), one rounding
//     of an exact residual).  The scaling is exact, so the pair represents every
//     element to <= 2^-23 |x| unless it is more than 2^16 below its pixel's max
//     (then to <= 2^-39 of that max) whatever the fmaps' scale — the r02 build
//     split unscaled values and lost precision below |x| ~ 2^-14.
//     Output per pair: SP [D/16][N][hi 16 k | lo 16 k] f16 (64 B per pixel and
//     16-channel block) and E [N] int32 exponents s.  A pixel with a non-finite
//     channel keeps s = 0: its inf/NaN reaches the accumulators and the build
//     recomputes those pages from the f32 operands on the exact-f32 MFMA.
// (2) corr_build_dma_kernel: 8 waves = two query blocks (waves 0-3, 4-7) x one
//     8x16 target tile, the tile shared by both (24 KB per 16-k step instead of
//     2 x 16 KB for two single-block pages).  The K loop moves operands only by
//     LDS-DMA (buffer_load ... lds, 16 B per lane) into a 3-stage ring, so no
//     VGPRs are held by loads in flight and no VALU splits in the loop: per step
//     a wave waits for its own 3 DMAs of the step (vmcnt), one barrier publishes
//     the tile, then 10 conflict-free ds_read_b128 and 12 f16 MFMAs — lo*hi,
//     hi*lo, hi*hi into ONE f32 accumulator (f16 x f16 products are exact in
//     f32; 3 roundings per 16 k against the exact-f32 MFMA's 8).  With a single
//     accumulator per output (64 VGPRs instead of the r02 split build's 128) the
//     kernel fits 4 waves per SIMD: two workgroups per CU.  The epilogue undoes
//     both pixels' scales (ldexp by -(s_q + s_t), exact) and writes the paged
//     pyramid as before.
// LDS image rows are 64 B (hi k0-7, hi k8-15, lo k0-7, lo k8-15 in 16-B slots);
// the slots of a row are XOR-permuted by a row key so that every 16-lane group
// of a ds_read_b128 hits 16 distinct bank slots; the DMA writes lane-linearly,
// so each lane fetches the logical slot its physical slot holds (the source
// side of the permutation).  Query rows: key (row >> 2) & 3 (lanes read rows
// j = lane & 31); target rows (LDS row = tile row * 16 + tile col): key
// ((row >> 2) & 1) | ((row >> 3) & 2) (MFMA row j reads tile row 2t + ((j>>2)&1),
// col (j & 3) + 4 (j >> 3)).
// ---------------------------------------------------------------------------
constexpr int SPLIT_S_TOP = 14;          // |x 2^s| < 2^SPLIT_S_TOP
constexpr int DMA_RING = 3;              // ring stages (k16 steps in LDS)
constexpr int DMA_TILE = 16384;          // tile offset in a stage: 8 waves x 2 KB queries
constexpr int DMA_STAGE = DMA_TILE + 8192;   // bytes per stage

__device__ __forceinline__ int pixel_scale(float m, bool finite) {
  if (!finite || !(m > 0.f)) return 0;
  int e;
  (void)__builtin_frexpf(m, &e);
  const int s = SPLIT_S_TOP - e;
  return s < -125 ? -125 : (s > 125 ? 125 : s);
}

// Split 16 consecutive channels of one pixel (already scaled) into the 64-B
// SP record: hi 16 f16 then lo 16 f16.  LO11: lo = RNE_f16((x - hi) 2^11) (the
// r02 pair, for experiments), else lo = RNE_f16(x - hi).
template <bool LO11 = false>
__device__ __forceinline__ void split_record(const float (&x)[16], uint4 (&rec)[4]) {
  uint32_t h[8], l[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if constexpr (LO11) {
      const Split2 p = split2h_mix(x[2 * e], x[2 * e + 1]);
      h[e] = p.h;
      l[e] = p.l;
    } else {
      h[e] = cvt_pk_f16(x[2 * e], x[2 * e + 1]);
      const f16x2_t hv = __builtin_bit_cast(f16x2_t, h[e]);
      f16x2_t lv;
      lv[0] = (_Float16)__builtin_fmaf((float)hv[0], -1.f, x[2 * e]);
      lv[1] = (_Float16)__builtin_fmaf((float)hv[1], -1.f, x[2 * e + 1]);
      l[e] = __builtin_bit_cast(uint32_t, lv);
    }
  }
  rec[0] = make_uint4(h[0], h[1], h[2], h[3]);
  rec[1] = make_uint4(h[4], h[5], h[6], h[7]);
  rec[2] = make_uint4(l[0], l[1], l[2], l[3]);
  rec[3] = make_uint4(l[4], l[5], l[6], l[7]);
}

// One thread per (pixel, 16-channel block): 1024-thread blocks of 64 pixels x
// 16 channel blocks (more blocks loop), grid (ceil(N / 64), B, 2 fmaps).  NCHW:
// wave = channel block, lane = pixel, so every load is 256 contiguous bytes;
// NHWC: 16 lanes per pixel read its channels as 64-byte runs.  The pixel max
// (and a non-finite flag, -1) is reduced through LDS; the values stay in
// registers between the two passes when D <= 256.
// Stores: the next kernel reads the records from every XCD, so they are
// written through (sc1) — in whole lines: a wave's 64 records (4 KB: 64
// consecutive pixels of one channel block, NCHW; 4 pixels x 16 blocks, NHWC)
// go through a per-wave LDS transpose (80-B pitch, conflict-free) so that each
// 16-B store instruction covers 1 KB of contiguous records.  (Per-lane 64-B
// records stored directly write every line in four partial pieces: 13.7 vs
// 9.5 us at Sintel B=1 against plain stores, which in turn leave the build's
// K loop evicting dirty lines.)
template <bool NHWC, bool LO11 = false, int PX = 64>
__global__ __launch_bounds__(PX * 16) void split_pairs_kernel(const float* __restrict__ f1,
                                                              const float* __restrict__ f2,
                                                              uint4* __restrict__ sp1,
                                                              uint4* __restrict__ sp2,
                                                              int* __restrict__ e1,
                                                              int* __restrict__ e2, int D, int N) {
  static_assert(PX == 64 || (!NHWC && PX == 32), "NHWC: 64 pixels per workgroup");
  __shared__ float red[16][PX + 1];
  __shared__ __attribute__((aligned(16))) uint4 tr[PX / 4][64 * 5];   // per wave: 64 records, 80-B pitch
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // NCHW: thread = (16-channel block kb0, pixel pl), pixels fastest (PX = 32:
  // a wave holds two channel blocks' 128-byte pixel runs)
  const int kb0 = NHWC ? (tid & 15) : (tid / PX), pl = NHWC ? (tid >> 4) : (tid % PX);
  const int p = blockIdx.x * PX + pl;
  const bool live = p < N;
  const int b = blockIdx.y;
  const float* src = (blockIdx.z == 0 ? f1 : f2) + (long long)b * D * N;
  uint4* sp = (blockIdx.z == 0 ? sp1 : sp2) + (long long)b * (D / 16) * N * 4;
  int* ex = (blockIdx.z == 0 ? e1 : e2) + (long long)b * N;
  const int nkb = D / 16;
  auto load16 = [&](int kb, float (&x)[16]) {
    if constexpr (NHWC) {
      const float4* s4 = reinterpret_cast<const float4*>(src + (long long)p * D + kb * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 v = s4[i];
        x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
      }
    } else {
      // channel stride N by 32-bit adds (a pair's plane is < 2^31 elements): no
      // quarter-rate 64-bit multiply in front of every load
      unsigned o = (unsigned)(kb * 16) * (unsigned)N + (unsigned)p;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        x[i] = src[o];
        o += (unsigned)N;
      }
    }
  };
  float x[16];
  // the pixel's max |x| over finite channels and whether any is not finite
  // (-1 below): the same value as the one-select-chain form, two ops per channel
  float m = 0.f;
  bool nonfin = false;
  for (int kb = kb0; kb < nkb && live; kb += 16) {
    load16(kb, x);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float a = __builtin_fabsf(x[i]);
      nonfin |= !(a <= 3.40282347e38f);
      m = __builtin_fmaxf(m, a <= 3.40282347e38f ? a : 0.f);
    }
  }
  if (nonfin) m = -1.f;
  red[kb0][pl] = m;
  __syncthreads();
  float mm = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const float v = red[k][pl];
    mm = (mm < 0.f || v < 0.f) ? -1.f : (v > mm ? v : mm);
  }
  const int s = pixel_scale(mm < 0.f ? 0.f : mm, mm >= 0.f);
  // per-pair resources (a pair's SP copy is D * N * 4 < 2^31 bytes)
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(sp, (short)0, 0x7fffffff, 0x00020000);
  if (live && kb0 == 0) {
    const __amdgpu_buffer_rsrc_t re =
        __builtin_amdgcn_make_buffer_rsrc(ex, (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)s, re, (unsigned)p * 4u, 0, 16);
  }
  uint4* tw = tr[wave];
  const int nit = (nkb + 15) / 16;               // wave-uniform trip count
  for (int it = 0; it < nit; ++it) {
    const int kb = kb0 + 16 * it;
    if (nkb > 16 && live && kb < nkb) load16(kb, x);   // D <= 256: the first pass's values
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = __builtin_ldexpf(x[i], s);
    uint4 rec[4];
    split_record<LO11>(x, rec);
    // the lane's record -> LDS record u (NCHW: u = pixel; NHWC: u = 4 block + pixel)
    const int u = NHWC ? (lane & 15) * 4 + (lane >> 4) : lane;
#pragma unroll
    for (int c = 0; c < 4; ++c) tw[u * 5 + c] = rec[c];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // 1 KB of contiguous records per instruction: LDS record u2, slot c
      const int u2 = 16 * i + (lane >> 2), c = lane & 3;
      const int kbs = NHWC ? 16 * it + (u2 >> 2) : 16 * it + (wave * 64 + u2) / PX;
      const int px = NHWC ? blockIdx.x * 64 + wave * 4 + (u2 & 3) : blockIdx.x * PX + u2 % PX;
      if (px < N && kbs < nkb) {
        const uint4 v = tw[u2 * 5 + c];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), rs,
                                               (unsigned)((kbs * N + px) * 64 + c * 16), 0, 16);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

typedef __attribute__((address_space(3))) void lds_void_t;

// Pyramid store policy of the DMA builds' epilogue (paged_epilogue EX), picked per
// launch (EXF; dma_stream_out): wave-private staging + write-through buffer stores (5),
// or non-temporal stores (3) for pyramids far beyond the Infinity Cache.

// LDS of corr_build_dma_kernel: ring | target scale exponents s (128 int).
constexpr int DMA_LDS_RING = DMA_RING * DMA_STAGE;
constexpr int DMA_LDS_BYTES = DMA_LDS_RING + NTGT * 4;
// Tail quarter units (dma_tail_split): the exchange region (two 32-query groups
// x four 32-target tiles of accumulators) and the epilogue staging after it.
constexpr int DMA_XS_BYTES = 2 * 4 * 16 * 64 * 4;
static_assert(DMA_XS_BYTES + WAVES * 16 * P0 * 4 <= DMA_LDS_RING, "tail exchange + staging fit");

// Unscale, divide by sqrt(D) and write one wave's 32 queries x 8x16 targets
// (f32 build), then — if the wave saw a non-finite sum — recompute them on
// the exact-f32 MFMA and write them again.  acc[t][r] is query qj x tile pixel
// (row 2t + kh, col r).  Shared by the whole-unit and the quarter-unit forms.
template <typename OT, bool DIV, int EXF = 5>
__device__ __forceinline__ void dma_finish_f32(f32x16 (&acc)[4], const BuildGeom& g,
                                               OT* __restrict__ pyr, float* stage, long long page,
                                               int w4, int lane, int sq, int qj,
                                               int trow0, int th0, int tw0, int b,
                                               const float* __restrict__ f1,
                                               const float* __restrict__ f2, int ps, int ks,
                                               const int* sexp) {
  const int kh = lane >> 5;
  // Non-finite sums (an inf/NaN operand pixel) are found per wave after the
  // epilogue from the level-3 cells, which pool every value of the lane's query
  // (round 5: one compare instead of 64 compares + 64 scalar ORs per wave and a
  // workgroup flag; the recompute only rewrites the wave's own pages anyway).
  // An exponent sum that overflows a finite value also reads as non-finite and
  // takes the exact path, whose f32 result overflows the same way.  Fewer than 4
  // levels: the unscaled values themselves are checked before the epilogue
  // consumes them (so an exponent-sum overflow takes the exact path either way).
  bool bad = false;
  // ldexp by the exponent sum -(s_q + s_t) + log2(1/sqrt(D)) (when that is
  // exact): one rounding of the exact value whatever the pixel magnitudes.
  // (Round 4 multiplied by 2^-s_q / sqrt(D), then by 2^-s_t: the same two VALU
  // ops per value, but the product overflowed or went subnormal between them for
  // pixel pairs of very different magnitudes)
  int eq = -sq;
  if constexpr (!DIV) {
    int e2;
    (void)__builtin_frexpf(g.recip, &e2);
    eq += e2 - 1;   // recip = 2^(e2 - 1)
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int4* se = reinterpret_cast<const int4*>(sexp + (2 * t + kh) * 16);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int4 s4 = se[u];
      acc[t][4 * u + 0] = __builtin_ldexpf(acc[t][4 * u + 0], eq - s4.x);
      acc[t][4 * u + 1] = __builtin_ldexpf(acc[t][4 * u + 1], eq - s4.y);
      acc[t][4 * u + 2] = __builtin_ldexpf(acc[t][4 * u + 2], eq - s4.z);
      acc[t][4 * u + 3] = __builtin_ldexpf(acc[t][4 * u + 3], eq - s4.w);
    }
  }
  if constexpr (DIV) scale_acc<DIV>(acc, g);
  if (g.levels < 4) {   // after the unscale, as the level-3 check
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) bad |= !(__builtin_fabsf(acc[t][r]) <= 3.40282347e38f);
  }
  const float l3 = paged_epilogue<OT, EXF>(acc, stage, pyr, g, page, w4, lane);
  if (g.levels >= 4) bad = !(__builtin_fabsf(l3) <= 3.40282347e38f);
  if (__ballot(bad) != 0) {   // wave-uniform
    // The wave saw a non-finite sum: its pages are recomputed on the
    // exact-f32 MFMA (v_mfma_f32_32x32x2_f32: each lane supplies channel k0 + kh
    // of its A row = target trow0 + 32 t and of its B column = query qj; same
    // output layout as the f16 products, nothing to undo) and written again over
    // the first pass's (each wave rewrites only its own rows, in program order).
    // Rare (non-finite inputs): operands straight from global memory by
    // range-checked buffer loads, off-map pixels reading as zero.
    int trw = trow0;
    asm volatile("" : "+v"(trw));   // keep this path's addressing out of the K loop
    const long long pb = (long long)b * g.D * g.N;
    const int nbytes = g.D * g.N * 4;
    const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(f1 + pb), (short)0, nbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(f2 + pb), (short)0, nbytes, 0x00020000);
    const unsigned qo = qj < g.N ? (unsigned)qj * (unsigned)ps * 4u : 0x80000000u;
    unsigned to[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int lrow = trw + 32 * t, hh = th0 + (lrow >> 4), ww = tw0 + (lrow & 15);
      to[t] = (hh < g.H && ww < g.W) ? (unsigned)(hh * g.W + ww) * (unsigned)ps * 4u : 0x80000000u;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    }
    const int kstep = ks * 4;
#pragma unroll 1
    for (int k = kh; k < g.D; k += 2) {
      const int ko = k * kstep;
      const float bq = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r1, qo, ko, 0));
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float at =
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r2, to[t], ko, 0));
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(at, bq, acc[t], 0, 0, 0);
      }
    }
    scale_acc<DIV>(acc, g);
    paged_epilogue<OT, EXF>(acc, stage, pyr, g, page, w4, lane);
  }
}

// Per-workgroup prologue of both forms: the lane's query exponent, the tile's
// 128 target exponents (LDS).
__device__ __forceinline__ void dma_scales(const BuildGeom& g, const int* __restrict__ ex1,
                                           const int* __restrict__ ex2, int b, int qj, int th0,
                                           int tw0, int tid, int& sq, int* sexp) {
  sq = qj < g.N ? ex1[(long long)b * g.N + qj] : 0;
  if (tid < NTGT) {
    // the target pixel's scale exponent s (in [-125, 125])
    const int r = tid >> 4, c = tid & 15;
    const bool in = th0 + r < g.H && tw0 + c < g.W;
    const int e = in ? ex2[(long long)b * g.N + (th0 + r) * g.W + tw0 + c] : 0;
    sexp[tid] = e;
  }
}

// Quarter units of the tail (dma_tail_split): workgroup blockIdx.x >= nmain
// takes query groups 2 sub, 2 sub + 1 (64 queries) of unit nmain + (x - nmain)/4
// against the unit's whole 8x16 tile; wave = (group gl, 32-target MFMA tile t).
// Every accumulator runs the whole-unit form's MFMA sequence on the same
// operands, so the pages are the same bits; the four tiles of a group meet in
// LDS and one wave per group runs the shared epilogue.  A quarter unit's K
// loop is a quarter of the MFMA work at the same per-step latency, so the
// last, partial dispatch round of whole units (1,568 units on 512 slots at
// Sintel B=1: 32 units alone for a whole unit time) becomes 128 short ones.
template <typename OT, bool DIV, bool BF, int EXF = 5>
__device__ __forceinline__ void dma_quarter(unsigned char* smem, const uint8_t* __restrict__ sp1,
                                            const uint8_t* __restrict__ sp2,
                                            const int* __restrict__ ex1,
                                            const int* __restrict__ ex2, OT* __restrict__ pyr,
                                            const float* __restrict__ f1,
                                            const float* __restrict__ f2, int ps, int ks, int pstr,
                                            int kstr, const BuildGeom& g) {
  int* const sexp = reinterpret_cast<int*>(smem + DMA_LDS_RING);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gl = wave >> 2, t = wave & 3;
  const long long xq = (long long)blockIdx.x - g.nmain;
  const int sub = (int)(xq & 3), half = sub >> 1;
  const PageCoord pc = unit_coord<2>(g, (long long)g.nmain + (xq >> 2));
  if (pc.qblk + half >= g.qt) return;                  // padding query block (uniform)
  const int qgrp = 2 * sub + gl, w4 = qgrp & 3;
  const int th0 = pc.tyi * TH, tw0 = pc.txi * TW;
  const int q0 = pc.qblk * BM + 64 * sub;              // first of the workgroup's 64 queries
  const int b = pc.b;
  const int j = lane & 31, kh = lane >> 5;
  const long long spstride = (long long)g.D * g.N * (BF ? 2 : 4);
  const int qj = q0 + gl * 32 + j;
  int sq = 0;
  if constexpr (!BF) dma_scales(g, ex1, ex2, b, qj, th0, tw0, tid, sq, sexp);

  const __amdgpu_buffer_rsrc_t rq =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp1 + b * spstride), (short)0,
                                        (int)spstride, 0x00020000);
  const __amdgpu_buffer_rsrc_t rt =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp2 + b * spstride), (short)0,
                                        (int)spstride, 0x00020000);
  // waves 0-3 stage the 64 query rows (16 each, the whole-unit form's LDS
  // image: group gl at gl * 2 KB), every wave its target tile row
  uint32_t vq = 0x80000000u, vt;
  {
    const int row = 16 * wave + (lane >> 2), sl = lane & 3;
    const int q = q0 + row;
    const int cq = sl ^ ((row >> 2) & 3);
    if (wave < 4 && q < g.N) vq = (uint32_t)q * (uint32_t)pstr + 16u * cq;
  }
  {
    const int sl = lane & 3, r = wave, col = lane >> 2, trow = r * 16 + col;
    const int ct = sl ^ (((trow >> 2) & 1) | ((trow >> 3) & 2));
    const int hh = th0 + r, ww = tw0 + col;
    vt = (hh < g.H && ww < g.W) ? (uint32_t)(hh * g.W + ww) * (uint32_t)pstr + 16u * ct
                                : 0x80000000u;
  }
  auto dma = [&](int kk) {
    unsigned char* st = smem + (kk % DMA_RING) * DMA_STAGE;
    const int so = kk * kstr;
    if (wave < 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rq, (lds_void_t*)(st + wave * 1024), 16, vq, so, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (lds_void_t*)(st + DMA_TILE + wave * 1024), 16,
                                             vt, so, 0, 0);
  };
  const int kq = (j >> 2) & 3;
  const int qh_off = gl * 2048 + j * 64 + 16 * (kh ^ kq);
  const int ql_off = gl * 2048 + j * 64 + 16 * ((2 + kh) ^ kq);
  const int trow0 = ((j >> 2) & 1) * 16 + (j & 3) + 4 * (j >> 3);
  const int kt = ((trow0 >> 2) & 1) | ((trow0 >> 3) & 2);
  const int th_off = DMA_TILE + t * 2048 + trow0 * 64 + 16 * (kh ^ kt);
  const int tl_off = DMA_TILE + t * 2048 + trow0 * 64 + 16 * ((2 + kh) ^ kt);

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int nk = g.D / (BF ? 2 * BKS : BKS);
  dma(0);
  if (nk > 1) dma(1);
  for (int kk = 0; kk < nk; ++kk) {
    if (kk + 1 < nk) {
      if (wave < 4) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kk + 2 < nk) dma(kk + 2);
    const unsigned char* st = smem + (kk % DMA_RING) * DMA_STAGE;
    if constexpr (BF) {
      const bf8v q0v = *reinterpret_cast<const bf8v*>(st + qh_off);
      const bf8v q1v = *reinterpret_cast<const bf8v*>(st + ql_off);
      const bf8v t0v = *reinterpret_cast<const bf8v*>(st + th_off);
      const bf8v t1v = *reinterpret_cast<const bf8v*>(st + tl_off);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t0v, q0v, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t1v, q1v, acc, 0, 0, 0);
    } else {
      const h8v qh = *reinterpret_cast<const h8v*>(st + qh_off);
      const h8v ql = *reinterpret_cast<const h8v*>(st + ql_off);
      const h8v th = *reinterpret_cast<const h8v*>(st + th_off);
      const h8v tl = *reinterpret_cast<const h8v*>(st + tl_off);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, qh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ql, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, qh, acc, 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // ring reads done: the LDS is free for reuse
  // the group's four tiles meet in LDS: [group][tile][r / 4][lane][4] f32
  float* const xs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int u = 0; u < 4; ++u)
    *reinterpret_cast<float4*>(xs + (((gl * 4 + t) * 4 + u) * 64 + lane) * 4) =
        make_float4(acc[4 * u], acc[4 * u + 1], acc[4 * u + 2], acc[4 * u + 3]);
  __syncthreads();
  if (t != 0) return;             // one wave per group writes (wave-local syncs below)
  f32x16 a4[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 v = *reinterpret_cast<const float4*>(xs + (((gl * 4 + tt) * 4 + u) * 64 + lane) * 4);
      a4[tt][4 * u] = v.x; a4[tt][4 * u + 1] = v.y; a4[tt][4 * u + 2] = v.z; a4[tt][4 * u + 3] = v.w;
    }
  const long long page = pc.page + (long long)half * g.tiles_h * g.tiles_w;
  float* const stage = reinterpret_cast<float*>(smem + DMA_XS_BYTES);
  if constexpr (BF) {
    scale_acc<DIV>(a4, g);
    paged_epilogue<OT, EXF>(a4, stage, pyr, g, page, w4, lane);
  } else {
    dma_finish_f32<OT, DIV, EXF>(a4, g, pyr, stage, page, w4, lane, sq, qj, trow0, th0, tw0, b, f1,
                            f2, ps, ks, sexp);
  }
}

// A wave whose sums are not finite (an inf/NaN operand pixel) recomputes
// its pages from the f32 operands (`f1`, `f2`: element (pixel p, channel k) at
// p * ps + k * ks of a pair's fmap) on the exact-f32 MFMA, in place: IEEE
// semantics as the reference's f32 matmul (inf x finite = inf, inf x 0 = NaN,
// NaN propagates).  Grid: dma_grid(g, B, stream) — [0, g.nmain) whole units in the
// XCD-banded order (page_coord<true, 2>), then the tail's quarter units.
//
// BF (bf16 mode, C3): the same K loop on bf16 operand records — a 64-B record
// is 32 consecutive channels of one pixel (k 0-7 | 8-15 | 16-23 | 24-31 in the
// four 16-B slots), so a stage is two 16-deep bf16 MFMA steps (slots kh, then
// 2 + kh), accumulated in the order of corr_build_bf16_q2_kernel: the same
// pages bit for bit.  Records come straight from channels-last bf16 fmaps
// (pixel stride D * 2 B, stage stride 64 B) or from the pack pass's blocked copy
// of NCHW fmaps (pixel stride 64 B, stage stride N * 64 B): `pstr` / `kstr`.
// No scales, no non-finite fallback (bf16 MFMA propagates inf/NaN itself), and
// the bf16 build's non-temporal pyramid stores.
template <typename OT, bool DIV, bool BF = false, int EXF = 5>
__global__ __launch_bounds__(2 * NT, 4) void corr_build_dma_kernel(
    const uint8_t* __restrict__ sp1, const uint8_t* __restrict__ sp2, const int* __restrict__ ex1,
    const int* __restrict__ ex2, OT* __restrict__ pyr, const float* __restrict__ f1,
    const float* __restrict__ f2, int ps, int ks, int pstr, int kstr, BuildGeom g) {
  static_assert(WAVES * 16 * P0 * 4 * 2 <= DMA_LDS_RING, "the epilogue staging aliases the ring");
  // one LDS array (cdna_hip_programming.md §5 item 4(a))
  __shared__ __attribute__((aligned(16))) unsigned char smem[DMA_LDS_BYTES];
  if (blockIdx.x >= (unsigned)g.nmain) {
    dma_quarter<OT, DIV, BF, EXF>(smem, sp1, sp2, ex1, ex2, pyr, f1, f2, ps, ks, pstr, kstr, g);
    return;
  }
  int* const sexp = reinterpret_cast<int*>(smem + DMA_LDS_RING);

  const int tid = threadIdx.x, lane = tid & 63;
  // wave-uniform (SGPR): the DMA's LDS base must be, or the compiler emits a
  // waterfall loop around every buffer_load ... lds
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave >> 2, w4 = wave & 3;
  const PageCoord pc = page_coord<true, 2>(g);
  const int th0 = pc.tyi * TH, tw0 = pc.txi * TW;
  const int q0 = pc.qblk * BM;                        // first of the two blocks
  const int b = pc.b;
  const int j = lane & 31, kh = lane >> 5;
  const long long spstride = (long long)g.D * g.N * (BF ? 2 : 4);   // operand bytes per pair

  // exponents: the lane's query, the tile's 128 targets (LDS, by tile pixel)
  const int qj = q0 + wave * 32 + j;
  int sq = 0;
  if constexpr (!BF) dma_scales(g, ex1, ex2, b, qj, th0, tw0, tid, sq, sexp);

  const __amdgpu_buffer_rsrc_t rq =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp1 + b * spstride), (short)0,
                                        (int)spstride, 0x00020000);
  const __amdgpu_buffer_rsrc_t rt =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp2 + b * spstride), (short)0,
                                        (int)spstride, 0x00020000);
  // DMA source offsets (fixed over K; the step's offset ks * kstr in soffset).
  // Query instruction i of this wave: LDS rows 16 i + (lane >> 2) of the wave's
  // 2 KB region; target instruction: tile row r = wave.
  uint32_t vq[2], vt;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * i + (lane >> 2), sl = lane & 3;
    const int q = q0 + wave * 32 + row;
    const int cq = sl ^ ((row >> 2) & 3);
    vq[i] = q < g.N ? (uint32_t)q * (uint32_t)pstr + 16u * cq : 0x80000000u;
  }
  {
    const int sl = lane & 3, r = wave, col = lane >> 2, trow = r * 16 + col;
    const int ct = sl ^ (((trow >> 2) & 1) | ((trow >> 3) & 2));
    const int hh = th0 + r, ww = tw0 + col;
    vt = (hh < g.H && ww < g.W) ? (uint32_t)(hh * g.W + ww) * (uint32_t)pstr + 16u * ct
                                : 0x80000000u;
  }
  auto dma = [&](int kk) {
    unsigned char* st = smem + (kk % DMA_RING) * DMA_STAGE;
    const int so = kk * kstr;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rq, (lds_void_t*)(st + wave * 2048 + i * 1024), 16, vq[i], so, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (lds_void_t*)(st + DMA_TILE + wave * 1024), 16,
                                             vt, so, 0, 0);
  };
  // fragment byte offsets within a stage (hi; lo = the other two slots)
  const int kq = (j >> 2) & 3;
  const int qh_off = wave * 2048 + j * 64 + 16 * (kh ^ kq);
  const int ql_off = wave * 2048 + j * 64 + 16 * ((2 + kh) ^ kq);
  const int trow0 = ((j >> 2) & 1) * 16 + (j & 3) + 4 * (j >> 3);     // tile t adds 32 rows
  const int kt = ((trow0 >> 2) & 1) | ((trow0 >> 3) & 2);
  const int th_off = DMA_TILE + trow0 * 64 + 16 * (kh ^ kt);
  const int tl_off = DMA_TILE + trow0 * 64 + 16 * ((2 + kh) ^ kt);

  f32x16 acc[4];
  // exponent loads and LDS writes above must not count against the ring's vmcnt
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int nk = g.D / (BF ? 2 * BKS : BKS);
  dma(0);
  if (nk > 1) dma(1);
  // one k step; the first starts every accumulator from the MFMA's inline zero
  // (no 64 v_mov per wave to clear them)
  auto kstep = [&](int kk, auto first_tag) {
    constexpr bool FIRST = decltype(first_tag)::value;
    // this wave's 3 DMAs of step kk have landed (those of kk + 1 stay in flight);
    // the barrier publishes every wave's, and orders the ring slot's previous
    // readers (step kk - 1) before the refill below
    if (kk + 1 < nk) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kk + 2 < nk) dma(kk + 2);
    const unsigned char* st = smem + (kk % DMA_RING) * DMA_STAGE;
    if constexpr (BF) {
      // k 0-15 of the stage for every tile, then k 16-31 (the q2 kernel's order)
      const bf8v q0v = *reinterpret_cast<const bf8v*>(st + qh_off);
      const bf8v q1v = *reinterpret_cast<const bf8v*>(st + ql_off);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf8v t0v = *reinterpret_cast<const bf8v*>(st + th_off + t * 2048);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t0v, q0v, FIRST ? f32x16{} : acc[t], 0, 0,
                                                         0);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf8v t1v = *reinterpret_cast<const bf8v*>(st + tl_off + t * 2048);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t1v, q1v, acc[t], 0, 0, 0);
      }
    } else {
      const h8v qh = *reinterpret_cast<const h8v*>(st + qh_off);
      const h8v ql = *reinterpret_cast<const h8v*>(st + ql_off);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const h8v th = *reinterpret_cast<const h8v*>(st + th_off + t * 2048);
        const h8v tl = *reinterpret_cast<const h8v*>(st + tl_off + t * 2048);
        // small terms first
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, qh, FIRST ? f32x16{} : acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ql, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, qh, acc[t], 0, 0, 0);
      }
    }
  };
  kstep(0, std::true_type{});
  for (int kk = 1; kk < nk; ++kk) kstep(kk, std::false_type{});
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // ring reads done: the LDS is free for reuse
  const bool live = pc.qblk + half < g.qt;            // this half's query block exists
  const long long page = pc.page + (live ? (long long)half * g.tiles_h * g.tiles_w : 0);
  float* const stage = reinterpret_cast<float*>(smem) + half * WAVES * 16 * P0;
  if constexpr (BF) {
    if (live) {
      scale_acc<DIV>(acc, g);
      paged_epilogue<OT, EXF>(acc, stage, pyr, g, page, w4, lane);
    }
    return;
  }

  // a half past the last query block has no page (the epilogue syncs per wave;
  // a wave whose sums are not finite recomputes its pages from the f32 operands)
  if (live)
    dma_finish_f32<OT, DIV, EXF>(acc, g, pyr, stage, page, w4, lane, sq, qj, trow0, th0, tw0, b, f1,
                            f2, ps, ks, sexp);
}

// Floor-mode 2x2 average pool of one pyramid level into the next, for levels
// beyond the fused four (any layout, addressed through dxr::cell_index).
__global__ __launch_bounds__(256) void pool_level_kernel(float* __restrict__ pyr,
                                                         dxr::LevelLayout src,
                                                         dxr::LevelLayout dst, int B, int N) {
  const long long per = (long long)dst.h * dst.w;
  const long long total = (long long)B * N * per;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(idx % dst.w);
    const int y = (int)((idx / dst.w) % dst.h);
    const long long bq = idx / per;
    const int b = (int)(bq / N), q = (int)(bq % N);
    const float v00 = pyr[dxr::cell_index(src, b, q, 2 * y, 2 * x)];
    const float v01 = pyr[dxr::cell_index(src, b, q, 2 * y, 2 * x + 1)];
    const float v10 = pyr[dxr::cell_index(src, b, q, 2 * y + 1, 2 * x)];
    const float v11 = pyr[dxr::cell_index(src, b, q, 2 * y + 1, 2 * x + 1)];
    pyr[dxr::cell_index(dst, b, q, y, x)] = (((v00 + v01) + v10) + v11) * 0.25f;
  }
}

// Row-major [planes, H, W] -> [planes, H/2, W/2] pool (AlternateCorrBlock's fmaps).
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

// Reference layout [B*N][h][w] <-> paged level (pack: UNPACK=false).
template <bool UNPACK, typename PT>
__global__ __launch_bounds__(256) void repack_kernel(PT* __restrict__ pyr, float* __restrict__ ref,
                                                     dxr::LevelLayout lay, int B, int N) {
  const long long per = (long long)lay.h * lay.w;
  const long long total = (long long)B * N * per;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(idx % lay.w);
    const int y = (int)((idx / lay.w) % lay.h);
    const long long bq = idx / per;
    const int b = (int)(bq / N), q = (int)(bq % N);
    const long long c = dxr::cell_index(lay, b, q, y, x);
    if constexpr (UNPACK) {
      if constexpr (sizeof(PT) == 2) ref[idx] = dxr::bf16_to_f32(pyr[c]);
      else ref[idx] = pyr[c];
    } else {
      if constexpr (sizeof(PT) == 2) pyr[c] = dxr::f32_to_bf16(ref[idx]);
      else pyr[c] = ref[idx];
    }
  }
}

// Pyramid backward: the gradient of every level (paged, as the pyramid) folded
// down the avg-pool chain (F.avg_pool2d backward: each covered cell of level l
// receives 1/4 of its level-(l+1) cell's total gradient; the floor-mode
// remainder row / column receives none), then divided by the divisor:
// dV[b*N + q][y][x] = (d0 + (d1 + (d2 + ...) / 4) / 4) / divisor, row-major.
struct LevelsArg {
  int n;
  dxr::LevelLayout lay[8];
};

// One workgroup per (query, pair) row of dV [B*N, H, W]: threads along x, a loop
// over y, so every dV row is one coalesced store and the query's page bases are
// block constants.  Per cell, levels from the coarsest down: level l gets its own
// gradient plus a quarter of its parent's total (floor-mode remainders have no
// parent), then / sqrt(D).  (r02: the flat one-thread-per-element form spent its
// time in 64-bit index division — 0.65 ms at Sintel for 450 MB of traffic.)
template <bool DIV>
__global__ __launch_bounds__(128) void pyramid_backward_kernel(const float* __restrict__ gp,
                                                               float* __restrict__ dv, LevelsArg L,
                                                               int N, int H, int W, float divisor,
                                                               float recip) {
  const int q = blockIdx.x, b = blockIdx.y;
  long long base[8];     // this query's element offset in each level
  int ysh[8];            // tiled levels: log2(tile rows); row-major levels: -1
  long long ystride[8];  // elements between tile rows of pages (tiled) / rows (row-major)
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k >= L.n) break;
    const dxr::LevelLayout& y = L.lay[k];
    const long long S = (long long)y.th * y.tw;
    base[k] = y.off + ((long long)b * y.qt + q / y.qb) * y.ty * y.tx * y.qb * S + (q % y.qb) * S;
    ysh[k] = y.qb > 1 ? __builtin_ctz(y.th) : -1;
    ystride[k] = y.qb > 1 ? (long long)y.tx * y.qb * S : y.w;
  }
  float* row = dv + ((long long)b * N + q) * H * W;
  for (int x = threadIdx.x; x < W; x += 128) {
    long long xo[8];     // x part of the cell offset per level
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k >= L.n) break;
      const dxr::LevelLayout& y = L.lay[k];
      const int cx = x >> k;
      xo[k] = ysh[k] >= 0 ? (long long)(cx >> __builtin_ctz(y.tw)) * y.qb * y.th * y.tw +
                                (cx & (y.tw - 1))
                          : cx;
    }
    // YU rows at a time: all their level loads are issued before any is used
    constexpr int YU = 4;
    for (int y0 = 0; y0 < H; y0 += YU) {
      float d[YU][8];
#pragma unroll
      for (int u = 0; u < YU; ++u) {
        const int yy = y0 + u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          d[u][k] = 0.f;
          if (k >= L.n || yy >= H) continue;
          const dxr::LevelLayout& y = L.lay[k];
          const int yk = yy >> k;
          if (yk >= y.h || (x >> k) >= y.w) continue;
          const long long yo = ysh[k] >= 0
                                   ? (long long)(yk >> ysh[k]) * ystride[k] + (yk & (y.th - 1)) * y.tw
                                   : (long long)yk * ystride[k];
          d[u][k] = gp[base[k] + yo + xo[k]];
        }
      }
#pragma unroll
      for (int u = 0; u < YU; ++u) {
        const int yy = y0 + u;
        if (yy >= H) break;
        float t = 0.f;
#pragma unroll
        for (int k = 7; k >= 0; --k) {
          if (k >= L.n) continue;
          if ((yy >> k) >= L.lay[k].h || (x >> k) >= L.lay[k].w) continue;
          const bool parent = k + 1 < L.n && (yy >> (k + 1)) < L.lay[k + 1].h &&
                              (x >> (k + 1)) < L.lay[k + 1].w;
          t = parent ? d[u][k] + 0.25f * t : d[u][k];
        }
        row[(long long)yy * W + x] = DIV ? t / divisor : t * recip;
      }
    }
  }
}

unsigned grid_for(long long total) {
  long long blocks = (total + 255) / 256;
  if (blocks > 2048 * 8) blocks = 2048 * 8;
  return (unsigned)(blocks < 1 ? 1 : blocks);
}

int launch_avg_pool(const float* in, float* out, long long planes, int H, int W,
                    hipStream_t stream) {
  const long long total = planes * (long long)(H / 2) * (W / 2);
  if (total == 0) return DXR_OK;
  hipLaunchKernelGGL(avg_pool2x2_kernel, dim3(grid_for(total)), dim3(256), 0, stream, in, out,
                     planes, H, W);
  return dxr::launch_status();
}

dim3 build_grid(const BuildGeom& g, int B) {
  return dim3((unsigned)(g.tiles_h * g.tiles_w), (unsigned)((g.N + BM - 1) / BM), (unsigned)B);
}

// 1-D grid of every page (REMAP launches), or of every group of QB pages along
// queries.
dim3 remap_grid(const BuildGeom& g, int B, int QB = 1) {
  return dim3((unsigned)((long long)B * ((g.qt + QB - 1) / QB) * g.tiles_h * g.tiles_w));
}

// Exact-f32 build: VEC = float4 staging (W % 4 == 0, aligned) at 3 waves/SIMD
// (r01: 247-258 us at Sintel against 278 at the compiler's choice); scalar
// staging at the compiler's choice.
template <bool PAGED, typename OT>
int launch_f32(bool vec, const float* f1, const float* f2, OT* pyr, const BuildGeom& g, int B,
               hipStream_t stream) {
  const dim3 grid = build_grid(g, B);
  if (grid.y > 65535) return DXR_EINVAL;
  const bool div = g.recip == 0.f;
  if (vec && div)
    hipLaunchKernelGGL((corr_build_f32_kernel<true, 16, PAGED, OT, 3, true>), grid, dim3(NT), 0,
                       stream, f1, f2, pyr, g);
  else if (vec)
    hipLaunchKernelGGL((corr_build_f32_kernel<true, 16, PAGED, OT, 3, false>), grid, dim3(NT), 0,
                       stream, f1, f2, pyr, g);
  else if (div)
    hipLaunchKernelGGL((corr_build_f32_kernel<false, 16, PAGED, OT, 0, true>), grid, dim3(NT), 0,
                       stream, f1, f2, pyr, g);
  else
    hipLaunchKernelGGL((corr_build_f32_kernel<false, 16, PAGED, OT, 0, false>), grid, dim3(NT), 0,
                       stream, f1, f2, pyr, g);
  return dxr::launch_status();
}

// bf16 build: launch bound 3 waves/SIMD (compiled at 120 VGPRs = 4, matching
// the 4 workgroups per CU its 40 KB of LDS allows) and the XCD-aware page order
// (r01 KITTI b8: 721 us vs 837 in grid order).  The scalar-staging path keeps
// the compiler's choice (it would spill at 3) and the grid order.
// Channels-last bf16 fmaps: the two-block kernel's NHWC form (D % 32 == 0,
// 16-byte aligned pixels; checked by the caller).
template <typename OT>
int launch_build_bf16_nhwc(const uint16_t* f1, const uint16_t* f2, OT* pyr, const BuildGeom& g,
                           int B, hipStream_t stream) {
  const dim3 rg = remap_grid(g, B, 2);
  if (g.recip == 0.f)
    hipLaunchKernelGGL((corr_build_bf16_q2_kernel<OT, true, 4, true>), rg, dim3(2 * NT), 0, stream,
                       f1, f2, pyr, g);
  else
    hipLaunchKernelGGL((corr_build_bf16_q2_kernel<OT, false, 4, true>), rg, dim3(2 * NT), 0, stream,
                       f1, f2, pyr, g);
  return dxr::launch_status();
}

template <typename OT>
int launch_build_bf16(bool vec, const uint16_t* f1, const uint16_t* f2, OT* pyr,
                      const BuildGeom& g, int B, hipStream_t stream) {
  const dim3 grid = build_grid(g, B);
  if (grid.y > 65535) return DXR_EINVAL;
  const bool div = g.recip == 0.f;
  if (vec) {
    // two query blocks per workgroup, XCD-banded group order
    const dim3 rg = remap_grid(g, B, 2);
    if (div)
      hipLaunchKernelGGL((corr_build_bf16_q2_kernel<OT, true, 4>), rg, dim3(2 * NT), 0, stream, f1,
                         f2, pyr, g);
    else
      hipLaunchKernelGGL((corr_build_bf16_q2_kernel<OT, false, 4>), rg, dim3(2 * NT), 0, stream, f1,
                         f2, pyr, g);
  } else if (div) {
    hipLaunchKernelGGL((corr_build_bf16_kernel<false, OT, true, 0, false>), grid, dim3(NT), 0,
                       stream, f1, f2, pyr, g);
  } else {
    hipLaunchKernelGGL((corr_build_bf16_kernel<false, OT, false, 0, false>), grid, dim3(NT), 0,
                       stream, f1, f2, pyr, g);
  }
  return dxr::launch_status();
}

// Split build on the f16 pair split (H2; overflowing pages re-run on the 3-way
// bf16 split) at 3 waves/SIMD: r02 Sintel 134-142 us against 151-154 for the
// 3-way bf16 split at 4 waves/SIMD, and 0.4-0.8x its max error against f64
// (scripts/xp_accuracy.py).
template <typename OT, int BV, bool NHWC = false>
int launch_split(const float* f1, const float* f2, OT* pyr, const BuildGeom& g, int B,
                 hipStream_t stream) {
  const dim3 grid = build_grid(g, B);
  if (grid.y > 65535) return DXR_EINVAL;
  if (g.recip == 0.f)
    hipLaunchKernelGGL((corr_build_split_kernel<OT, true, 3, BV, NHWC, true>), grid, dim3(NT),
                       0, stream, f1, f2, pyr, g);
  else
    hipLaunchKernelGGL((corr_build_split_kernel<OT, false, 3, BV, NHWC, true>), grid, dim3(NT),
                       0, stream, f1, f2, pyr, g);
  return dxr::launch_status();
}

// Dispatch slots of the DMA build: two workgroups per CU (74.8 KB of LDS and 4
// waves per SIMD each), per device (cached) — the launch stream's device, which
// a C-API caller's current device need not be.
int dma_slots(hipStream_t stream) {
  static int cache[64] = {0};
  int dev = 0;
  if (hipStreamGetDevice(stream, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess) return 512;
  if (dev < 0 || dev >= 64) return 512;
  if (cache[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
      cus = 256;
    cache[dev] = 2 * cus;
  }
  return cache[dev];
}

// Grid of a DMA build (corr_build_dma_kernel) and its tail split.  U units (two
// query blocks x one target tile each) on S dispatch slots leave T = U mod S
// units for a last, partial round in which most CUs idle while T units take a
// whole unit time (Sintel B=1: 1,568 = 3 x 512 + 32).  Those T units run as 4T
// quarter units instead (dma_quarter: the same bits).  `tail`: split when
// 8 T <= tail * S (0: never; 8: always).  Same-process A/B (round 5, µs per
// build incl. the split pass, scripts/ab_build.py): Sintel B=1 (T = S/16) 107.5
// never -> 103.4 split; Sintel B=8 (T = S/2) 870.5 -> 883.2; KITTI B=8 bf16
// (T = S/5.3) 394.0 -> 395.9; Chairs (U < S) 35.2 -> 38.6: split only a short tail.
constexpr int DMA_TAIL_DEFAULT = 1;
dim3 dma_grid(BuildGeom& g, int B, hipStream_t stream, int tail = DMA_TAIL_DEFAULT) {
  const long long U = (long long)B * ((g.qt + 1) / 2) * g.tiles_h * g.tiles_w;
  const long long S = dma_slots(stream);
  long long T = U % S;
  if (8 * T > (long long)tail * S) T = 0;
  g.nmain = (int)(U - T);
  return dim3((unsigned)(U + 3 * T));
}

// Pyramid store policy of a DMA build (round 5, in the step with 12 lookups,
// scripts/ab_step.py -6; profiles/r05/experiments/r6n_build_store_policy.jsonl,
// r6q_bf16_build_store_policy.jsonl): write-through keeps part of a pyramid up to
// about twice the Infinity Cache resident for the lookups (f32 Sintel B=1, 261 MB:
// non-temporal +2.2 % per step; bf16 Sintel / KITTI / Chairs B=1: write-through
// -8.9 / -4.0 / -20.5 % against the bf16 build's earlier non-temporal stores,
// KITTI B=2 -2.0 %); beyond that nothing stays, and non-temporal stores stream it
// out faster (f32 Sintel B=8, 2.1 GB: -9.3 % per step; bf16 KITTI B=8, 1.1 GB,
// build alone: 393.7 vs 421.4 us).
template <typename OT>
bool dma_stream_out(const BuildGeom& g, int B) {
  const double pyr_bytes = (double)B * g.qt * BM * g.tiles_h * g.tiles_w * NTGT * (4.0 / 3.0) *
                           sizeof(OT);   // paged level 0 (queries x cells) + levels 1-3
  return pyr_bytes > 512.0 * (1 << 20);
}

// Launch corr_build_dma_kernel<OT, DIV, BF, EXF> with DIV from g.recip and EXF
// from dma_stream_out.
template <typename OT, bool BF, typename... A>
void launch_dma_kernel(const dim3& rg, const BuildGeom& g, int B, hipStream_t stream, A... args) {
  const bool so = dma_stream_out<OT>(g, B);
  auto go = [&](auto div_tag, auto ex_tag) {
    constexpr bool DV = decltype(div_tag)::value;
    constexpr int EXF = decltype(ex_tag)::value;
    hipLaunchKernelGGL((corr_build_dma_kernel<OT, DV, BF, EXF>), rg, dim3(2 * NT), 0, stream,
                       args..., g);
  };
  using T5 = std::integral_constant<int, 5>;
  using T3 = std::integral_constant<int, 3>;
  if (g.recip == 0.f) {
    if (so) go(std::true_type{}, T3{});
    else go(std::true_type{}, T5{});
  } else {
    if (so) go(std::false_type{}, T3{});
    else go(std::false_type{}, T5{});
  }
}

// Pre-split + LDS-DMA f32 build (round 3): workspace = SP1 | SP2 | E1 | E2.
long long align256(long long x) { return (x + 255) & ~255LL; }
long long dma_workspace_bytes(long long B, long long D, long long H, long long W) {
  const long long N = H * W;
  return 2 * align256(B * D * N * 4) + 2 * align256(B * N * 4);
}

template <typename OT, bool NHWC>
int launch_dma(const float* f1, const float* f2, OT* pyr, BuildGeom g, int B, void* ws,
               hipStream_t stream, int tail = DMA_TAIL_DEFAULT) {
  const dim3 grid = build_grid(g, B);
  if (grid.y > 65535) return DXR_EINVAL;
  const long long N = g.N, spb = align256((long long)B * g.D * N * 4), eb = align256((long long)B * N * 4);
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint8_t* sp1 = w;
  uint8_t* sp2 = w + spb;
  int* e1 = reinterpret_cast<int*>(w + 2 * spb);
  int* e2 = reinterpret_cast<int*>(w + 2 * spb + eb);
  // NCHW: 32 pixels per workgroup, two workgroups per CU (round 4, same-process
  // whole-build A/B: Sintel B=1 115.5 -> 114.4 us, split kernel 13.6 -> 12.4 us)
  constexpr int PX = NHWC ? 64 : 32;
  hipLaunchKernelGGL((split_pairs_kernel<NHWC, false, PX>),
                     dim3((unsigned)((N + PX - 1) / PX), (unsigned)B, 2), dim3(PX * 16), 0, stream,
                     f1, f2, reinterpret_cast<uint4*>(sp1), reinterpret_cast<uint4*>(sp2), e1, e2,
                     g.D, g.N);
  int st = dxr::launch_status();
  if (st != DXR_OK) return st;
  const dim3 rg = dma_grid(g, B, stream, tail);
  const int ps = NHWC ? g.D : 1, ks = NHWC ? 1 : g.N;   // fallback operand strides
  launch_dma_kernel<OT, false>(rg, g, B, stream, (const uint8_t*)sp1, (const uint8_t*)sp2,
                               (const int*)e1, (const int*)e2, pyr, f1, f2, ps, ks, 64, g.N * 64);
  return dxr::launch_status();
}

// bf16 operand records by LDS-DMA (corr_build_dma_kernel<.., BF>): channels-last
// bf16 fmaps are read in place (pixel stride D * 2 B, stage stride 64 B).
template <typename OT>
int launch_dma_bf16_nhwc(const uint16_t* f1, const uint16_t* f2, OT* pyr, BuildGeom g, int B,
                         hipStream_t stream, int tail = DMA_TAIL_DEFAULT) {
  const dim3 rg = dma_grid(g, B, stream, tail);
  const uint8_t* a = reinterpret_cast<const uint8_t*>(f1);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(f2);
  launch_dma_kernel<OT, true>(rg, g, B, stream, a, c, (const int*)nullptr, (const int*)nullptr, pyr,
                              (const float*)nullptr, (const float*)nullptr, 0, 0, g.D * 2, 64);
  return dxr::launch_status();
}

// Pack pass of the bf16 DMA build for NCHW fmaps: [D][N] bf16 -> blocked
// records [D/32][N][32 k] (64 B per pixel and 32-channel block, the layout a
// channels-last fmap already has per pixel).  Workgroup = 256 pixels x one
// 32-channel block; thread = 4 pixels x 8 channels: eight 8-byte loads along
// pixels (a wave reads 512 contiguous bytes per channel row; VEC: N % 4 == 0
// and 8-byte aligned rows), a register transpose, then the workgroup's 16 KB
// of records go through LDS so that every 16-byte write-through store
// instruction covers 1 KB of contiguous records (per-lane record pieces were
// partial-line write-throughs: 65 us at KITTI B=8).  Grid (ceil(N / 256), D / 32, 2 B).
template <bool VEC>
__global__ __launch_bounds__(256) void pack_bf16_kernel(const uint16_t* __restrict__ f1,
                                                        const uint16_t* __restrict__ f2,
                                                        uint8_t* __restrict__ o1,
                                                        uint8_t* __restrict__ o2, int D, int N) {
  __shared__ __attribute__((aligned(16))) uint4 rec[256 * 4];   // [pixel][4 x 16 B]
  const int tid = threadIdx.x, quad = tid & 63, cg = tid >> 6;
  const int kb = blockIdx.y, b = blockIdx.z >> 1, which = blockIdx.z & 1;
  const long long pbase = (long long)b * D * N;
  const uint16_t* src = (which ? f2 : f1) + pbase + (long long)(kb * 32 + cg * 8) * N;
  uint8_t* dst = (which ? o2 : o1) + pbase * 2;
  const int pw = blockIdx.x * 256;                 // first pixel of the workgroup
  const int p0 = pw + quad * 4;
  uint16_t v[8][4];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    if constexpr (VEC) {
      uint2 u = make_uint2(0u, 0u);
      if (p0 < N) u = *reinterpret_cast<const uint2*>(src + (long long)c * N + p0);
      v[c][0] = (uint16_t)u.x; v[c][1] = (uint16_t)(u.x >> 16);
      v[c][2] = (uint16_t)u.y; v[c][3] = (uint16_t)(u.y >> 16);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[c][i] = p0 + i < N ? src[(long long)c * N + p0 + i] : (uint16_t)0;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
    rec[(quad * 4 + i) * 4 + cg] = make_uint4((uint32_t)v[0][i] | ((uint32_t)v[1][i] << 16),
                                              (uint32_t)v[2][i] | ((uint32_t)v[3][i] << 16),
                                              (uint32_t)v[4][i] | ((uint32_t)v[5][i] << 16),
                                              (uint32_t)v[6][i] | ((uint32_t)v[7][i] << 16));
  __syncthreads();
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, 0x7fffffff, 0x00020000);
  const unsigned base = (unsigned)(((long long)kb * N + pw) * 64);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = i * 256 + tid;                   // 16-B piece of the workgroup's records
    if (pw + (e >> 2) < N)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, rec[e]), r,
                                             base + (unsigned)e * 16u, 0, 16);
  }
}

long long bf16_pack_bytes(long long B, long long D, long long H, long long W) {
  return 2 * align256(B * D * H * W * 2);
}

// NCHW bf16 fmaps with a workspace: pack pass + the bf16 DMA build
// (blocked records: pixel stride 64 B, stage stride N * 64 B).
template <typename OT>
int launch_dma_bf16_nchw(const uint16_t* f1, const uint16_t* f2, OT* pyr, BuildGeom g, int B,
                         void* ws, hipStream_t stream, int tail = DMA_TAIL_DEFAULT) {
  const long long half = align256((long long)B * g.D * g.N * 2);
  uint8_t* o1 = static_cast<uint8_t*>(ws);
  uint8_t* o2 = o1 + half;
  const dim3 pg((unsigned)((g.N + 255) / 256), (unsigned)(g.D / 32), (unsigned)(2 * B));
  const bool vec = g.N % 4 == 0 && ((uintptr_t)f1 % 8) == 0 && ((uintptr_t)f2 % 8) == 0;
  if (vec)
    hipLaunchKernelGGL(pack_bf16_kernel<true>, pg, dim3(256), 0, stream, f1, f2, o1, o2, g.D, g.N);
  else
    hipLaunchKernelGGL(pack_bf16_kernel<false>, pg, dim3(256), 0, stream, f1, f2, o1, o2, g.D, g.N);
  int st = dxr::launch_status();
  if (st != DXR_OK) return st;
  const dim3 rg = dma_grid(g, B, stream, tail);
  launch_dma_kernel<OT, true>(rg, g, B, stream, (const uint8_t*)o1, (const uint8_t*)o2,
                              (const int*)nullptr, (const int*)nullptr, pyr, (const float*)nullptr,
                              (const float*)nullptr, 0, 0, 64, g.N * 64);
  return dxr::launch_status();
}

// f32 fmaps: the split build when its layout conditions hold (D % 16 == 0;
// float4 target units for W % 4 == 0, float2 units for even W), else — or on
// request (DXR_BUILD_EXACT_F32) — the exact-f32 MFMA build.
template <typename OT>
int launch_build_f32(bool vec, const float* f1, const float* f2, OT* pyr, const BuildGeom& g,
                     int B, int algo, hipStream_t stream) {
  if (algo == DXR_BUILD_AUTO && g.D % 16 == 0 && (long long)g.D * g.N < (1LL << 29)) {
    if (vec) return launch_split<OT, 4>(f1, f2, pyr, g, B, stream);
    if (g.W % 2 == 0 && ((uintptr_t)f1 % 8) == 0 && ((uintptr_t)f2 % 8) == 0 &&
        ((uintptr_t)pyr % 16) == 0)
      return launch_split<OT, 2>(f1, f2, pyr, g, B, stream);
  }
  return launch_f32<true>(vec, f1, f2, pyr, g, B, stream);
}

BuildGeom make_geom(int64_t D, int64_t H, int64_t W, float divisor, const dxr::Levels& L) {
  BuildGeom g;
  g.D = (int)D; g.H = (int)H; g.W = (int)W; g.N = (int)(H * W);
  g.levels = L.n < 4 ? L.n : 4;
  g.tiles_w = (int)((W + TW - 1) / TW);
  g.tiles_h = (int)((H + TH - 1) / TH);
  g.qt = (int)((H * W + BM - 1) / BM);
  g.strip = STRIP;
  g.nmain = 0x7fffffff;
  g.divisor = divisor;
  int e2 = 0;
  g.recip = (std::frexp(divisor, &e2) == 0.5f) ? 1.f / divisor : 0.f;  // exact iff 2^k
  for (int l = 0; l < 4; ++l) {
    g.lh[l] = l < L.n ? L.h[l] : 1;
    g.lw[l] = l < L.n ? L.w[l] : 1;
    g.loff[l] = l < L.n ? L.off[l] : 0;
  }
  return g;
}

bool aligned16(const void* p) { return ((uintptr_t)p % 16) == 0; }

constexpr int PROCEED = -100;

int check_build_args(const void* fmap1, const void* fmap2, int in_dtype, int64_t B, int64_t D,
                     float divisor, const void* out, int out_dtype) {
  if (D < 1 || D > (1 << 20) || !(divisor == divisor) || divisor == 0.f) return DXR_EINVAL;
  if (B > 65535) return DXR_EINVAL;
  if ((in_dtype != DXR_F32 && in_dtype != DXR_BF16) ||
      (out_dtype != DXR_F32 && out_dtype != DXR_BF16))
    return DXR_EINVAL;
  if (B == 0) return DXR_OK;
  if (!fmap1 || !fmap2 || !out) return DXR_EINVAL;
  return PROCEED;
}

}  // namespace

extern "C" int dxr_avg_pool2x2(const float* in, float* out, int64_t planes, int64_t H, int64_t W,
                               hipStream_t stream) {
  if (planes < 0 || H < 1 || W < 1 || H > (1 << 30) || W > (1 << 30)) return DXR_EINVAL;
  if (planes == 0 || H < 2 || W < 2) return DXR_OK;
  if (!in || !out) return DXR_EINVAL;
  return launch_avg_pool(in, out, planes, (int)H, (int)W, stream);
}

namespace {
int pyramid_build(const void* fmap1, const void* fmap2, int in_dtype, int fmap_layout, int64_t B,
                  int64_t D, int64_t H, int64_t W, int num_levels, float divisor, void* pyramid,
                  int pyr_dtype, int algo, void* workspace, int64_t workspace_bytes,
                  hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L)) return DXR_EINVAL;
  if (fmap_layout != DXR_NCHW && fmap_layout != DXR_NHWC) return DXR_EINVAL;
  if (algo != DXR_BUILD_AUTO && algo != DXR_BUILD_EXACT_F32) return DXR_EINVAL;
  const int chk = check_build_args(fmap1, fmap2, in_dtype, B, D, divisor, pyramid, pyr_dtype);
  if (chk != PROCEED) return chk;
  // Levels beyond the fused four are pooled by f32 passes: f32 pyramids only.
  if (L.n > dxr::TILED_LEVELS && pyr_dtype != DXR_F32) return DXR_EUNSUPPORTED;
  if (algo == DXR_BUILD_EXACT_F32 && in_dtype != DXR_F32) return DXR_EUNSUPPORTED;
  const BuildGeom g = make_geom(D, H, W, divisor, L);
  int st = PROCEED;
  // f32 operands with a workspace: pre-split f16 pairs + the LDS-DMA build
  // (any W; D % 16 == 0; NHWC rows 16-byte aligned).
  const bool dma_ok = in_dtype == DXR_F32 && algo == DXR_BUILD_AUTO && D % 16 == 0 &&
                      D * H * W < (1LL << 29) && workspace != nullptr && aligned16(workspace) &&
                      workspace_bytes >= dma_workspace_bytes(B, D, H, W) && aligned16(pyramid);
  if (dma_ok) {
    const float* f1 = static_cast<const float*>(fmap1);
    const float* f2 = static_cast<const float*>(fmap2);
    float* pf = static_cast<float*>(pyramid);
    uint16_t* ph = static_cast<uint16_t*>(pyramid);
    const bool f32p = pyr_dtype == DXR_F32;
    // NCHW operands are read as scalars by the split pass; NHWC as float4
    if (fmap_layout == DXR_NCHW)
      st = f32p ? launch_dma<float, false>(f1, f2, pf, g, (int)B, workspace, stream)
                : launch_dma<uint16_t, false>(f1, f2, ph, g, (int)B, workspace, stream);
    else if (aligned16(f1) && aligned16(f2))
      st = f32p ? launch_dma<float, true>(f1, f2, pf, g, (int)B, workspace, stream)
                : launch_dma<uint16_t, true>(f1, f2, ph, g, (int)B, workspace, stream);
  }
  // bf16 NCHW operands with a workspace: pack pass + the bf16 DMA build (D % 32,
  // D * N * 2 < 2^31 per pair)
  if (st == PROCEED && in_dtype == DXR_BF16 && fmap_layout == DXR_NCHW && D % 32 == 0 &&
      D * H * W < (1LL << 30) && L.n <= dxr::TILED_LEVELS && workspace != nullptr &&
      aligned16(workspace) && workspace_bytes >= bf16_pack_bytes(B, D, H, W) &&
      aligned16(pyramid)) {
    const uint16_t* f1 = static_cast<const uint16_t*>(fmap1);
    const uint16_t* f2 = static_cast<const uint16_t*>(fmap2);
    st = pyr_dtype == DXR_F32
             ? launch_dma_bf16_nchw(f1, f2, static_cast<float*>(pyramid), g, (int)B, workspace,
                                    stream)
             : launch_dma_bf16_nchw(f1, f2, static_cast<uint16_t*>(pyramid), g, (int)B, workspace,
                                    stream);
  }
  if (st != PROCEED) {
    // done by a DMA build
  } else if (fmap_layout == DXR_NHWC && in_dtype == DXR_BF16) {
    // channels-last bf16 operands (the bf16 mode's encoders, core/extractor.py:168-192):
    // the two-block bf16 build's NHWC form, bit-identical to the NCHW build;
    // D % 32 == 0 (whole 32-channel stages) and 16-byte aligned pixels
    if (D % 32 != 0 || D * H * W >= (1LL << 30) || !aligned16(fmap1) || !aligned16(fmap2) ||
        !aligned16(pyramid))
      return DXR_EUNSUPPORTED;
    const uint16_t* f1 = static_cast<const uint16_t*>(fmap1);
    const uint16_t* f2 = static_cast<const uint16_t*>(fmap2);
    st = pyr_dtype == DXR_F32
             ? launch_dma_bf16_nhwc(f1, f2, static_cast<float*>(pyramid), g, (int)B, stream)
             : launch_dma_bf16_nhwc(f1, f2, static_cast<uint16_t*>(pyramid), g, (int)B, stream);
  } else if (fmap_layout == DXR_NHWC) {
    // channels-last f32 operands: the split build's NHWC form, where the NCHW build
    // would also be the split build (f32 fmaps, D % 16 == 0, even W: same bits),
    // with 16-byte aligned rows; other requests are unsupported (callers transpose)
    if (algo != DXR_BUILD_AUTO || D % 16 != 0 || W % 2 != 0 ||
        D * H * W >= (1LL << 29) || !aligned16(fmap1) || !aligned16(fmap2) || !aligned16(pyramid))
      return DXR_EUNSUPPORTED;
    const float* f1 = static_cast<const float*>(fmap1);
    const float* f2 = static_cast<const float*>(fmap2);
    st = pyr_dtype == DXR_F32
             ? launch_split<float, 4, true>(f1, f2, static_cast<float*>(pyramid), g, (int)B, stream)
             : launch_split<uint16_t, 4, true>(f1, f2, static_cast<uint16_t*>(pyramid), g, (int)B,
                                               stream);
  } else if (in_dtype == DXR_F32) {
    const float* f1 = static_cast<const float*>(fmap1);
    const float* f2 = static_cast<const float*>(fmap2);
    const bool vec = (W % 4) == 0 && aligned16(f1) && aligned16(f2) && aligned16(pyramid);
    st = pyr_dtype == DXR_F32
             ? launch_build_f32(vec, f1, f2, static_cast<float*>(pyramid), g, (int)B, algo, stream)
             : launch_build_f32(vec, f1, f2, static_cast<uint16_t*>(pyramid), g, (int)B, algo,
                                stream);
  } else {
    const uint16_t* f1 = static_cast<const uint16_t*>(fmap1);
    const uint16_t* f2 = static_cast<const uint16_t*>(fmap2);
    const bool vec = (W % 4) == 0 && ((uintptr_t)f1 % 8) == 0 && ((uintptr_t)f2 % 8) == 0 &&
                     aligned16(pyramid) && D * H * W < (1LL << 30);
    st = pyr_dtype == DXR_F32
             ? launch_build_bf16(vec, f1, f2, static_cast<float*>(pyramid), g, (int)B, stream)
             : launch_build_bf16(vec, f1, f2, static_cast<uint16_t*>(pyramid), g, (int)B, stream);
  }
  if (st != DXR_OK) return st;
  float* pyr = static_cast<float*>(pyramid);
  // Levels beyond the fused four: plain pooling passes, level l from level l-1.
  for (int l = dxr::TILED_LEVELS; l < L.n; ++l) {
    const long long total = B * H * W * (long long)L.h[l] * L.w[l];
    hipLaunchKernelGGL(pool_level_kernel, dim3(grid_for(total)), dim3(256), 0, stream, pyr,
                       L.lay[l - 1], L.lay[l], (int)B, (int)(H * W));
    st = dxr::launch_status();
    if (st != DXR_OK) return st;
  }
  return DXR_OK;
}
}  // namespace

extern "C" int64_t dxr_build_workspace_bytes(int in_dtype, int64_t B, int64_t D, int64_t H,
                                             int64_t W) {
  if (B < 0 || D < 1 || H < 1 || W < 1 || H * W > (1LL << 30)) return -1;
  if (in_dtype == DXR_BF16) return D % 32 == 0 ? bf16_pack_bytes(B, D, H, W) : 0;
  if (in_dtype != DXR_F32 || D % 16 != 0) return 0;
  return dma_workspace_bytes(B, D, H, W);
}

extern "C" int dxr_corr_pyramid_build_ws(const void* fmap1, const void* fmap2, int in_dtype,
                                         int fmap_layout, int64_t B, int64_t D, int64_t H,
                                         int64_t W, int num_levels, float divisor, void* pyramid,
                                         int pyr_dtype, int algo, void* workspace,
                                         int64_t workspace_bytes, hipStream_t stream) {
  return pyramid_build(fmap1, fmap2, in_dtype, fmap_layout, B, D, H, W, num_levels, divisor,
                       pyramid, pyr_dtype, algo, workspace, workspace_bytes, stream);
}

extern "C" int dxr_corr_pyramid_build(const void* fmap1, const void* fmap2, int in_dtype,
                                      int fmap_layout, int64_t B, int64_t D, int64_t H,
                                      int64_t W, int num_levels, float divisor, void* pyramid,
                                      int pyr_dtype, int algo, hipStream_t stream) {
  return pyramid_build(fmap1, fmap2, in_dtype, fmap_layout, B, D, H, W, num_levels, divisor,
                       pyramid, pyr_dtype, algo, nullptr, 0, stream);
}

extern "C" int dxr_corr_volume(const void* fmap1, const void* fmap2, int in_dtype, int64_t B,
                               int64_t D, int64_t H, int64_t W, float divisor, float* out,
                               hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, 1, &L)) return DXR_EINVAL;
  const int chk = check_build_args(fmap1, fmap2, in_dtype, B, D, divisor, out, DXR_F32);
  if (chk != PROCEED) return chk;
  if (in_dtype != DXR_F32) return DXR_EUNSUPPORTED;
  const BuildGeom g = make_geom(D, H, W, divisor, L);
  const float* f1 = static_cast<const float*>(fmap1);
  const float* f2 = static_cast<const float*>(fmap2);
  const bool vec = (W % 4) == 0 && aligned16(f1) && aligned16(f2) && aligned16(out);
  return launch_f32<false>(vec, f1, f2, out, g, (int)B, stream);
}

extern "C" int dxr_pyramid_unpack(const void* pyramid, int pyr_dtype, int64_t B, int64_t H,
                                  int64_t W, int num_levels, int level, float* out,
                                  hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L) || level < 0 || level >= num_levels)
    return DXR_EINVAL;
  if (pyr_dtype != DXR_F32 && pyr_dtype != DXR_BF16) return DXR_EINVAL;
  if (B == 0) return DXR_OK;
  if (!pyramid || !out) return DXR_EINVAL;
  const long long total = B * H * W * (long long)L.h[level] * L.w[level];
  if (pyr_dtype == DXR_F32)
    hipLaunchKernelGGL((repack_kernel<true, float>), dim3(grid_for(total)), dim3(256), 0, stream,
                       const_cast<float*>(static_cast<const float*>(pyramid)), out, L.lay[level],
                       (int)B, (int)(H * W));
  else
    hipLaunchKernelGGL((repack_kernel<true, uint16_t>), dim3(grid_for(total)), dim3(256), 0,
                       stream, const_cast<uint16_t*>(static_cast<const uint16_t*>(pyramid)), out,
                       L.lay[level], (int)B, (int)(H * W));
  return dxr::launch_status();
}

extern "C" int dxr_pyramid_pack(const float* level_data, int64_t B, int64_t H, int64_t W,
                                int num_levels, int level, void* pyramid, int pyr_dtype,
                                hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L) || level < 0 || level >= num_levels)
    return DXR_EINVAL;
  if (pyr_dtype != DXR_F32 && pyr_dtype != DXR_BF16) return DXR_EINVAL;
  if (B == 0) return DXR_OK;
  if (!pyramid || !level_data) return DXR_EINVAL;
  const long long total = B * H * W * (long long)L.h[level] * L.w[level];
  float* src = const_cast<float*>(level_data);
  if (pyr_dtype == DXR_F32)
    hipLaunchKernelGGL((repack_kernel<false, float>), dim3(grid_for(total)), dim3(256), 0, stream,
                       static_cast<float*>(pyramid), src, L.lay[level], (int)B, (int)(H * W));
  else
    hipLaunchKernelGGL((repack_kernel<false, uint16_t>), dim3(grid_for(total)), dim3(256), 0,
                       stream, static_cast<uint16_t*>(pyramid), src, L.lay[level], (int)B,
                       (int)(H * W));
  return dxr::launch_status();
}

extern "C" int dxr_pyramid_backward(const void* grad_pyramid, int grad_dtype, int64_t B,
                                    int64_t H, int64_t W, int num_levels, float divisor,
                                    float* grad_volume, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L)) return DXR_EINVAL;
  if (grad_dtype != DXR_F32) return grad_dtype == DXR_BF16 ? DXR_EUNSUPPORTED : DXR_EINVAL;
  if (!(divisor == divisor) || divisor == 0.f || B > 65535) return DXR_EINVAL;
  if (B == 0) return DXR_OK;
  if (!grad_pyramid || !grad_volume) return DXR_EINVAL;
  LevelsArg la;
  la.n = L.n;
  for (int l = 0; l < L.n; ++l) la.lay[l] = L.lay[l];
  int e2 = 0;
  const float recip = (std::frexp(divisor, &e2) == 0.5f) ? 1.f / divisor : 0.f;
  const float* gp = static_cast<const float*>(grad_pyramid);
  const dim3 grid((unsigned)(H * W), (unsigned)B);
  if (recip != 0.f)
    hipLaunchKernelGGL(pyramid_backward_kernel<false>, grid, dim3(128), 0, stream, gp, grad_volume,
                       la, (int)(H * W), (int)H, (int)W, divisor, recip);
  else
    hipLaunchKernelGGL(pyramid_backward_kernel<true>, grid, dim3(128), 0, stream, gp, grad_volume,
                       la, (int)(H * W), (int)H, (int)W, divisor, recip);
  return dxr::launch_status();
}

