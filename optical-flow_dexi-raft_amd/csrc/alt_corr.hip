// Stage (d): on-the-fly ("alternate") correlation lookup — no O((HW)^2) volume.
//
// Replaces alt_cuda_corr/correlation_kernel.cu:18-119 (corr_forward_kernel) +
// :260-286 (corr_cuda_forward), reached through alt_cuda_corr/correlation.cpp:23-33,
// and the Python loop around it, core/corr.py:74-91 (AlternateCorrBlock.__call__).
//
// Semantics (restated from correlation_kernel.cu:59-114): for a query pixel with
// level coordinate (x, y), x0 = floor(x), dx = x - x0 (same for y), the (2r+2)^2
// integer cells (h2, w2) = (y0 - r + iy, x0 - r + ix), iy, ix in [0, 2r+1], each
// get s = <fmap1[q], fmap2[h2, w2]> (0 outside the map), and output channel
// oy + (2r+1)*ox receives the bilinear combination of cells (oy..oy+1, ox..ox+1):
//   s(oy,ox)(1-dy)(1-dx) + s(oy,ox+1)(1-dy)dx + s(oy+1,ox)dy(1-dx) + s(oy+1,ox+1)dy dx
// i.e. bilinear sampling at (x - r + ox, y - r + oy) of the implicit correlation.
//
// MI355X mapping.  A workgroup owns 64 consecutive query pixels of one
// (pair, level).  Each wave takes one query at a time: lane L holds channels
// [4L, 4L+4) (+256 m) of fmap1[q] in registers and reads, per cell, the 16-byte
// slice of fmap2[cell] — one fully coalesced 1 KiB wave load per cell vector.
// Partial dot products of 16 cells are reduced across the wave by a 17-shuffle
// butterfly transpose (each lane ends with one cell's sum), cell sums go to LDS,
// and after one barrier every thread emits outputs for one query with coalesced
// 256-byte wave stores along the query dimension.
#include <algorithm>
#include <cmath>
#include <cstdint>

#include <type_traits>

#include "dxr_common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;

struct AltLevel {
  const float* f2;        // [Bf, H2, W2, C]
  int H2, W2;
  float inv;              // coordinate scale (1 / 2^l)
  int ch_off;             // first output channel of this level
};

struct AltGeom {
  int N;                  // query pixels per coordinate set (H1 * W1)
  int C;
  int Nc;                 // coordinate sets per pair (reference FFI); 1 for the fused form
  int cout;               // channels per output image
  float divisor;
  float div_recip = 0.f;  // 1 / divisor when divisor is a power of two (exact), else 0
  long long f1_bstride;   // H1 * W1 * C
  long long coord_zstride, coord_cstride, coord_qstride;
  AltLevel lv[8];
  dxr::LevelLayout vlay{};  // FULL: the volume's paged level layout (offset from the volume buffer)
};

template <int R>
struct Cells {
  static constexpr int RD = 2 * R + 1;
  static constexpr int RD1 = RD + 1;
  static constexpr int NCELL = RD1 * RD1;
  static constexpr int NB = (NCELL + 15) / 16;   // 16-cell batches
  static constexpr int LD = NCELL + 1;           // LDS row pitch (odd: no bank aliasing)
};

template <int R, bool VEC>
__global__ __launch_bounds__(256) void alt_corr_kernel(const float* __restrict__ f1,
                                                       const float* __restrict__ coords,
                                                       float* __restrict__ out, AltGeom g) {
  using CL = Cells<R>;
  constexpr int RD = CL::RD, RD1 = CL::RD1, NCELL = CL::NCELL;
  __shared__ float cells[64 * CL::LD];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q0 = blockIdx.x * 64;
  const AltLevel lv = g.lv[blockIdx.y];
  const int z = blockIdx.z;           // coordinate-set index (b * Nc + n)
  const int bf = z / g.Nc;            // fmap batch index
  const float* cz = coords + (long long)z * g.coord_zstride;
  const float* f1b = f1 + (long long)bf * g.f1_bstride;
  const float* f2b = lv.f2 + (long long)bf * lv.H2 * lv.W2 * g.C;
  const int nslab = VEC ? (g.C + 255) / 256 : (g.C + 63) / 64;

  for (int qq = wave; qq < 64; qq += 4) {
    const int q = q0 + qq;
    if (q >= g.N) break;  // wave-uniform
    const float x = cz[(long long)q * g.coord_qstride] * lv.inv;
    const float y = cz[(long long)q * g.coord_qstride + g.coord_cstride] * lv.inv;
    const float xf = floorf(x), yf = floorf(y);
    const bool near = fabsf(xf) < 1.0e8f && fabsf(yf) < 1.0e8f;
    const int xb = near ? (int)xf - R : -(1 << 28);
    const int yb = near ? (int)yf - R : -(1 << 28);

    for (int cb = 0; cb < CL::NB; ++cb) {
      float p[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) p[i] = 0.f;
      for (int m = 0; m < nslab; ++m) {
        if constexpr (VEC) {
          const int c = 4 * lane + 256 * m;
          if (c < g.C) {
            const float4 a = *reinterpret_cast<const float4*>(f1b + (long long)q * g.C + c);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int cell = cb * 16 + i;
              if (cell < NCELL) {
                const int hh = yb + cell / RD1, ww = xb + cell % RD1;
                if ((unsigned)hh < (unsigned)lv.H2 && (unsigned)ww < (unsigned)lv.W2) {
                  const float4 v = *reinterpret_cast<const float4*>(
                      f2b + ((long long)hh * lv.W2 + ww) * g.C + c);
                  p[i] += a.x * v.x + a.y * v.y + a.z * v.z + a.w * v.w;
                }
              }
            }
          }
        } else {
          const int c = lane + 64 * m;
          if (c < g.C) {
            const float a = f1b[(long long)q * g.C + c];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int cell = cb * 16 + i;
              if (cell < NCELL) {
                const int hh = yb + cell / RD1, ww = xb + cell % RD1;
                if ((unsigned)hh < (unsigned)lv.H2 && (unsigned)ww < (unsigned)lv.W2)
                  p[i] += a * f2b[((long long)hh * lv.W2 + ww) * g.C + c];
              }
            }
          }
        }
      }
      // Butterfly transpose-reduce: 16 partials x 64 lanes -> one cell per lane.
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bool hi = lane & 32;
        const float send = hi ? p[i] : p[i + 8], keep = hi ? p[i + 8] : p[i];
        p[i] = keep + __shfl_xor(send, 32);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool hi = lane & 16;
        const float send = hi ? p[i] : p[i + 4], keep = hi ? p[i + 4] : p[i];
        p[i] = keep + __shfl_xor(send, 16);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool hi = lane & 8;
        const float send = hi ? p[i] : p[i + 2], keep = hi ? p[i + 2] : p[i];
        p[i] = keep + __shfl_xor(send, 8);
      }
      {
        const bool hi = lane & 4;
        const float send = hi ? p[0] : p[1], keep = hi ? p[1] : p[0];
        p[0] = keep + __shfl_xor(send, 4);
      }
      p[0] += __shfl_xor(p[0], 2);
      p[0] += __shfl_xor(p[0], 1);
      const int cell = cb * 16 + ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 +
                       ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
      if ((lane & 3) == 0 && cell < NCELL) cells[qq * CL::LD + cell] = p[0];
    }
  }
  __syncthreads();

  // Output phase: thread -> (query = tid % 64, x-offset class = tid / 64).
  const int qq = tid & 63;
  const int q = q0 + qq;
  if (q >= g.N) return;
  const float x = cz[(long long)q * g.coord_qstride] * lv.inv;
  const float y = cz[(long long)q * g.coord_qstride + g.coord_cstride] * lv.inv;
  const float dx = x - floorf(x), dy = y - floorf(y);
  const float* s = cells + qq * CL::LD;
  float* o = out + (long long)z * g.cout * g.N + (long long)lv.ch_off * g.N + q;
  for (int ox = wave; ox < RD; ox += 4) {
#pragma unroll
    for (int oy = 0; oy < RD; ++oy) {
      // Reference accumulation order: se, sw, ne, nw (cell loop iy-major, ix-minor).
      const float s00 = s[oy * RD1 + ox], s01 = s[oy * RD1 + ox + 1];
      const float s10 = s[(oy + 1) * RD1 + ox], s11 = s[(oy + 1) * RD1 + ox + 1];
      float v = __fmul_rn(__fmul_rn(s00, 1.f - dy), 1.f - dx);
      v = __fadd_rn(v, __fmul_rn(__fmul_rn(s01, 1.f - dy), dx));
      v = __fadd_rn(v, __fmul_rn(__fmul_rn(s10, dy), 1.f - dx));
      v = __fadd_rn(v, __fmul_rn(__fmul_rn(s11, dy), dx));
      o[(long long)(oy + RD * ox) * g.N] = v / g.divisor;
    }
  }
}

// ---------------------------------------------------------------------------
// MFMA form (default when C % 16 == 0, C <= 256).  A workgroup owns a 4 x 8
// tile of query pixels and one level.  The queries' (2r+2)^2 windows overlap,
// so it computes the dot products of its 32 queries with every cell of the
// windows' union bounding box (clipped to the level) as a small GEMM on the
// matrix cores, cells x queries x C, and keeps the entries that fall in each
// query's own window.  Every fmap2 cell vector is then read once per workgroup
// instead of once per query (the per-query form above re-reads 100 cell vectors
// per query: 6.7 GB per 1080p lookup, 1.37 ms).  f32 class: both operands are
// split into f16 pairs (H2, as the split build, csrc/corr_build.hip; r01: a 3-way
// bf16 split with six products, still the overflow fallback) and accumulated in
// f32; the query planes are split once into LDS, cell vectors in registers as
// they arrive (one k step ahead).  Box
// cells are walked in chunks of 4 waves x 32*NRB.  The bilinear combination and
// the output follow the per-query form exactly.
// ---------------------------------------------------------------------------
typedef __bf16 abf8 __attribute__((ext_vector_type(8)));
typedef float af16 __attribute__((ext_vector_type(16)));
typedef __bf16 abf2 __attribute__((ext_vector_type(2)));
typedef float af2 __attribute__((ext_vector_type(2)));

constexpr int TQY = 4, TQX = 8, TQ = TQY * TQX;    // query tile (32 pixels)

__device__ __forceinline__ uint32_t alt_cvt_pk(float a, float b) {
  const af2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, abf2));
}

// Exact hi/mid/lo split of 8 floats into three 8 x bf16 operands.
__device__ __forceinline__ void alt_split8(const float (&x)[8], uint4& h, uint4& m, uint4& l) {
  uint32_t hh[4], mm[4], ll[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a = x[2 * e], b = x[2 * e + 1];
    const uint32_t hp = alt_cvt_pk(a, b);
    const float ha = __uint_as_float(hp << 16), hb = __uint_as_float(hp & 0xffff0000u);
    const float ra = __builtin_isinf(ha) ? 0.f : a - ha, rb = __builtin_isinf(hb) ? 0.f : b - hb;
    const uint32_t mp = alt_cvt_pk(ra, rb);
    const float la = ra - __uint_as_float(mp << 16), lb = rb - __uint_as_float(mp & 0xffff0000u);
    hh[e] = hp;
    mm[e] = mp;
    ll[e] = __builtin_amdgcn_perm(__float_as_uint(lb), __float_as_uint(la), 0x07060302u);
  }
  h = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  m = make_uint4(mm[0], mm[1], mm[2], mm[3]);
  l = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

// f16 pair split of 8 floats (csrc/corr_build.hip split2h): x = hi + 2^-11 lo,
// hi = RNE_f16(x), lo = RNE_f16((x - hi) * 2^11); valid while |x| < 65520.
typedef _Float16 ah2 __attribute__((ext_vector_type(2)));
typedef _Float16 ah8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint32_t alt_cvt_pk_h(float a, float b) {
  const af2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, ah2));
}
__device__ __forceinline__ void alt_split8h(const float (&x)[8], uint4& h, uint4& l) {
  uint32_t hh[4], ll[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a = x[2 * e], b = x[2 * e + 1];
    hh[e] = alt_cvt_pk_h(a, b);
    const ah2 hv = __builtin_bit_cast(ah2, hh[e]);
    ll[e] = alt_cvt_pk_h((a - (float)hv[0]) * 2048.f, (b - (float)hv[1]) * 2048.f);
  }
  h = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  l = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

// H2: the f16 pair split (3 f16 products, cross terms in a second accumulator),
// as the split build; a chunk whose sums are not finite (an operand beyond f16
// range, or inf/NaN) is recomputed by its wave on the 3-way bf16 split, with
// the query operand split from fmap1 in registers.
// BIN: the workgroup's 32 queries are not a 4 x 8 pixel tile but 32 consecutive
// entries of `ord` — this coordinate set's and level's query list in the order
// alt_bin_*_kernel chose (grouped by window position, or the tile order), each
// entry {query, x, y, -} carrying the query's coordinates, so a workgroup's
// first global read gives it both.
// PF: k steps of cell-vector loads kept in flight (a ring of PF register stages).
// XP (experiments only; 0 in the product): bit 0 feeds the cell vectors' raw
// bits to the f16 MFMAs instead of splitting them (and skips the non-finite
// fallback) — a timing ablation of the split's VALU work, results meaningless;
// bit 1 stores only outputs that are exactly 12345.0 (none: an ablation of the
// output stores).
// FULL (round 6, the coarse-level volumes of dxr_alt_coarse_volumes): the box is
// the whole level and every (cell, query) sum is stored, raw (not divided), into
// `out` in the pyramid's paged layout of that level (g.vlay, dxr_common.h
// cell_index): the same products in the same order as the windowed form, so a
// lookup that reads its windows from the volume reproduces the on-the-fly
// outputs bit for bit (finite operands inside the f16 pair's range; a chunk with
// a non-finite sum is recomputed on the bf16 split in either form, and chunks
// group different cells in the two forms).  Tile order only (BIN = false);
// coordinates are not read.
template <int R, int NRB, int CMAX, bool H2 = false, int MINW = 2, bool BIN = false, int PF = 1,
          int DMA = 0, int XP = 0, bool FULL = false>
__global__ __launch_bounds__(256, MINW) void alt_corr_mfma_kernel(const float* __restrict__ f1,
                                                               const float* __restrict__ coords,
                                                               float* __restrict__ out,
                                                               AltGeom g, int W1, int tiles_x,
                                                               const int4* __restrict__ ord,
                                                               long long ord_stride, int XL) {
  constexpr int RD = 2 * R + 1, RD1 = RD + 1, NCELL = RD1 * RD1;
  constexpr int CHUNK = 4 * 32 * NRB;                       // box cells per chunk
  constexpr int KB = CMAX / 8;                              // 8-channel blocks
  constexpr int NPL = H2 ? 2 : 3;                           // query operand planes
  __shared__ __attribute__((aligned(16))) uint4 qplanes[NPL * KB * TQ]; // [plane][kb][q]
  // window dot products, row pitch SP: odd (round 6), so the 32 lanes of a
  // half-wave reading S[q * SP + cell] for 32 queries hit 32 banks (pitch 100:
  // 4 q mod 32, a 4-way conflict on every phase-2 read).  XP bit 4: the old pitch.
  constexpr int SP = (XP & 16) ? NCELL : NCELL + 1;
  __shared__ float S[TQ * SP];
  __shared__ int4 qinfo[TQ];                                // {x0, y0, live, -}
  __shared__ int box[4];                                    // bx0, by0, bw, bh
  __shared__ int qlist[TQ];                                 // BIN: query index or -1
  __shared__ float2 qxy[TQ];                                // BIN: its coordinates
  // DMA 1: per wave two 4 KB buffers of 32 cells x 128 B (two k steps), swizzled 16-B slots;
  // DMA 2: per wave a ring of 4 one-k-step stages of 32 cells x 64 B (round 6)
  __shared__ __attribute__((aligned(16))) unsigned char cbuf[DMA ? 4 * 2 * 4096 : 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // Workgroups are dealt round-robin to the 8 XCDs; XCD k takes the k-th
  // contiguous band of tiles instead, so neighbouring tiles (whose boxes overlap)
  // share one L2 (the bijection of csrc/corr_build.hip's page_coord; r01 1080p:
  // FETCH 424 -> 162 MB per lookup).  XL (levels dividing 8, levels x tiles a
  // multiple of 8): the XCDs are shared out by level too — 8 / levels XCDs per
  // level, each taking a contiguous band of that level's list — so one output
  // line (32 pixels of one channel, written by the workgroups holding those
  // pixels' queries) is written from one or two XCDs' L2s: with queries ordered
  // by window position a line's 32 queries sit in bins of several bands, and
  // partial dirty lines written back from several L2s multiplied the output's
  // write traffic (r03 1080p: WRITE 137 MB per lookup for a 42 MB output).
  // Measured slower (the levels cost different amounts): experiments only.
  int tile = blockIdx.x, lvl = blockIdx.y;
  if (XL) {
    const int T = gridDim.x, L = gridDim.y;
    const int lin = blockIdx.x + T * blockIdx.y, xcd = lin % 8, k = lin / 8;
    const int xpl = 8 / L;
    lvl = xcd / xpl;
    tile = (xcd % xpl) * (T / xpl) + k;
  } else {
    const int n = gridDim.x, q8 = n / 8, r8 = n % 8, xcd = tile % 8;
    tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + tile / 8;
  }
  const int tx = tile % tiles_x, ty = tile / tiles_x;
  const AltLevel lv = g.lv[lvl];
  const int z = blockIdx.z, bf = z / g.Nc;
  const float* cz = coords + (long long)z * g.coord_zstride;
  const float* f1b = f1 + (long long)bf * g.f1_bstride;
  const float* f2b = lv.f2 + (long long)bf * lv.H2 * lv.W2 * g.C;
  const int H1 = g.N / W1;
  const int nkb = g.C / 8;
  // query of lane/slot qq: a pixel of the 4 x 8 tile, or (BIN) entry tile*32 + qq of
  // the sorted list; -1 past the image / the list
  auto query_of = [&](int qq) -> int {
    if constexpr (BIN) {
      return qlist[qq];
    } else {
      const int qy = ty * TQY + qq / TQX, qx = tx * TQX + qq % TQX;
      return (qy < H1 && qx < W1) ? qy * W1 + qx : -1;
    }
  };
  if constexpr (BIN) {
    if (tid < TQ) {
      // per (coordinate set, level) gridDim.x * 32 entries, query -1 = padding
      const int4 e = ord[((long long)z * gridDim.y + lvl) * ord_stride + tile * TQ + tid];
      qlist[tid] = e.x;
      qxy[tid] = make_float2(__int_as_float(e.y), __int_as_float(e.z));
    }
    __syncthreads();
  }

  // ---- query coordinates, window origins, the windows' union box
  if constexpr (FULL) {
    static_assert(!BIN, "the full-level box runs in tile order");
    if (tid < TQ) qinfo[tid] = make_int4(0, 0, 0, 0);
    if (tid == 0) {
      box[0] = 0;
      box[1] = 0;
      box[2] = lv.W2;
      box[3] = lv.H2;
    }
  } else if (tid < TQ) {
    const int qsel = query_of(tid);
    int x0 = 0, y0 = 0, live = 0;
    if (qsel >= 0) {
      const int q = qsel;
      float x, y;
      if constexpr (BIN) {
        x = qxy[tid].x * lv.inv;
        y = qxy[tid].y * lv.inv;
      } else {
        x = cz[(long long)q * g.coord_qstride] * lv.inv;
        y = cz[(long long)q * g.coord_qstride + g.coord_cstride] * lv.inv;
      }
      const float xf = floorf(x), yf = floorf(y);
      if (fabsf(xf) < 1.0e8f && fabsf(yf) < 1.0e8f) {
        x0 = (int)xf - R;
        y0 = (int)yf - R;
        // windows entirely off the level need no dot products
        live = (x0 + RD1 > 0 && x0 < lv.W2 && y0 + RD1 > 0 && y0 < lv.H2) ? 1 : 0;
      }
    }
    qinfo[tid] = make_int4(x0, y0, live, 0);
    int lx0 = live ? max(x0, 0) : 0x7fffffff, ly0 = live ? max(y0, 0) : 0x7fffffff;
    int lx1 = live ? min(x0 + RD1, lv.W2) : -1, ly1 = live ? min(y0 + RD1, lv.H2) : -1;
#pragma unroll
    for (int o = 1; o < TQ; o <<= 1) {
      lx0 = min(lx0, __shfl_xor(lx0, o));
      ly0 = min(ly0, __shfl_xor(ly0, o));
      lx1 = max(lx1, __shfl_xor(lx1, o));
      ly1 = max(ly1, __shfl_xor(ly1, o));
    }
    if (tid == 0) {
      const bool any = lx1 > lx0;
      box[0] = any ? lx0 : 0;
      box[1] = any ? ly0 : 0;
      box[2] = any ? lx1 - lx0 : 0;
      box[3] = any ? ly1 - ly0 : 0;
    }
  }
  if constexpr (!FULL)
    for (int i = tid; i < TQ * SP; i += 256) S[i] = 0.f;
  // query operand planes: unit (kb, q) -> f1[q][8 kb .. 8 kb + 8), split once
  for (int u = tid; u < nkb * TQ; u += 256) {
    const int kb = u / TQ, qq = u - kb * TQ;
    int qsrc0;   // padding slots read a valid query (their outputs are not stored)
    if constexpr (BIN) {
      qsrc0 = max(query_of(qq), 0);
    } else {
      const int qy = min(ty * TQY + qq / TQX, H1 - 1), qx = min(tx * TQX + qq % TQX, W1 - 1);
      qsrc0 = qy * W1 + qx;
    }
    const float* src = f1b + (long long)qsrc0 * g.C + kb * 8;
    const float4 a = *reinterpret_cast<const float4*>(src);
    const float4 c = *reinterpret_cast<const float4*>(src + 4);
    const float x[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
    if constexpr (H2) {
      uint4 h, l;
      alt_split8h(x, h, l);
      qplanes[(0 * KB + kb) * TQ + qq] = h;
      qplanes[(1 * KB + kb) * TQ + qq] = l;
    } else {
      uint4 h, m, l;
      alt_split8(x, h, m, l);
      qplanes[(0 * KB + kb) * TQ + qq] = h;
      qplanes[(1 * KB + kb) * TQ + qq] = m;
      qplanes[(2 * KB + kb) * TQ + qq] = l;
    }
  }
  __syncthreads();

  const int bx0 = box[0], by0 = box[1], bw = box[2], bh = box[3];
  // c / bw for box cells (c < 2^24): a float estimate corrected to the exact quotient
  const float rbw = 1.f / (float)max(bw, 1);
  auto divbw = [&](int c) -> int {
    int q = (int)((float)c * rbw);
    q -= (q * bw > c) ? 1 : 0;
    q += ((q + 1) * bw <= c) ? 1 : 0;
    return q;
  };
  const int ncells = bw * bh;
  const int j = lane & 31, kh = lane >> 5;
  const int4 qi = qinfo[j];                   // this lane's accumulator column (query j)
  for (int c0 = 0; c0 < ncells; c0 += CHUNK) {
    af16 acc[NRB];
    const float* src[NRB];
#pragma unroll
    for (int rb = 0; rb < NRB; ++rb) {
      // A operand lane -> cell c0 + 32 (wave NRB + rb) + j, channels 8 kh .. + 8 per k16
      const int c = min(c0 + (wave * NRB + rb) * 32 + j, ncells - 1);
      const int cy = divbw(c), cx = c - cy * bw;
      src[rb] = f2b + ((long long)(by0 + cy) * lv.W2 + bx0 + cx) * g.C + 8 * kh;
      if constexpr ((XP & 4) != 0) src[rb] = f2b + (long long)(j & 7) * g.C + 8 * kh;   // ablation: 8 hot cells
    }
    // DMA (f16 pair form): the wave's 32 cell vectors move by LDS-DMA, two k steps (128 B per cell)
    // per batch into a double-buffered wave region: an instruction covers 8 cells x 128 B (8 lanes
    // per cell: 8 line segments instead of the 32 cells x 32 B of a register load), and slot
    // s of cell row r holds logical 16-B piece s ^ ((r >> 1) & 7), so the operand reads below
    // (row j, pieces 4 step + 2 kh, + 1) are conflict-free ds_read_b128.  Same operands, same
    // split, same products in the same order: bit-identical to the register form.
    auto kloop_dma = [&]() {
      static_assert(NRB == 1, "the DMA form stages one 32-cell block per wave");
      af16 acc2 = {};
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[0][r] = 0.f;
      const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(f2b), (short)0, lv.H2 * lv.W2 * g.C * 4, 0x00020000);
      uint32_t voff[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 8 * i + (lane >> 3), slot = lane & 7;
        const int c = min(c0 + wave * 32 + row, ncells - 1);
        const int cy = divbw(c), cx = c - cy * bw;
        const int piece = slot ^ ((row >> 1) & 7);
        voff[i] = (uint32_t)(((by0 + cy) * lv.W2 + bx0 + cx) * g.C) * 4u + 16u * piece;
      }
      // readfirstlane: the DMA's LDS destination must be wave-uniform (an SGPR)
      unsigned char* wreg = cbuf + __builtin_amdgcn_readfirstlane(wave) * 8192;
      auto issue = [&](int bt) {
        unsigned char* dst = wreg + (bt & 1) * 4096;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rf, (lds_void_t*)(dst + i * 1024), 16, voff[i],
                                                   bt * 128, 0, 0);
      };
      const int nbt = nkb / 4;                     // batches of two k16 steps
      const int sw = (j >> 1) & 7;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      issue(0);
      for (int bt = 0; bt < nbt; ++bt) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads of the buffer refilled next
        if (bt + 1 < nbt) {
          issue(bt + 1);
          asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const unsigned char* rb0 = wreg + (bt & 1) * 4096 + j * 128;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const int ks = 2 * bt + st;
          const int p0 = 4 * st + 2 * kh;
          const float4 a = *reinterpret_cast<const float4*>(rb0 + 16 * (p0 ^ sw));
          const float4 b = *reinterpret_cast<const float4*>(rb0 + 16 * ((p0 + 1) ^ sw));
          const ah8 qh = __builtin_bit_cast(ah8, qplanes[(0 * KB + 2 * ks + kh) * TQ + j]);
          const ah8 ql = __builtin_bit_cast(ah8, qplanes[(1 * KB + 2 * ks + kh) * TQ + j]);
          const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
          uint4 h, l;
          alt_split8h(x, h, l);
          const ah8 th = __builtin_bit_cast(ah8, h), tl = __builtin_bit_cast(ah8, l);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, qh, acc2, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ql, acc2, 0, 0, 0);
          acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, qh, acc[0], 0, 0, 0);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[0][r] = __builtin_fmaf(acc2[r], 0x1p-11f, acc[0][r]);
    };
    // DMA 2 (round 6, experiments): one k step (32 cells x 64 B) per stage, a ring of
    // NS = 4 stages per wave, so three k steps of cell data are in flight (DMA 1 keeps
    // one two-step batch ahead).  An instruction covers 16 cells x 64 B (4 lanes per
    // cell); physical slot p of cell row r holds logical 16-B piece p ^ ((r >> 2) & 3),
    // so the fragment reads (row j, pieces 2 kh, 2 kh + 1) are conflict-free
    // ds_read_b128.  Same operands, split and products: bit-identical.
    auto kloop_dma2 = [&]() {
      static_assert(NRB == 1, "the DMA form stages one 32-cell block per wave");
      constexpr int NS = 4;
      af16 acc2 = {};
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[0][r] = 0.f;
      const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(f2b), (short)0, lv.H2 * lv.W2 * g.C * 4, 0x00020000);
      uint32_t voff[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = 16 * i + (lane >> 2), slot = lane & 3;
        const int c = min(c0 + wave * 32 + row, ncells - 1);
        const int cy = divbw(c), cx = c - cy * bw;
        const int piece = slot ^ ((row >> 2) & 3);
        voff[i] = (uint32_t)(((by0 + cy) * lv.W2 + bx0 + cx) * g.C) * 4u + 16u * piece;
      }
      unsigned char* wreg = cbuf + __builtin_amdgcn_readfirstlane(wave) * (NS * 2048);
      auto issue = [&](int ks) {
        unsigned char* dst = wreg + (ks % NS) * 2048;
#pragma unroll
        for (int i = 0; i < 2; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rf, (lds_void_t*)(dst + i * 1024), 16, voff[i],
                                                   ks * 64, 0, 0);
      };
      const int nst = nkb / 2;
      const int sw = (j >> 2) & 3;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < NS - 1; ++u)
        if (u < nst) issue(u);
      for (int ks = 0; ks < nst; ++ks) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads of the slot refilled next
        if (ks + NS - 1 < nst) {
          issue(ks + NS - 1);
          asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // stage ks landed (3 stages behind it)
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const unsigned char* rb0 = wreg + (ks % NS) * 2048 + j * 64;
        const float4 a = *reinterpret_cast<const float4*>(rb0 + 16 * ((2 * kh) ^ sw));
        const float4 b = *reinterpret_cast<const float4*>(rb0 + 16 * ((2 * kh + 1) ^ sw));
        const ah8 qh = __builtin_bit_cast(ah8, qplanes[(0 * KB + 2 * ks + kh) * TQ + j]);
        const ah8 ql = __builtin_bit_cast(ah8, qplanes[(1 * KB + 2 * ks + kh) * TQ + j]);
        const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint4 h, l;
        alt_split8h(x, h, l);
        const ah8 th = __builtin_bit_cast(ah8, h), tl = __builtin_bit_cast(ah8, l);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, qh, acc2, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ql, acc2, 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, qh, acc[0], 0, 0, 0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[0][r] = __builtin_fmaf(acc2[r], 0x1p-11f, acc[0][r]);
    };
    // cell vectors one k step ahead in registers
    auto kloop = [&](auto h2tag) {
      constexpr bool M2 = decltype(h2tag)::value;
      af16 acc2[NRB];
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[rb][r] = acc2[rb][r] = 0.f;
      const int nst = nkb / 2;
      float4 ra[PF][NRB], rv[PF][NRB];   // ring of in-flight k steps
#pragma unroll
      for (int u = 0; u < PF; ++u)
        if (u < nst) {
#pragma unroll
          for (int rb = 0; rb < NRB; ++rb) {
            ra[u][rb] = *reinterpret_cast<const float4*>(src[rb] + u * 16);
            rv[u][rb] = *reinterpret_cast<const float4*>(src[rb] + u * 16 + 4);
          }
        }
      // fallback form: this lane's query operand straight from fmap1
      int fq;
      if constexpr (BIN) {
        fq = max(query_of(j), 0);
      } else {
        const int fqy = min(ty * TQY + j / TQX, H1 - 1), fqx = min(tx * TQX + j % TQX, W1 - 1);
        fq = fqy * W1 + fqx;
      }
      const float* qsrc = f1b + (long long)fq * g.C + 8 * kh;
      for (int ks0 = 0; ks0 < nst; ks0 += PF)
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int ks = ks0 + u;
        if (ks >= nst) break;
        float4 ca[NRB], cb[NRB];
#pragma unroll
        for (int rb = 0; rb < NRB; ++rb) {
          ca[rb] = ra[u][rb];
          cb[rb] = rv[u][rb];
        }
        if (ks + PF < nst) {
#pragma unroll
          for (int rb = 0; rb < NRB; ++rb) {
            ra[u][rb] = *reinterpret_cast<const float4*>(src[rb] + (ks + PF) * 16);
            rv[u][rb] = *reinterpret_cast<const float4*>(src[rb] + (ks + PF) * 16 + 4);
          }
        }
        if constexpr (M2) {
          const ah8 qh = __builtin_bit_cast(ah8, qplanes[(0 * KB + 2 * ks + kh) * TQ + j]);
          const ah8 ql = __builtin_bit_cast(ah8, qplanes[(1 * KB + 2 * ks + kh) * TQ + j]);
#pragma unroll
          for (int rb = 0; rb < NRB; ++rb) {
            const float4 a = ca[rb], b = cb[rb];
            uint4 h, l;
            if constexpr ((XP & 1) != 0) {
              h = __builtin_bit_cast(uint4, a);
              l = __builtin_bit_cast(uint4, b);
            } else {
              const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
              alt_split8h(x, h, l);
            }
            const ah8 th = __builtin_bit_cast(ah8, h), tl = __builtin_bit_cast(ah8, l);
            if constexpr ((XP & 8) != 0) {   // ablation: no MFMAs (results meaningless)
              acc[rb][0] += __uint_as_float(h.x ^ l.y) + (float)qh[0] + (float)ql[1];
            } else {
            acc2[rb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, qh, acc2[rb], 0, 0, 0);
            acc2[rb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ql, acc2[rb], 0, 0, 0);
            acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, qh, acc[rb], 0, 0, 0);
            }
          }
        } else {
          abf8 qh, qm, ql;
          if constexpr (H2) {     // fallback: split the query operand here
            const float4 u = *reinterpret_cast<const float4*>(qsrc + ks * 16);
            const float4 w = *reinterpret_cast<const float4*>(qsrc + ks * 16 + 4);
            const float x[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
            uint4 h, m, l;
            alt_split8(x, h, m, l);
            qh = __builtin_bit_cast(abf8, h);
            qm = __builtin_bit_cast(abf8, m);
            ql = __builtin_bit_cast(abf8, l);
          } else {
            qh = __builtin_bit_cast(abf8, qplanes[(0 * KB + 2 * ks + kh) * TQ + j]);
            qm = __builtin_bit_cast(abf8, qplanes[(1 * KB + 2 * ks + kh) * TQ + j]);
            ql = __builtin_bit_cast(abf8, qplanes[(2 * KB + 2 * ks + kh) * TQ + j]);
          }
#pragma unroll
          for (int rb = 0; rb < NRB; ++rb) {
            const float4 a = ca[rb], b = cb[rb];
            const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            uint4 h, m, l;
            alt_split8(x, h, m, l);
            const abf8 th = __builtin_bit_cast(abf8, h), tm = __builtin_bit_cast(abf8, m),
                       tl = __builtin_bit_cast(abf8, l);
            // small terms first
            acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tm, qm, acc[rb], 0, 0, 0);
            acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tl, qh, acc[rb], 0, 0, 0);
            acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, ql, acc[rb], 0, 0, 0);
            acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tm, qh, acc[rb], 0, 0, 0);
            acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, qm, acc[rb], 0, 0, 0);
            acc[rb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, qh, acc[rb], 0, 0, 0);
          }
        }
      }
      if constexpr (M2) {
#pragma unroll
        for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[rb][r] = __builtin_fmaf(acc2[rb][r], 0x1p-11f, acc[rb][r]);
      }
    };
    if constexpr (H2) {
      if constexpr (DMA == 2 && NRB == 1) {
        if (nkb % 2 == 0) kloop_dma2();
        else kloop(std::integral_constant<bool, true>{});
      } else if constexpr (DMA == 1 && NRB == 1) {
        if (nkb % 4 == 0) kloop_dma();
        else kloop(std::integral_constant<bool, true>{});
      } else {
        kloop(std::integral_constant<bool, true>{});
      }
      bool bad = false;
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int r = 0; r < 16; ++r) bad |= !(__builtin_fabsf(acc[rb][r]) <= 3.40282347e38f);
      if ((XP & 13) == 0 && __ballot(bad) != 0)
        kloop(std::integral_constant<bool, false>{});   // wave-uniform
    } else {
      kloop(std::integral_constant<bool, false>{});
    }
    if constexpr (FULL) {
      // every sum of query j to its row of the volume: D rows (r & 3) + 8 (r >> 2)
      // + 4 kh, i.e. four runs of four consecutive cells per lane
      const int qv = query_of(j);
      if (qv >= 0) {
#pragma unroll
        for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int c = c0 + (wave * NRB + rb) * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
            if (c < ncells) {
              const int cy = divbw(c), cx = c - cy * bw;
              out[dxr::cell_index(g.vlay, bf, qv, cy, cx)] = acc[rb][r];
            }
          }
      }
      continue;
    }
    // keep the entries inside query j's window: D row = (r & 3) + 8 (r >> 2) + 4 kh
    if (qi.z) {
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = c0 + (wave * NRB + rb) * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
          if (c < ncells) {
            const int cy = divbw(c), cx = c - cy * bw;
            const int iy = by0 + cy - qi.y, ix = bx0 + cx - qi.x;
            if ((unsigned)iy < (unsigned)RD1 && (unsigned)ix < (unsigned)RD1)
              S[j * SP + iy * RD1 + ix] = acc[rb][r];
          }
        }
    }
  }
  if constexpr (FULL) return;
  __syncthreads();

  // ---- bilinear combination, as the per-query form (reference order)
  const int qq = tid & (TQ - 1), cls = tid / TQ;
  const int q = query_of(qq);
  if (q < 0) return;
  float x, y;
  if constexpr (BIN) {
    x = qxy[qq].x * lv.inv;
    y = qxy[qq].y * lv.inv;
  } else {
    x = cz[(long long)q * g.coord_qstride] * lv.inv;
    y = cz[(long long)q * g.coord_qstride + g.coord_cstride] * lv.inv;
  }
  const float dx = x - floorf(x), dy = y - floorf(y);
  const float* s = S + qq * SP;
  float* o = out + (long long)z * g.cout * g.N + (long long)lv.ch_off * g.N + q;
  for (int ox = cls; ox < RD; ox += 256 / TQ) {
#pragma unroll
    for (int oy = 0; oy < RD; ++oy) {
      const float s00 = s[oy * RD1 + ox], s01 = s[oy * RD1 + ox + 1];
      const float s10 = s[(oy + 1) * RD1 + ox], s11 = s[(oy + 1) * RD1 + ox + 1];
      float v = __fmul_rn(__fmul_rn(s00, 1.f - dy), 1.f - dx);
      v = __fadd_rn(v, __fmul_rn(__fmul_rn(s01, 1.f - dy), dx));
      v = __fadd_rn(v, __fmul_rn(__fmul_rn(s10, dy), 1.f - dx));
      v = __fadd_rn(v, __fmul_rn(__fmul_rn(s11, dy), dx));
      // v / divisor; a power-of-two divisor (sqrt(256) = 16) scales exactly by its reciprocal
      const float res = g.div_recip != 0.f ? v * g.div_recip : v / g.divisor;
      if ((XP & 2) == 0 || res == 12345.0f) o[(long long)(oy + RD * ox) * g.N] = res;
    }
  }
}

// ---------------------------------------------------------------------------
// Query order of the on-the-fly lookup (round 3).  The union box of a 4 x 8
// query tile is compact for smooth flow fields but ~10x its windows' cells at
// level 0 for flows that vary pixel to pixel (the bench's i.i.d. N(0, 4^2)
// model): neighbouring queries' windows are unrelated.  Grouping the queries by
// window position instead keeps every box near one window whatever the flow.
// Three launches over OB blocks of whole tiles per (coordinate set, level):
//   K1 alt_bin_count_kernel   thread = query (tile-major): bin by window origin
//      (bins of ~32 queries: 2^by x 2^bx origin cells, snake order over bin
//      rows; non-finite coordinates in a last bin), bin ids to the workspace,
//      the block's histogram (LDS) to cnt[block][bin], and the block's tiles'
//      union box areas (the cells the tile order would multiply) to cost[block];
//   K2 alt_bin_scan_kernel    thread = bin: its exclusive prefix over the
//      blocks (in place) and its total;
//   K3 alt_bin_scatter_kernel chooses the bin order when the tiles' boxes
//      average more than 1.5x a bin group's estimated box ((2^by + 2r + 1) x
//      (2^bx + 2r + 1)), else the tile order (then the lookup multiplies exactly
//      the spatial form's boxes); in bin order each block scans the bins' totals
//      itself and writes its queries' entries {query, x, y, 0} at bin base +
//      block prefix + an LDS rank, in tile order at their tile slots.
// Queries of a bin land in any order: the box GEMM's per-(cell, query) sums do
// not depend on which queries share a workgroup, so the lookup's outputs are
// bit-identical to the tile order's.  (A one-workgroup-per-list form ran the
// whole job on 4 CUs: 76 us per 1080p lookup.)
// ---------------------------------------------------------------------------
constexpr int BIN_MAX = 4096;
constexpr int OB = 64;            // blocks per list

struct BinGeom {
  int bsx[8], bsy[8], nbx[8], nby[8];
};

BinGeom make_bins(int N, const AltGeom& g, int levels) {
  BinGeom b{};
  for (int l = 0; l < levels; ++l) {
    const int h2 = g.lv[l].H2, w2 = g.lv[l].W2;
    const double dens = (double)N / ((double)h2 * w2);
    int lg = 0;
    while ((1 << lg) * dens < 32.0 && lg < 12) ++lg;   // bin area 2^lg ~ 32 queries
    int by = lg / 2, bx = lg - by;
    while (((w2 + (1 << bx) - 1) >> bx) * ((h2 + (1 << by) - 1) >> by) > BIN_MAX) {
      if (bx <= by) ++bx; else ++by;
    }
    b.bsx[l] = bx;
    b.bsy[l] = by;
    b.nbx[l] = (w2 + (1 << bx) - 1) >> bx;
    b.nby[l] = (h2 + (1 << by) - 1) >> by;
  }
  return b;
}

// Workspace of one list (coordinate set, level): entries int4[NP] | bin ids
// int[NP] | cnt int[OB][BIN_MAX + 1] | tot int[BIN_MAX + 1] | cost float[OB]
// (16-B aligned).
struct OrderWs {
  long long np, ents, ids, cnt, tot, cost, bytes;   // byte offsets within a list
};
__host__ __device__ inline OrderWs order_ws(long long np) {
  OrderWs w;
  w.np = np;
  w.ents = 0;
  w.ids = w.ents + 16 * np;
  w.cnt = w.ids + 4 * np;
  w.tot = w.cnt + 4LL * OB * (BIN_MAX + 1);
  w.cost = w.tot + 4LL * (BIN_MAX + 1);
  w.bytes = (w.cost + 4LL * OB + 15) & ~15LL;
  return w;
}

struct OrderArgs {
  unsigned char* ws;   // lists [Z][L] of OrderWs.bytes each
  long long list_bytes, np;
  int W1, tiles_x, ntiles, tpb;   // tiles per block
};

// slot i of a block -> (tile, slot within the 4 x 8 tile) -> query (or -1)
__device__ __forceinline__ int order_query(int blk, int i, const OrderArgs& o, int H1, int& tile,
                                           int& slot) {
  tile = blk * o.tpb + i / TQ;
  slot = i % TQ;
  const int qy = (tile / o.tiles_x) * TQY + slot / TQX, qx = (tile % o.tiles_x) * TQX + slot % TQX;
  return (tile < o.ntiles && qy < H1 && qx < o.W1) ? qy * o.W1 + qx : -1;
}

template <int R>
__global__ __launch_bounds__(256) void alt_bin_count_kernel(const float* __restrict__ coords,
                                                            AltGeom g, BinGeom bg, OrderArgs o) {
  constexpr int RD1 = 2 * R + 2;
  __shared__ int hist[BIN_MAX + 1];
  __shared__ float wcost[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = blockIdx.x, l = blockIdx.y, z = blockIdx.z;
  const AltLevel lv = g.lv[l];
  const int nbx = bg.nbx[l], nb = nbx * bg.nby[l], bsx = bg.bsx[l], bsy = bg.bsy[l];
  const float* cz = coords + (long long)z * g.coord_zstride;
  const int H1 = g.N / o.W1;
  unsigned char* lw = o.ws + ((long long)z * gridDim.y + l) * o.list_bytes;
  const OrderWs w = order_ws(o.np);
  int* ids = reinterpret_cast<int*>(lw + w.ids);
  for (int i = tid; i <= nb; i += 256) hist[i] = 0;
  __syncthreads();
  float cost = 0.f;
  // 32 consecutive lanes = one tile: its union box by a 32-lane reduction
  for (int i = tid; i < o.tpb * TQ; i += 256) {
    int tile, slot;
    const int q = order_query(blk, i, o, H1, tile, slot);
    const int qc = max(q, 0);
    const float x = cz[(long long)qc * g.coord_qstride] * lv.inv;
    const float y = cz[(long long)qc * g.coord_qstride + g.coord_cstride] * lv.inv;
    const float xf = floorf(x), yf = floorf(y);
    int bin = nb;
    int lx0 = 0x7fffffff, ly0 = 0x7fffffff, lx1 = -1, ly1 = -1;
    if (q >= 0 && fabsf(xf) < 1.0e8f && fabsf(yf) < 1.0e8f) {
      const int cx = min(max((int)xf, 0), lv.W2 - 1), cy = min(max((int)yf, 0), lv.H2 - 1);
      const int byi = cy >> bsy;
      int bxi = cx >> bsx;
      if (byi & 1) bxi = nbx - 1 - bxi;
      bin = byi * nbx + bxi;
      const int x0 = (int)xf - R, y0 = (int)yf - R;
      if (x0 + RD1 > 0 && x0 < lv.W2 && y0 + RD1 > 0 && y0 < lv.H2) {   // live window
        lx0 = max(x0, 0);
        ly0 = max(y0, 0);
        lx1 = min(x0 + RD1, lv.W2);
        ly1 = min(y0 + RD1, lv.H2);
      }
    }
    if (q >= 0) {
      atomicAdd(&hist[bin], 1);
      ids[(long long)blk * o.tpb * TQ + i] = bin;
    }
#pragma unroll
    for (int d = 1; d < TQ; d <<= 1) {
      lx0 = min(lx0, __shfl_xor(lx0, d));
      ly0 = min(ly0, __shfl_xor(ly0, d));
      lx1 = max(lx1, __shfl_xor(lx1, d));
      ly1 = max(ly1, __shfl_xor(ly1, d));
    }
    if ((lane & 31) == 0 && lx1 > lx0) cost += (float)(lx1 - lx0) * (float)(ly1 - ly0);
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) cost += __shfl_xor(cost, d);
  if (lane == 0) wcost[wave] = cost;
  __syncthreads();
  int* cnt = reinterpret_cast<int*>(lw + w.cnt) + (long long)blk * (BIN_MAX + 1);
  for (int i = tid; i <= nb; i += 256) cnt[i] = hist[i];
  if (tid == 0)
    reinterpret_cast<float*>(lw + w.cost)[blk] = wcost[0] + wcost[1] + wcost[2] + wcost[3];
}

// K2: thread = bin: exclusive prefix of its count over the OB blocks, in place
// (64 loads in flight), and the bin's total.  Grid (ceil(bins / 256), L, Z).
__global__ __launch_bounds__(256) void alt_bin_scan_kernel(BinGeom bg, OrderArgs o) {
  const int l = blockIdx.y, z = blockIdx.z;
  const int bin = blockIdx.x * 256 + threadIdx.x;
  const int nb = bg.nbx[l] * bg.nby[l];
  if (bin > nb) return;
  unsigned char* lw = o.ws + ((long long)z * gridDim.y + l) * o.list_bytes;
  const OrderWs w = order_ws(o.np);
  int* cnt = reinterpret_cast<int*>(lw + w.cnt) + bin;
  int c[OB];
#pragma unroll
  for (int b = 0; b < OB; ++b) c[b] = cnt[(long long)b * (BIN_MAX + 1)];
  int run = 0;
#pragma unroll
  for (int b = 0; b < OB; ++b) {
    const int t = c[b];
    cnt[(long long)b * (BIN_MAX + 1)] = run;
    run += t;
  }
  reinterpret_cast<int*>(lw + w.tot)[bin] = run;
}

// K3: every block scans the bins' totals itself (<= 4097 values from L2) into
// LDS bases, decides the order from the blocks' box costs (the same decision in
// every block), then writes its queries' entries: at base[bin] + its block
// prefix + an LDS rank (bin order), or at their tile slots (tile order).
template <int R>
__global__ __launch_bounds__(256) void alt_bin_scatter_kernel(const float* __restrict__ coords,
                                                              AltGeom g, BinGeom bg, OrderArgs o) {
  constexpr int RD1 = 2 * R + 2;
  __shared__ int off[BIN_MAX + 1];
  __shared__ int wsum[4];
  __shared__ int binned_s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = blockIdx.x, l = blockIdx.y, z = blockIdx.z;
  const int nb = bg.nbx[l] * bg.nby[l];
  const float* cz = coords + (long long)z * g.coord_zstride;
  const int H1 = g.N / o.W1;
  unsigned char* lw = o.ws + ((long long)z * gridDim.y + l) * o.list_bytes;
  const OrderWs w = order_ws(o.np);
  int4* ents = reinterpret_cast<int4*>(lw + w.ents);
  const int* ids = reinterpret_cast<const int*>(lw + w.ids);
  if (tid == 0) {
    float c = 0.f;
    const float* cost = reinterpret_cast<const float*>(lw + w.cost);
    for (int b = 0; b < OB; ++b) c += cost[b];
    const float chunk = (float)((1 << bg.bsy[l]) + RD1 - 1) * (float)((1 << bg.bsx[l]) + RD1 - 1);
    binned_s = c > 1.5f * chunk * (float)o.ntiles ? 1 : 0;
  }
  __syncthreads();
  const bool binned = binned_s != 0;
  if (binned) {
    // exclusive scan of the totals: thread t owns bins [t * per, t * per + per)
    const int* tot = reinterpret_cast<const int*>(lw + w.tot);
    const int per = (nb + 1 + 255) / 256;    // <= 17
    int loc = 0;
    for (int k = 0; k < per; ++k) {
      const int b = tid * per + k;
      if (b <= nb) loc += tot[b];
    }
    int v = loc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(v, d);
      if (lane >= d) v += t;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    int base = v - loc;
    for (int i = 0; i < wave; ++i) base += wsum[i];
    const int* cnt = reinterpret_cast<const int*>(lw + w.cnt) + (long long)blk * (BIN_MAX + 1);
    for (int k = 0; k < per; ++k) {
      const int b = tid * per + k;
      if (b <= nb) {
        off[b] = base + cnt[b];
        base += tot[b];
      }
    }
    __syncthreads();
  }
  for (int i = tid; i < o.tpb * TQ; i += 256) {
    int tile, slot;
    const int q = order_query(blk, i, o, H1, tile, slot);
    if (tile >= o.ntiles) break;
    int4 e = make_int4(-1, 0, 0, 0);
    if (q >= 0)
      e = make_int4(q, __float_as_int(cz[(long long)q * g.coord_qstride]),
                    __float_as_int(cz[(long long)q * g.coord_qstride + g.coord_cstride]), 0);
    if (!binned)
      ents[(long long)tile * TQ + slot] = e;
    else if (q >= 0)
      ents[atomicAdd(&off[ids[(long long)blk * o.tpb * TQ + i]], 1)] = e;
  }
  if (binned && blk == 0)   // entries past the queries: padding
    for (long long i = g.N + tid; i < o.np; i += 256) ents[i] = make_int4(-1, 0, 0, 0);
}

long long alt_order_entries(long long H, long long W) {
  return ((W + TQX - 1) / TQX) * ((H + TQY - 1) / TQY) * (long long)TQ;
}

long long alt_order_bytes(long long H, long long W) {
  return order_ws(alt_order_entries(H, W)).bytes;
}

// PF: cell loads of the ordered form kept 4 k steps ahead (round 3: with compact boxes the
// waves wait on L2 latency, 62 % of wave cycles at PF = 1; 1080p 12 lookups 2,033 -> 1,972 us,
// Sintel 626 -> 612 us in the step).  The tile-order form stays at 1 (its boxes are L1/TA-bound).
// Occupancy bound of the f16-pair form: 3 workgroups per CU (the 1080p r02
// A/B); from r = 6 the window buffers and index registers do not fit that bound
// (hipcc: "desired occupancy 3, final 2"), so those radii ask for 2.
constexpr int alt_minw(int r) { return r >= 6 ? 2 : 3; }

template <int R, int NRB, int DMA = 0, int PF = 4, int XP = 0>
int launch_alt_mfma_r(const float* f1, const float* coords, float* out, const AltGeom& g,
                      int levels, int Z, int W1, hipStream_t stream, void* ws = nullptr,
                      int xl = -1) {
  const int H1 = g.N / W1;
  const int tiles_x = (W1 + TQX - 1) / TQX, tiles_y = (H1 + TQY - 1) / TQY;
  const int ntiles = tiles_x * tiles_y;
  // XCDs shared out by level (alt_corr_mfma_kernel XL) where the split is exact:
  // experiments only — round 4, 1080p i.i.d. flows, 12 ordered lookups in the
  // step: 2,567 us with it against 1,990 us without (the levels' lists cost
  // different amounts, so the XCDs of the cheap levels idle)
  const int xl_ok = (8 % levels == 0 && ((long long)levels * ntiles) % 8 == 0) ? 1 : 0;
  const int XL = xl < 0 ? 0 : (xl & xl_ok);
  const dim3 grid((unsigned)ntiles, (unsigned)levels, (unsigned)Z);
  if (g.C > 256) return DXR_EUNSUPPORTED;
  // f16 pair split (r02, 1080p: 227 vs 275 us for the 3-way bf16 split), 3 workgroups/CU
  if (ws != nullptr && Z <= 65535) {
    OrderArgs o;
    o.ws = static_cast<unsigned char*>(ws);
    o.np = (long long)ntiles * TQ;
    o.list_bytes = order_ws(o.np).bytes;
    o.W1 = W1;
    o.tiles_x = tiles_x;
    o.ntiles = ntiles;
    o.tpb = (ntiles + OB - 1) / OB;
    const BinGeom bg = make_bins(g.N, g, levels);
    const dim3 bgrid(OB, (unsigned)levels, (unsigned)Z);
    hipLaunchKernelGGL((alt_bin_count_kernel<R>), bgrid, dim3(256), 0, stream, coords, g, bg, o);
    int st = dxr::launch_status();
    if (st != DXR_OK) return st;
    int nbmax = 0;
    for (int l = 0; l < levels; ++l) nbmax = std::max(nbmax, bg.nbx[l] * bg.nby[l]);
    hipLaunchKernelGGL(alt_bin_scan_kernel, dim3((unsigned)((nbmax + 1 + 255) / 256),
                       (unsigned)levels, (unsigned)Z), dim3(256), 0, stream, bg, o);
    st = dxr::launch_status();
    if (st != DXR_OK) return st;
    hipLaunchKernelGGL((alt_bin_scatter_kernel<R>), bgrid, dim3(256), 0, stream, coords, g, bg, o);
    st = dxr::launch_status();
    if (st != DXR_OK) return st;
    // entries of list (z, l) start at list (z * levels + l) * list_bytes: the kernel
    // indexes int4 entries by ((z * levels + l) * np + i), so lists are laid out
    // with a stride of list_bytes / 16 entries
    if constexpr (DMA != 0)
      hipLaunchKernelGGL((alt_corr_mfma_kernel<R, NRB, 256, true, 2, true, 1, DMA>), grid,
                         dim3(256), 0, stream, f1, coords, out, g, W1, tiles_x,
                         reinterpret_cast<const int4*>(ws), o.list_bytes / 16, XL);
    else
      hipLaunchKernelGGL((alt_corr_mfma_kernel<R, NRB, 256, true, alt_minw(R), true, PF, 0, XP>), grid, dim3(256),
                         0, stream, f1, coords, out, g, W1, tiles_x,
                         reinterpret_cast<const int4*>(ws), o.list_bytes / 16, XL);
    return dxr::launch_status();
  }
  hipLaunchKernelGGL((alt_corr_mfma_kernel<R, NRB, 256, true, alt_minw(R)>), grid, dim3(256), 0, stream, f1,
                     coords, out, g, W1, tiles_x, nullptr, 0, 0);
  return dxr::launch_status();
}

template <int R>
int launch_alt_r(const float* f1, const float* coords, float* out, const AltGeom& g, int levels,
                 int Z, bool vec, hipStream_t stream) {
  const dim3 grid((unsigned)((g.N + 63) / 64), (unsigned)levels, (unsigned)Z);
  if (vec)
    hipLaunchKernelGGL((alt_corr_kernel<R, true>), grid, dim3(256), 0, stream, f1, coords, out, g);
  else
    hipLaunchKernelGGL((alt_corr_kernel<R, false>), grid, dim3(256), 0, stream, f1, coords, out, g);
  return dxr::launch_status();
}

int launch_alt(const float* f1, const float* coords, float* out, const AltGeom& g, int levels,
               int Z, int radius, bool vec, hipStream_t stream, int W1 = 0,
               void* ord = nullptr) {
  // MFMA form: C a multiple of 16 (k16 steps) up to 256, 16-byte aligned rows;
  // the per-query VALU form otherwise.  With a workspace (`ord`) the queries are
  // ordered first (alt_bin_*_kernel).
  if (vec && W1 > 0 && g.C % 16 == 0 && g.C <= 256) {
    switch (radius) {
      case 0: return launch_alt_mfma_r<0, 1>(f1, coords, out, g, levels, Z, W1, stream, ord);
      case 1: return launch_alt_mfma_r<1, 1>(f1, coords, out, g, levels, Z, W1, stream, ord);
      case 2: return launch_alt_mfma_r<2, 1>(f1, coords, out, g, levels, Z, W1, stream, ord);
      case 3: return launch_alt_mfma_r<3, 1>(f1, coords, out, g, levels, Z, W1, stream, ord);
      case 4: return launch_alt_mfma_r<4, 1>(f1, coords, out, g, levels, Z, W1, stream, ord);
      case 5: return launch_alt_mfma_r<5, 1>(f1, coords, out, g, levels, Z, W1, stream, ord);
      case 6: return launch_alt_mfma_r<6, 1>(f1, coords, out, g, levels, Z, W1, stream, ord);
      default: return DXR_EUNSUPPORTED;
    }
  }
  switch (radius) {
    case 0: return launch_alt_r<0>(f1, coords, out, g, levels, Z, vec, stream);
    case 1: return launch_alt_r<1>(f1, coords, out, g, levels, Z, vec, stream);
    case 2: return launch_alt_r<2>(f1, coords, out, g, levels, Z, vec, stream);
    case 3: return launch_alt_r<3>(f1, coords, out, g, levels, Z, vec, stream);
    case 4: return launch_alt_r<4>(f1, coords, out, g, levels, Z, vec, stream);
    case 5: return launch_alt_r<5>(f1, coords, out, g, levels, Z, vec, stream);
    case 6: return launch_alt_r<6>(f1, coords, out, g, levels, Z, vec, stream);
    default: return DXR_EUNSUPPORTED;
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p % 16) == 0; }

// 1 / d when d is a (normal) power of two — then x * (1 / d) == x / d exactly — else 0.
float pow2_recip(float d) {
  int e;
  const float m = std::frexp(d, &e);
  return (m == 0.5f && e > -125 && e < 126) ? 1.f / d : 0.f;
}

// ---------------------------------------------------------------------------
// alt_cuda_corr.backward, reference-FFI form (correlation_kernel.cu:122-256,
// launched by :288-320).  For query q of pair b and coordinate set n, cell
// (iy, ix) in [0, 2r+1]^2 — (h2, w2) = (floor(y) - r + iy, floor(x) - r + ix) —
// receives the transpose of the forward's bilinear scatter (:197-216):
//   g = [iy>0, ix>0]  G(iy-1, ix-1) dy dx   + [iy>0, ix<rd]  G(iy-1, ix) dy (1-dx)
//     + [iy<rd, ix>0] G(iy, ix-1) (1-dy) dx + [iy<rd, ix<rd] G(iy, ix) (1-dy)(1-dx)
// with G(oy, ox) = corr_grad[b][n][oy + rd*ox][q]; every in-bounds cell then adds
// g * fmap2[cell] to fmap1_grad[q] and g * fmap1[q] to fmap2_grad[cell]
// (:218-233; atomics there too).  coords_grad is zero (:307).
//
// MI355X mapping: one wave per query pixel.  Lane L owns channels c0 + L + 64j
// (j < 4) of a 256-channel slab, so each fmap2[cell] read is four 256-byte
// coalesced dword loads and each fmap2_grad update four 256-byte hardware
// global_atomic_add_f32 (full rate on contiguous lines).  The (2r+1)^2 weights of
// the query are loaded once across the lanes and broadcast per cell with
// v_readlane (the cell loops are unrolled, so the lane index is a constant).
// fmap1_grad[q] is owned by the wave: written once per slab, no atomics.
template <int R>
__global__ __launch_bounds__(256) void alt_corr_backward_kernel(
    const float* __restrict__ f1, const float* __restrict__ f2, const float* __restrict__ coords,
    const float* __restrict__ cgrad, float* __restrict__ f1g, float* __restrict__ f2g, int N,
    int H2, int W2, int C, int Nc) {
  constexpr int RD = 2 * R + 1, RR = RD * RD, NG = (RR + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  const int b = blockIdx.y;
  if (q >= N) return;  // whole wave; the kernel has no block barrier
  const float* f1q = f1 + ((long long)b * N + q) * C;
  float* f1gq = f1g + ((long long)b * N + q) * C;
  const float* f2b = f2 + (long long)b * H2 * W2 * C;
  float* f2gb = f2g + (long long)b * H2 * W2 * C;
  for (int c0 = 0; c0 < C; c0 += 256) {
    float a[4], acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + lane + 64 * j;
      a[j] = c < C ? f1q[c] : 0.f;
      acc[j] = 0.f;
    }
    for (int n = 0; n < Nc; ++n) {
      const long long z = (long long)b * Nc + n;
      const float x = coords[(z * N + q) * 2], y = coords[(z * N + q) * 2 + 1];
      const float fx = floorf(x), fy = floorf(y);
      const float dx = x - fx, dy = y - fy;
      const int x0 = (int)fx - R, y0 = (int)fy - R;
      int gv[NG];
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        const int i = lane + 64 * k;
        gv[k] = i < RR ? __float_as_int(cgrad[(z * RR + i) * N + q]) : 0;
      }
      auto G = [&](int oy, int ox) {
        const int i = oy + RD * ox;
        return __int_as_float(__builtin_amdgcn_readlane(gv[i / 64], i % 64));
      };
#pragma unroll
      for (int iy = 0; iy <= RD; ++iy) {
        const int h2 = y0 + iy;
        if (h2 < 0 || h2 >= H2) continue;
#pragma unroll
        for (int ix = 0; ix <= RD; ++ix) {
          const int w2 = x0 + ix;
          if (w2 < 0 || w2 >= W2) continue;
          float g = 0.f;
          if (iy > 0 && ix > 0) g += G(iy - 1, ix - 1) * dy * dx;
          if (iy > 0 && ix < RD) g += G(iy - 1, ix) * dy * (1.f - dx);
          if (iy < RD && ix > 0) g += G(iy, ix - 1) * (1.f - dy) * dx;
          if (iy < RD && ix < RD) g += G(iy, ix) * (1.f - dy) * (1.f - dx);
          const long long cell = ((long long)h2 * W2 + w2) * C;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int c = c0 + lane + 64 * j;
            if (c < C) {
              acc[j] += g * f2b[cell + c];
              unsafeAtomicAdd(f2gb + cell + c, g * a[j]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + lane + 64 * j;
      if (c < C) f1gq[c] = acc[j];
    }
  }
}

struct AltBwd {
  const float *f1, *f2, *coords, *cgrad;
  float *f1g, *f2g;
  int B, N, H2, W2, C, Nc;
};

template <int R>
int launch_alt_backward_r(const AltBwd& a, hipStream_t stream) {
  const dim3 grid((unsigned)((a.N + 3) / 4), (unsigned)a.B);
  hipLaunchKernelGGL((alt_corr_backward_kernel<R>), grid, dim3(256), 0, stream, a.f1, a.f2,
                     a.coords, a.cgrad, a.f1g, a.f2g, a.N, a.H2, a.W2, a.C, a.Nc);
  return dxr::launch_status();
}

// ---------------------------------------------------------------------------
// Layout kernels for channels-last (NHWC) fmaps.
//
// Batched transpose [B, rows, cols] -> [B, cols, rows] (NCHW -> NHWC is rows = C,
// cols = H*W; NHWC -> NCHW the reverse).  One workgroup moves a 64x64 tile
// through LDS (row pitch 65 elements: the column reads are conflict-free); a
// wave reads one 64-element row segment and writes one 64-element column
// segment, so both HBM streams are contiguous.  Pure data movement: bit-exact.
template <typename T>
__global__ __launch_bounds__(256) void transpose_tile_kernel(const T* __restrict__ in,
                                                             T* __restrict__ out, int rows,
                                                             int cols) {
  __shared__ T tile[64][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  const long long base = (long long)blockIdx.z * rows * cols;
  const T* src = in + base;
  T* dst = out + base;
  const int c = c0 + tx;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = r0 + ty + 4 * i;
    if (r < rows && c < cols) tile[ty + 4 * i][tx] = src[(long long)r * cols + c];
  }
  __syncthreads();
  const int r = r0 + tx;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int cc = c0 + ty + 4 * i;
    if (cc < cols && r < rows) dst[(long long)cc * rows + r] = tile[tx][ty + 4 * i];
  }
}

// float32 form for rows % 4 == 0 and cols % 4 == 0 (fmaps: C and H*W): 16-byte
// loads along cols and 16-byte stores along rows, 16 lanes per 256-byte row
// segment.  The scalar kernel moved 1080p fmaps at 3.8 TB/s.
__global__ __launch_bounds__(256) void transpose_tile_v4_kernel(const float* __restrict__ in,
                                                                float* __restrict__ out, int rows,
                                                                int cols) {
  __shared__ float tile[64][65];
  const int tq = threadIdx.x & 15, tr = threadIdx.x >> 4;   // float4 slot, row in pass
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  const long long base = (long long)blockIdx.z * rows * cols;
  const float* src = in + base;
  float* dst = out + base;
  const int c = c0 + 4 * tq;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int lr = tr + 16 * i, r = r0 + lr;
    if (r < rows && c < cols) {
      const float4 v = *reinterpret_cast<const float4*>(src + (long long)r * cols + c);
      tile[lr][4 * tq] = v.x;
      tile[lr][4 * tq + 1] = v.y;
      tile[lr][4 * tq + 2] = v.z;
      tile[lr][4 * tq + 3] = v.w;
    }
  }
  __syncthreads();
  const int r = r0 + 4 * tq;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int lc = tr + 16 * i, cc = c0 + lc;
    if (cc < cols && r < rows) {
      const float4 v = make_float4(tile[4 * tq][lc], tile[4 * tq + 1][lc], tile[4 * tq + 2][lc],
                                   tile[4 * tq + 3][lc]);
      *reinterpret_cast<float4*>(dst + (long long)cc * rows + r) = v;
    }
  }
}

// 2x2 / stride-2 floor-mode average pool of [B, H, W, C] into [B, H/2, W/2, C]:
// F.avg_pool2d on a channels-last tensor (core/corr.py:70-71), the same four
// values summed in the same order as avg_pool2x2_kernel (corr_build.hip), so
// the result is bit-identical to pooling the NCHW tensor.  Four channels per
// thread (float4) when C % 4 == 0.
template <int V>
__global__ __launch_bounds__(256) void avg_pool2x2_nhwc_kernel(const float* __restrict__ in,
                                                               float* __restrict__ out,
                                                               int B, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2, Cv = C / V;
  const long long total = (long long)B * Ho * Wo * Cv;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int cv = (int)(idx % Cv);
    long long r = idx / Cv;
    const int x = (int)(r % Wo);
    r /= Wo;
    const int y = (int)(r % Ho);
    const long long b = r / Ho;
    const long long row = (b * H + 2 * y) * W + 2 * x;
    if constexpr (V == 4) {
      const float4* s = reinterpret_cast<const float4*>(in);
      const long long cs = C / 4;
      const float4 a = s[row * cs + cv], bb = s[(row + 1) * cs + cv];
      const float4 cc = s[(row + W) * cs + cv], d = s[(row + W + 1) * cs + cv];
      float4 o;
      o.x = (((a.x + bb.x) + cc.x) + d.x) * 0.25f;
      o.y = (((a.y + bb.y) + cc.y) + d.y) * 0.25f;
      o.z = (((a.z + bb.z) + cc.z) + d.z) * 0.25f;
      o.w = (((a.w + bb.w) + cc.w) + d.w) * 0.25f;
      reinterpret_cast<float4*>(out)[idx] = o;
    } else {
      const float* s = in + row * C + cv;
      out[idx] = (((s[0] + s[C]) + s[(long long)W * C]) + s[(long long)(W + 1) * C]) * 0.25f;
    }
  }
}

}  // namespace

extern "C" int dxr_alt_corr_forward(const float* fmap1, const float* fmap2, const float* coords,
                                    float* corr, int64_t B, int64_t H1, int64_t W1, int64_t H2,
                                    int64_t W2, int64_t C, int64_t Nc, int radius,
                                    hipStream_t stream) {
  if (B < 0 || H1 < 1 || W1 < 1 || H2 < 1 || W2 < 1 || C < 1 || Nc < 0 || radius < 0)
    return DXR_EINVAL;
  if (radius > 6) return DXR_EUNSUPPORTED;
  if (H1 * W1 > (1LL << 30) || H2 * W2 > (1LL << 30) || B * Nc > 65535 || C > (1 << 20))
    return DXR_EINVAL;
  if (B == 0 || Nc == 0) return DXR_OK;
  if (!fmap1 || !fmap2 || !coords || !corr) return DXR_EINVAL;
  const int rd = 2 * radius + 1;
  AltGeom g;
  g.N = (int)(H1 * W1);
  g.C = (int)C;
  g.Nc = (int)Nc;
  g.cout = rd * rd;
  g.divisor = 1.f;
  g.div_recip = 1.f;
  g.f1_bstride = H1 * W1 * C;
  g.coord_zstride = H1 * W1 * 2;
  g.coord_cstride = 1;
  g.coord_qstride = 2;
  g.lv[0] = AltLevel{fmap2, (int)H2, (int)W2, 1.f, 0};
  const bool vec = (C % 4 == 0) && aligned16(fmap1) && aligned16(fmap2);
  return launch_alt(fmap1, coords, corr, g, 1, (int)(B * Nc), radius, vec, stream, (int)W1);
}

extern "C" int dxr_alt_corr_backward(const float* fmap1, const float* fmap2, const float* coords,
                                     const float* corr_grad, float* fmap1_grad,
                                     float* fmap2_grad, int64_t B, int64_t H1, int64_t W1,
                                     int64_t H2, int64_t W2, int64_t C, int64_t Nc, int radius,
                                     hipStream_t stream) {
  if (B < 0 || H1 < 1 || W1 < 1 || H2 < 1 || W2 < 1 || C < 1 || Nc < 0 || radius < 0)
    return DXR_EINVAL;
  if (radius > 6) return DXR_EUNSUPPORTED;
  if (H1 * W1 > (1LL << 30) || H2 * W2 > (1LL << 30) || B > 65535 || C > (1 << 20))
    return DXR_EINVAL;
  if (B == 0) return DXR_OK;
  if (!fmap1 || !fmap2 || !fmap1_grad || !fmap2_grad) return DXR_EINVAL;
  if (Nc > 0 && (!coords || !corr_grad)) return DXR_EINVAL;
  // fmap2_grad accumulates atomically from zero, as the reference's torch::zeros output.
  hipError_t e = hipMemsetAsync(fmap2_grad, 0, (size_t)(B * H2 * W2 * C) * sizeof(float), stream);
  if (e != hipSuccess) {
    dxr::set_last_hip_error(e);
    return DXR_EHIP;
  }
  const AltBwd a{fmap1, fmap2, coords, corr_grad, fmap1_grad, fmap2_grad, (int)B,
                 (int)(H1 * W1), (int)H2, (int)W2, (int)C, (int)Nc};
  switch (radius) {
    case 0: return launch_alt_backward_r<0>(a, stream);
    case 1: return launch_alt_backward_r<1>(a, stream);
    case 2: return launch_alt_backward_r<2>(a, stream);
    case 3: return launch_alt_backward_r<3>(a, stream);
    case 4: return launch_alt_backward_r<4>(a, stream);
    case 5: return launch_alt_backward_r<5>(a, stream);
    default: return launch_alt_backward_r<6>(a, stream);
  }
}

extern "C" int dxr_transpose(const void* in, void* out, int dtype, int64_t B, int64_t rows,
                             int64_t cols, hipStream_t stream) {
  if (B < 0 || rows < 0 || cols < 0 || (dtype != DXR_F32 && dtype != DXR_BF16)) return DXR_EINVAL;
  if (rows * cols > (1LL << 40) || B > 65535 || (rows + 63) / 64 > 65535 ||
      (cols + 63) / 64 > (1LL << 31) - 1)
    return DXR_EINVAL;
  if (B == 0 || rows == 0 || cols == 0) return DXR_OK;
  if (!in || !out || rows > INT32_MAX || cols > INT32_MAX) return DXR_EINVAL;
  const dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64), (unsigned)B);
  if (dtype == DXR_F32 && rows % 4 == 0 && cols % 4 == 0 && aligned16(in) && aligned16(out))
    hipLaunchKernelGGL(transpose_tile_v4_kernel, grid, dim3(256), 0, stream,
                       static_cast<const float*>(in), static_cast<float*>(out), (int)rows,
                       (int)cols);
  else if (dtype == DXR_F32)
    hipLaunchKernelGGL((transpose_tile_kernel<float>), grid, dim3(256), 0, stream,
                       static_cast<const float*>(in), static_cast<float*>(out), (int)rows,
                       (int)cols);
  else
    hipLaunchKernelGGL((transpose_tile_kernel<uint16_t>), grid, dim3(256), 0, stream,
                       static_cast<const uint16_t*>(in), static_cast<uint16_t*>(out), (int)rows,
                       (int)cols);
  return dxr::launch_status();
}

extern "C" int dxr_avg_pool2x2_nhwc(const float* in, float* out, int64_t B, int64_t H, int64_t W,
                                    int64_t C, hipStream_t stream) {
  if (B < 0 || H < 0 || W < 0 || C < 1 || B > INT32_MAX || H > INT32_MAX || W > INT32_MAX ||
      C > INT32_MAX)
    return DXR_EINVAL;
  const long long total = B * (H / 2) * (W / 2) * C;
  if (total == 0) return DXR_OK;
  if (!in || !out) return DXR_EINVAL;
  const bool vec = (C % 4 == 0) && aligned16(in) && aligned16(out);
  long long blocks = (total / (vec ? 4 : 1) + 255) / 256;
  if (blocks > 2048 * 8) blocks = 2048 * 8;
  if (vec)
    hipLaunchKernelGGL((avg_pool2x2_nhwc_kernel<4>), dim3((unsigned)blocks), dim3(256), 0, stream,
                       in, out, (int)B, (int)H, (int)W, (int)C);
  else
    hipLaunchKernelGGL((avg_pool2x2_nhwc_kernel<1>), dim3((unsigned)blocks), dim3(256), 0, stream,
                       in, out, (int)B, (int)H, (int)W, (int)C);
  return dxr::launch_status();
}

namespace {
// n_levels < 0: every level; else only levels [0, n_levels) of a num_levels-level
// output (the rest come from dxr_alt_volume_lookup).
int alt_lookup(const float* fmap1, const float* const* fmap2_levels, const float* coords, float* out,
               int64_t B, int64_t H, int64_t W, int64_t C, int num_levels, int radius,
               float divisor, void* workspace, int64_t workspace_bytes, hipStream_t stream,
               int n_levels = -1) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L)) return DXR_EINVAL;
  if (n_levels > num_levels || n_levels == 0) return DXR_EINVAL;
  const int nl = n_levels < 0 ? num_levels : n_levels;
  if (C < 1 || radius < 0 || !(divisor == divisor) || divisor == 0.f) return DXR_EINVAL;
  if (radius > 6) return DXR_EUNSUPPORTED;
  if (H * W > (1LL << 30) || B > 65535 || C > (1 << 20)) return DXR_EINVAL;
  if (B == 0) return DXR_OK;
  if (!fmap1 || !fmap2_levels || !coords || !out) return DXR_EINVAL;
  const int rd = 2 * radius + 1;
  AltGeom g;
  g.N = (int)(H * W);
  g.C = (int)C;
  g.Nc = 1;
  g.cout = num_levels * rd * rd;
  g.divisor = divisor;
  g.div_recip = pow2_recip(divisor);
  g.f1_bstride = H * W * C;
  g.coord_zstride = 2 * H * W;
  g.coord_cstride = H * W;
  g.coord_qstride = 1;
  bool vec = (C % 4 == 0) && aligned16(fmap1);
  for (int l = 0; l < nl; ++l) {
    if (!fmap2_levels[l]) return DXR_EINVAL;
    vec = vec && aligned16(fmap2_levels[l]);
    g.lv[l] = AltLevel{fmap2_levels[l], L.h[l], L.w[l], 1.f / (float)(1 << l), l * rd * rd};
  }
  void* ord = nullptr;
  if (workspace != nullptr && aligned16(workspace) &&
      workspace_bytes >= (long long)B * nl * alt_order_bytes(H, W))
    ord = workspace;
  return launch_alt(fmap1, coords, out, g, nl, (int)B, radius, vec, stream, (int)W, ord);
}

// ---------------------------------------------------------------------------
// A coarse level's whole volume as one tiled GEMM (round 6): every (query, cell)
// sum of the level, raw, into that level's pages of the volume buffer — the FULL
// form's output (and so the on-the-fly lookup's dot products) bit for bit, since
// each sum is the same three f16 products per k step (alt_split8h operands, cell
// vectors as the A rows, queries as the B columns of v_mfma_f32_32x32x16_f16,
// cross terms in a second accumulator folded by 2^-11 at the end) in the same k
// order; only the tiling differs.  The FULL form streams every cell of the level
// through each 32-query workgroup (1080p level 2: 337 us per block); here one
// workgroup = one page's 128 queries x 128 cells (128 / T whole tiles of the
// level, T = th * tw cells per tile, i.e. 128 / T consecutive pages), four waves
// of 64 cells x 64 queries (2 x 2 MFMA tiles), so each loaded operand feeds 64
// MFMA columns instead of 32 and the split is paid once per workgroup.
// K runs in stages of 32 channels: every thread loads 8 float4 (4 of cells, 4 of
// queries) one stage ahead, splits them and writes hi / lo to a double-buffered
// LDS stage laid out [operand][plane][k step][row][kh] x 16 B, so every MFMA
// fragment read is a conflict-free ds_read_b128 over 1 KB contiguous per wave
// (blocks padded by 128 B so the split's 8-B writes of the two k steps of a row
// land in different banks).  A 32 x 32 tile whose sums are not finite is redone
// from fmap1 / fmap2 on the 3-way bf16 split (six products, the windowed form's
// fallback arithmetic).  Rows past the level or the query count compute zeros;
// pages past the level's last tile are not written.  C % 32 == 0.
constexpr int VG_BLK = 4096 + 128;            // one [row][kh] block of 128 rows x 32 B
constexpr int VG_STAGE = 8 * VG_BLK;          // [operand][plane][k step] blocks

// XA (experiments only; 0 in the product): bit 0 stores only sums equal to
// 12345.0 (none: an ablation of the stores), bit 1 writes the raw f32 bits as the
// hi / lo planes (no split VALU; results meaningless), bit 2 skips the MFMAs.
template <int T, bool DMA, int XA = 0>
__global__ __launch_bounds__(256, 2) void alt_volume_gemm_kernel(
    const float* __restrict__ f1, const float* __restrict__ f2, float* __restrict__ out,
    dxr::LevelLayout vl, int N, int C, int ngroups, const _Float16* __restrict__ p1,
    const _Float16* __restrict__ p2) {
  static_assert(T == 2 || T == 8 || T == 32 || T == 128, "tiled levels 0-3 only");
  constexpr int TPG = 128 / T;                 // level tiles (pages) per workgroup
  __shared__ __attribute__((aligned(16))) unsigned char lds[DMA ? 4 * 16384 : 2 * VG_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, kh = lane >> 5;
  const int wc = wave & 1, wq = wave >> 1;     // the wave's 64-cell / 64-query half
  // contiguous bands of (query block, cell group) per XCD (csrc/corr_build.hip's
  // page_coord bijection): one XCD's workgroups share their query block's operand in L2
  const int n = gridDim.x, q8 = n / 8, r8 = n % 8, xcd = (int)blockIdx.x % 8;
  const int idx = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) +
                  (int)blockIdx.x / 8;
  const int qblk = idx / ngroups, grp = idx - qblk * ngroups;
  const int b = blockIdx.z;
  const int ntiles = vl.ty * vl.tx;
  const float* f1b = f1 + (long long)b * N * C;
  const float* f2b = f2 + (long long)b * vl.h * vl.w * C;
  // element offset of cell row i (0..127) of this workgroup's group, -1 past the level
  auto cell_off = [&](int i) -> int {
    const int tile = grp * TPG + i / T, c = i % T;
    if (tile >= ntiles) return -1;
    const int ty = tile / vl.tx, tx = tile - ty * vl.tx;
    const int cy = ty * vl.th + c / vl.tw, cx = tx * vl.tw + c % vl.tw;
    return (cy < vl.h && cx < vl.w) ? (cy * vl.w + cx) * C : -1;
  };
  auto query_off = [&](int i) -> int {
    const int q = qblk * 128 + i;
    return q < N ? q * C : -1;
  };
  af16 acc[2][2], acc2[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][q][r] = acc2[a][q][r] = 0.f;
  // one k step of the wave's 2 x 2 tiles: the windowed form's three products
  auto mfma_step = [&](const ah8 (&th)[2], const ah8 (&tl)[2], const ah8 (&qh)[2],
                       const ah8 (&ql)[2]) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if constexpr ((XA & 4) != 0) {
          acc[a][q][0] += (float)th[a][0] * (float)qh[q][1] + (float)tl[a][2] * (float)ql[q][3];
          continue;
        }
        acc2[a][q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl[a], qh[q], acc2[a][q], 0, 0, 0);
        acc2[a][q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th[a], ql[q], acc2[a][q], 0, 0, 0);
        acc[a][q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th[a], qh[q], acc[a][q], 0, 0, 0);
      }
  };
  if constexpr (DMA) {
    // operands pre-split (alt_split_planes_kernel: [pair][hi | lo][k step][row][16]
    // f16) and staged by LDS-DMA, one k step (16 channels) per ring slot, NS slots: no
    // staging VGPRs and no split VALU in the loop, NS - 1 k steps of loads in flight.
    // Slot layout [operand][plane][row block of 32][row][kh] x 16 B: one DMA
    // instruction (lane l -> row 32 rb + l / 2, kh = l % 2, 16 B) fills one 1 KB row
    // block — from 32 consecutive 32-B records of one k step, so queries read whole
    // lines — and every fragment read is a conflict-free ds_read_b128 of 1 KB per
    // wave.  Wave w moves operand w / 2 (0 cells, 1 queries), plane w % 2; rows past
    // the level or the query count read out of the buffer's range, i.e. zeros.
    constexpr int NS = 4, SLOT = 16384;
    const int o = wave >> 1, pl = wave & 1;
    const int rows_o = o == 0 ? vl.h * vl.w : N;
    const _Float16* pbase = (o == 0 ? p2 : p1) + ((long long)b * 2 + pl) * rows_o * C;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<_Float16*>(pbase), (short)0, rows_o * C * 2, 0x00020000);
    uint32_t voff[4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const int row = rb * 32 + (lane >> 1);
      const int e = o == 0 ? cell_off(row) : query_off(row);   // row * C, or -1
      voff[rb] = e >= 0 ? (uint32_t)(e / C) * 32u + (uint32_t)(lane & 1) * 16u : 0x80000000u;
    }
    const int kstride = rows_o * 32;               // bytes per k step of a plane
    const int wslot = __builtin_amdgcn_readfirstlane((o * 2 + pl) * 4096);
    auto issue = [&](int ks) {
      unsigned char* dst = lds + (ks % NS) * SLOT + wslot;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + rb * 1024), 16, voff[rb],
                                                 ks * kstride, 0, 0);
    };
    const int nks = C / 16;
#pragma unroll
    for (int u = 0; u < NS - 1; ++u)
      if (u < nks) issue(u);
    for (int ks = 0; ks < nks; ++ks) {
      // this wave's DMAs of step ks done (those of the younger steps may fly), then
      // everyone's: the barrier also retires the reads of the slot refilled below
      const int younger = min(NS - 2, nks - 1 - ks);
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (ks + NS - 1 < nks) issue(ks + NS - 1);
      const unsigned char* st = lds + (ks % NS) * SLOT;
      ah8 th[2], tl[2], qh[2], ql[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int rc = (wc * 2 + a) * 1024 + j * 32 + kh * 16;
        const int rq = (wq * 2 + a) * 1024 + j * 32 + kh * 16;
        th[a] = __builtin_bit_cast(ah8, *reinterpret_cast<const uint4*>(st + 0 * 4096 + rc));
        tl[a] = __builtin_bit_cast(ah8, *reinterpret_cast<const uint4*>(st + 1 * 4096 + rc));
        qh[a] = __builtin_bit_cast(ah8, *reinterpret_cast<const uint4*>(st + 2 * 4096 + rq));
        ql[a] = __builtin_bit_cast(ah8, *reinterpret_cast<const uint4*>(st + 3 * 4096 + rq));
      }
      mfma_step(th, tl, qh, ql);
    }
  } else {
    // this thread's 8 load slots: slot i < 4 cells, else queries; piece t + 256 (i % 4)
    // -> row piece / 8, channels 4 (piece % 8) .. + 4 of the stage
    int off[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int piece = tid + 256 * (i & 3), row = piece >> 3;
      off[i] = i < 4 ? cell_off(row) : query_off(row);
    }
    const int f4 = tid & 7;
    const int ch = 4 * f4;
    // LDS byte offset of this thread's 8-B hi write for slot i (lo: + 2 VG_BLK)
    auto wr_addr = [&](int i) -> int {
      const int row = (tid + 256 * (i & 3)) >> 3, o = i >> 2;
      return ((o * 2 + 0) * 2 + (f4 >> 2)) * VG_BLK + row * 32 + ((f4 >> 1) & 1) * 16 + (f4 & 1) * 8;
    };
    float4 pre[8];
    auto load_stage = [&](int s) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float* base = i < 4 ? f2b : f1b;
        pre[i] = off[i] >= 0 ? *reinterpret_cast<const float4*>(base + off[i] + 32 * s + ch)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    auto write_stage = [&](int buf) {
      unsigned char* st = lds + buf * VG_STAGE;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 v = pre[i];
        uint32_t h0, h1, l0, l1;
        if constexpr ((XA & 2) != 0) {
          h0 = __float_as_uint(v.x); h1 = __float_as_uint(v.y);
          l0 = __float_as_uint(v.z); l1 = __float_as_uint(v.w);
        } else {
          h0 = alt_cvt_pk_h(v.x, v.y);
          h1 = alt_cvt_pk_h(v.z, v.w);
          const ah2 a0 = __builtin_bit_cast(ah2, h0), a1 = __builtin_bit_cast(ah2, h1);
          l0 = alt_cvt_pk_h((v.x - (float)a0[0]) * 2048.f, (v.y - (float)a0[1]) * 2048.f);
          l1 = alt_cvt_pk_h((v.z - (float)a1[0]) * 2048.f, (v.w - (float)a1[1]) * 2048.f);
        }
        const int a = wr_addr(i);
        *reinterpret_cast<uint2*>(st + a) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(st + a + 2 * VG_BLK) = make_uint2(l0, l1);
      }
    };
    const int nst = C / 32;
    load_stage(0);
    write_stage(0);
    __syncthreads();
    for (int s = 0; s < nst; ++s) {
      if (s + 1 < nst) load_stage(s + 1);
      const unsigned char* st = lds + (s & 1) * VG_STAGE;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        ah8 th[2], tl[2], qh[2], ql[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const int rc = (wc * 64 + a * 32 + j) * 32 + kh * 16;
          const int rq = (wq * 64 + a * 32 + j) * 32 + kh * 16;
          th[a] = __builtin_bit_cast(ah8, *reinterpret_cast<const uint4*>(st + (0 + ks) * VG_BLK + rc));
          tl[a] = __builtin_bit_cast(ah8, *reinterpret_cast<const uint4*>(st + (2 + ks) * VG_BLK + rc));
          qh[a] = __builtin_bit_cast(ah8, *reinterpret_cast<const uint4*>(st + (4 + ks) * VG_BLK + rq));
          ql[a] = __builtin_bit_cast(ah8, *reinterpret_cast<const uint4*>(st + (6 + ks) * VG_BLK + rq));
        }
        mfma_step(th, tl, qh, ql);
      }
      if (s + 1 < nst) write_stage((s + 1) & 1);
      __syncthreads();
    }
  }
  const long long page0 = ((long long)b * vl.qt + qblk) * ntiles + (long long)grp * TPG;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      bool bad = false;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[a][q][r] = __builtin_fmaf(acc2[a][q][r], 0x1p-11f, acc[a][q][r]);
        bad |= !(__builtin_fabsf(acc[a][q][r]) <= 3.40282347e38f);
      }
      if ((XA & 6) == 0 && __ballot(bad) != 0) {   // wave-uniform: the tile on the 3-way bf16 split
        const int co = cell_off(wc * 64 + a * 32 + j), qo = query_off(wq * 64 + q * 32 + j);
        af16 f = {};
        for (int ks = 0; ks < C / 16; ++ks) {
          float x[8], y[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            x[e] = co >= 0 ? f2b[co + 16 * ks + 8 * kh + e] : 0.f;
            y[e] = qo >= 0 ? f1b[qo + 16 * ks + 8 * kh + e] : 0.f;
          }
          uint4 h, m, l, uh, um, ul;
          alt_split8(x, h, m, l);
          alt_split8(y, uh, um, ul);
          const abf8 th = __builtin_bit_cast(abf8, h), tm = __builtin_bit_cast(abf8, m),
                     tl = __builtin_bit_cast(abf8, l);
          const abf8 qh = __builtin_bit_cast(abf8, uh), qm = __builtin_bit_cast(abf8, um),
                     ql = __builtin_bit_cast(abf8, ul);
          f = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tm, qm, f, 0, 0, 0);
          f = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tl, qh, f, 0, 0, 0);
          f = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, ql, f, 0, 0, 0);
          f = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tm, qh, f, 0, 0, 0);
          f = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, qm, f, 0, 0, 0);
          f = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, qh, f, 0, 0, 0);
        }
        acc[a][q] = f;
      }
      // lane (j, kh) holds rows (r & 3) + 8 (r >> 2) + 4 kh of column j: runs of four
      // consecutive cells, i.e. one 16-B store into one page (T >= 4) or two 8-B
      // stores into two (T = 2)
      const int ql_ = wq * 64 + q * 32 + j;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int row = wc * 64 + a * 32 + 8 * g4 + 4 * kh;
        const float4 v = make_float4(acc[a][q][4 * g4], acc[a][q][4 * g4 + 1],
                                     acc[a][q][4 * g4 + 2], acc[a][q][4 * g4 + 3]);
        if constexpr ((XA & 1) != 0)
          if (v.x != 12345.f) continue;
        if constexpr (T >= 4) {
          const int t = row / T;
          if (grp * TPG + t < ntiles)
            *reinterpret_cast<float4*>(out + vl.off + ((page0 + t) * 128 + ql_) * T + row % T) = v;
        } else {
          const int t = row / 2;
          if (grp * TPG + t < ntiles)
            *reinterpret_cast<float2*>(out + vl.off + ((page0 + t) * 128 + ql_) * 2) =
                make_float2(v.x, v.y);
          if (grp * TPG + t + 1 < ntiles)
            *reinterpret_cast<float2*>(out + vl.off + ((page0 + t + 1) * 128 + ql_) * 2) =
                make_float2(v.z, v.w);
        }
      }
    }
}

// f16 pair planes of `rows` f32 rows of C channels per pair, k-step-major so one
// k step (16 channels) of consecutive rows is contiguous: out[pair][plane][ks][row][16]
// with plane 0 = RNE_f16(x), plane 1 = RNE_f16((x - hi) * 2^11) — alt_split8h per
// element, so the DMA form's products are the register form's.  Thread = 4
// channels of a row, row-major (a wave reads 1 KB contiguous; its 8-B writes form
// 32-B runs whose neighbours — the next rows' — the next waves write).
__global__ __launch_bounds__(256) void alt_split_planes_kernel(const float* __restrict__ in,
                                                               _Float16* __restrict__ out,
                                                               long long rows, int C,
                                                               long long n4) {
  const int c4n = C / 4;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < n4;
       t += (long long)gridDim.x * 256) {
    const long long prow = t / c4n;
    const int c = (int)(t - prow * c4n) * 4;
    const long long pair = prow / rows, row = prow - pair * rows;
    const float4 v = *reinterpret_cast<const float4*>(in + 4 * t);
    const uint32_t h0 = alt_cvt_pk_h(v.x, v.y), h1 = alt_cvt_pk_h(v.z, v.w);
    const ah2 a0 = __builtin_bit_cast(ah2, h0), a1 = __builtin_bit_cast(ah2, h1);
    const uint32_t l0 = alt_cvt_pk_h((v.x - (float)a0[0]) * 2048.f, (v.y - (float)a0[1]) * 2048.f);
    const uint32_t l1 = alt_cvt_pk_h((v.z - (float)a1[0]) * 2048.f, (v.w - (float)a1[1]) * 2048.f);
    _Float16* o = out + pair * 2 * rows * C + ((long long)(c >> 4) * rows + row) * 16 + (c & 15);
    *reinterpret_cast<uint2*>(o) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(o + rows * C) = make_uint2(l0, l1);
  }
}

int launch_split_planes(const float* in, _Float16* out, long long B, long long rows, int C,
                        hipStream_t stream) {
  const long long n4 = B * rows * C / 4;
  const long long blocks = std::min<long long>((n4 + 255) / 256, 16384);
  hipLaunchKernelGGL(alt_split_planes_kernel, dim3((unsigned)std::max<long long>(blocks, 1)),
                     dim3(256), 0, stream, in, out, rows, C, n4);
  return dxr::launch_status();
}

// one level's volume by alt_volume_gemm_kernel (tiled levels 0-3, C % 32 == 0);
// with f16 pair planes of both operands (p1, p2) the LDS-DMA form
template <int XA = 0>
int launch_alt_volume_gemm(const float* f1, const float* f2, float* vol, const dxr::LevelLayout& vl,
                           int B, int N, int C, hipStream_t stream,
                           const _Float16* p1 = nullptr, const _Float16* p2 = nullptr) {
  const int T = vl.th * vl.tw;
  const int ngroups = (vl.ty * vl.tx + 128 / T - 1) / (128 / T);
  const long long nwg = (long long)vl.qt * ngroups;
  if (nwg > 0x7fffffffLL || (long long)N * C > 0x3fffffffLL ||
      (long long)vl.h * vl.w * C > 0x3fffffffLL)
    return DXR_EUNSUPPORTED;
  const dim3 grid((unsigned)nwg, 1u, (unsigned)B);
  const bool dma = p1 != nullptr && p2 != nullptr;
#define DXR_VG(TT)                                                                              \
  if (dma)                                                                                      \
    hipLaunchKernelGGL((alt_volume_gemm_kernel<TT, true, XA>), grid, dim3(256), 0, stream, f1, \
                       f2, vol, vl, N, C, ngroups, p1, p2);                                     \
  else                                                                                          \
    hipLaunchKernelGGL((alt_volume_gemm_kernel<TT, false, XA>), grid, dim3(256), 0, stream, f1,\
                       f2, vol, vl, N, C, ngroups, p1, p2);
  switch (T) {
    case 2: DXR_VG(2) break;
    case 8: DXR_VG(8) break;
    case 32: DXR_VG(32) break;
    case 128: DXR_VG(128) break;
    default: return DXR_EUNSUPPORTED;
  }
#undef DXR_VG
  return dxr::launch_status();
}
}  // namespace

// ---------------------------------------------------------------------------
// Coarse-level volumes (round 6).  An on-the-fly lookup pays each level's box
// GEMMs again on every call, ~26 us per level and 1080p lookup whatever the
// level's size; a coarse level's whole correlation volume costs less than one
// such lookup to compute once per block.  dxr_alt_coarse_volumes computes levels
// [first_level, num_levels) of fmap1 against the pooled fmap2 levels (the
// alternate block's own operands) — the tiled levels (0-3) by
// alt_volume_gemm_kernel when C % 32 == 0, others by the FULL form of the box
// kernel, the same sums either way — and
// stores them, raw, in the paged layout of those pyramid levels, one buffer of
// dxr_alt_volume_numel floats; dxr_alt_volume_lookup (csrc/corr_lookup.hip)
// reads its windows from there with the alternate block's arithmetic.
extern "C" int64_t dxr_alt_volume_numel(int64_t B, int64_t H, int64_t W, int num_levels,
                                        int first_level) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L) || first_level < 0 || first_level >= num_levels)
    return -1;
  return L.numel - L.off[first_level];
}

namespace {
// Bytes of the f16 pair planes the DMA form of the volume GEMM reads (fmap1 and
// each tiled level >= first_level of fmap2, 2 x 2 B per element, 256-B aligned
// regions); 0 when no level takes the GEMM.
long long alt_volume_planes_bytes(const dxr::Levels& L, int64_t B, int64_t H, int64_t W, int64_t C,
                                  int num_levels, int first_level, long long* level_off) {
  if (C % 32 != 0 || first_level >= dxr::TILED_LEVELS) return 0;
  auto up = [](long long x) { return (x + 255) / 256 * 256; };
  long long off = up(B * H * W * C * 4);
  for (int l = first_level; l < num_levels && l < dxr::TILED_LEVELS; ++l) {
    if (level_off) level_off[l] = off;
    off += up(B * (long long)L.h[l] * L.w[l] * C * 4);
  }
  return off;
}

// full_form: every level by the FULL box kernel (experiments: the round-6 first form);
// ws (>= alt_volume_planes_bytes): the GEMM's LDS-DMA form on pre-split planes
int alt_coarse_volumes(const float* fmap1, const float* const* fmap2_levels, int64_t B, int64_t H,
                       int64_t W, int64_t C, int num_levels, int first_level, float* volumes,
                       hipStream_t stream, bool full_form, void* ws = nullptr,
                       int64_t ws_bytes = 0) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L) || first_level < 0 || first_level >= num_levels)
    return DXR_EINVAL;
  if (C < 1 || B > 65535 || H * W > (1LL << 30)) return DXR_EINVAL;
  if (C % 16 != 0 || C > 256) return DXR_EUNSUPPORTED;
  if (B == 0) return DXR_OK;
  if (!fmap1 || !fmap2_levels || !volumes || !aligned16(fmap1)) return DXR_EINVAL;
  AltGeom g;
  g.N = (int)(H * W);
  g.C = (int)C;
  g.Nc = 1;
  g.cout = 0;
  g.divisor = 1.f;
  g.f1_bstride = H * W * C;
  g.coord_zstride = g.coord_cstride = 0;
  g.coord_qstride = 0;
  const int tiles_x = (int)((W + TQX - 1) / TQX);
  const int ntiles = tiles_x * (int)((H + TQY - 1) / TQY);
  long long loff[8] = {};
  const long long pbytes = alt_volume_planes_bytes(L, B, H, W, C, num_levels, first_level, loff);
  _Float16* planes = nullptr;
  if (!full_form && pbytes > 0 && ws != nullptr && ws_bytes >= pbytes && aligned16(ws)) {
    planes = static_cast<_Float16*>(ws);
    int st = launch_split_planes(fmap1, planes, B, H * W, (int)C, stream);
    if (st != DXR_OK) return st;
  }
  for (int l = first_level; l < num_levels; ++l) {
    if (!fmap2_levels[l] || !aligned16(fmap2_levels[l])) return DXR_EINVAL;
    g.lv[0] = AltLevel{fmap2_levels[l], L.h[l], L.w[l], 1.f, 0};
    g.vlay = L.lay[l];
    g.vlay.off -= L.off[first_level];
    if (l < dxr::TILED_LEVELS && C % 32 == 0 && !full_form) {
      _Float16* p2 = nullptr;
      if (planes) {
        p2 = reinterpret_cast<_Float16*>(static_cast<unsigned char*>(ws) + loff[l]);
        const int st = launch_split_planes(fmap2_levels[l], p2, B, (long long)L.h[l] * L.w[l],
                                           (int)C, stream);
        if (st != DXR_OK) return st;
      }
      const int st = launch_alt_volume_gemm(fmap1, fmap2_levels[l], volumes, g.vlay, (int)B, g.N,
                                            (int)C, stream, planes, p2);
      if (st != DXR_OK) return st;
      continue;
    }
    hipLaunchKernelGGL((alt_corr_mfma_kernel<0, 1, 256, true, 3, false, 4, 0, 0, true>),
                       dim3((unsigned)ntiles, 1u, (unsigned)B), dim3(256), 0, stream, fmap1,
                       (const float*)nullptr, volumes, g, (int)W, tiles_x, (const int4*)nullptr,
                       0LL, 0);
    const int st = dxr::launch_status();
    if (st != DXR_OK) return st;
  }
  return DXR_OK;
}
}  // namespace

extern "C" int dxr_alt_coarse_volumes(const float* fmap1, const float* const* fmap2_levels,
                                      int64_t B, int64_t H, int64_t W, int64_t C, int num_levels,
                                      int first_level, float* volumes, hipStream_t stream) {
  return alt_coarse_volumes(fmap1, fmap2_levels, B, H, W, C, num_levels, first_level, volumes,
                            stream, false);
}

extern "C" int64_t dxr_alt_coarse_volumes_ws_bytes(int64_t B, int64_t H, int64_t W, int64_t C,
                                                   int num_levels, int first_level) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L) || first_level < 0 ||
      first_level >= num_levels || C < 1)
    return -1;
  return alt_volume_planes_bytes(L, B, H, W, C, num_levels, first_level, nullptr);
}

extern "C" int dxr_alt_coarse_volumes_ws(const float* fmap1, const float* const* fmap2_levels,
                                         int64_t B, int64_t H, int64_t W, int64_t C,
                                         int num_levels, int first_level, float* volumes,
                                         void* workspace, int64_t workspace_bytes,
                                         hipStream_t stream) {
  return alt_coarse_volumes(fmap1, fmap2_levels, B, H, W, C, num_levels, first_level, volumes,
                            stream, false, workspace, workspace_bytes);
}

extern "C" int dxr_alt_corr_lookup(const float* fmap1, const float* const* fmap2_levels,
                                   const float* coords, float* out, int64_t B, int64_t H,
                                   int64_t W, int64_t C, int num_levels, int radius,
                                   float divisor, hipStream_t stream) {
  return alt_lookup(fmap1, fmap2_levels, coords, out, B, H, W, C, num_levels, radius, divisor,
                    nullptr, 0, stream);
}

extern "C" int64_t dxr_alt_workspace_bytes(int64_t B, int64_t H, int64_t W, int num_levels) {
  if (B < 0 || H < 1 || W < 1 || num_levels < 1 || num_levels > 8 || H * W > (1LL << 30))
    return -1;
  return B * num_levels * alt_order_bytes(H, W);
}

extern "C" int dxr_alt_corr_lookup_ws(const float* fmap1, const float* const* fmap2_levels,
                                      const float* coords, float* out, int64_t B, int64_t H,
                                      int64_t W, int64_t C, int num_levels, int radius,
                                      float divisor, void* workspace, int64_t workspace_bytes,
                                      hipStream_t stream) {
  return alt_lookup(fmap1, fmap2_levels, coords, out, B, H, W, C, num_levels, radius, divisor,
                    workspace, workspace_bytes, stream);
}

extern "C" int dxr_alt_corr_lookup_levels_ws(const float* fmap1, const float* const* fmap2_levels,
                                             const float* coords, float* out, int64_t B, int64_t H,
                                             int64_t W, int64_t C, int num_levels, int n_levels,
                                             int radius, float divisor, void* workspace,
                                             int64_t workspace_bytes, hipStream_t stream) {
  if (n_levels < 1) return DXR_EINVAL;
  return alt_lookup(fmap1, fmap2_levels, coords, out, B, H, W, C, num_levels, radius, divisor,
                    workspace, workspace_bytes, stream, n_levels);
}

