// Stage (c): radius-r bilinear lookup into every pyramid level.
//
// Replaces core/corr.py:29-50 (CorrBlock.__call__) and the helper it calls,
// core/utils/utils.py:57-71 (bilinear_sampler -> F.grid_sample with
// align_corners=True, bilinear, zero padding).  The reference builds a
// (2r+1)^2 delta grid on the host and copies it to the device per level per
// call (core/corr.py:37-39), runs one grid_sample per level, then cat + permute
// + contiguous.  Here one launch writes the final [B, L*(2r+1)^2, H, W] tensor.
//
// Arithmetic is the reference's, sample by sample (bit-exact on its golden vectors):
//   c   = coords / 2^l + (o - r)                            (core/corr.py:41-43)
//   g   = 2*c / (S_l - 1) - 1                               (utils.py:61-62)
//   u   = (g + 1) * ((S_l - 1) / 2)                         (grid_sample unnormalise)
//   taps at floor(u), floor(u)+1 with weights 1-f, f (f = u - floor(u)); taps off
//   the level contribute 0; the four products are summed as the fused chain
//   fma(se, v_se, fma(sw, v_sw, fma(ne, v_ne, nw*v_nw))) — the arithmetic of the
//   reference's compiled CPU grid sampler.
// The round trip moves a sample by a few ulps, so for integer-valued coordinates
// (RAFT's first iteration) floor(u) of neighbouring samples need not step by
// exactly one.  Every sample therefore uses its own floor, and the staged window
// is (2r+3)^2 cells: the per-sample floors span at most one extra row/column.
//
// MI355X mapping: one workgroup = QB consecutive query pixels x one level.
//   phase 0  QB threads compute the 2(2r+1) sample positions of their query and
//            the window origin (LDS);
//   phase 1  each wave gathers whole windows of one query at a time into LDS —
//            lanes walk consecutive cells of a window row, so one wave load
//            touches a handful of 128-B lines instead of 64 (lane-per-query
//            gathers thrash the 32 KiB L1 and become L2-bandwidth bound);
//   phase 2  thread = (query, x-offset class): taps from LDS, fused sum, and
//            every output store is a coalesced 256-B wave store along queries.
#include "dxr_common.h"

namespace {

constexpr int FAR_ORIGIN = -(1 << 29);  // window origin of far / non-finite queries

// Paged-pyramid addressing of one level (dxr_common.h), in shift/mask form:
//   index = off + (b*qt + (q >> lqb)) * qstride + (q & (2^lqb - 1)) * S
//         + ((y >> lth) * tx + (x >> ltw)) * pageS + (y & mh) * tw + (x & mw)
// Row-major levels use lth = ltw = 30 (tile index 0 for in-range cells).
struct LevelAddr {
  int h, w;                 // true level size
  int lth, ltw, mh, mw;     // tile shifts / masks
  int tw, tx, lqb, qt;
  long long off, qstride, S, pageS;
};

struct LookupGeom {
  int N;          // H * W query pixels per pair
  int levels;
  int cout;       // levels * (2r+1)^2
  LevelAddr lv[8];
};

LevelAddr level_addr(const dxr::LevelLayout& y) {
  LevelAddr a;
  a.h = y.h; a.w = y.w; a.tw = y.tw; a.tx = y.tx; a.qt = y.qt; a.off = y.off;
  a.S = (long long)y.th * y.tw;
  if (y.qb > 1) {  // paged level: power-of-two tile dims and page size
    a.lth = __builtin_ctz(y.th); a.ltw = __builtin_ctz(y.tw);
    a.mh = y.th - 1; a.mw = y.tw - 1;
    a.lqb = __builtin_ctz(y.qb);
    a.pageS = (long long)y.qb * a.S;
    a.qstride = (long long)y.ty * y.tx * a.pageS;
  } else {         // row-major level
    a.lth = 30; a.ltw = 30; a.mh = 0x3fffffff; a.mw = 0x3fffffff;
    a.lqb = 0; a.pageS = 0; a.qstride = a.S;
  }
  return a;
}

template <typename PT>
__device__ __forceinline__ float load_cell(const PT* p) {
  if constexpr (sizeof(PT) == 2) return dxr::bf16_to_f32(*reinterpret_cast<const uint16_t*>(p));
  else return *p;
}

// Reference coordinate round trip for one sample (see file comment).
__device__ __forceinline__ float sample_coord(float c, float sm1, float half_sm1) {
  const float gn = __fsub_rn(__fdiv_rn(__fmul_rn(2.f, c), sm1), 1.f);
  return __fmul_rn(__fadd_rn(gn, 1.f), half_sm1);
}

template <int R>
struct LookupCfg {
  static constexpr int RD = 2 * R + 1;     // samples per axis
  static constexpr int WD = RD + 2;        // staged window side
  static constexpr int NC = WD * WD;       // cells per window (odd: bank-friendly pitch)
  static constexpr int NTHR = 128;         // two waves
  static constexpr int QB = R <= 4 ? 32 : 16;  // queries per workgroup
  static constexpr int NG = NTHR / QB;     // x-offset classes in phase 2
  static constexpr int QPW = QB / (NTHR / 64);  // queries gathered per wave
  static constexpr int CPL = (NC + 63) / 64;    // window cells per lane per query
};

template <int R, typename PT>
__global__ __launch_bounds__(LookupCfg<R>::NTHR) void corr_lookup_kernel(const PT* __restrict__ pyr,
                                                           const float* __restrict__ coords,
                                                           float* __restrict__ out,
                                                           LookupGeom g) {
  using C = LookupCfg<R>;
  constexpr int RD = C::RD, WD = C::WD, NC = C::NC, QB = C::QB, NG = C::NG;
  constexpr int QPW = C::QPW, CPL = C::CPL;
  __shared__ float cells[QB * NC];
  __shared__ float sx[RD * QB];
  __shared__ float sy[RD * QB];
  __shared__ int org[2 * QB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * QB;
  const LevelAddr A = g.lv[l];
  const int Hl = A.h, Wl = A.w;

  // ---- phase 0: sample positions and window origin per query
  if (tid < QB) {
    const int q = q0 + tid;
    float x = 0.f, y = 0.f;
    if (q < g.N) {
      const float inv = 1.f / (float)(1 << l);  // exact power of two
      x = coords[((long long)b * 2 + 0) * g.N + q] * inv;
      y = coords[((long long)b * 2 + 1) * g.N + q] * inv;
    }
    const float wm1 = (float)(Wl - 1), hm1 = (float)(Hl - 1);
    const float whalf = wm1 / 2.f, hhalf = hm1 / 2.f;
    bool far = false;
    int mx = 1 << 30, my = 1 << 30;
#pragma unroll
    for (int j = 0; j < RD; ++j) {
      const float u = sample_coord(__fadd_rn(x, (float)(j - R)), wm1, whalf);
      const float v = sample_coord(__fadd_rn(y, (float)(j - R)), hm1, hhalf);
      sx[j * QB + tid] = u;
      sy[j * QB + tid] = v;
      const float fu = floorf(u), fv = floorf(v);
      if (!(fabsf(fu) < 1.0e7f) || !(fabsf(fv) < 1.0e7f)) {
        far = true;
      } else {
        mx = min(mx, (int)fu - j);
        my = min(my, (int)fv - j);
      }
    }
    // Windows entirely off the level hold only zeros: skip their loads.
    if (!far && (mx + WD <= 0 || mx >= Wl || my + WD <= 0 || my >= Hl)) far = true;
    org[tid] = far ? FAR_ORIGIN : mx;
    org[QB + tid] = far ? FAR_ORIGIN : my;
  }
  __syncthreads();

  // ---- phase 1: gather each query's window into LDS (zeros off the level).
  // All of a wave's loads are issued before its first LDS store, so the
  // QPW x CPL gathers are in flight together (one memory latency per wave).
  float cellv[QPW][CPL];
#pragma unroll
  for (int i = 0; i < QPW; ++i) {
    const int qq = wave * QPW + i;
    const int q = q0 + qq;
    const int xlo = org[qq], ylo = org[QB + qq];
    const bool live = q < g.N && xlo != FAR_ORIGIN;
    const int qs = live ? q : 0;
    const PT* img = pyr + A.off + ((long long)b * A.qt + (qs >> A.lqb)) * A.qstride +
                    (long long)(qs & ((1 << A.lqb) - 1)) * A.S;
#pragma unroll
    for (int m = 0; m < CPL; ++m) {
      const int c = m * 64 + lane;
      const int yy = ylo + c / WD, xx = xlo + c % WD;
      const bool in = live && c < NC && (unsigned)yy < (unsigned)Hl && (unsigned)xx < (unsigned)Wl;
      const long long e = ((long long)(yy >> A.lth) * A.tx + (xx >> A.ltw)) * A.pageS +
                          (yy & A.mh) * A.tw + (xx & A.mw);
      cellv[i][m] = in ? load_cell(img + e) : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < QPW; ++i)
#pragma unroll
    for (int m = 0; m < CPL; ++m) {
      const int c = m * 64 + lane;
      if (c < NC) cells[(wave * QPW + i) * NC + c] = cellv[i][m];
    }
  __syncthreads();

  // ---- phase 2: bilinear taps from LDS, coalesced stores along queries
  const int qq = tid % QB;
  const int q = q0 + qq;
  if (q >= g.N) return;
  const int xlo = org[qq], ylo = org[QB + qq];
  const bool live = xlo != FAR_ORIGIN;
  const float* cq = cells + qq * NC;
  int row[RD];
  float fn[RD], fs[RD];
#pragma unroll
  for (int oy = 0; oy < RD; ++oy) {
    const float v = sy[oy * QB + qq];
    const float fl = floorf(v);
    fn[oy] = __fsub_rn(v, fl);
    fs[oy] = __fsub_rn(1.f, fn[oy]);
    row[oy] = live ? ((int)fl - ylo) * WD : 0;
  }
  float* ob = out + ((long long)b * g.cout + (long long)l * RD * RD) * g.N + q;
  for (int ox = tid / QB; ox < RD; ox += NG) {
    const float u = sx[ox * QB + qq];
    const float fl = floorf(u);
    const float fx = __fsub_rn(u, fl);
    const float ex = __fsub_rn(1.f, fx);
    const int col = live ? (int)fl - xlo : 0;
#pragma unroll
    for (int oy = 0; oy < RD; ++oy) {
      float v00 = 0.f, v01 = 0.f, v10 = 0.f, v11 = 0.f;
      if (live) {
        const float* p = cq + row[oy] + col;
        v00 = p[0]; v01 = p[1]; v10 = p[WD]; v11 = p[WD + 1];
      }
      const float nw = __fmul_rn(fs[oy], ex), ne = __fmul_rn(fs[oy], fx);
      const float sw = __fmul_rn(fn[oy], ex), se = __fmul_rn(fn[oy], fx);
      float v = __fmul_rn(nw, v00);
      v = __builtin_fmaf(ne, v01, v);
      v = __builtin_fmaf(sw, v10, v);
      v = __builtin_fmaf(se, v11, v);
      ob[(long long)(ox * RD + oy) * g.N] = v;
    }
  }
}

template <int R, typename PT>
int launch_lookup_r(const PT* pyr, const float* coords, float* out, const LookupGeom& g, int B,
                    hipStream_t stream) {
  using C = LookupCfg<R>;
  const dim3 grid((unsigned)((g.N + C::QB - 1) / C::QB), (unsigned)g.levels, (unsigned)B);
  hipLaunchKernelGGL((corr_lookup_kernel<R, PT>), grid, dim3(C::NTHR), 0, stream, pyr, coords,
                     out, g);
  return dxr::launch_status();
}

template <typename PT>
int launch_lookup(const PT* pyr, const float* coords, float* out, const LookupGeom& g, int B,
                  int radius, hipStream_t stream) {
  switch (radius) {
    case 0: return launch_lookup_r<0, PT>(pyr, coords, out, g, B, stream);
    case 1: return launch_lookup_r<1, PT>(pyr, coords, out, g, B, stream);
    case 2: return launch_lookup_r<2, PT>(pyr, coords, out, g, B, stream);
    case 3: return launch_lookup_r<3, PT>(pyr, coords, out, g, B, stream);
    case 4: return launch_lookup_r<4, PT>(pyr, coords, out, g, B, stream);
    case 5: return launch_lookup_r<5, PT>(pyr, coords, out, g, B, stream);
    case 6: return launch_lookup_r<6, PT>(pyr, coords, out, g, B, stream);
    case 7: return launch_lookup_r<7, PT>(pyr, coords, out, g, B, stream);
    case 8: return launch_lookup_r<8, PT>(pyr, coords, out, g, B, stream);
    default: return DXR_EUNSUPPORTED;
  }
}

}  // namespace

extern "C" int dxr_corr_lookup(const void* pyramid, int pyr_dtype, int64_t B, int64_t H,
                               int64_t W, int num_levels, int radius, const float* coords,
                               float* out, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L)) return DXR_EINVAL;
  if (radius < 0) return DXR_EINVAL;
  if (radius > 8) return DXR_EUNSUPPORTED;
  if (B > 65535 || H * W > (1LL << 30)) return DXR_EINVAL;
  if (B == 0) return DXR_OK;
  if (!pyramid || !coords || !out) return DXR_EINVAL;
  const int rd = 2 * radius + 1;
  LookupGeom g;
  g.N = (int)(H * W);
  g.levels = num_levels;
  g.cout = num_levels * rd * rd;
  for (int l = 0; l < L.n; ++l) g.lv[l] = level_addr(L.lay[l]);
  if (pyr_dtype == DXR_F32)
    return launch_lookup(static_cast<const float*>(pyramid), coords, out, g, (int)B, radius, stream);
  if (pyr_dtype == DXR_BF16)
    return launch_lookup(static_cast<const uint16_t*>(pyramid), coords, out, g, (int)B, radius,
                         stream);
  return DXR_EINVAL;
}
