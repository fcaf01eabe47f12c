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
//   phase 0  threads compute the 2(2r+1) sample positions of their query and
//            the window origin (LDS);
//   phase 1  the windows are gathered into LDS as aligned 4-cell vectors;
//   phase 2  thread = (query, output class): taps from LDS, fused sum, and
//            every output store is a coalesced wave store along queries.
// The product lookup (round 6) is corr_lookup_qm_kernel, which stages the
// windows query-minor so the phase-2 tap reads are bank-conflict-free;
// corr_lookup_wide_kernel (per-query LDS blocks, rounds 1-5) stays for the
// experiments target, and its phase 0 / gathers serve the lookup backward and
// the fused motion kernel.
#include <cmath>
#include <type_traits>

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
  int lS, lpS;              // paged levels: log2 S, log2 pageS (shifts, not multiplies)
  long long off, qstride, S, pageS;
};

struct LookupGeom {
  int N;          // H * W query pixels per pair
  int levels;
  int cout;       // levels * (2r+1)^2
  int out_nt = 0; // wide lookup: non-temporal output stores (launch_lookup_r decides)
  int l0 = 0;     // level of blockIdx.y == 0 (the alternate block's volume lookup: its first coarse level)
  float divisor = 1.f, div_recip = 0.f;   // ALT: the alternate block's division of each output
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
    a.lS = __builtin_ctzll(a.S);
    a.lpS = __builtin_ctzll(a.pageS);
  } else {         // row-major level
    a.lth = 30; a.ltw = 30; a.mh = 0x3fffffff; a.mw = 0x3fffffff;
    a.lqb = 0; a.pageS = 0; a.qstride = a.S;
    a.lS = a.lpS = -1;
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

// ---------------------------------------------------------------------------
// Lookup.  The work of a workgroup (QB queries x one level) is spread over
// NT = 512 threads so that no phase is a long per-thread chain:
//   phase 0  one thread per (query, sample index j): both axes' coordinate
//            round trips, floors and fractions; the window origin
//            min_j(floor_j - j) and the far test are reduced over the query's
//            G-lane group by shuffles; per-sample tap data {cell offset, f, 1-f}
//            goes to LDS;
//   phase 1  the QB windows are gathered as aligned vectors of V cells (V = 4 on
//            the paged levels 0-2, whose tile rows hold >= 4 cells; 2 on level 3;
//            1 on row-major levels), with 32-bit offsets from the workgroup's page
//            base, into LDS rows of RS cells starting at the origin rounded down
//            to a multiple of 4;
//   phase 2  thread = (query, output class), stores along queries.
// A narrow predecessor (128 threads per 32 queries; r01, sintel: 1,600 VALU
// instructions per wave, 1.7 waves per SIMD, 8.8 of 11.6 us left with gathers
// and stores removed) was bound by its per-thread instruction chains.
// ---------------------------------------------------------------------------
template <int R, int NT_ = 512, int QB_ = 0>
struct WideCfg {
  static constexpr int RD = 2 * R + 1;
  static constexpr int WD = RD + 2;                      // window side (cells)
  static constexpr int RS = (WD + 3 + 3) & ~3;           // LDS row: 4-aligned start + WD
  static constexpr int NQ = RS / 4;                      // 4-cell vectors per LDS row
  static constexpr int QS = WD * RS + 4;                 // LDS cells per query (bank skew)
  static constexpr int K = RD * RD;                      // outputs per query and level
  static constexpr int NT = NT_;
  static constexpr int QB = QB_ ? QB_ : (R <= 4 ? 32 : 16);   // queries per workgroup
  static constexpr int LG = RD <= 2 ? 1 : RD <= 4 ? 2 : RD <= 8 ? 3 : RD <= 16 ? 4 : 5;
  static constexpr int G = 1 << LG;                      // lanes per query in phase 0
  static constexpr int VSLOTS = QB * WD * NQ;            // 4-cell vectors per workgroup
  static constexpr int VIT = (VSLOTS + NT - 1) / NT;
  static constexpr int NCLS = NT / QB;                   // output classes
  static constexpr int SIT = (QB * G + NT - 1) / NT;     // phase-0 slots per thread
  static_assert((QB * G) % NT == 0 || QB * G < NT, "whole waves per phase-0 pass");
  static_assert(G <= 64, "a query's lane group must sit in one wave");
  static_assert(QB <= dxr::PAGE_Q && dxr::PAGE_Q % QB == 0, "a workgroup stays in one page");
};

// V consecutive cells of one tile row (or of a row-major level), widened to f32.
template <int V, typename PT>
__device__ __forceinline__ void load_vec(const PT* p, float* v) {
  if constexpr (sizeof(PT) == 4 && V == 4) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  } else if constexpr (sizeof(PT) == 4 && V == 2) {
    const float2 x = *reinterpret_cast<const float2*>(p);
    v[0] = x.x; v[1] = x.y;
  } else if constexpr (sizeof(PT) == 2 && V == 4) {
    const uint2 x = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
    v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
  } else if constexpr (sizeof(PT) == 2 && V == 2) {
    const uint32_t x = *reinterpret_cast<const uint32_t*>(p);
    v[0] = __uint_as_float(x << 16); v[1] = __uint_as_float(x & 0xffff0000u);
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = load_cell(p + i);
  }
}

// Phase 1 for one level type: V-cell vectors, 4 per LDS vector slot.  Split in
// a load half (registers) and a store half (LDS) so a caller can keep several
// levels' gathers in flight at once (the fused motion kernel).
// Slot order: QMAJ = false walks one query's window row by row (consecutive
// lanes read consecutive 16-B pieces of one window row: levels 0/1, whose tile
// rows are 32-64 B of one query); QMAJ = true walks the queries fastest, so a
// wave instruction reads the same window piece of 32 consecutive queries —
// on levels 2/3, whose pages interleave queries at 32 / 8 B per tile, those
// are neighbours in one or a few lines instead of 64 separate lines.
template <int R, int NT_, bool QMAJ, int QB_ = 0>
__device__ __forceinline__ void gather_slot(int s, int& qq, int& rem) {
  using C = WideCfg<R, NT_, QB_>;
  if constexpr (QMAJ) {
    qq = s % C::QB;
    rem = s / C::QB;
  } else {
    qq = s / (C::WD * C::NQ);
    rem = s - qq * (C::WD * C::NQ);
  }
}

template <int R, int NT_, int V, typename PT, bool QMAJ = false, int QB_ = 0>
__device__ __forceinline__ void gather_load(const PT* __restrict__ base, int qb0, const LevelAddr& A,
                                            const int2* org, int q0, int N, int tid,
                                            float4 (&v)[WideCfg<R, NT_, QB_>::VIT]) {
  using C = WideCfg<R, NT_, QB_>;
#pragma unroll
  for (int i = 0; i < C::VIT; ++i) {
    const int s = tid + i * C::NT;
    int qq, rem;
    gather_slot<R, NT_, QMAJ, QB_>(s, qq, rem);
    const int r = rem / C::NQ, k = rem - r * C::NQ;
    float c[4] = {0.f, 0.f, 0.f, 0.f};
    if (s < C::VSLOTS && q0 + qq < N) {
      const int2 o = org[qq];
      const int yy = o.y + r, x0 = (o.x & ~3) + 4 * k;
      if (o.x != FAR_ORIGIN && (unsigned)yy < (unsigned)A.h && x0 >= 0 && x0 < A.w) {
        // V > 1: a paged level (power-of-two S, pageS, tw): shifts and a 24-bit
        // multiply instead of quarter-rate 32-bit ones (round 4)
        const unsigned qoff = V > 1 ? (unsigned)(qb0 + qq) << A.lS : (unsigned)(qb0 + qq) * (unsigned)A.S;
        const unsigned yoff = V > 1 ? __umul24((unsigned)(yy >> A.lth), (unsigned)A.tx)
                                    : (unsigned)(yy >> A.lth) * (unsigned)A.tx;
        const unsigned yin = V > 1 ? (unsigned)(yy & A.mh) << A.ltw : (unsigned)((yy & A.mh) * A.tw);
#pragma unroll
        for (int h = 0; h < 4; h += V) {
          const int x = x0 + h;
          const unsigned tl = yoff + (unsigned)(x >> A.ltw);
          const unsigned e = qoff + (V > 1 ? tl << A.lpS : tl * (unsigned)A.pageS) + yin +
                             (unsigned)(x & A.mw);
          if (V == 4 || x < A.w) load_vec<V, PT>(base + e, c + h);
        }
#pragma unroll
        for (int h = 1; h < 4; ++h)
          if (x0 + h >= A.w) c[h] = 0.f;   // past the level's right edge (tile padding)
      }
    }
    v[i] = make_float4(c[0], c[1], c[2], c[3]);
  }
}

template <int R, int NT_, bool QMAJ = false, int QB_ = 0>
__device__ __forceinline__ void gather_store(const float4 (&v)[WideCfg<R, NT_, QB_>::VIT], float* cells,
                                             int tid) {
  using C = WideCfg<R, NT_, QB_>;
#pragma unroll
  for (int i = 0; i < C::VIT; ++i) {
    const int s = tid + i * C::NT;
    if (s < C::VSLOTS) {
      int qq, rem;
      gather_slot<R, NT_, QMAJ, QB_>(s, qq, rem);
      *reinterpret_cast<float4*>(cells + qq * C::QS + rem * 4) = v[i];
    }
  }
}

template <int R, int NT_, int V, typename PT, bool QMAJ = false, int QB_ = 0>
__device__ __forceinline__ void gather_windows(const PT* __restrict__ base, int qb0, const LevelAddr& A,
                                               const int2* org, float* cells, int q0, int N,
                                               int tid) {
  float4 v[WideCfg<R, NT_, QB_>::VIT];
  gather_load<R, NT_, V, PT, QMAJ, QB_>(base, qb0, A, org, q0, N, tid, v);
  gather_store<R, NT_, QMAJ, QB_>(v, cells, tid);
}

// Phase 0 of the wide lookup (forward and backward): per (query, sample) the
// coordinate round trip, floor and fractions; per query the window origin and
// the far flag.  Tap data goes to xs / ys, origins to org.  Split into the
// coordinate loads and the rest so the multi-set backward can load the next
// set's coordinates a pass ahead.
template <int R, int NT_, int QB_ = 0>
struct Phase0Coords {
  float x[WideCfg<R, NT_, QB_>::SIT], y[WideCfg<R, NT_, QB_>::SIT];
};

template <int R, int NT_, int QB_ = 0>
__device__ __forceinline__ void wide_phase0_load(const float* __restrict__ coords, const LookupGeom& g,
                                                 int b, int q0, int tid, Phase0Coords<R, NT_, QB_>& c) {
  using C = WideCfg<R, NT_, QB_>;
  constexpr int QB = C::QB, G = C::G;
#pragma unroll
  for (int it = 0; it < C::SIT; ++it) {
    const int slot = tid + it * C::NT;
    c.x[it] = c.y[it] = 0.f;
    if (slot >= QB * G) break;   // whole waves
    const int q = q0 + (slot >> C::LG);
    if (q < g.N) {
      c.x[it] = coords[((long long)b * 2 + 0) * g.N + q];
      c.y[it] = coords[((long long)b * 2 + 1) * g.N + q];
    }
  }
}

// min over the aligned group of G lanes (G = 2, 4, 8, 16: DPP within a row of
// 16 lanes, no LDS round trip; 32: cross-row shuffles).  Order-free, so the same
// value as any other reduction order.
template <int G>
__device__ __forceinline__ int group_min(int v) {
  if constexpr (G >= 2) v = min(v, __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));  // quad [1,0,3,2]
  if constexpr (G >= 4) v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));  // quad [2,3,0,1]
  if constexpr (G >= 8) v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false)); // row_half_mirror
  if constexpr (G >= 16) v = min(v, __builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false)); // row_mirror
  if constexpr (G >= 32) v = min(v, __shfl_xor(v, 16));
  if constexpr (G >= 64) v = min(v, __shfl_xor(v, 32));
  return v;
}

// XPITCH: pitch of the tap arrays (xs[j * XPITCH + qq]; 0 = QB).  A query's
// samples are written by consecutive lanes, so at pitch QB every lane of an
// 8-lane ds_write_b128 group hits one bank group (8-way); QB + 1 spreads them
// (round 6: the lookup backward and the fused motion kernel).
template <int R, int NT_, int QB_ = 0, int XPITCH = 0>
__device__ __forceinline__ void wide_phase0_taps(const Phase0Coords<R, NT_, QB_>& c, const LevelAddr& A,
                                                 int l, int tid, float4* xs, float4* ys, int2* org) {
  using C = WideCfg<R, NT_, QB_>;
  constexpr int RD = C::RD, WD = C::WD, RS = C::RS, QB = C::QB, G = C::G;
  constexpr int XPB = XPITCH ? XPITCH : QB;
  const int Hl = A.h, Wl = A.w;
#pragma unroll
  for (int it = 0; it < C::SIT; ++it) {
    const int slot = tid + it * C::NT;
    if (slot >= QB * G) break;   // whole waves
    const int j = slot & (G - 1), qq = slot >> C::LG;
    const float cx = c.x[it], cy = c.y[it];
    const float inv = __builtin_ldexpf(1.f, -l);  // 2^-l, exact (no division)
    const float wm1 = (float)(Wl - 1), hm1 = (float)(Hl - 1);
    const float ux = sample_coord(__fadd_rn(cx * inv, (float)(j - R)), wm1, wm1 / 2.f);
    const float uy = sample_coord(__fadd_rn(cy * inv, (float)(j - R)), hm1, hm1 / 2.f);
    const float flx = floorf(ux), fly = floorf(uy);
    const bool act = j < RD;
    // a non-finite or huge sample makes its query far: FAR_ORIGIN propagates through the min
    int mx = 0x7fffffff, my = 0x7fffffff;
    if (act) {
      const bool bad = !(fabsf(flx) < 1.0e7f) || !(fabsf(fly) < 1.0e7f);
      mx = bad ? FAR_ORIGIN : (int)flx - j;
      my = bad ? FAR_ORIGIN : (int)fly - j;
    }
    mx = group_min<G>(mx);
    my = group_min<G>(my);
    // windows entirely off the level hold only zeros: no loads
    const bool far = mx + WD <= 0 || mx >= Wl || my + WD <= 0 || my >= Hl;
    if (j == 0) org[qq] = far ? make_int2(FAR_ORIGIN, FAR_ORIGIN) : make_int2(mx, my);
    if (act) {
      const float fx = __fsub_rn(ux, flx), fy = __fsub_rn(uy, fly);
      const int col = far ? 0 : (int)flx - (mx & ~3);
      const int row = far ? 0 : ((int)fly - my) * RS;
      xs[j * XPB + qq] = make_float4(__int_as_float(col), fx, __fsub_rn(1.f, fx), 0.f);
      ys[j * XPB + qq] = make_float4(__int_as_float(row), fy, __fsub_rn(1.f, fy), 0.f);
    }
  }
}

template <int R, int NT_, int QB_ = 0, int XPITCH = 0>
__device__ __forceinline__ void wide_phase0(const float* __restrict__ coords, const LookupGeom& g,
                                            const LevelAddr& A, int b, int l, int q0, int tid,
                                            float4* xs, float4* ys, int2* org) {
  Phase0Coords<R, NT_, QB_> c;
  wide_phase0_load<R, NT_, QB_>(coords, g, b, q0, tid, c);
  wide_phase0_taps<R, NT_, QB_, XPITCH>(c, A, l, tid, xs, ys, org);
}

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int R, typename PT, int NT_ = 512, int QB_ = 0>
__global__ __launch_bounds__(NT_) void corr_lookup_wide_kernel(
    const PT* __restrict__ pyr, const float* __restrict__ coords, float* __restrict__ out,
    LookupGeom g) {
  using C = WideCfg<R, NT_, QB_>;
  constexpr int RD = C::RD, RS = C::RS, K = C::K, QB = C::QB;
  __shared__ __attribute__((aligned(16))) float cells[QB * C::QS];
  __shared__ float4 xs[RD * QB];   // {column in the LDS row (int bits), fx, 1-fx, -}
  __shared__ float4 ys[RD * QB];   // {row offset in LDS (int bits), fy, 1-fy, -}
  __shared__ int2 org[QB];         // window origin (x, y) or FAR_ORIGIN

  const int tid = threadIdx.x;
  const int l = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * QB;
  const LevelAddr A = g.lv[l];
  // One-dispatch-round grids (the 256 x 16 shape): wave priority by level, finest
  // first (3 / 2 / 1 / 0), so co-resident level-0 waves, which move the most
  // lines, issue ahead.  Same-process A/B in the step (r4af): Sintel B=1 203.1 ->
  // 201.2 us; on multi-round grids (Sintel B=8, KITTI B=8) it cost 0.7-1.5 %.
  if constexpr (QB_ != 0 && QB_ <= 16) {
    if (l == 0) __builtin_amdgcn_s_setprio(3);
    else if (l == 1) __builtin_amdgcn_s_setprio(2);
    else if (l == 2) __builtin_amdgcn_s_setprio(1);
  }

  // ---- phase 0
  wide_phase0<R, NT_, QB_>(coords, g, A, b, l, q0, tid, xs, ys, org);
  __syncthreads();

  // ---- phase 1 (zeros off the level and for far queries)
  {
    const PT* base = pyr + A.off + ((long long)b * A.qt + (q0 >> A.lqb)) * A.qstride;
    const int qb0 = q0 & ((1 << A.lqb) - 1);
    // levels 2/3 (tile rows of 4 / 2 cells): query-major slots (round 3: Sintel
    // B=8 51.5 -> 50.1 us, KITTI B=8 bf16 54.1 -> 51.6 us, bit-identical)
    if (A.lth == 30)
      gather_windows<R, NT_, 1, PT, false, QB_>(base, qb0, A, org, cells, q0, g.N, tid);
    else if (A.tw >= 8)
      gather_windows<R, NT_, 4, PT, false, QB_>(base, qb0, A, org, cells, q0, g.N, tid);
    else if (A.tw == 4)
      gather_windows<R, NT_, 4, PT, true, QB_>(base, qb0, A, org, cells, q0, g.N, tid);
    else if (A.tw == 2)
      gather_windows<R, NT_, 2, PT, true, QB_>(base, qb0, A, org, cells, q0, g.N, tid);
    else
      gather_windows<R, NT_, 1, PT, false, QB_>(base, qb0, A, org, cells, q0, g.N, tid);
  }
  __syncthreads();

  // ---- phase 2
  const int qq = tid % QB, cls = tid / QB;
  if (q0 + qq >= g.N) return;
  const float* cq = cells + qq * C::QS;
  float* ob = out + ((long long)b * g.cout + (long long)l * K) * g.N + q0 + qq;
  // output k at ob + k N: a pointer stepped by NCLS N (no per-store multiply)
  float* op = ob + (long long)cls * g.N;
  const long long ostep = (long long)C::NCLS * g.N;
  // (round 4: unrolled and branch-free over the thread's outputs, every LDS read
  // issued before the first sum, was slower in the step: Sintel B=1 207.3 vs
  // 204.7 us, Chairs 102.9 vs 100.5, Sintel B=8 1,541 vs 1,519, KITTI B=8 bf16
  // 1,136 vs 1,107 us)
  for (int k = cls; k < K; k += C::NCLS) {
    const int ox = k / RD, oy = k - ox * RD;
    const float4 xd = xs[ox * QB + qq], yd = ys[oy * QB + qq];
    const float* p = cq + __float_as_int(yd.x) + __float_as_int(xd.x);
    const float v00 = p[0], v01 = p[1], v10 = p[RS], v11 = p[RS + 1];
    const float nw = __fmul_rn(yd.z, xd.z), ne = __fmul_rn(yd.z, xd.y);
    const float sw = __fmul_rn(yd.y, xd.z), se = __fmul_rn(yd.y, xd.y);
    float r = __fmul_rn(nw, v00);
    r = __builtin_fmaf(ne, v01, r);
    r = __builtin_fmaf(sw, v10, r);
    r = __builtin_fmaf(se, v11, r);
    // write-through (sc1) output stores (round 2): the outputs leave the XCD's
    // L2 while the kernel runs instead of as dirty lines the next kernel
    // boundary writes back (Sintel B=1 9.5 -> 8.5 us, B=8 58.0 -> 54.6 us).
    // Round 5: non-temporal stores where a wave's output segments are whole or
    // aligned half lines (g.out_nt, launch_lookup_r) — they leave the caches
    // entirely, so the pyramid lines the next lookups gather stay resident.
    // Round 4: routing them through LDS as 16-byte stores of 4 queries was
    // slower in the step (Sintel B=1 237.9 vs 222.8 us, B=8 1,623 vs 1,583 us,
    // KITTI B=8 bf16 1,268 vs 1,193 us).
    if (g.out_nt) __builtin_nontemporal_store(r, op);
    else __hip_atomic_store(op, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    op += ostep;
  }
}

// ---------------------------------------------------------------------------
// Query-minor lookup (round 6).  The wide kernel stages each query's window as
// its own block of rows (qq * 180 + row * 16 + col floats), so the phase-2 tap
// reads of a half-wave (32 lanes = 32 queries at one output) fall on banks set
// by each query's own window origin: ~2.7 LDS cycles per read where 1 is the
// floor (PMC r05: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 0.42).  Here the
// window cells are staged query-minor, cell (row, col) of query qq at
//   ((row * RSC + col) * QB + qq)
// so a lane's bank is qq + QB * (cell index) mod 32: with QB = 32 every tap read
// of a half-wave is conflict-free whatever the windows; with QB = 16 (the
// one-round 256 x 16 shape) a half-wave holds outputs k and k + 1 of 16 queries,
// whose cells are one row apart, and the odd row pitch RSC = 17 puts them in
// opposite bank halves.  Gathers walk the queries fastest on every level, so
// each 4-cell vector goes out as four conflict-free ds_write_b32.  Tap data is
// 8 bytes per sample ({LDS offset, f}, 1 - f recomputed with the same rounding).
// Same arithmetic, same outputs bit for bit.
// ---------------------------------------------------------------------------
template <int R, int NT_ = 512, int QB_ = 32>
struct QmCfg {
  using C = WideCfg<R, NT_, QB_>;
  static constexpr int RD = C::RD, WD = C::WD, K = C::K, QB = C::QB, NT = NT_;
  static constexpr int NQ = C::NQ;                    // 4-cell vectors per staged row
  static constexpr int RSC = 4 * NQ + 1;              // odd row pitch (cells)
  static constexpr int NCELL = WD * RSC;
  // gather slots: query fastest, then the window row over an even count WDE >= WD
  // (row WD is a dummy when WD is odd), then the vector: the two slots of a
  // 16-query half-wave are always rows r, r + 1 of one vector column
  static constexpr int WDE = (WD + 1) & ~1;
  static constexpr int VSLOTS = QB * WDE * NQ;
  static constexpr int VIT = (VSLOTS + NT - 1) / NT;
  static constexpr int NCLS = NT / QB;
  // tap data pitch: phase 0 writes a query's samples from 16 consecutive lanes
  // (xs[j * XP + qq]); with XP = QB every one of them hit one bank (16-way)
  static constexpr int XP = QB + 1;
  static_assert(QB == 16 || QB == 32, "bank arithmetic assumes 16 or 32 queries");
};

// Phase 0 taps in the query-minor form: per sample {LDS offset in floats, f}.
template <int R, int NT_, int QB_>
__device__ __forceinline__ void qm_phase0_taps(const Phase0Coords<R, NT_, QB_>& c, const LevelAddr& A,
                                               int l, int tid, float2* xs, float2* ys, int2* org) {
  using C = WideCfg<R, NT_, QB_>;
  using Q = QmCfg<R, NT_, QB_>;
  constexpr int RD = C::RD, WD = C::WD, QB = C::QB, G = C::G;
  const int Hl = A.h, Wl = A.w;
#pragma unroll
  for (int it = 0; it < C::SIT; ++it) {
    const int slot = tid + it * C::NT;
    if (slot >= QB * G) break;   // whole waves
    const int j = slot & (G - 1), qq = slot >> C::LG;
    const float cx = c.x[it], cy = c.y[it];
    const float inv = __builtin_ldexpf(1.f, -l);
    const float wm1 = (float)(Wl - 1), hm1 = (float)(Hl - 1);
    const float ux = sample_coord(__fadd_rn(cx * inv, (float)(j - R)), wm1, wm1 / 2.f);
    const float uy = sample_coord(__fadd_rn(cy * inv, (float)(j - R)), hm1, hm1 / 2.f);
    const float flx = floorf(ux), fly = floorf(uy);
    const bool act = j < RD;
    int mx = 0x7fffffff, my = 0x7fffffff;
    if (act) {
      const bool bad = !(fabsf(flx) < 1.0e7f) || !(fabsf(fly) < 1.0e7f);
      mx = bad ? FAR_ORIGIN : (int)flx - j;
      my = bad ? FAR_ORIGIN : (int)fly - j;
    }
    mx = group_min<G>(mx);
    my = group_min<G>(my);
    const bool far = mx + WD <= 0 || mx >= Wl || my + WD <= 0 || my >= Hl;
    if (j == 0) org[qq] = far ? make_int2(FAR_ORIGIN, FAR_ORIGIN) : make_int2(mx, my);
    if (act) {
      const int col = far ? 0 : (int)flx - (mx & ~3);
      const int row = far ? 0 : (int)fly - my;
      xs[j * Q::XP + qq] = make_float2(__int_as_float(col * QB), __fsub_rn(ux, flx));
      ys[j * Q::XP + qq] = make_float2(__int_as_float(row * Q::RSC * QB), __fsub_rn(uy, fly));
    }
  }
}

// Phase 0 of the ALT form: every sample of a query shares its window origin
// floor(c / 2^l) - r and its fractions (no per-sample floors, no reduction);
// outside +-1e8 or with the window wholly off the level the query is far (its
// staged cells are zeros, its outputs 0 or NaN as the fractions make them, as
// alt_corr_mfma_kernel's).
template <int R, int NT_, int QB_>
__device__ __forceinline__ void qm_phase0_alt(const Phase0Coords<R, NT_, QB_>& c, const LevelAddr& A,
                                              int l, int tid, float2* xs, float2* ys, int2* org) {
  using C = WideCfg<R, NT_, QB_>;
  using Q = QmCfg<R, NT_, QB_>;
  constexpr int RD = C::RD, QB = C::QB, G = C::G;
#pragma unroll
  for (int it = 0; it < C::SIT; ++it) {
    const int slot = tid + it * C::NT;
    if (slot >= QB * G) break;   // whole waves
    const int j = slot & (G - 1), qq = slot >> C::LG;
    const float inv = __builtin_ldexpf(1.f, -l);   // alt_corr: 1 / 2^l, exact
    const float x = c.x[it] * inv, y = c.y[it] * inv;
    const float xf = floorf(x), yf = floorf(y);
    int x0 = 0, y0 = 0;
    bool live = false;
    if (fabsf(xf) < 1.0e8f && fabsf(yf) < 1.0e8f) {
      x0 = (int)xf - R;
      y0 = (int)yf - R;
      live = x0 + RD + 1 > 0 && x0 < A.w && y0 + RD + 1 > 0 && y0 < A.h;
    }
    if (j == 0) org[qq] = live ? make_int2(x0, y0) : make_int2(FAR_ORIGIN, FAR_ORIGIN);
    if (j < RD) {
      const int col = live ? j + (x0 & 3) : 0, row = live ? j : 0;
      xs[j * Q::XP + qq] = make_float2(__int_as_float(col * QB), __fsub_rn(x, xf));
      ys[j * Q::XP + qq] = make_float2(__int_as_float(row * Q::RSC * QB), __fsub_rn(y, yf));
    }
  }
}

// One 4-cell window vector (row r, vector k of the staged row) of query qq:
// the wide kernel's gather_load arithmetic for one slot.
template <int V, typename PT>
__device__ __forceinline__ void qm_load_vec(const PT* __restrict__ base, int qb0, const LevelAddr& A,
                                            int2 o, int qq, int r, int k, float (&c)[4]) {
  c[0] = c[1] = c[2] = c[3] = 0.f;
  const int yy = o.y + r, x0 = (o.x & ~3) + 4 * k;
  if (o.x != FAR_ORIGIN && (unsigned)yy < (unsigned)A.h && x0 >= 0 && x0 < A.w) {
    const unsigned qoff = V > 1 ? (unsigned)(qb0 + qq) << A.lS : (unsigned)(qb0 + qq) * (unsigned)A.S;
    const unsigned yoff = V > 1 ? __umul24((unsigned)(yy >> A.lth), (unsigned)A.tx)
                                : (unsigned)(yy >> A.lth) * (unsigned)A.tx;
    const unsigned yin = V > 1 ? (unsigned)(yy & A.mh) << A.ltw : (unsigned)((yy & A.mh) * A.tw);
#pragma unroll
    for (int h = 0; h < 4; h += V) {
      const int x = x0 + h;
      const unsigned tl = yoff + (unsigned)(x >> A.ltw);
      const unsigned e = qoff + (V > 1 ? tl << A.lpS : tl * (unsigned)A.pageS) + yin +
                         (unsigned)(x & A.mw);
      if (V == 4 || x < A.w) load_vec<V, PT>(base + e, c + h);
    }
#pragma unroll
    for (int h = 1; h < 4; ++h)
      if (x0 + h >= A.w) c[h] = 0.f;
  }
}

// The same vector by a range-checked buffer load (paged levels, V = 4): an
// invalid slot (off the level, far query, padding) gets an out-of-range offset
// and reads as zeros, so the load needs no branch.
template <typename PT>
__device__ __forceinline__ void qm_load_vec_buf(__amdgpu_buffer_rsrc_t rs, int qb0, const LevelAddr& A,
                                                int2 o, int qq, int r, int k, bool live,
                                                float (&c)[4]) {
  const int yy = o.y + r, x0 = (o.x & ~3) + 4 * k;
  unsigned voff = 0x80000000u;
  if (live && o.x != FAR_ORIGIN && (unsigned)yy < (unsigned)A.h && x0 >= 0 && x0 < A.w) {
    const unsigned tl = __umul24((unsigned)(yy >> A.lth), (unsigned)A.tx) + (unsigned)(x0 >> A.ltw);
    const unsigned e = ((unsigned)(qb0 + qq) << A.lS) + (tl << A.lpS) +
                       ((unsigned)(yy & A.mh) << A.ltw) + (unsigned)(x0 & A.mw);
    voff = e * (unsigned)sizeof(PT);
  }
  if constexpr (sizeof(PT) == 4) {
    const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0);
    c[0] = __uint_as_float(v[0]); c[1] = __uint_as_float(v[1]);
    c[2] = __uint_as_float(v[2]); c[3] = __uint_as_float(v[3]);
  } else {
    typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
    const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, 0, 0);
    c[0] = __uint_as_float(v[0] << 16); c[1] = __uint_as_float(v[0] & 0xffff0000u);
    c[2] = __uint_as_float(v[1] << 16); c[3] = __uint_as_float(v[1] & 0xffff0000u);
  }
#pragma unroll
  for (int h = 1; h < 4; ++h)
    if (x0 + h >= A.w) c[h] = 0.f;   // tile padding past the level's right edge
}

// Phase 1, query-minor: slot s -> query s % QB, (vector, row) s / QB with the
// row fastest over WDE rows (so the two slots of a 16-query half-wave are one
// row = RSC cells apart: opposite bank halves); all loads in flight before the
// LDS writes.
template <int R, int NT_, int QB_, int V, typename PT, bool BUF = false>
__device__ __forceinline__ void qm_gather(const PT* __restrict__ base, int qb0, const LevelAddr& A,
                                          const int2* org, float* cells, int q0, int N, int tid) {
  using Q = QmCfg<R, NT_, QB_>;
  constexpr int QB = Q::QB, RSC = Q::RSC;
  float c[Q::VIT][4];
  if constexpr (BUF && V == 4) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<PT*>(base), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int i = 0; i < Q::VIT; ++i) {
      const int s = tid + i * Q::NT;
      const int qq = s % QB, rem = s / QB, k = rem / Q::WDE, r = rem - k * Q::WDE;
      const bool live = s < Q::VSLOTS && r < Q::WD && q0 + qq < N;
      qm_load_vec_buf<PT>(rs, qb0, A, org[live ? qq : 0], qq, r, k, live, c[i]);
    }
  } else {
#pragma unroll
  for (int i = 0; i < Q::VIT; ++i) {
    const int s = tid + i * Q::NT;
    const int qq = s % QB, rem = s / QB, k = rem / Q::WDE, r = rem - k * Q::WDE;
    if (s < Q::VSLOTS && r < Q::WD && q0 + qq < N) {
      qm_load_vec<V, PT>(base, qb0, A, org[qq], qq, r, k, c[i]);
    } else {
      c[i][0] = c[i][1] = c[i][2] = c[i][3] = 0.f;
    }
  }
  }
#pragma unroll
  for (int i = 0; i < Q::VIT; ++i) {
    const int s = tid + i * Q::NT;
    if (s < Q::VSLOTS) {
      const int qq = s % QB, rem = s / QB, k = rem / Q::WDE, r = rem - k * Q::WDE;
      if (r >= Q::WD) continue;
      float* d = cells + (r * RSC + 4 * k) * QB + qq;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e * QB] = c[i][e];
    }
  }
}

// XA: timing ablations for the experiments target (0 in the product): bit 0 skips
// the window gathers, bit 1 the output stores (only values equal to 12345 are
// stored), bit 2 returns after phase 0.
// ALT (round 6, dxr_alt_volume_lookup): the alternate block's arithmetic on
// coarse-level volumes of raw dot products (dxr_alt_coarse_volumes): window origin
// floor(c / 2^l) - r with no coordinate round trip, the (2r+2)^2 window cells
// weighted by the fractions of c / 2^l and combined in correlation_kernel.cu's
// order (as alt_corr_mfma_kernel's last phase), then divided by sqrt(D).
template <int R, typename PT, int NT_ = 512, int QB_ = 32, int UNR = 1, bool BUF = false, int XA = 0,
          bool ALT = false>
__global__ __launch_bounds__(NT_) void corr_lookup_qm_kernel(
    const PT* __restrict__ pyr, const float* __restrict__ coords, float* __restrict__ out,
    LookupGeom g) {
  using Q = QmCfg<R, NT_, QB_>;
  constexpr int RD = Q::RD, K = Q::K, QB = Q::QB, RSC = Q::RSC;
  __shared__ __attribute__((aligned(16))) float cells[Q::NCELL * QB];
  __shared__ float2 xs[RD * Q::XP];   // {LDS column offset (int bits), fx}
  __shared__ float2 ys[RD * Q::XP];   // {LDS row offset (int bits), fy}
  __shared__ int2 org[QB];

  const int tid = threadIdx.x;
  const int l = blockIdx.y + g.l0, b = blockIdx.z;
  const int q0 = blockIdx.x * QB;
  const LevelAddr A = g.lv[l];
  if constexpr (QB_ == 16) {   // one-round grids: finest level first (as the wide kernel)
    if (l == 0) __builtin_amdgcn_s_setprio(3);
    else if (l == 1) __builtin_amdgcn_s_setprio(2);
    else if (l == 2) __builtin_amdgcn_s_setprio(1);
  }

  {
    Phase0Coords<R, NT_, QB_> c;
    wide_phase0_load<R, NT_, QB_>(coords, g, b, q0, tid, c);
    if constexpr (ALT) qm_phase0_alt<R, NT_, QB_>(c, A, l, tid, xs, ys, org);
    else qm_phase0_taps<R, NT_, QB_>(c, A, l, tid, xs, ys, org);
  }
  __syncthreads();
  if constexpr ((XA & 4) != 0) {
    if (xs[tid % (RD * Q::XP)].y == 1234.5f) out[tid] = 0.f;
    return;
  }
  if constexpr ((XA & 1) == 0) {
    const PT* base = pyr + A.off + ((long long)b * A.qt + (q0 >> A.lqb)) * A.qstride;
    const int qb0 = q0 & ((1 << A.lqb) - 1);
    if (A.lth == 30 || A.tw == 1)
      qm_gather<R, NT_, QB_, 1, PT>(base, qb0, A, org, cells, q0, g.N, tid);
    else if (A.tw >= 4)
      qm_gather<R, NT_, QB_, 4, PT, BUF>(base, qb0, A, org, cells, q0, g.N, tid);
    else
      qm_gather<R, NT_, QB_, 2, PT>(base, qb0, A, org, cells, q0, g.N, tid);
  }
  __syncthreads();

  const int qq = tid % QB, cls = tid / QB;
  if (q0 + qq >= g.N) return;
  const float* cq = cells + qq;
  float* op = out + ((long long)b * g.cout + (long long)l * K + cls) * g.N + q0 + qq;
  const long long ostep = (long long)Q::NCLS * g.N;
#pragma unroll UNR
  for (int k = cls; k < K; k += Q::NCLS) {
    const int ox = k / RD, oy = k - ox * RD;
    const float2 xd = xs[ox * Q::XP + qq], yd = ys[oy * Q::XP + qq];
    const float* p = cq + __float_as_int(yd.x) + __float_as_int(xd.x);
    const float v00 = p[0], v01 = p[QB], v10 = p[RSC * QB], v11 = p[RSC * QB + QB];
    const float gx = __fsub_rn(1.f, xd.y), gy = __fsub_rn(1.f, yd.y);
    float r;
    if constexpr (ALT) {
      // correlation_kernel.cu:92-114's order, as alt_corr_mfma_kernel
      r = __fmul_rn(__fmul_rn(v00, gy), gx);
      r = __fadd_rn(r, __fmul_rn(__fmul_rn(v01, gy), xd.y));
      r = __fadd_rn(r, __fmul_rn(__fmul_rn(v10, yd.y), gx));
      r = __fadd_rn(r, __fmul_rn(__fmul_rn(v11, yd.y), xd.y));
      r = g.div_recip != 0.f ? r * g.div_recip : r / g.divisor;
    } else {
      const float nw = __fmul_rn(gy, gx), ne = __fmul_rn(gy, xd.y);
      const float sw = __fmul_rn(yd.y, gx), se = __fmul_rn(yd.y, xd.y);
      r = __fmul_rn(nw, v00);
      r = __builtin_fmaf(ne, v01, r);
      r = __builtin_fmaf(sw, v10, r);
      r = __builtin_fmaf(se, v11, r);
    }
    if ((XA & 2) == 0 || r == 12345.f) {
      if (g.out_nt) __builtin_nontemporal_store(r, op);
      else __hip_atomic_store(op, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    op += ostep;
  }
}

// ---------------------------------------------------------------------------
// Lookup backward (training: train.py:175-178 backpropagates through the
// grid_sample calls of core/utils/utils.py:65).  The gradient of one query's
// level-l image comes only from that query's (2r+1)^2 samples at level l, so a
// workgroup (QB queries x one level, as the forward) owns its windows: the
// bilinear transpose is accumulated in LDS and added into the gradient pyramid
// (same paged layout as the pyramid) with plain read-modify-writes, no atomics.
// The transpose is separable — every tap weight is the product of a row factor
// (1-fy or fy) and a column factor (1-fx or fx) of the forward — so per query
//   T[cy][ox]  = sum_oy  wy(oy, cy) * g[ox][oy]
//   dW[cy][cx] = sum_ox  T[cy][ox] * wx(ox, cx)
// a deterministic order (no LDS atomics).  Taps off the level get no gradient
// (zero padding); far and non-finite queries contribute nothing.
// ---------------------------------------------------------------------------
// Several lookups' backwards in one launch (round 3): a workgroup applies the
// sets in the given order, one read-modify-write pass each, so the result is
// the one-set launches' bit for bit; its window lines stay in L2 between passes,
// and the next set's coordinates and output gradient load during this pass's
// sums and stores.  Eight waves per SIMD (four workgroups per CU) beat six with
// no spill: 0.323 vs 0.337 ms for Sintel's 12 lookups (0.373 without the
// prefetch; scripts/ab_lookup_backward.sh).
constexpr int BW_MAX_SETS = 16;
struct BwSets {
  const float* coords[BW_MAX_SETS];
  const float* gout[BW_MAX_SETS];
  int n;
};

// Minimum waves per SIMD by radius: 8 (<= 64 VGPRs) up to r = 5 — r = 4 then
// keeps 44 B/lane in scratch (52 with the bound slots; r = 5: 0 / 12) and still
// ran faster than six waves without a spill (0.323 vs 0.337 ms, Sintel's 12
// lookups); r = 6 spilled 44 B/lane at that bound and r = 7 / 8 need 86 / 109
// VGPRs, so r >= 6 asks for 4 (<= 128 VGPRs, no spill).
// (BW_WAVES_SMALL_R: the experiments target rebuilds this file with another
// value for the r <= 5 bound; the product keeps 8)
#ifndef BW_WAVES_SMALL_R
#define BW_WAVES_SMALL_R 8
#endif
constexpr int bw_min_waves(int r) { return r <= 5 ? BW_WAVES_SMALL_R : 4; }

// BOUND: also add to bound_slots[workgroup] a bound on the magnitude of what this
// launch adds to the workgroup's cells: a cell hears from at most three samples
// per axis, each with a tap weight <= 1, so per set |added| <= 9 max|grad_out|
// over the workgroup's queries at its level (non-finite -> +inf).  The sets'
// maxima are summed in set order and the slot read-add-written (the workgroup
// owns it), so over zero-initialised slots the slots' maximum bounds max|G|
// after any number of launches: the gradient pyramid's magnitude bound the f16
// pair fmap-gradient GEMMs scale by (dxr_fmap_grads_bounded).  Taken from the
// output gradients as they arrive, off the read-modify-write path; deterministic.
template <int R, bool BOUND = false>
__global__ __launch_bounds__(512, bw_min_waves(R)) void corr_lookup_backward_kernel(BwSets sets,
                                                                   float* __restrict__ gpyr,
                                                                   LookupGeom g,
                                                                   float* __restrict__ bound_slots) {
  using C = WideCfg<R, 512>;
  constexpr int RD = C::RD, WD = C::WD, RS = C::RS, K = C::K, QB = C::QB, NT = C::NT;
  constexpr int XPB = QB + 1;              // tap-array pitch (wide_phase0_taps)
  __shared__ float4 xs[RD * XPB];
  __shared__ float4 ys[RD * XPB];
  __shared__ int2 org[QB];
  __shared__ float G[K * QB];              // [k][qq]
  __shared__ float T[QB * WD * RD];        // [qq][cy][ox]
  __shared__ float4 xq[QB * RD];           // xs query-major
  __shared__ unsigned wmax[BW_MAX_SETS];   // BOUND: float bits of each set's max |grad_out|

  const int l = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * QB;
  const LevelAddr A = g.lv[l];
  // a set's coordinates and output gradient, loaded a pass ahead
  constexpr int GIT = (K * QB + NT - 1) / NT;
  Phase0Coords<R, 512> cc;
  float gv[GIT];
  auto load_set = [&](int set) {
    const int t0 = threadIdx.x;
    wide_phase0_load<R, 512>(sets.coords[set], g, b, q0, t0, cc);
    const float* __restrict__ gout = sets.gout[set];
#pragma unroll
    for (int it = 0; it < GIT; ++it) {
      const int i = t0 + it * NT, k = i / QB, qq = i - k * QB, q = q0 + qq;
      gv[it] = (i < K * QB && q < g.N) ? gout[((long long)b * g.cout + (long long)l * K + k) * g.N + q]
                                       : 0.f;
    }
  };
  if (BOUND && threadIdx.x < BW_MAX_SETS) wmax[threadIdx.x] = 0u;   // published by the first barrier
  load_set(0);
  for (int set = 0; set < sets.n; ++set) {
  if (set > 0) {
    // the previous pass's stores are complete before any wave of the workgroup
    // reads them back (one CU, one L1: workgroup scope; an agent-scope fence
    // writes the XCD's L2 back and cost 5x the kernel)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  // thread-index arithmetic stays inside the pass (hoisted out of the set loop
  // it would hold ~100 VGPRs across passes and halve the resident workgroups)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  wide_phase0_taps<R, 512, 0, XPB>(cc, A, l, tid, xs, ys, org);
#pragma unroll
  for (int it = 0; it < GIT; ++it) {
    const int i = tid + it * NT;
    if (i < K * QB) G[i] = gv[it];
  }
  if constexpr (BOUND) {
    float m = 0.f;
#pragma unroll
    for (int it = 0; it < GIT; ++it) {
      const float a = __builtin_fabsf(gv[it]);   // padding slots hold 0
      m = a <= 3.40282347e38f ? __builtin_fmaxf(m, a) : __builtin_inff();
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = __builtin_fmaxf(m, __shfl_xor(m, o));
    if ((tid & 63) == 0) __hip_atomic_fetch_max(&wmax[set], __float_as_uint(m), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  if (set + 1 < sets.n) load_set(set + 1);  // in flight during this pass's sums and stores

  // Sample oy's taps sit on window rows row(oy) and row(oy)+1 with row(oy) in
  // {oy, oy+1} (row = floor_oy - min_j(floor_j - j)), so row cy hears only from
  // oy in {cy-2, cy-1, cy}: three candidates instead of all RD, in the same
  // ascending order (the skipped terms had weight 0, and 0 * inf/NaN gradients
  // no longer leak into untapped cells, as in grid_sample's backward).
  // query fastest across lanes: G and ys reads are lane-contiguous and the T
  // stores 90 floats apart (26 banks, all distinct); the (cy, ox)-fastest order
  // read G 288 floats apart and spent 82 % of the kernel's LDS cycles in conflicts
  for (int e = tid; e < QB * WD * RD; e += NT) {
    const int qq = e % QB, rem = e / QB;
    const int cy = rem / RD, ox = rem - cy * RD;
    float acc = 0.f;
#pragma unroll
    for (int d = 2; d >= 0; --d) {
      const int oy = cy - d;
      if (oy < 0 || oy >= RD) continue;
      const float4 yd = ys[oy * XPB + qq];
      const int row = __float_as_int(yd.x) / RS;
      if (row == cy || row + 1 == cy)
        acc = __builtin_fmaf(G[(ox * RD + oy) * QB + qq], row == cy ? yd.z : yd.y, acc);
    }
    T[(qq * WD + cy) * RD + ox] = acc;
  }
  // the x factors query-major for the column pass (lanes there walk a window row)
  for (int i = tid; i < RD * QB; i += NT) {
    const int ox = i / QB, qq = i - ox * QB;
    xq[qq * RD + ox] = xs[ox * XPB + qq];
  }
  __syncthreads();

  float* base = gpyr + A.off + ((long long)b * A.qt + (q0 >> A.lqb)) * A.qstride;
  const int qb0 = q0 & ((1 << A.lqb) - 1);
  // Every (query, cell) of the workgroup is a distinct gradient-pyramid element
  // (each query owns its images), so the read-modify-writes are independent:
  // all sums first, then all reads in flight together, then all writes
  // (round 2; one dependent round trip per element before).  Round 4: a thread
  // takes V consecutive cells of a window row (V = 4 on levels 0-2, whose tile
  // rows are >= 4 cells; 2 on level 3; 1 on row-major levels): one V-wide load
  // and store, the V + 2 column candidates read from LDS once.  Cells of the
  // vector outside the window or the level keep their old bits; each cell's sum
  // is the one-cell form's, term for term.
  auto colpass = [&](auto vtag) {
    constexpr int V = decltype(vtag)::value;
    constexpr int NGR = RS / V, NE = QB * WD * NGR, ITER = (NE + NT - 1) / NT;
    typedef float vf __attribute__((ext_vector_type(V)));
    vf accv[ITER];
    unsigned offv[ITER], okm[ITER];
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int e = tid + i * NT;
      okm[i] = 0u;
      offv[i] = 0u;
#pragma unroll
      for (int v = 0; v < V; ++v) accv[i][v] = 0.f;
      if (e >= NE) continue;
      const int qq = e / (WD * NGR), rem = e - qq * (WD * NGR);
      const int cy = rem / NGR, cx0 = (rem - cy * NGR) * V;
      const int2 o = org[qq];
      if (q0 + qq >= g.N || o.x == FAR_ORIGIN) continue;
      const int s0 = o.x & 3, c0 = cx0 - s0;   // window column of the vector's first cell
      const int yy = o.y + cy, xx0 = (o.x & ~3) + cx0;
      // xx0 is V-aligned: a vector starting left of the level lies wholly off it
      if ((unsigned)yy >= (unsigned)A.h || xx0 < 0 || xx0 >= A.w) continue;
      if (c0 + V <= 0 || c0 >= WD) continue;    // no window column in the vector
      const float* t = T + (qq * WD + cy) * RD;
      // col(ox) - s0 is ox or ox+1: window column c hears from ox in {c-2, c-1, c}
      float tk[V + 2];
      float4 xk[V + 2];
#pragma unroll
      for (int k = 0; k < V + 2; ++k) {
        const int ox = c0 - 2 + k;
        const bool in = ox >= 0 && ox < RD;
        tk[k] = in ? t[in ? ox : 0] : 0.f;
        xk[k] = in ? xq[qq * RD + (in ? ox : 0)] : make_float4(__int_as_float(-100), 0.f, 0.f, 0.f);
      }
      unsigned m = 0u;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int cx = cx0 + v, c = c0 + v;
        if (c < 0 || c >= WD || xx0 + v >= A.w) continue;
        float acc = 0.f;
#pragma unroll
        for (int d = 2; d >= 0; --d) {
          const int ox = c - d;
          if (ox < 0 || ox >= RD) continue;
          const float4 xd = xk[v + 2 - d];
          const int col = __float_as_int(xd.x);
          if (col == cx || col + 1 == cx) acc = __builtin_fmaf(tk[v + 2 - d], col == cx ? xd.z : xd.y, acc);
        }
        accv[i][v] = acc;
        m |= 1u << v;
      }
      okm[i] = m;
      offv[i] = (unsigned)(qb0 + qq) * (unsigned)A.S +
                ((unsigned)((yy >> A.lth) * A.tx + (xx0 >> A.ltw))) * (unsigned)A.pageS +
                (unsigned)((yy & A.mh) * A.tw + (xx0 & A.mw));
    }
    vf old[ITER];
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      if (okm[i]) {
        if constexpr (V == 1) old[i][0] = base[offv[i]];
        else old[i] = *reinterpret_cast<const vf*>(base + offv[i]);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) old[i][v] = 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      if (!okm[i]) continue;
      vf nv = old[i];
#pragma unroll
      for (int v = 0; v < V; ++v)
        if (okm[i] & (1u << v)) nv[v] = old[i][v] + accv[i][v];
      if constexpr (V == 1) base[offv[i]] = nv[0];
      else *reinterpret_cast<vf*>(base + offv[i]) = nv;
    }
  };
  if (A.lth == 30) colpass(std::integral_constant<int, 1>{});
  else if (A.tw >= 4) colpass(std::integral_constant<int, 4>{});
  else if (A.tw == 2) colpass(std::integral_constant<int, 2>{});
  else colpass(std::integral_constant<int, 1>{});
  }
  if constexpr (BOUND) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const long long w = blockIdx.x + (long long)gridDim.x * (blockIdx.y + (long long)gridDim.y * blockIdx.z);
      float t = bound_slots[w];
      for (int k = 0; k < sets.n; ++k) t += 9.f * __uint_as_float(wmax[k]);
      bound_slots[w] = t;
    }
  }
}

template <int R>
dim3 lookup_backward_grid(const LookupGeom& g, int B) {
  using W = WideCfg<R, 512>;
  return dim3((unsigned)((g.N + W::QB - 1) / W::QB), (unsigned)g.levels, (unsigned)B);
}

template <int R>
int launch_lookup_backward_r(const BwSets& sets, float* gpyr, const LookupGeom& g, int B,
                             float* bound_slots, hipStream_t stream) {
  const dim3 grid = lookup_backward_grid<R>(g, B);
  if (bound_slots)
    hipLaunchKernelGGL((corr_lookup_backward_kernel<R, true>), grid, dim3(512), 0, stream, sets, gpyr,
                       g, bound_slots);
  else
    hipLaunchKernelGGL((corr_lookup_backward_kernel<R, false>), grid, dim3(512), 0, stream, sets,
                       gpyr, g, bound_slots);
  return dxr::launch_status();
}

// Round-5 product launcher of the wide kernel (kept for the experiments target).
// Workgroup shape: 512 threads x 32 queries (4 resident per CU), or — when that
// grid fits in one dispatch round (<= 1024 workgroups: Sintel / Chairs B=1) —
// 256 threads x 16 queries, the same 16 threads per query in twice the
// workgroups, so the per-CU load evens out (3.44 -> 6.9 workgroups per CU at
// Sintel B=1: one CU in four no longer runs a fourth workgroup after the rest).
// Round 3, same-process A/B (bit-identical): Sintel B=1 8.0 -> 7.4 us, Chairs
// 5.6 -> 5.2 us; multi-round grids keep 512 x 32 (Sintel B=8 50.4 vs 53.3 us).
// Output store policy (round 5, same-process A/Bs in the step, scripts/ab_step.py,
// profiles/r05/experiments/r6e_lookup_output_nt.jsonl): non-temporal stores
// gained 2-9 % per step wherever a wave stores whole lines (the 512 x 32 shape: 32
// consecutive queries of a channel = 128 B; Sintel B=8 -2.3 %, KITTI B=8 bf16
// -5.6 %, Chairs B=4 -8.9 %, Sintel B=2 -2.3 %) and with the 256 x 16 shape
// (64-B segments) when those are half-line aligned (N % 32 == 0: Sintel B=1 f32
// -4.0 %, bf16 -4.4 %); with misaligned 64-B segments (KITTI, Chairs at B=1)
// write-through stores, which L2 merges, were 2-12 % faster — except with a large
// pyramid (>= 128 MB: KITTI B=1, 286 MB f32 / 143 MB bf16), where the 512 x 32 shape
// with non-temporal stores beat both (-6.3 % / -3.9 %, r6k); a small one (Chairs
// B=1, 43 MB, resident anyway) keeps 256 x 16 with write-through (+13 % otherwise).
template <int R, typename PT>
int launch_lookup_wide_r(const PT* pyr, const float* coords, float* out, const LookupGeom& g0, int B,
                    hipStream_t stream) {
  using W = WideCfg<R>;
  LookupGeom g = g0;
  const long long wg32 = (long long)((g.N + W::QB - 1) / W::QB) * g.levels * B;
  // pyramid bytes as the build's store rule counts them (dma_stream_out): padded
  // level-0 pages (qt x 128 queries x whole tiles), x 4/3 for levels 1-3
  const double pyr_bytes = (double)B * g.lv[0].qt * (double)g.lv[0].qstride * sizeof(PT) * (4.0 / 3.0);
  const bool big_misaligned = g.N % 32 != 0 && pyr_bytes >= 128.0 * (1 << 20);
  if (R <= 4 && wg32 <= 1024 && !big_misaligned) {
    using S = WideCfg<R, 256, 16>;
    g.out_nt = g.N % 32 == 0 ? 1 : 0;
    const dim3 grid((unsigned)((g.N + S::QB - 1) / S::QB), (unsigned)g.levels, (unsigned)B);
    hipLaunchKernelGGL((corr_lookup_wide_kernel<R, PT, 256, 16>), grid, dim3(256), 0, stream, pyr,
                       coords, out, g);
    return dxr::launch_status();
  }
  g.out_nt = 1;
  const dim3 grid((unsigned)((g.N + W::QB - 1) / W::QB), (unsigned)g.levels, (unsigned)B);
  hipLaunchKernelGGL((corr_lookup_wide_kernel<R, PT>), grid, dim3(W::NT), 0, stream, pyr, coords,
                     out, g);
  return dxr::launch_status();
}

// The product lookup (round 6): the query-minor kernel with the round-5 shape
// and output policy below (launch_lookup_wide_r).  One-round grids (256 x 16)
// load their window vectors with plain global loads, multi-round grids (512 x
// 32) with range-checked buffer loads (BUF; the loads need no branch).  Same
// process, in the step (build + 12 lookups, scripts/ab_step.py, outputs checked
// bit-identical; profiles/r06/experiments/r6d_*): Sintel B=1 184.9 -> 177.0 us
// (plain) / 178.8 (buffer), B=8 1,288.4 -> 1,280.1 / 1,258.0, KITTI B=8 bf16
// 913.1 -> 884.6 / 854.0, 1080p full 2,176 -> 2,170 / 2,149, Chairs 98.2 -> 96.4
// / 97.4, Sintel B=2 348.2 -> 355.6 / 349.7.  `ONE_QB` / `UNR` / `MULTI_BUF`:
// experiment knobs (queries per one-round workgroup, phase-2 unroll, buffer loads
// on multi-round grids); `ONE_BUF`: buffer loads on one-round grids too.
template <int R, typename PT, int ONE_QB = 16, int UNR = 1, bool ONE_BUF = false, bool MULTI_BUF = true,
          int XA = 0, int MULTI_NT = 512, int MULTI_QB = 0>
int launch_lookup_r(const PT* pyr, const float* coords, float* out, const LookupGeom& g0, int B,
                       hipStream_t stream) {
  using W = WideCfg<R>;
  LookupGeom g = g0;
  const long long wg32 = (long long)((g.N + W::QB - 1) / W::QB) * g.levels * B;
  const double pyr_bytes = (double)B * g.lv[0].qt * (double)g.lv[0].qstride * sizeof(PT) * (4.0 / 3.0);
  const bool big_misaligned = g.N % 32 != 0 && pyr_bytes >= 128.0 * (1 << 20);
  if (R <= 4 && wg32 <= 1024 && !big_misaligned) {
    g.out_nt = g.N % 32 == 0 ? 1 : 0;
    const dim3 grid((unsigned)((g.N + ONE_QB - 1) / ONE_QB), (unsigned)g.levels, (unsigned)B);
    hipLaunchKernelGGL((corr_lookup_qm_kernel<R, PT, 256, ONE_QB, UNR, ONE_BUF, XA>), grid, dim3(256), 0, stream, pyr,
                       coords, out, g);
    return dxr::launch_status();
  }
  g.out_nt = 1;
  constexpr int MQB = MULTI_QB ? MULTI_QB : W::QB;
  const dim3 grid((unsigned)((g.N + MQB - 1) / MQB), (unsigned)g.levels, (unsigned)B);
  hipLaunchKernelGGL((corr_lookup_qm_kernel<R, PT, MULTI_NT, MQB, UNR, MULTI_BUF, XA>), grid,
                     dim3(MULTI_NT), 0, stream, pyr, coords, out, g);
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

// ---------------------------------------------------------------------------
// Lookup fused with the motion encoder's first 1x1 convolution (SURVEY.md
// §8(f) row 2):
//   out[b, o, q] = act(bias[o] + sum_c Wt[o, c] * corr[b, c, q])
// where corr is this file's lookup output (channel c = l*(2r+1)^2 + ix*(2r+1) + iy,
// core/corr.py:29-50) and Wt the convc1 weight of core/update.py:83 / :90
// (BasicMotionEncoder, F.relu(self.convc1(corr)), 324 -> 256) or :66 / :71
// (SmallMotionEncoder, 196 -> 96).  The reference writes the 9.1 MB lookup
// tensor (Sintel), reads it back in the convolution and writes the conv output
// before a separate ReLU pass; here the lookup vector of a query never leaves
// the CU.
//
// One workgroup = 32 query pixels, 8 waves.  Per level: the lookup's phase 0
// and phase 1 (the forward kernel's code), then phase 2 computes the samples
// with the same arithmetic (bit-identical values) and stores each as an exact
// hi/mid/lo bf16 split into LDS planes [plane][k/8][query][8] — the B operand
// of v_mfma_f32_32x32x16_bf16 as it stands.  Then a (Cout x 32 x Cin) GEMM on
// the matrix cores, f32 class like the build (six bf16 products per f32
// product, small terms first, f32 accumulation): wave w owns output rows
// 32w.., its A operand the pre-split weight planes (dxr_conv1x1_split_weight,
// [plane][k/8][Cout] uint4, hot in L2), bias + ReLU in registers, coalesced
// 128-B stores along queries into [B, Cout, H, W].
// ---------------------------------------------------------------------------
typedef __bf16 mbf8 __attribute__((ext_vector_type(8)));
typedef float mf16 __attribute__((ext_vector_type(16)));

template <int R>
struct MotionCfg {
  using C = WideCfg<R, 512>;
  static constexpr int LMAX = 4;                          // levels staged in LDS
  static constexpr int KP = (LMAX * C::K + 15) & ~15;     // input channels, padded to k steps
  static constexpr int KB = KP / 8;                       // 8-channel blocks
  static constexpr int NKS = KP / 16;                     // k steps
  static_assert(C::QB == 32, "one 32-query MFMA column block per workgroup");
};

// hi / mid / lo bf16 bits of x (each round-to-nearest; x = hi + mid + lo exactly
// for finite x up to the bf16 range of the residuals).
__device__ __forceinline__ void split3(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = dxr::f32_to_bf16(x);
  const float r1 = __fsub_rn(x, dxr::bf16_to_f32(h));
  m = dxr::f32_to_bf16(r1);
  l = dxr::f32_to_bf16(__fsub_rn(r1, dxr::bf16_to_f32(m)));
}

// The convc1 weight [Cout, Cin] f32 rearranged as [Cin_pad/8][Cout][8] (zero
// padded): one k step of a lane's A operand is 32 contiguous bytes.  Kept in
// f32 and split in registers by the fused kernel: 4 bytes per weight streamed
// from L2 instead of 6 for pre-split planes (the stream is the GEMM's bound:
// ~70 GB/s of L2 reads per CU, MI355X_MICROARCH.md "gather into LDS").
// Round 2: the same [Cin_pad/8][Cout][8] layout twice — f32 (the 3-way bf16
// fallback's operand) and then f16 pairs (8 x f16 hi, 8 x f16 lo in the same 32
// bytes: the f16-pair GEMM's operand, split once here instead of per k step).
__device__ __forceinline__ void lk_split8h(const float (&x)[8], uint4& h, uint4& l) {
  typedef _Float16 h2t __attribute__((ext_vector_type(2)));
  typedef float f2t __attribute__((ext_vector_type(2)));
  uint32_t hh[4], ll[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const f2t v = {x[2 * e], x[2 * e + 1]};
    hh[e] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, h2t));
    const h2t hv = __builtin_bit_cast(h2t, hh[e]);
    const f2t r = {(x[2 * e] - (float)hv[0]) * 2048.f, (x[2 * e + 1] - (float)hv[1]) * 2048.f};
    ll[e] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, h2t));
  }
  h = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  l = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

__global__ __launch_bounds__(256) void conv1x1_pack_weight_kernel(const float* __restrict__ w,
                                                                  int cout, int cin, int kbw,
                                                                  float4* __restrict__ packed) {
  const int u = blockIdx.x * 256 + threadIdx.x;
  if (u >= kbw * cout) return;
  const int kb = u / cout, o = u - kb * cout;
  float x[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = kb * 8 + e;
    x[e] = c < cin ? w[(long long)o * cin + c] : 0.f;
  }
  packed[2LL * u] = make_float4(x[0], x[1], x[2], x[3]);
  packed[2LL * u + 1] = make_float4(x[4], x[5], x[6], x[7]);
  uint4 h, l;
  lk_split8h(x, h, l);
  uint4* pairs = reinterpret_cast<uint4*>(packed + 2LL * kbw * cout);
  pairs[2LL * u] = h;
  pairs[2LL * u + 1] = l;
}

// ---------------------------------------------------------------------------
// Round-2 form: two workgroups per CU.  The r01 kernel staged all four levels'
// tap data and kept three bf16 sample planes (125 KB of LDS: one workgroup per
// CU, both halves latency-bound).  Here phase 0 runs per level just before its
// gather (one level's tap data), the samples stay f32 in LDS (43 KB, split into
// f16 pairs per k step in registers) and the weights arrive pre-split as f16
// pairs (dxr_conv1x1_pack_weight): ~76 KB, so one workgroup's GEMM overlaps the
// other's gathers.  The GEMM runs on the f16 pair split (3 products, cross terms
// in a second accumulator, as the split build); a workgroup whose sums are not
// finite re-runs the GEMM on the 3-way bf16 split from the f32 samples and the
// f32 weight copy.  Samples are the lookup's, bit for bit.
// ---------------------------------------------------------------------------
typedef _Float16 mh8 __attribute__((ext_vector_type(8)));

template <int R, typename PT, int NT = 512, int PF = 4>
__global__ __launch_bounds__(NT, 4) void corr_lookup_conv1x1_h2_kernel(
    const PT* __restrict__ pyr, const float* __restrict__ coords, const float4* __restrict__ wpk,
    const float* __restrict__ bias, float* __restrict__ out, LookupGeom g, int cout, int relu) {
  using C = WideCfg<R, NT>;
  using M = MotionCfg<R>;
  constexpr int RD = C::RD, RS = C::RS, K = C::K, QB = C::QB, KB = M::KB;
  constexpr int NW = NT / 64, KSPLIT = NW >= 16 ? 2 : 1;
  static_assert(NW == 8 || NW == 16, "8 output blocks of 32 per pass");
  constexpr int XPB = QB + 1;   // tap-array pitch (wide_phase0_taps)
  constexpr int CELLS_B = QB * C::QS * 4, XS_B = RD * XPB * 16, ORG_B = QB * 8;
  constexpr int STAGE_B = CELLS_B + 2 * XS_B + ORG_B, RED_B = KSPLIT > 1 ? 8 * 16 * 64 * 4 : 0;
  __shared__ __attribute__((aligned(16))) char stage[STAGE_B > RED_B ? STAGE_B : RED_B];
  __shared__ __attribute__((aligned(16))) float spl[KB * QB * 8];   // samples [k/8][q][8], f32
  __shared__ int nonfinite;
  float* cells = reinterpret_cast<float*>(stage);
  float4* xs = reinterpret_cast<float4*>(stage + CELLS_B);
  float4* ys = reinterpret_cast<float4*>(stage + CELLS_B + XS_B);
  int2* org = reinterpret_cast<int2*>(stage + CELLS_B + 2 * XS_B);
  float* red = reinterpret_cast<float*>(stage);

  const int tid = threadIdx.x;
  const int b = blockIdx.y;
  const int q0 = blockIdx.x * QB;
  const int cin = g.cout;
  const int kpad = (cin + 15) & ~15;
  const int lane = tid & 63, wave = tid >> 6, j = lane & 31, kh = lane >> 5;
  const int wob = wave & 7, khalf = wave >> 3;
  const int nks = kpad / 16;
  const int kbeg = khalf * nks / KSPLIT, kend = (khalf + 1) * nks / KSPLIT;
  const int nob = cout / 32;
  const int kbw = nks * 2;
  const uint4* wpair = reinterpret_cast<const uint4*>(wpk + 2LL * kbw * cout);

  if (tid == 0) nonfinite = 0;
  for (int i = tid; i < QB * (kpad - cin); i += NT) {      // channel padding: zeros
    const int np = kpad - cin, qq = i / np, c = cin + i - qq * np;
    spl[((c >> 3) * QB + qq) * 8 + (c & 7)] = 0.f;
  }
  // ---- per level: phase 0, gather, samples -> spl
  for (int l = 0; l < g.levels; ++l) {
    const LevelAddr& A = g.lv[l];
    wide_phase0<R, NT, 0, XPB>(coords, g, A, b, l, q0, tid, xs, ys, org);
    __syncthreads();
    {
      float4 win[C::VIT];
      const PT* base = pyr + A.off + ((long long)b * A.qt + (q0 >> A.lqb)) * A.qstride;
      const int qb0 = q0 & ((1 << A.lqb) - 1);
      if (l < 2) {
        gather_load<R, NT, 4>(base, qb0, A, org, q0, g.N, tid, win);
        gather_store<R, NT>(win, cells, tid);
      } else {   // levels 2/3: query-major slots, as the lookup
        if (l == 2)
          gather_load<R, NT, 4, PT, true>(base, qb0, A, org, q0, g.N, tid, win);
        else
          gather_load<R, NT, 2, PT, true>(base, qb0, A, org, q0, g.N, tid, win);
        gather_store<R, NT, true>(win, cells, tid);
      }
    }
    __syncthreads();
    {
      const int qq = tid % QB, cls = tid / QB;
      const bool live = q0 + qq < g.N;
      const float* cq = cells + qq * C::QS;
      for (int k = cls; k < K; k += C::NCLS) {
        const int ox = k / RD, oy = k - ox * RD;
        const float4 xd = xs[ox * XPB + qq], yd = ys[oy * XPB + qq];
        const float* p = cq + __float_as_int(yd.x) + __float_as_int(xd.x);
        const float v00 = p[0], v01 = p[1], v10 = p[RS], v11 = p[RS + 1];
        const float nw = __fmul_rn(yd.z, xd.z), ne = __fmul_rn(yd.z, xd.y);
        const float sw = __fmul_rn(yd.y, xd.z), se = __fmul_rn(yd.y, xd.y);
        float r = __fmul_rn(nw, v00);
        r = __builtin_fmaf(ne, v01, r);
        r = __builtin_fmaf(sw, v10, r);
        r = __builtin_fmaf(se, v11, r);
        if (!live) r = 0.f;                // queries past N: finite zeros
        const int c = l * K + k;
        spl[((c >> 3) * QB + qq) * 8 + (c & 7)] = r;
      }
    }
    __syncthreads();   // the next level rewrites xs / ys / org / cells
  }

  // ---- (Cout x 32 queries x Cin) GEMM: f16 pairs, then (rarely) the 3-way bf16 split
  const int q = q0 + j;
  auto gemm = [&](auto mode) {
    constexpr bool M2 = decltype(mode)::value;
    for (int ob0 = 0; ob0 < nob; ob0 += 8) {   // uniform trip count: barriers inside
      const int ob = ob0 + wob;
      const bool act = ob < nob;
      mf16 acc, acc2;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = acc2[r] = 0.f;
      if (act) {
        uint4 wb[PF][2];
        auto wload = [&](uint4* dst, int ks) {
          const long long u = 2 * ((long long)(2 * ks + kh) * cout + ob * 32 + j);
          if constexpr (M2) {
            dst[0] = wpair[u];
            dst[1] = wpair[u + 1];
          } else {
            dst[0] = __builtin_bit_cast(uint4, wpk[u]);
            dst[1] = __builtin_bit_cast(uint4, wpk[u + 1]);
          }
        };
#pragma unroll
        for (int sl = 0; sl < PF; ++sl) wload(wb[sl], min(kbeg + sl, kend - 1));
        auto kstep = [&](int ks, int sl, bool refill) {
          __builtin_amdgcn_sched_barrier(0);
          const int kb = 2 * ks + kh;
          const float4* sp = reinterpret_cast<const float4*>(spl + ((long long)kb * QB + j) * 8);
          const float4 sa = sp[0], sb = sp[1];
          const float xq[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
          if constexpr (M2) {
            uint4 qh4, ql4;
            lk_split8h(xq, qh4, ql4);
            const mh8 th = __builtin_bit_cast(mh8, wb[sl][0]), tl = __builtin_bit_cast(mh8, wb[sl][1]);
            if (refill) wload(wb[sl], min(ks + PF, kend - 1));
            const mh8 qh = __builtin_bit_cast(mh8, qh4), ql = __builtin_bit_cast(mh8, ql4);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, qh, acc2, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ql, acc2, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, qh, acc, 0, 0, 0);
          } else {
            uint4 wh, wm, wl, qh4, qm4, ql4;
            {
              const float4 a = __builtin_bit_cast(float4, wb[sl][0]);
              const float4 c = __builtin_bit_cast(float4, wb[sl][1]);
              const float x[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
              dxr::split8(x, wh, wm, wl);
            }
            dxr::split8(xq, qh4, qm4, ql4);
            if (refill) wload(wb[sl], min(ks + PF, kend - 1));
            const mbf8 th = __builtin_bit_cast(mbf8, wh), tm = __builtin_bit_cast(mbf8, wm),
                       tl = __builtin_bit_cast(mbf8, wl);
            const mbf8 qh = __builtin_bit_cast(mbf8, qh4), qm = __builtin_bit_cast(mbf8, qm4),
                       ql = __builtin_bit_cast(mbf8, ql4);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tm, qm, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tl, qh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, ql, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tm, qh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, qm, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(th, qh, acc, 0, 0, 0);
          }
        };
        const int nfull = kbeg + (kend - kbeg) / PF * PF;
#pragma unroll 1
        for (int k0 = kbeg; k0 < nfull; k0 += PF) {
#pragma unroll
          for (int sl = 0; sl < PF; ++sl) kstep(k0 + sl, sl, true);
        }
#pragma unroll
        for (int sl = 0; sl < PF; ++sl)
          if (nfull + sl < kend) kstep(nfull + sl, sl, false);
        if constexpr (M2) {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] = __builtin_fmaf(acc2[r], 0x1p-11f, acc[r]);
        }
      }
      if constexpr (KSPLIT > 1) {
        if (khalf == 1 && act) {
#pragma unroll
          for (int r = 0; r < 16; ++r) red[(wob * 16 + r) * 64 + lane] = acc[r];
        }
        __syncthreads();
        if (khalf == 0 && act) {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] += red[(wob * 16 + r) * 64 + lane];
        }
        __syncthreads();
      }
      if (khalf == 0 && act && q < g.N) {
        if constexpr (M2) {
          bool bad = false;
#pragma unroll
          for (int r = 0; r < 16; ++r) bad |= !(__builtin_fabsf(acc[r]) <= 3.40282347e38f);
          if (bad) nonfinite = 1;
        }
        float* ob_out = out + (long long)b * cout * g.N + q;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int orow = ob * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
          float v = acc[r] + (bias ? bias[orow] : 0.f);
          if (relu && v < 0.f) v = 0.f;      // NaN stays NaN, as torch.relu
          ob_out[(long long)orow * g.N] = v;
        }
      }
    }
  };
  gemm(std::integral_constant<bool, true>{});
  __syncthreads();
  if (nonfinite) gemm(std::integral_constant<bool, false>{});   // workgroup-uniform
}

template <int R, typename PT>
int launch_lookup_conv1x1_r(const PT* pyr, const float* coords, const float4* wpl,
                            const float* bias, float* out, const LookupGeom& g, int B, int cout,
                            int relu, hipStream_t stream) {
  using C = WideCfg<R, 1024>;
  if (g.cout > MotionCfg<R>::KP) return DXR_EUNSUPPORTED;
  const dim3 grid((unsigned)((g.N + C::QB - 1) / C::QB), (unsigned)B);
  // Grids up to one workgroup per CU (Sintel B=1: 220) run the 1024-thread form
  // (more waves per workgroup: 24 vs 26 us); larger grids the 512-thread form,
  // ~76 KB LDS and 128 VGPRs, two workgroups per CU (Sintel B=2: 35 vs 47 us,
  // KITTI-shape B=8: 136 vs 190 us; r01 kernel 52 / 214 us).
  if ((long long)grid.x * grid.y <= 256)
    hipLaunchKernelGGL((corr_lookup_conv1x1_h2_kernel<R, PT, 1024, 4>), grid, dim3(1024), 0,
                       stream, pyr, coords, wpl, bias, out, g, cout, relu);
  else
    hipLaunchKernelGGL((corr_lookup_conv1x1_h2_kernel<R, PT, 512, 4>), grid, dim3(512), 0, stream,
                       pyr, coords, wpl, bias, out, g, cout, relu);
  return dxr::launch_status();
}

template <typename PT>
int launch_lookup_conv1x1(const PT* pyr, const float* coords, const float4* wpl, const float* bias,
                          float* out, const LookupGeom& g, int B, int radius, int cout, int relu,
                          hipStream_t stream) {
  switch (radius) {
    case 3: return launch_lookup_conv1x1_r<3, PT>(pyr, coords, wpl, bias, out, g, B, cout, relu, stream);
    case 4: return launch_lookup_conv1x1_r<4, PT>(pyr, coords, wpl, bias, out, g, B, cout, relu, stream);
    default: return DXR_EUNSUPPORTED;
  }
}

}  // namespace

namespace {
// The alternate block's coarse levels from their volumes (dxr_alt_coarse_volumes),
// levels [first, num_levels): launch_lookup_r's shapes and output policy.
template <int R>
int launch_alt_volume_r(const float* vol, const float* coords, float* out, const LookupGeom& g0,
                        int first, int B, hipStream_t stream) {
  using W = WideCfg<R>;
  LookupGeom g = g0;
  const int nl = g.levels - first;
  const long long wg32 = (long long)((g.N + W::QB - 1) / W::QB) * nl * B;
  if (R <= 4 && wg32 <= 1024) {
    g.out_nt = g.N % 32 == 0 ? 1 : 0;
    const dim3 grid((unsigned)((g.N + 15) / 16), (unsigned)nl, (unsigned)B);
    hipLaunchKernelGGL((corr_lookup_qm_kernel<R, float, 256, 16, 1, false, 0, true>), grid, dim3(256), 0,
                       stream, vol, coords, out, g);
    return dxr::launch_status();
  }
  g.out_nt = 1;
  const dim3 grid((unsigned)((g.N + W::QB - 1) / W::QB), (unsigned)nl, (unsigned)B);
  hipLaunchKernelGGL((corr_lookup_qm_kernel<R, float, 512, W::QB, 1, true, 0, true>), grid, dim3(512), 0,
                     stream, vol, coords, out, g);
  return dxr::launch_status();
}
}  // namespace

extern "C" int dxr_alt_volume_lookup(const float* volumes, const float* coords, float* out,
                                     int64_t B, int64_t H, int64_t W, int num_levels,
                                     int first_level, int radius, float divisor,
                                     hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L) || first_level < 0 || first_level >= num_levels)
    return DXR_EINVAL;
  if (radius < 0 || !(divisor == divisor) || divisor == 0.f) return DXR_EINVAL;
  if (radius > 8) return DXR_EUNSUPPORTED;
  if (B > 65535) return DXR_EINVAL;
  if (B == 0) return DXR_OK;
  if (!volumes || !coords || !out) return DXR_EINVAL;
  const int rd = 2 * radius + 1;
  LookupGeom g;
  g.N = (int)(H * W);
  g.levels = num_levels;
  g.cout = num_levels * rd * rd;
  g.l0 = first_level;
  g.divisor = divisor;
  {
    int e;
    const float m = std::frexp(divisor, &e);
    g.div_recip = (m == 0.5f && e > -125 && e < 126) ? 1.f / divisor : 0.f;   // exact: a power of two
  }
  for (int l = 0; l < L.n; ++l) {
    g.lv[l] = level_addr(L.lay[l]);
    g.lv[l].off -= L.off[first_level];
  }
  switch (radius) {
    case 0: return launch_alt_volume_r<0>(volumes, coords, out, g, first_level, (int)B, stream);
    case 1: return launch_alt_volume_r<1>(volumes, coords, out, g, first_level, (int)B, stream);
    case 2: return launch_alt_volume_r<2>(volumes, coords, out, g, first_level, (int)B, stream);
    case 3: return launch_alt_volume_r<3>(volumes, coords, out, g, first_level, (int)B, stream);
    case 4: return launch_alt_volume_r<4>(volumes, coords, out, g, first_level, (int)B, stream);
    case 5: return launch_alt_volume_r<5>(volumes, coords, out, g, first_level, (int)B, stream);
    case 6: return launch_alt_volume_r<6>(volumes, coords, out, g, first_level, (int)B, stream);
    case 7: return launch_alt_volume_r<7>(volumes, coords, out, g, first_level, (int)B, stream);
    case 8: return launch_alt_volume_r<8>(volumes, coords, out, g, first_level, (int)B, stream);
    default: return DXR_EUNSUPPORTED;
  }
}

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

namespace {
int lookup_backward(const BwSets& sets, int64_t B, int64_t H, int64_t W, int num_levels, int radius,
                    void* grad_pyramid, int grad_dtype, float* bound_slots, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L)) return DXR_EINVAL;
  if (radius < 0) return DXR_EINVAL;
  if (radius > 8) return DXR_EUNSUPPORTED;
  if (grad_dtype != DXR_F32) return grad_dtype == DXR_BF16 ? DXR_EUNSUPPORTED : DXR_EINVAL;
  if (B > 65535 || H * W > (1LL << 30)) return DXR_EINVAL;
  if (B == 0 || sets.n == 0) return DXR_OK;
  if (!grad_pyramid) return DXR_EINVAL;
  for (int i = 0; i < sets.n; ++i)
    if (!sets.coords[i] || !sets.gout[i]) return DXR_EINVAL;
  const int rd = 2 * radius + 1;
  LookupGeom g;
  g.N = (int)(H * W);
  g.levels = num_levels;
  g.cout = num_levels * rd * rd;
  for (int l = 0; l < L.n; ++l) g.lv[l] = level_addr(L.lay[l]);
  float* gp = static_cast<float*>(grad_pyramid);
  switch (radius) {
    case 0: return launch_lookup_backward_r<0>(sets, gp, g, (int)B, bound_slots, stream);
    case 1: return launch_lookup_backward_r<1>(sets, gp, g, (int)B, bound_slots, stream);
    case 2: return launch_lookup_backward_r<2>(sets, gp, g, (int)B, bound_slots, stream);
    case 3: return launch_lookup_backward_r<3>(sets, gp, g, (int)B, bound_slots, stream);
    case 4: return launch_lookup_backward_r<4>(sets, gp, g, (int)B, bound_slots, stream);
    case 5: return launch_lookup_backward_r<5>(sets, gp, g, (int)B, bound_slots, stream);
    case 6: return launch_lookup_backward_r<6>(sets, gp, g, (int)B, bound_slots, stream);
    case 7: return launch_lookup_backward_r<7>(sets, gp, g, (int)B, bound_slots, stream);
    default: return launch_lookup_backward_r<8>(sets, gp, g, (int)B, bound_slots, stream);
  }
}
}  // namespace

extern "C" int dxr_corr_lookup_backward(const float* coords, const float* grad_out, int64_t B,
                                        int64_t H, int64_t W, int num_levels, int radius,
                                        void* grad_pyramid, int grad_dtype, hipStream_t stream) {
  BwSets sets{};
  sets.coords[0] = coords;
  sets.gout[0] = grad_out;
  sets.n = 1;
  return lookup_backward(sets, B, H, W, num_levels, radius, grad_pyramid, grad_dtype, nullptr,
                         stream);
}

extern "C" int dxr_corr_lookup_backward_multi(const float* const* coords, const float* const* grad_out,
                                              int n_sets, int64_t B, int64_t H, int64_t W,
                                              int num_levels, int radius, void* grad_pyramid,
                                              int grad_dtype, hipStream_t stream) {
  if (n_sets < 0) return DXR_EINVAL;
  if (n_sets > BW_MAX_SETS) return DXR_EUNSUPPORTED;
  if (n_sets > 0 && (!coords || !grad_out)) return DXR_EINVAL;
  BwSets sets{};
  for (int i = 0; i < n_sets; ++i) {
    sets.coords[i] = coords[i];
    sets.gout[i] = grad_out[i];
  }
  sets.n = n_sets;
  return lookup_backward(sets, B, H, W, num_levels, radius, grad_pyramid, grad_dtype, nullptr,
                         stream);
}

extern "C" int64_t dxr_lookup_backward_bound_slots(int64_t B, int64_t H, int64_t W, int num_levels,
                                                   int radius) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L) || radius < 0 || radius > 8) return -1;
  if (B > 65535 || H * W > (1LL << 30)) return -1;
  LookupGeom g;
  g.N = (int)(H * W);
  g.levels = num_levels;
  dim3 d;
  switch (radius) {
    case 0: d = lookup_backward_grid<0>(g, (int)B); break;
    case 1: d = lookup_backward_grid<1>(g, (int)B); break;
    case 2: d = lookup_backward_grid<2>(g, (int)B); break;
    case 3: d = lookup_backward_grid<3>(g, (int)B); break;
    case 4: d = lookup_backward_grid<4>(g, (int)B); break;
    case 5: d = lookup_backward_grid<5>(g, (int)B); break;
    case 6: d = lookup_backward_grid<6>(g, (int)B); break;
    case 7: d = lookup_backward_grid<7>(g, (int)B); break;
    default: d = lookup_backward_grid<8>(g, (int)B); break;
  }
  return (int64_t)d.x * d.y * d.z;
}

extern "C" int dxr_corr_lookup_backward_multi_bound(const float* const* coords,
                                                    const float* const* grad_out, int n_sets,
                                                    int64_t B, int64_t H, int64_t W, int num_levels,
                                                    int radius, void* grad_pyramid, int grad_dtype,
                                                    float* bound_slots, hipStream_t stream) {
  if (n_sets < 0) return DXR_EINVAL;
  if (n_sets > BW_MAX_SETS) return DXR_EUNSUPPORTED;
  if (n_sets > 0 && (!coords || !grad_out)) return DXR_EINVAL;
  if (!bound_slots) return DXR_EINVAL;
  BwSets sets{};
  for (int i = 0; i < n_sets; ++i) {
    sets.coords[i] = coords[i];
    sets.gout[i] = grad_out[i];
  }
  sets.n = n_sets;
  return lookup_backward(sets, B, H, W, num_levels, radius, grad_pyramid, grad_dtype, bound_slots,
                         stream);
}

extern "C" int64_t dxr_conv1x1_packed_bytes(int64_t cout, int64_t cin) {
  if (cout < 1 || cin < 1) return -1;
  return ((cin + 15) / 16 * 16) * cout * 4 * 2;   // f32 copy + f16-pair copy
}

extern "C" int dxr_conv1x1_pack_weight(const float* weight, int64_t cout, int64_t cin,
                                       void* packed, hipStream_t stream) {
  if (cout < 1 || cin < 1 || cout > (1 << 20) || cin > (1 << 20)) return DXR_EINVAL;
  if (!weight || !packed) return DXR_EINVAL;
  const int kbw = (int)((cin + 15) / 16 * 2);
  const long long units = (long long)kbw * cout;
  hipLaunchKernelGGL(conv1x1_pack_weight_kernel, dim3((unsigned)((units + 255) / 256)), dim3(256),
                     0, stream, weight, (int)cout, (int)cin, kbw, static_cast<float4*>(packed));
  return dxr::launch_status();
}

extern "C" int dxr_corr_lookup_conv1x1(const void* pyramid, int pyr_dtype, int64_t B, int64_t H,
                                       int64_t W, int num_levels, int radius, const float* coords,
                                       const void* weight_packed, const float* bias, int64_t cout,
                                       int relu, float* out, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L)) return DXR_EINVAL;
  if (radius < 0 || cout < 1) return DXR_EINVAL;
  if (radius != 3 && radius != 4) return DXR_EUNSUPPORTED;
  if (num_levels > 4 || cout % 32 != 0 || cout > 4096) return DXR_EUNSUPPORTED;
  if (B > 65535 || H * W > (1LL << 30)) return DXR_EINVAL;
  if (B == 0) return DXR_OK;
  if (!pyramid || !coords || !weight_packed || !out) return DXR_EINVAL;
  const int rd = 2 * radius + 1;
  LookupGeom g;
  g.N = (int)(H * W);
  g.levels = num_levels;
  g.cout = num_levels * rd * rd;
  for (int l = 0; l < L.n; ++l) g.lv[l] = level_addr(L.lay[l]);
  const float4* wpl = static_cast<const float4*>(weight_packed);
  if (pyr_dtype == DXR_F32)
    return launch_lookup_conv1x1(static_cast<const float*>(pyramid), coords, wpl, bias, out, g,
                                 (int)B, radius, (int)cout, relu, stream);
  if (pyr_dtype == DXR_BF16)
    return launch_lookup_conv1x1(static_cast<const uint16_t*>(pyramid), coords, wpl, bias, out, g,
                                 (int)B, radius, (int)cout, relu, stream);
  return DXR_EINVAL;
}

