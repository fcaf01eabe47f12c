// Fmap gradients of the correlation pyramid on MFMA, with no [N x N] dV.
//
// Training backpropagates through matmul -> / sqrt(D) -> avg_pool2d chain ->
// grid_sample (train.py:175-178, core/corr.py:13-27,52-60).  The lookups'
// backwards leave one gradient pyramid G (paged like the pyramid, dxr_common.h).
// Folding it down the pooling chain gives
//   dV[q][t] = (G0 + (G1 + (G2 + G3/4)/4)/4)[q][t] / sqrt(D)   (floor-mode masks)
// and the fmap gradients are two GEMMs against dV:
//   dF1[d][q] = sum_t F2[d][t] dV[q][t]      (kernel KT: K runs over targets)
//   dF2[d][t] = sum_q F1[d][q] dV[q][t]      (kernel !KT: K runs over queries)
// (r02 formed dV in HBM with dxr_pyramid_backward — 189 MB per Sintel pair —
// and ran the two GEMMs on rocBLAS f32.)
//
// Here a workgroup owns 256 channels x one n-block of 128 (a query block for
// dF1, a level-0 target tile for dF2) and walks a chunk of k-blocks.  A k-block
// is one page of each level: 128 queries x one 8 x 16 target tile (and its 4 x 8,
// 2 x 4, 1 x 2 pooled tiles), all contiguous.  Four fold waves turn the pages,
// half a k-block per stage, into the dV operand: folded, split three ways into
// bf16 (hi, mid, lo) MFMA B-operand records in LDS, one stage ahead of eight
// MFMA waves that run v_mfma_f32_32x32x16_bf16 with six products (the f32-class
// split of dxr_common.h split8) against the fmap operand, which comes pre-split
// from a pack pass, one 1 KiB-contiguous record block per wave and k-step.
// Chunks of k-blocks (split K, so ~256 workgroups fill the chip) write partial
// sums that a last pass adds in a fixed order: deterministic.
//
// Bounded form (round 4, dxr_fmap_grads_bounded): when the caller knows a bound
// on |G| (the lookup backwards' per-workgroup maxima), both operands run as
// power-of-two-scaled f16 pairs x = hi + lo (x 2^s < 2^14: hi = RNE_f16(x 2^s),
// lo = RNE_f16(x 2^s - hi)) — one scale per fmap channel (the GEMM's M rows),
// one for all of dV (its n columns and k rows) — and three f16 products
// (lo*hi, hi*lo, hi*hi) replace the six bf16 ones: half the MFMA work and
// two-thirds of the fold's records.  Error per element <= 2^-22 |x| + 2^-39 of
// the scale's bound (f16 subnormals keep an absolute step); the scales are
// undone exactly (ldexp) per output row.  A pair whose fmap has a non-finite
// channel, or a non-finite bound, runs the six-product path inside the same
// kernel, splitting the fmap operand from f32 in registers: IEEE propagation as
// the unbounded form.
#include <cmath>
#include <type_traits>

#include "dxr_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

constexpr int PQ = dxr::PAGE_Q;           // queries per page
constexpr int TH = dxr::PAGE_H;           // level-0 tile rows
constexpr int TW = dxr::PAGE_W;           // level-0 tile cols
constexpr int NB = 128;                   // n per workgroup
constexpr int KSTEPS = 8;                 // 16-k steps per k-block (128)
constexpr int DS = 256;                   // channels per workgroup (8 waves x 32)
constexpr int MW = 8;                     // MFMA waves (32 channels each)
constexpr int LW = 4;                     // fold waves
constexpr int NTHR = (MW + LW) * 64;
constexpr int HK = 4;                     // k-steps per stage (half a k-block)
constexpr int REC = HK * NB * 2;          // 16-B records per split part per stage
static_assert(PQ == NB && TH * TW == NB, "a k-block is one page");

struct GradGeom {
  int B, D, H, W, N;
  int qt, tyn, txn;       // query blocks, tile rows, tile cols per pair
  int nlev;               // tiled levels in the pyramid (1..4)
  int lh[4], lw[4];
  long long loff[4];
  float divisor, recip;   // recip = 1/divisor when exact, else 0
  int nblk, kbt, S;       // n blocks, k blocks, k chunks
  int nslab;              // 256-channel slabs
  long long ks;           // k steps of the packed operand
  float* out0;            // chunk 0's sums: the output itself (chunks >= 1: the workspace)
};

__device__ __forceinline__ uint4 ld4(const float* p) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  return make_uint4(__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                    __float_as_uint(v.w));
}

// Page element offsets of (pair b, query block qb, tile (ty, tx)) at each level.
__device__ __forceinline__ void page_bases(const GradGeom& g, int b, int qb, int ty, int tx,
                                           long long (&base)[4]) {
  const long long page = (((long long)b * g.qt + qb) * g.tyn + ty) * g.txn + tx;
#pragma unroll
  for (int l = 0; l < 4; ++l) base[l] = g.loff[l] + page * PQ * (NB >> (2 * l));
}

// One dV element from its four level gradients (pyramid_backward_kernel's order:
// from the coarsest level down, t = g_l + t/4; masked levels contribute 0).
template <bool DIV>
__device__ __forceinline__ float fold(const GradGeom& g, int y, int x, bool qok, float g0, float g1,
                                      float g2, float g3) {
  float t = 0.f;
  if (g.nlev > 3 && (y >> 3) < g.lh[3] && (x >> 3) < g.lw[3]) t = g3;
  if (g.nlev > 2) t = (((y >> 2) < g.lh[2] && (x >> 2) < g.lw[2]) ? g2 : 0.f) + 0.25f * t;
  if (g.nlev > 1) t = (((y >> 1) < g.lh[1] && (x >> 1) < g.lw[1]) ? g1 : 0.f) + 0.25f * t;
  t = ((y < g.H && x < g.W && qok) ? g0 : 0.f) + 0.25f * t;
  return DIV ? t / g.divisor : t * g.recip;
}

// Raw page values one fold thread (lt = 0..255) folds for a stage (half a
// k-block).  KT (dF1, n = query, k = target): query lt&127, tile rows
// 4*half + 2(lt>>7), +1, all 16 cols.  !KT (dF2, n = target, k = query): queries
// 64*half + 8(lt>>5).. +7, targets 4(lt&31).. +3.
template <bool KT>
struct Raw;

template <>
struct Raw<true> {
  uint4 g0[8];
  uint4 g1[2];
  uint4 g2;
  float g3[2];
};

template <>
struct Raw<false> {
  uint4 g0[8];
  float g1[8][2];
  float g2[8];
  float g3[8];
};

template <bool KT>
__device__ __forceinline__ void load_raw(const GradGeom& g, const float* __restrict__ gp, int b,
                                         int qb, int tile, int half, int lt, Raw<KT>& r) {
  long long base[4];
  page_bases(g, b, qb, tile / g.txn, tile % g.txn, base);
  if constexpr (KT) {
    const int q = lt & 127, k = 2 * half + (lt >> 7);   // level-1 row of the pair of rows
    const float* p0 = gp + base[0] + q * 128 + k * 32;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.g0[i] = ld4(p0 + 4 * i);
    r.g1[0] = r.g1[1] = make_uint4(0, 0, 0, 0);
    r.g2 = make_uint4(0, 0, 0, 0);
    r.g3[0] = r.g3[1] = 0.f;
    if (g.nlev > 1) {
      const float* p1 = gp + base[1] + q * 32 + k * 8;
      r.g1[0] = ld4(p1);
      r.g1[1] = ld4(p1 + 4);
    }
    if (g.nlev > 2) r.g2 = ld4(gp + base[2] + q * 8 + half * 4);
    if (g.nlev > 3) {
      const float2 v = *reinterpret_cast<const float2*>(gp + base[3] + q * 2);
      r.g3[0] = v.x;
      r.g3[1] = v.y;
    }
  } else {
    const int tg = lt & 31, q0 = 64 * half + (lt >> 5) * 8, rr = tg >> 2, cq = tg & 3;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = q0 + i;
      r.g0[i] = ld4(gp + base[0] + q * 128 + 4 * tg);
      r.g1[i][0] = r.g1[i][1] = r.g2[i] = r.g3[i] = 0.f;
      if (g.nlev > 1) {
        const float2 v = *reinterpret_cast<const float2*>(gp + base[1] + q * 32 + (rr >> 1) * 8 + 2 * cq);
        r.g1[i][0] = v.x;
        r.g1[i][1] = v.y;
      }
      if (g.nlev > 2) r.g2[i] = gp[base[2] + q * 8 + (rr >> 2) * 4 + cq];
      if (g.nlev > 3) r.g3[i] = gp[base[3] + q * 2 + (cq >> 1)];
    }
  }
}

__device__ __forceinline__ float u2f(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ float comp(const uint4& v, int e) {
  return u2f(e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w);
}

// f16 pair of 8 values scaled by 2^e (|x 2^e| < 2^14 by the choice of e).
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split8h(const float (&v)[8], int e, uint4& hi, uint4& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = __builtin_ldexpf(v[2 * i], e), b = __builtin_ldexpf(v[2 * i + 1], e);
    const f2v ab = {a, b};
    const h2v hv = __builtin_convertvector(ab, h2v);
    const f2v r = {__builtin_fmaf((float)hv[0], -1.f, a), __builtin_fmaf((float)hv[1], -1.f, b)};
    h[i] = __builtin_bit_cast(uint32_t, hv);
    l[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, h2v));
  }
  hi = make_uint4(h[0], h[1], h[2], h[3]);
  lo = make_uint4(l[0], l[1], l[2], l[3]);
}

// The 8 fmap values of operand record (k-step s, half h) of channel row `src`
// (one channel's plane of a pair): TORD, k = target in tile order; else k = query.
template <bool TORD>
__device__ __forceinline__ void load_fmap8(const float* __restrict__ src, const GradGeom& g,
                                           long long s, int h, float (&x)[8]) {
  auto two4 = [&](const float* p) {   // 16-B aligned: two float4 loads
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
    x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  };
  if constexpr (TORD) {
    const int tile = (int)(s / KSTEPS);
    const int y = (tile / g.txn) * TH + (int)(s % KSTEPS), xx = (tile % g.txn) * TW + 8 * h;
    if ((g.W & 3) == 0 && y < g.H && xx + 8 <= g.W) {   // plane and row bases 16-B aligned
      two4(src + y * g.W + xx);
      return;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = (y < g.H && xx + e < g.W) ? src[y * g.W + xx + e] : 0.f;
  } else {
    const long long q = s * 16 + 8 * h;
    if ((g.N & 3) == 0 && q + 8 <= g.N) {
      two4(src + q);
      return;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = q + e < g.N ? src[q + e] : 0.f;
  }
}

// Is every cell of k-block (qb, tile) inside every level (no floor-mode mask,
// no padding query)?  Then the fold needs no masks, and the coarse levels fold
// once per level-1 cell instead of once per dV element.
__device__ __forceinline__ bool interior(const GradGeom& g, int qb, int tile) {
  const int y1 = (tile / g.txn) * TH + TH - 1, x1 = (tile % g.txn) * TW + TW - 1;
  bool in = (qb + 1) * PQ <= g.N && y1 < g.H && x1 < g.W;
#pragma unroll
  for (int l = 1; l < 4; ++l)
    if (l < g.nlev) in = in && (y1 >> l) < g.lh[l] && (x1 >> l) < g.lw[l];
  return in;
}

__device__ __forceinline__ void store_split(const float (&v)[8], int rec, uint4* __restrict__ sb) {
  uint4 hi, mi, lo;
  dxr::split8(v, hi, mi, lo);
  sb[rec] = hi;
  sb[REC + rec] = mi;
  sb[2 * REC + rec] = lo;
}

// Fold a stage's raw values into dV, split, write the stage's LDS records
// (part p, k-step s of the stage, half h of the k-step, n) at
// sb[p*REC + (s*2 + h)*128 + n]: an MFMA operand read is two 512-B runs and a
// fold thread's store is lane-contiguous, both free of bank conflicts
// (the [n][h] order, 32-B lane stride, spent half the LDS cycles in conflicts).  Interior k-blocks: the same arithmetic in the
// same order (levels absent beyond nlev were loaded as 0, and x + 0.25*0 = x).
// F16: the records are the f16 pair of dV 2^ev (parts hi, lo) instead of the
// three-way bf16 split.
template <bool F16>
__device__ __forceinline__ void store_rec(const float (&v)[8], int rec, uint4* __restrict__ sb,
                                          int ev) {
  if constexpr (F16) {
    uint4 hi, lo;
    split8h(v, ev, hi, lo);
    sb[rec] = hi;
    sb[REC + rec] = lo;
  } else {
    store_split(v, rec, sb);
  }
}

template <bool KT, bool DIV, bool F16 = false>
__device__ __forceinline__ void fold_store(const GradGeom& g, const Raw<KT>& r, int qb, int tile,
                                           int half, int lt, uint4* __restrict__ sb, int ev = 0) {
  const int y0 = (tile / g.txn) * TH, x0 = (tile % g.txn) * TW;
  const bool inner = interior(g, qb, tile);
  auto scale = [&](float t) { return DIV ? t / g.divisor : t * g.recip; };
  if constexpr (KT) {
    const int q = lt & 127, k = lt >> 7;
    const bool qok = qb * PQ + q < g.N;
    float p1[8];  // this thread's level-1 row, coarser levels folded in
#pragma unroll
    for (int c1 = 0; c1 < 8; ++c1) {
      const float p2 = comp(r.g2, c1 >> 1) + 0.25f * r.g3[c1 >> 2];
      p1[c1] = comp(r.g1[c1 >> 2], c1 & 3) + 0.25f * p2;
    }
    auto body = [&](auto in_c) {
      constexpr bool IN = decltype(in_c)::value;
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int y = y0 + 4 * half + 2 * k + rr;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int c = 8 * h + e, i = rr * 16 + c;
            if constexpr (IN)
              v[e] = scale(comp(r.g0[i >> 2], i & 3) + 0.25f * p1[c >> 1]);
            else
              v[e] = fold<DIV>(g, y, x0 + c, qok, comp(r.g0[i >> 2], i & 3),
                               comp(r.g1[c >> 3], (c >> 1) & 3), comp(r.g2, c >> 2), r.g3[c >> 3]);
          }
          store_rec<F16>(v, ((2 * k + rr) * 2 + h) * NB + q, sb, ev);
        }
      }
    };
    if (inner)
      body(std::true_type{});
    else
      body(std::false_type{});
  } else {
    const int tg = lt & 31, qg = lt >> 5, rr = tg >> 2, cq = tg & 3;
    const int y = y0 + rr;
    float p1[8][2];  // per query: its two level-1 cells, coarser levels folded in
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float p2 = r.g2[i] + 0.25f * r.g3[i];
      p1[i][0] = r.g1[i][0] + 0.25f * p2;
      p1[i][1] = r.g1[i][1] + 0.25f * p2;
    }
    auto body = [&](auto in_c) {
      constexpr bool IN = decltype(in_c)::value;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = 4 * cq + j;
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if constexpr (IN) {
            v[i] = scale(comp(r.g0[i], j) + 0.25f * p1[i][j >> 1]);
          } else {
            const bool qok = qb * PQ + 64 * half + qg * 8 + i < g.N;
            v[i] = fold<DIV>(g, y, x0 + c, qok, comp(r.g0[i], j), r.g1[i][j >> 1], r.g2[i], r.g3[i]);
          }
        }
        store_rec<F16>(v, qg * NB + j * 32 + tg, sb, ev);
      }
    };
    if (inner)
      body(std::true_type{});
    else
      body(std::false_type{});
  }
}

// XCD-aware linear order (workgroup w runs on XCD w % 8): each XCD takes a
// contiguous range of (pair, slab, chunk, n block), n block fastest, so the
// workgroups an XCD holds share one chunk's fmap operand in its L2.
__device__ __forceinline__ long long xcd_linear(long long w, long long nwg) {
  const long long q8 = nwg / 8, r8 = nwg % 8, xcd = w % 8;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + w / 8;
}

// Warp-specialised: LW fold waves turn gradient pages into dV operand stages
// (two LDS buffers, one stage ahead), MW MFMA waves stream the fmap operand
// from L2 and multiply.  The fold waves' page loads never sit in front of the
// MFMA waves' operand loads in a vmcnt queue, and their VALU work overlaps the
// MFMAs.  One barrier per stage: at barrier st the fold waves have published
// stage st and the MFMA waves have finished stage st-1, whose buffer the fold
// waves fill next.
template <bool KT, bool DIV>
__global__ __launch_bounds__(NTHR) void fmap_grad_kernel(const float* __restrict__ gp,
                                                         const uint4* __restrict__ fp,
                                                         float* __restrict__ out, GradGeom g) {
  __shared__ uint4 sb[2][3 * REC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long wl = xcd_linear(blockIdx.x, gridDim.x);
  const int nb = (int)(wl % g.nblk);
  wl /= g.nblk;
  const int chunk = (int)(wl % g.S);
  wl /= g.S;
  const int slab = (int)(wl % g.nslab);
  const int b = (int)(wl / g.nslab);
  const int kb0 = (int)((long long)chunk * g.kbt / g.S);
  const int kb1 = (int)((long long)(chunk + 1) * g.kbt / g.S);
  const int nst = 2 * (kb1 - kb0);

  if (wave >= MW) {  // fold waves
    // KT: two register sets, stage st+1's pages are in flight while stage st
    // folds and the MFMA waves finish stage st-1 (stage st = k-block kb0 + st/2,
    // half st%2)
    const int lt = tid - MW * 64;
    auto load = [&](int st, Raw<KT>& r) {
      const int kb = kb0 + (st >> 1);
      load_raw<KT>(g, gp, b, KT ? nb : kb, KT ? kb : nb, st & 1, lt, r);
    };
    auto fold = [&](int st, const Raw<KT>& r) {
      const int kb = kb0 + (st >> 1);
      fold_store<KT, DIV>(g, r, KT ? nb : kb, KT ? kb : nb, st & 1, lt, sb[st & 1]);
    };
    Raw<KT> r0;
    if (nst > 0) load(0, r0);
    if constexpr (KT) {
      Raw<KT> r1;
      for (int st = 0; st < nst; st += 2) {  // nst is even
        load(st + 1, r1);
        fold(st, r0);
        __syncthreads();
        if (st + 2 < nst) load(st + 2, r0);
        fold(st + 1, r1);
        __syncthreads();
      }
    } else {  // 64 raw values a thread: one set (two would spill)
      for (int st = 0; st < nst; ++st) {
        fold(st, r0);
        if (st + 1 < nst) load(st + 1, r0);
        __syncthreads();
      }
    }
    return;
  }

  const int d0 = slab * DS + wave * 32;
  const bool active = d0 < g.D;  // D % 32 == 0: whole waves
  f32x16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[j][v] = 0.f;

  // fmap operand records: (((b*3 + p)*ks + k-step)*D + d)*2 + half
  const long long pstride = g.ks * g.D * 2, kstride = (long long)g.D * 2;
  const uint4* fa = fp + (long long)b * 3 * pstride + (long long)(d0 + (lane & 31)) * 2 +
                    (lane >> 5) + (long long)kb0 * KSTEPS * kstride;
  const int bl = (lane >> 5) * NB + (lane & 31);
  // fmap operand: a stage's four k-steps in registers; each k-step's slot is
  // reloaded with the next stage's k-step as soon as its MFMAs have issued (a
  // stage of cover; no register rotation, so no wait for a load in flight)
  uint4 A[HK][3];
  auto load_a = [&](int st, int s, uint4 (&a)[3]) {
    const uint4* f = fa + (long long)(st * HK + s) * kstride;
    a[0] = f[0];
    a[1] = f[pstride];
    a[2] = f[2 * pstride];
  };
  if (active && nst > 0) {
#pragma unroll
    for (int s = 0; s < HK; ++s) load_a(0, s, A[s]);
  }
  for (int st = 0; st < nst; ++st) {
    __syncthreads();  // stage st published
    if (!active) continue;
    const uint4* sp = sb[st & 1] + bl;
#pragma unroll
    for (int s = 0; s < HK; ++s) {
      const bf8v qh = __builtin_bit_cast(bf8v, A[s][0]), qm = __builtin_bit_cast(bf8v, A[s][1]),
                 ql = __builtin_bit_cast(bf8v, A[s][2]);
      bf8v th[4], tm[4], tl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint4* bp = sp + s * 2 * NB + 32 * j;
        th[j] = __builtin_bit_cast(bf8v, bp[0]);
        tm[j] = __builtin_bit_cast(bf8v, bp[REC]);
        tl[j] = __builtin_bit_cast(bf8v, bp[2 * REC]);
      }
      // per accumulator small terms first; the four tiles interleaved so no
      // MFMA waits on the one before it
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm, tm[j], acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ql, th[j], acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, tl[j], acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm, th[j], acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, tm[j], acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, th[j], acc[j], 0, 0, 0);
      if (st + 1 < nst) load_a(st + 1, s, A[s]);
    }
  }
  if (!active) return;
  // C/D map: column n = lane & 31 (+32 j), row d = (v&3) + 8(v>>2) + 4(lane>>5)
  float* o = chunk == 0 ? g.out0 + (long long)b * g.D * g.N
                        : out + ((long long)(chunk - 1) * g.B + b) * g.D * g.N;
  const int ty = nb / g.txn, tx = nb % g.txn;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int px;
    if constexpr (KT) {
      const int q = nb * PQ + 32 * j + (lane & 31);
      px = q < g.N ? q : -1;
    } else {
      const int t = 4 * (lane & 31) + j, y = ty * TH + (t >> 4), x = tx * TW + (t & 15);
      px = (y < g.H && x < g.W) ? y * g.W + x : -1;
    }
    if (px < 0) continue;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int d = d0 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
      o[(long long)d * g.N + px] = acc[j][v];
    }
  }
}

// ---------------------------------------------------------------------------
// Bounded form: f16 pair operands, three products (see the file comment).
// Scales (workspace, int32): [0] dV's exponent ev, [1] 1 when the bound is
// finite, [2 + b D + d] the exponent of channel d of pair b, or SCALE_BAD when
// that channel holds a non-finite value.
constexpr int SCALE_BAD = -2147483647 - 1;
constexpr int SCALE_TOP = 14;     // |x 2^s| < 2^SCALE_TOP for every |x| <= m

__device__ __forceinline__ int scale_for(float m) {   // m finite, >= 0
  if (!(m > 0.f)) return 0;
  int e;
  (void)__builtin_frexpf(m, &e);
  const int s = SCALE_TOP - e;
  return s < -125 ? -125 : (s > 125 ? 125 : s);
}

// One kernel body for both arithmetics (F16: f16 pairs from the pre-split
// records `fp`, three products; else the six-product bf16 split with the fmap
// operand split from f32 (`fsrc`) in registers — the non-finite path).
template <bool KT, bool DIV, bool F16>
__device__ __forceinline__ void grad_body(const float* __restrict__ gp, const uint4* __restrict__ fp,
                                          const float* __restrict__ fsrc,
                                          const int* __restrict__ scales, float* __restrict__ out,
                                          const GradGeom& g, uint4* __restrict__ sbase, int nb,
                                          int chunk, int slab, int b, int ev) {
  constexpr int NP = F16 ? 2 : 3;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kb0 = (int)((long long)chunk * g.kbt / g.S);
  const int kb1 = (int)((long long)(chunk + 1) * g.kbt / g.S);
  const int nst = 2 * (kb1 - kb0);
  auto stage = [&](int st) { return sbase + (st & 1) * (3 * REC); };

  if (wave >= MW) {  // fold waves (as fmap_grad_kernel)
    const int lt = tid - MW * 64;
    auto load = [&](int st, Raw<KT>& r) {
      const int kb = kb0 + (st >> 1);
      load_raw<KT>(g, gp, b, KT ? nb : kb, KT ? kb : nb, st & 1, lt, r);
    };
    auto fold = [&](int st, const Raw<KT>& r) {
      const int kb = kb0 + (st >> 1);
      fold_store<KT, DIV, F16>(g, r, KT ? nb : kb, KT ? kb : nb, st & 1, lt, stage(st), ev);
    };
    Raw<KT> r0;
    if (nst > 0) load(0, r0);
    if constexpr (KT) {
      Raw<KT> r1;
      for (int st = 0; st < nst; st += 2) {
        load(st + 1, r1);
        fold(st, r0);
        __syncthreads();
        if (st + 2 < nst) load(st + 2, r0);
        fold(st + 1, r1);
        __syncthreads();
      }
    } else {
      for (int st = 0; st < nst; ++st) {
        fold(st, r0);
        if (st + 1 < nst) load(st + 1, r0);
        __syncthreads();
      }
    }
    return;
  }

  const int d0 = slab * DS + wave * 32;
  const bool active = d0 < g.D;
  f32x16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[j][v] = 0.f;

  // F16 records: (((b*2 + p)*ks + k-step)*D + d)*2 + half
  const long long pstride = g.ks * g.D * 2, kstride = (long long)g.D * 2;
  const int dl = active ? d0 + (lane & 31) : 0, hl = lane >> 5;
  const uint4* fa = fp + (long long)b * 2 * pstride + (long long)dl * 2 + hl +
                    (long long)kb0 * KSTEPS * kstride;
  const float* plane = fsrc + ((long long)b * g.D + dl) * g.N;
  const int bl = hl * NB + (lane & 31);
  uint4 A[HK][NP];
  auto load_a = [&](int st, int s, uint4 (&a)[NP]) {
    if constexpr (F16) {
      const uint4* f = fa + (long long)(st * HK + s) * kstride;
      a[0] = f[0];
      a[1] = f[pstride];
    } else {
      float x[8];
      load_fmap8<KT>(plane, g, (long long)kb0 * KSTEPS + st * HK + s, hl, x);
      dxr::split8(x, a[0], a[1], a[NP - 1]);
    }
  };
  if (active && nst > 0) {
#pragma unroll
    for (int s = 0; s < HK; ++s) load_a(0, s, A[s]);
  }
  for (int st = 0; st < nst; ++st) {
    __syncthreads();  // stage st published
    if (!active) continue;
    const uint4* sp = stage(st) + bl;
#pragma unroll
    for (int s = 0; s < HK; ++s) {
      if constexpr (F16) {
        const h8v ah = __builtin_bit_cast(h8v, A[s][0]), al = __builtin_bit_cast(h8v, A[s][1]);
        h8v th[4], tl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint4* bp = sp + s * 2 * NB + 32 * j;
          th[j] = __builtin_bit_cast(h8v, bp[0]);
          tl[j] = __builtin_bit_cast(h8v, bp[REC]);
        }
        // small terms first, the four tiles interleaved
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, th[j], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, tl[j], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, th[j], acc[j], 0, 0, 0);
      } else {
        const bf8v qh = __builtin_bit_cast(bf8v, A[s][0]), qm = __builtin_bit_cast(bf8v, A[s][1]),
                   ql = __builtin_bit_cast(bf8v, A[s][NP - 1]);
        bf8v th[4], tm[4], tl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint4* bp = sp + s * 2 * NB + 32 * j;
          th[j] = __builtin_bit_cast(bf8v, bp[0]);
          tm[j] = __builtin_bit_cast(bf8v, bp[REC]);
          tl[j] = __builtin_bit_cast(bf8v, bp[2 * REC]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm, tm[j], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ql, th[j], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, tl[j], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qm, th[j], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, tm[j], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qh, th[j], acc[j], 0, 0, 0);
      }
      if (st + 1 < nst) load_a(st + 1, s, A[s]);
    }
  }
  if (!active) return;
  // undo the scales: row d's exponent + dV's
  int un[16];
#pragma unroll
  for (int v = 0; v < 16; ++v)
    un[v] = F16 ? -(scales[2 + b * g.D + d0 + (v & 3) + 8 * (v >> 2) + 4 * hl] + ev) : 0;
  float* o = chunk == 0 ? g.out0 + (long long)b * g.D * g.N
                        : out + ((long long)(chunk - 1) * g.B + b) * g.D * g.N;
  const int ty = nb / g.txn, tx = nb % g.txn;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int px;
    if constexpr (KT) {
      const int q = nb * PQ + 32 * j + (lane & 31);
      px = q < g.N ? q : -1;
    } else {
      const int t = 4 * (lane & 31) + j, y = ty * TH + (t >> 4), x = tx * TW + (t & 15);
      px = (y < g.H && x < g.W) ? y * g.W + x : -1;
    }
    if (px < 0) continue;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int d = d0 + (v & 3) + 8 * (v >> 2) + 4 * hl;
      o[(long long)d * g.N + px] = F16 ? __builtin_ldexpf(acc[j][v], un[v]) : acc[j][v];
    }
  }
}

template <bool KT, bool DIV>
__global__ __launch_bounds__(NTHR) void fmap_grad_bounded_kernel(const float* __restrict__ gp,
                                                                 const uint4* __restrict__ fp,
                                                                 const float* __restrict__ fsrc,
                                                                 const int* __restrict__ scales,
                                                                 float* __restrict__ out, GradGeom g) {
  __shared__ uint4 sb[2 * 3 * REC];
  __shared__ int s_ok;
  const int tid = threadIdx.x;
  long long wl = xcd_linear(blockIdx.x, gridDim.x);
  const int nb = (int)(wl % g.nblk);
  wl /= g.nblk;
  const int chunk = (int)(wl % g.S);
  wl /= g.S;
  const int slab = (int)(wl % g.nslab);
  const int b = (int)(wl / g.nslab);
  if (tid == 0) s_ok = scales[1];
  __syncthreads();
  for (int i = tid; i < g.D; i += NTHR)
    if (scales[2 + b * g.D + i] == SCALE_BAD) s_ok = 0;   // same value from every writer
  __syncthreads();
  const int ev = scales[0];
  if (s_ok)
    grad_body<KT, DIV, true>(gp, fp, fsrc, scales, out, g, sb, nb, chunk, slab, b, ev);
  else
    grad_body<KT, DIV, false>(gp, fp, fsrc, scales, out, g, sb, nb, chunk, slab, b, ev);
}

// Fmap -> f16 pair records of the bounded form, grid (ceil(D / 4), B, slices),
// 1024 threads: four waves per channel find its max |x| (its scale; float4
// loads, four in flight per lane), then the workgroup writes its slice of the
// four channels' records, eight threads per 128-B line.  Workgroup (0, 0) also
// reduces the bound slots to dV's scale: |dV| <= vfac max|G|.
template <bool TORD>
__global__ __launch_bounds__(1024) void fmap_split16_kernel(const float* __restrict__ f,
                                                            uint4* __restrict__ fp,
                                                            int* __restrict__ scales,
                                                            const float* __restrict__ slots,
                                                            long long n_slots, float vfac, GradGeom g) {
  __shared__ float pm[16];
  __shared__ int pbad[16];
  __shared__ int se[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.y, dbase = blockIdx.x * 4;
  const int slice = blockIdx.z, nslice = gridDim.z;   // this workgroup's share of the records
  auto wave_reduce = [&](float m, bool bad) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = __builtin_fmaxf(m, __shfl_xor(m, o));
    bad = __any(bad);
    if (lane == 0) {
      pm[w] = m;
      pbad[w] = bad;
    }
  };
  auto absmax = [&](float v, float& m, bool& bad) {
    const float a = __builtin_fabsf(v);
    if (a <= 3.40282347e38f) m = __builtin_fmaxf(m, a);
    else bad = true;
  };
  {
    const int d = dbase + (w >> 2), part = w & 3;
    float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;
    bool bad = false;
    if (d < g.D) {
      const float* src = f + ((long long)b * g.D + d) * g.N;
      if ((g.N & 3) == 0) {   // 16-B aligned planes: float4 loads, four in flight
        const float4* s4 = reinterpret_cast<const float4*>(src);
        const int n4 = g.N >> 2;
        int q = part * 64 + lane;
        for (; q + 768 < n4; q += 1024) {
          const float4 a = s4[q], c = s4[q + 256], e = s4[q + 512], h = s4[q + 768];
          absmax(a.x, m0, bad); absmax(a.y, m1, bad); absmax(a.z, m2, bad); absmax(a.w, m3, bad);
          absmax(c.x, m0, bad); absmax(c.y, m1, bad); absmax(c.z, m2, bad); absmax(c.w, m3, bad);
          absmax(e.x, m0, bad); absmax(e.y, m1, bad); absmax(e.z, m2, bad); absmax(e.w, m3, bad);
          absmax(h.x, m0, bad); absmax(h.y, m1, bad); absmax(h.z, m2, bad); absmax(h.w, m3, bad);
        }
        for (; q < n4; q += 256) {
          const float4 a = s4[q];
          absmax(a.x, m0, bad); absmax(a.y, m1, bad); absmax(a.z, m2, bad); absmax(a.w, m3, bad);
        }
      } else {
        int p = part * 64 + lane;
        for (; p + 768 < g.N; p += 1024) {   // four independent loads per step
          const float v0 = src[p], v1 = src[p + 256], v2 = src[p + 512], v3 = src[p + 768];
          absmax(v0, m0, bad);
          absmax(v1, m1, bad);
          absmax(v2, m2, bad);
          absmax(v3, m3, bad);
        }
        for (; p < g.N; p += 256) absmax(src[p], m0, bad);
      }
    }
    wave_reduce(__builtin_fmaxf(__builtin_fmaxf(m0, m1), __builtin_fmaxf(m2, m3)), bad);
  }
  __syncthreads();
  if (tid < 4) {
    const float m = __builtin_fmaxf(__builtin_fmaxf(pm[4 * tid], pm[4 * tid + 1]),
                                    __builtin_fmaxf(pm[4 * tid + 2], pm[4 * tid + 3]));
    const bool bad = pbad[4 * tid] | pbad[4 * tid + 1] | pbad[4 * tid + 2] | pbad[4 * tid + 3];
    se[tid] = bad ? SCALE_BAD : scale_for(m);
    if (slice == 0 && dbase + tid < g.D) scales[2 + b * g.D + dbase + tid] = se[tid];
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && slice == 0) {
    __syncthreads();   // pm / pbad reused
    float m = 0.f;
    bool bad = false;
    for (long long i = tid; i < n_slots; i += 1024) {
      const float v = slots[i];
      if (v <= 3.40282347e38f) m = __builtin_fmaxf(m, v);
      else bad = true;
    }
    wave_reduce(m, bad);
    __syncthreads();
    if (tid == 0) {   // (slice-0 workgroup (0, 0) only)
      float mm = 0.f;
      bool bb = false;
      for (int i = 0; i < 16; ++i) {
        mm = __builtin_fmaxf(mm, pm[i]);
        bb |= pbad[i] != 0;
      }
      const float bound = mm * vfac;
      const bool ok = !bb && bound <= 3.40282347e38f;
      scales[0] = ok ? scale_for(bound) : 0;
      scales[1] = ok ? 1 : 0;
    }
  }
  __syncthreads();
  const long long pstride = g.ks * g.D * 2;
  const long long items = g.ks * 8;
  const long long i0 = items * slice / nslice, i1 = items * (slice + 1) / nslice;
  for (long long it = i0 + tid; it < i1; it += 1024) {
    const int h = (int)(it & 1), dd = (int)((it >> 1) & 3);
    const long long s = it >> 3;
    const int d = dbase + dd;
    if (d >= g.D || se[dd] == SCALE_BAD) continue;
    float x[8];
    load_fmap8<TORD>(f + ((long long)b * g.D + d) * g.N, g, s, h, x);
    uint4 hi, lo;
    split8h(x, se[dd], hi, lo);
    const long long rec = (((long long)b * 2 * g.ks + s) * g.D + d) * 2 + h;
    fp[rec] = hi;
    fp[rec + pstride] = lo;
  }
}

// Fmap -> three-way bf16 split operand records in the GEMM's k order.
// TORD: k = target in tile order (tile*128 + row*16 + col); else k = query.
template <bool TORD>
__global__ __launch_bounds__(256) void fmap_split_kernel(const float* __restrict__ f,
                                                         uint4* __restrict__ fp, GradGeom g) {
  const long long total = (long long)g.B * g.ks * g.D * 2;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int h = (int)(idx & 1);
    long long r = idx >> 1;
    const int d = (int)(r % g.D);
    r /= g.D;
    const long long s = r % g.ks;
    const int b = (int)(r / g.ks);
    const float* src = f + ((long long)b * g.D + d) * g.N;
    float x[8];
    if constexpr (TORD) {
      const int tile = (int)(s / KSTEPS);
      const int y = (tile / g.txn) * TH + (int)(s % KSTEPS), xx = (tile % g.txn) * TW + 8 * h;
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = (y < g.H && xx + e < g.W) ? src[y * g.W + xx + e] : 0.f;
    } else {
      const long long q = s * 16 + 8 * h;
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = q + e < g.N ? src[q + e] : 0.f;
    }
    uint4 hi, mi, lo;
    dxr::split8(x, hi, mi, lo);
    const long long rec = (((long long)b * 3 * g.ks + s) * g.D + d) * 2 + h;
    const long long ps = g.ks * g.D * 2;
    fp[rec] = hi;
    fp[rec + ps] = mi;
    fp[rec + 2 * ps] = lo;
  }
}

// out[i] = sum over chunks s (ascending) of chunk s's sums: chunk 0's are out[i]
// itself, chunk s >= 1's part[s - 1][i] (one [B, D, H*W] buffer fewer in the
// workspace than S separate partials; the same additions in the same order).
__global__ __launch_bounds__(256) void chunk_sum_kernel(const float* __restrict__ part,
                                                        float* __restrict__ out, long long n, int S) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float t = out[i];
    for (int s = 1; s < S; ++s) t += part[(s - 1) * n + i];
    out[i] = t;
  }
}

long long align256(long long x) { return (x + 255) / 256 * 256; }

bool make_geom(int64_t B, int64_t D, int64_t H, int64_t W, int num_levels, float divisor,
               GradGeom* g) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L)) return false;
  g->B = (int)B;
  g->D = (int)D;
  g->H = (int)H;
  g->W = (int)W;
  g->N = (int)(H * W);
  g->qt = L.lay[0].qt;
  g->tyn = L.lay[0].ty;
  g->txn = L.lay[0].tx;
  g->nlev = num_levels;
  for (int l = 0; l < 4; ++l) {
    const int k = l < num_levels ? l : 0;
    g->lh[l] = L.lay[k].h;
    g->lw[l] = L.lay[k].w;
    g->loff[l] = L.lay[k].off;
  }
  g->divisor = divisor;
  int e2 = 0;
  g->recip = (std::frexp(divisor, &e2) == 0.5f) ? 1.f / divisor : 0.f;
  g->nslab = (int)((D + DS - 1) / DS);
  return true;
}

// KT: n blocks = query blocks, k blocks = tiles; else the other way round.
void set_kernel(GradGeom* g, bool kt) {
  const int tiles = g->tyn * g->txn;
  g->nblk = kt ? g->qt : tiles;
  g->kbt = kt ? tiles : g->qt;
  g->ks = (long long)g->kbt * KSTEPS;
  const long long units = (long long)g->nblk * g->B * g->nslab;
  long long S = units >= 256 ? 1 : 256 / units;
  if (S > g->kbt) S = g->kbt;
  g->S = (int)S;
}

long long operand_bytes(const GradGeom& g) { return align256((long long)g.B * 3 * g.ks * g.D * 32); }
long long partial_bytes(const GradGeom& g) {
  return g.S > 1 ? align256((long long)(g.S - 1) * g.B * g.D * g.N * 4) : 0;
}

bool grads_supported(int64_t D, int num_levels) {
  return D > 0 && D % 32 == 0 && num_levels >= 1 && num_levels <= dxr::TILED_LEVELS;
}

unsigned grid_for(long long total) {
  long long blocks = (total + 255) / 256;
  if (blocks > 2048 * 8) blocks = 2048 * 8;
  return (unsigned)(blocks < 1 ? 1 : blocks);
}

long long scales_bytes(const GradGeom& g) { return align256((2 + (long long)g.B * g.D) * 4); }
long long operand16_bytes(const GradGeom& g) { return align256((long long)g.B * 2 * g.ks * g.D * 32); }

}  // namespace

namespace {
// form 0: dxr_fmap_grads (three-part operand); 1: the bounded form (scales +
// two-part operand); either adds the chunks' partial sums
long long grads_workspace(int64_t B, int64_t D, int64_t H, int64_t W, int num_levels, int form) {
  GradGeom g;
  if (!grads_supported(D, num_levels) || !make_geom(B, D, H, W, num_levels, 1.f, &g)) return -1;
  long long ws = 0;
  for (int kt = 0; kt < 2; ++kt) {
    set_kernel(&g, kt == 1);
    const long long need = (form ? scales_bytes(g) + operand16_bytes(g) : operand_bytes(g)) +
                           partial_bytes(g);
    if (need > ws) ws = need;
  }
  return ws;
}
}  // namespace

// The larger of both forms' workspace (the bounded form needs less: its own query below).
extern "C" int64_t dxr_fmap_grads_workspace_bytes(int64_t B, int64_t D, int64_t H, int64_t W,
                                                  int num_levels) {
  const long long a = grads_workspace(B, D, H, W, num_levels, 0);
  const long long b = grads_workspace(B, D, H, W, num_levels, 1);
  return a < b ? b : a;
}

extern "C" int64_t dxr_fmap_grads_bounded_workspace_bytes(int64_t B, int64_t D, int64_t H,
                                                          int64_t W, int num_levels) {
  return grads_workspace(B, D, H, W, num_levels, 1);
}

extern "C" int dxr_fmap_grads_bounded(const void* grad_pyramid, int grad_dtype, const float* fmap1,
                                      const float* fmap2, int64_t B, int64_t D, int64_t H, int64_t W,
                                      int num_levels, float divisor, const float* bound_slots,
                                      int64_t n_slots, float* grad_fmap1, float* grad_fmap2,
                                      void* workspace, int64_t workspace_bytes, hipStream_t stream) {
  if (grad_dtype != DXR_F32) return grad_dtype == DXR_BF16 ? DXR_EUNSUPPORTED : DXR_EINVAL;
  if (D < 1 || B < 0 || B > 65535 || !(divisor == divisor) || divisor == 0.f) return DXR_EINVAL;
  if (!grads_supported(D, num_levels)) return DXR_EUNSUPPORTED;
  GradGeom g;
  if (!make_geom(B, D, H, W, num_levels, divisor, &g)) return DXR_EINVAL;
  if (B == 0 || (!grad_fmap1 && !grad_fmap2)) return DXR_OK;
  if (!grad_pyramid || !workspace || !bound_slots || n_slots < 1) return DXR_EINVAL;
  if (workspace_bytes < grads_workspace(B, D, H, W, num_levels, 1)) return DXR_EINVAL;
  const float* gp = static_cast<const float*>(grad_pyramid);
  // |dV| <= (1 + 1/4 + 1/16 + 1/64) max|G| / divisor (the fold), with headroom
  const float vfac = 1.34f / __builtin_fabsf(divisor);
  for (int kt = 1; kt >= 0; --kt) {
    float* dst = kt ? grad_fmap1 : grad_fmap2;
    const float* src = kt ? fmap2 : fmap1;
    if (!dst) continue;
    if (!src) return DXR_EINVAL;
    set_kernel(&g, kt == 1);
    g.out0 = dst;
    char* w = static_cast<char*>(workspace);
    int* scales = reinterpret_cast<int*>(w);
    uint4* fp = reinterpret_cast<uint4*>(w + scales_bytes(g));
    float* part = g.S > 1 ? reinterpret_cast<float*>(w + scales_bytes(g) + operand16_bytes(g)) : dst;
    const long long nwg = (long long)g.nblk * g.S * g.nslab * g.B;
    // ~256 split workgroups: the four channels' records in slices (each slice
    // recomputes the four maxima, L2 hits after the first)
    const long long cwg = (g.D + 3) / 4 * (long long)g.B;
    const unsigned nsl = (unsigned)(cwg >= 256 ? 1 : (256 + cwg - 1) / cwg);
    const dim3 sg((unsigned)((g.D + 3) / 4), (unsigned)g.B, nsl), gg((unsigned)nwg);
    const bool div = g.recip == 0.f;
    if (kt)
      hipLaunchKernelGGL(fmap_split16_kernel<true>, sg, dim3(1024), 0, stream, src, fp, scales,
                         bound_slots, (long long)n_slots, vfac, g);
    else
      hipLaunchKernelGGL(fmap_split16_kernel<false>, sg, dim3(1024), 0, stream, src, fp, scales,
                         bound_slots, (long long)n_slots, vfac, g);
    if (kt) {
      if (div)
        hipLaunchKernelGGL((fmap_grad_bounded_kernel<true, true>), gg, dim3(NTHR), 0, stream, gp, fp,
                           src, scales, part, g);
      else
        hipLaunchKernelGGL((fmap_grad_bounded_kernel<true, false>), gg, dim3(NTHR), 0, stream, gp,
                           fp, src, scales, part, g);
    } else {
      if (div)
        hipLaunchKernelGGL((fmap_grad_bounded_kernel<false, true>), gg, dim3(NTHR), 0, stream, gp,
                           fp, src, scales, part, g);
      else
        hipLaunchKernelGGL((fmap_grad_bounded_kernel<false, false>), gg, dim3(NTHR), 0, stream, gp,
                           fp, src, scales, part, g);
    }
    if (g.S > 1) {
      const long long n = (long long)g.B * g.D * g.N;
      hipLaunchKernelGGL(chunk_sum_kernel, dim3(grid_for(n)), dim3(256), 0, stream, part, dst, n, g.S);
    }
    const int st = dxr::launch_status();
    if (st != DXR_OK) return st;
  }
  return DXR_OK;
}

extern "C" int dxr_fmap_grads(const void* grad_pyramid, int grad_dtype, const float* fmap1,
                              const float* fmap2, int64_t B, int64_t D, int64_t H, int64_t W,
                              int num_levels, float divisor, float* grad_fmap1, float* grad_fmap2,
                              void* workspace, int64_t workspace_bytes, hipStream_t stream) {
  if (grad_dtype != DXR_F32) return grad_dtype == DXR_BF16 ? DXR_EUNSUPPORTED : DXR_EINVAL;
  if (D < 1 || B < 0 || B > 65535 || !(divisor == divisor) || divisor == 0.f) return DXR_EINVAL;
  if (!grads_supported(D, num_levels)) return DXR_EUNSUPPORTED;
  GradGeom g;
  if (!make_geom(B, D, H, W, num_levels, divisor, &g)) return DXR_EINVAL;
  if (B == 0 || (!grad_fmap1 && !grad_fmap2)) return DXR_OK;
  if (!grad_pyramid || !workspace) return DXR_EINVAL;
  if (workspace_bytes < dxr_fmap_grads_workspace_bytes(B, D, H, W, num_levels)) return DXR_EINVAL;
  const float* gp = static_cast<const float*>(grad_pyramid);
  for (int kt = 1; kt >= 0; --kt) {
    float* dst = kt ? grad_fmap1 : grad_fmap2;
    const float* src = kt ? fmap2 : fmap1;
    if (!dst) continue;
    if (!src) return DXR_EINVAL;
    set_kernel(&g, kt == 1);
    g.out0 = dst;
    uint4* fp = static_cast<uint4*>(workspace);
    float* part = g.S > 1 ? reinterpret_cast<float*>(static_cast<char*>(workspace) + operand_bytes(g))
                          : dst;
    const long long nwg = (long long)g.nblk * g.S * g.nslab * g.B;
    const dim3 pg(grid_for(g.B * g.ks * g.D * 2)), gg((unsigned)nwg);
    const bool div = g.recip == 0.f;
    if (kt) {
      hipLaunchKernelGGL(fmap_split_kernel<true>, pg, dim3(256), 0, stream, src, fp, g);
      if (div)
        hipLaunchKernelGGL((fmap_grad_kernel<true, true>), gg, dim3(NTHR), 0, stream, gp, fp, part, g);
      else
        hipLaunchKernelGGL((fmap_grad_kernel<true, false>), gg, dim3(NTHR), 0, stream, gp, fp, part, g);
    } else {
      hipLaunchKernelGGL(fmap_split_kernel<false>, pg, dim3(256), 0, stream, src, fp, g);
      if (div)
        hipLaunchKernelGGL((fmap_grad_kernel<false, true>), gg, dim3(NTHR), 0, stream, gp, fp, part, g);
      else
        hipLaunchKernelGGL((fmap_grad_kernel<false, false>), gg, dim3(NTHR), 0, stream, gp, fp, part, g);
    }
    if (g.S > 1) {
      const long long n = (long long)g.B * g.D * g.N;
      hipLaunchKernelGGL(chunk_sum_kernel, dim3(grid_for(n)), dim3(256), 0, stream, part, dst, n, g.S);
    }
    const int st = dxr::launch_status();
    if (st != DXR_OK) return st;
  }
  return DXR_OK;
}
