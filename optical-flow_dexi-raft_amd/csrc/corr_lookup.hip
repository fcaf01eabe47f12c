// Stage (c): radius-r bilinear lookup into every pyramid level, one launch.
//
// Replaces core/corr.py:29-50 (CorrBlock.__call__) and the helper it calls,
// core/utils/utils.py:57-71 (bilinear_sampler -> F.grid_sample with
// align_corners=True, bilinear, zero padding).  The reference builds a
// (2r+1)^2 delta grid on the host and copies it to the device per level per
// call (core/corr.py:37-39), runs one grid_sample per level, then cat + permute
// + contiguous.  Here one kernel writes the final [B, L*(2r+1)^2, H, W] tensor.
//
// Arithmetic follows the reference sample by sample:
//   c   = coords / 2^l + (o - r)                            (core/corr.py:41-43)
//   g   = 2*c / (S_l - 1) - 1                               (utils.py:61-62)
//   u   = (g + 1) * ((S_l - 1) / 2)                         (grid_sample unnormalise)
//   taps at floor(u), floor(u)+1, weights (1-f, f), f = u - floor(u), out-of-range
//   taps contribute 0, and the four products are summed as the fused chain
//   fma(se, v_se, fma(sw, v_sw, fma(ne, v_ne, nw*v_nw))) — the exact arithmetic of
//   the reference's compiled CPU grid sampler (bit-exact on the golden vectors).
// Consecutive samples of one query share taps, so a thread loads a
// (2r+2) x (OXG+1) window once and produces OXG x (2r+1) outputs.  A sample whose
// normalise/unnormalise round trip lands a few ulps across an integer keeps the
// window's cell and gets a fraction of -eps or 1+eps: the value equals the
// reference's up to eps * |cell difference|.
//
// Thread mapping: lanes = consecutive query pixels of one (pair, level, x-group),
// so every output store is a coalesced 256-byte wave store.
#include "dxr_common.h"

namespace {

struct LookupGeom {
  int N;          // H * W query pixels per pair
  int levels;
  int groups;     // x-offset groups per level
  int cout;       // levels * (2r+1)^2
  int lh[8], lw[8];
  long long loff[8];
};

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

template <int R, int OXG, typename PT>
__global__ __launch_bounds__(256) void corr_lookup_kernel(const PT* __restrict__ pyr,
                                                          const float* __restrict__ coords,
                                                          float* __restrict__ out,
                                                          LookupGeom g) {
  constexpr int RD = 2 * R + 1;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= g.N) return;
  const int l = blockIdx.y / g.groups;
  const int grp = blockIdx.y % g.groups;
  const int b = blockIdx.z;
  const int ox0 = grp * OXG;

  const int Hl = g.lh[l], Wl = g.lw[l];
  float* obase = out + ((long long)b * g.cout + (long long)l * RD * RD) * g.N + q;

  if (Hl == 1 || Wl == 1) {
    // bilinear_sampler divides by zero (utils.py:61-62): the reference returns NaN.
#pragma unroll
    for (int j = 0; j < OXG; ++j) {
      if (ox0 + j >= RD) break;
#pragma unroll
      for (int oy = 0; oy < RD; ++oy)
        obase[(long long)((ox0 + j) * RD + oy) * g.N] = __builtin_nanf("");
    }
    return;
  }

  const float inv = 1.f / (float)(1 << l);  // exact power of two
  const float xc = coords[((long long)b * 2 + 0) * g.N + q] * inv;
  const float yc = coords[((long long)b * 2 + 1) * g.N + q] * inv;
  const float wm1 = (float)(Wl - 1), hm1 = (float)(Hl - 1);
  const float whalf = wm1 / 2.f, hhalf = hm1 / 2.f;

  float ys[RD], xs[OXG];
#pragma unroll
  for (int oy = 0; oy < RD; ++oy) ys[oy] = sample_coord(__fadd_rn(yc, (float)(oy - R)), hm1, hhalf);
#pragma unroll
  for (int j = 0; j < OXG; ++j) xs[j] = sample_coord(__fadd_rn(xc, (float)(ox0 + j - R)), wm1, whalf);

  const float ybf = floorf(ys[0]);
  const float xbf = floorf(xs[0]);
  // Far-away or non-finite windows: every tap is outside the level (weights
  // still carry NaN/inf through, as in the reference).
  const bool near = fabsf(ybf) < 1.0e8f && fabsf(xbf) < 1.0e8f;
  const int yb = near ? (int)ybf : -(1 << 28);
  const int xb = near ? (int)xbf : -(1 << 28);

  float fx[OXG], ex[OXG];
#pragma unroll
  for (int j = 0; j < OXG; ++j) {
    fx[j] = __fsub_rn(xs[j], __fadd_rn(xbf, (float)j));
    ex[j] = __fsub_rn(1.f, fx[j]);
  }

  const PT* img = pyr + g.loff[l] + ((long long)b * g.N + q) * ((long long)Hl * Wl);
  bool colok[OXG + 1];
#pragma unroll
  for (int c = 0; c <= OXG; ++c) colok[c] = (unsigned)(xb + c) < (unsigned)Wl;

  float prev[OXG + 1];
#pragma unroll
  for (int rr = 0; rr <= RD; ++rr) {
    const int yy = yb + rr;
    const bool rowok = (unsigned)yy < (unsigned)Hl;
    float cur[OXG + 1];
#pragma unroll
    for (int c = 0; c <= OXG; ++c)
      cur[c] = (rowok && colok[c]) ? load_cell(img + (long long)yy * Wl + (xb + c)) : 0.f;
    if (rr > 0) {
      const int oy = rr - 1;
      const float n = __fsub_rn(ys[oy], __fadd_rn(ybf, (float)oy));
      const float s = __fsub_rn(1.f, n);
#pragma unroll
      for (int j = 0; j < OXG; ++j) {
        if (ox0 + j >= RD) break;
        const float nw = __fmul_rn(s, ex[j]), ne = __fmul_rn(s, fx[j]);
        const float sw = __fmul_rn(n, ex[j]), se = __fmul_rn(n, fx[j]);
        float v = __fmul_rn(nw, prev[j]);
        v = __builtin_fmaf(ne, prev[j + 1], v);
        v = __builtin_fmaf(sw, cur[j], v);
        v = __builtin_fmaf(se, cur[j + 1], v);
        obase[(long long)((ox0 + j) * RD + oy) * g.N] = v;
      }
    }
#pragma unroll
    for (int c = 0; c <= OXG; ++c) prev[c] = cur[c];
  }
}

template <int R, typename PT>
int launch_lookup_r(const PT* pyr, const float* coords, float* out, LookupGeom g, int B,
                    hipStream_t stream) {
  constexpr int RD = 2 * R + 1;
  constexpr int OXG = RD <= 3 ? RD : (RD % 3 == 0 ? 3 : 4);
  g.groups = (RD + OXG - 1) / OXG;
  const dim3 grid((unsigned)((g.N + 255) / 256), (unsigned)(g.levels * g.groups), (unsigned)B);
  hipLaunchKernelGGL((corr_lookup_kernel<R, OXG, PT>), grid, dim3(256), 0, stream, pyr, coords,
                     out, g);
  return dxr::launch_status();
}

template <typename PT>
int launch_lookup(const PT* pyr, const float* coords, float* out, LookupGeom g, int B, int radius,
                  hipStream_t stream) {
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
  g.groups = 1;
  g.cout = num_levels * rd * rd;
  for (int l = 0; l < 8; ++l) {
    g.lh[l] = l < L.n ? L.h[l] : 1;
    g.lw[l] = l < L.n ? L.w[l] : 1;
    g.loff[l] = l < L.n ? L.off[l] : 0;
  }
  if (pyr_dtype == DXR_F32)
    return launch_lookup(static_cast<const float*>(pyramid), coords, out, g, (int)B, radius, stream);
  if (pyr_dtype == DXR_BF16)
    return launch_lookup(static_cast<const uint16_t*>(pyramid), coords, out, g, (int)B, radius,
                         stream);
  return DXR_EINVAL;
}
