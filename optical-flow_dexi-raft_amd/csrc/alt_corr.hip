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
#include "dxr_common.h"

namespace {

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
  long long f1_bstride;   // H1 * W1 * C
  long long coord_zstride, coord_cstride, coord_qstride;
  AltLevel lv[8];
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
               int Z, int radius, bool vec, hipStream_t stream) {
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
  g.f1_bstride = H1 * W1 * C;
  g.coord_zstride = H1 * W1 * 2;
  g.coord_cstride = 1;
  g.coord_qstride = 2;
  g.lv[0] = AltLevel{fmap2, (int)H2, (int)W2, 1.f, 0};
  const bool vec = (C % 4 == 0) && aligned16(fmap1) && aligned16(fmap2);
  return launch_alt(fmap1, coords, corr, g, 1, (int)(B * Nc), radius, vec, stream);
}

extern "C" int dxr_alt_corr_lookup(const float* fmap1, const float* const* fmap2_levels,
                                   const float* coords, float* out, int64_t B, int64_t H,
                                   int64_t W, int64_t C, int num_levels, int radius,
                                   float divisor, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L)) return DXR_EINVAL;
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
  g.f1_bstride = H * W * C;
  g.coord_zstride = 2 * H * W;
  g.coord_cstride = H * W;
  g.coord_qstride = 1;
  bool vec = (C % 4 == 0) && aligned16(fmap1);
  for (int l = 0; l < num_levels; ++l) {
    if (!fmap2_levels[l]) return DXR_EINVAL;
    vec = vec && aligned16(fmap2_levels[l]);
    g.lv[l] = AltLevel{fmap2_levels[l], L.h[l], L.w[l], 1.f / (float)(1 << l), l * rd * rd};
  }
  return launch_alt(fmap1, coords, out, g, num_levels, (int)B, radius, vec, stream);
}
