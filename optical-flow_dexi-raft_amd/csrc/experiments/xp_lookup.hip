// Experiments target only (libdexiraft_corr_exp.so, build.py --experiments):
// timing ablations and layout variants of the lookup (csrc/corr_lookup.hip).
// Never loaded by the package.  The lookup backward's r <= 5 launch bound is 6
// waves per SIMD here (the product: 8), so this library's
// dxr_corr_lookup_backward_multi[_bound] is that A/B variant.
#define BW_WAVES_SMALL_R 6
#include "../corr_lookup.hip"

namespace {

// XP bits: 0 skip the window gathers, 1 skip phase 2 (return after the gather),
// 2 return after phase 0, 3 synthetic coordinates (the grid: no coords loads),
// 5 query-major gather slots on levels 2/3 (gather_slot QMAJ; now the product's),
// 64 / 128: the product kernel at 256 threads x 16 queries / 1024 x 64,
// 8 record a per-workgroup timeline (s_memrealtime at start, after phase 0,
// after the gather, at the end; plus the hardware id) into `trace`.
template <int R, typename PT, int XP>
__global__ __launch_bounds__(512) void xp_lookup_kernel(const PT* __restrict__ pyr,
                                                        const float* __restrict__ coords,
                                                        float* __restrict__ out, LookupGeom g,
                                                        unsigned long long* __restrict__ trace) {
  using C = WideCfg<R, 512>;
  constexpr int RD = C::RD, RS = C::RS, K = C::K, QB = C::QB;
  __shared__ __attribute__((aligned(16))) float cells[QB * C::QS];
  __shared__ float4 xs[RD * QB];
  __shared__ float4 ys[RD * QB];
  __shared__ int2 org[QB];
  const unsigned long long t0 = (XP & 256) ? __builtin_amdgcn_s_memrealtime() : 0ull;

  const int tid = threadIdx.x;
  const int l = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * QB;
  const LevelAddr A = g.lv[l];

  if constexpr ((XP & 8) != 0) {
    // synthetic coordinates: the identity grid scaled, no global loads
    using CC = WideCfg<R, 512>;
    const int slot = tid;
    if (slot < QB * CC::G) {
      const int j = slot & (CC::G - 1), qq = slot >> CC::LG, q = q0 + qq;
      const int W1 = 128;
      const float cx = (float)(q % W1) + 0.37f, cy = (float)(q / W1) + 0.61f;
      const float inv = 1.f / (float)(1 << l);
      const float wm1 = (float)(A.w - 1), hm1 = (float)(A.h - 1);
      const float ux = sample_coord(__fadd_rn(cx * inv, (float)(j - R)), wm1, wm1 / 2.f);
      const float uy = sample_coord(__fadd_rn(cy * inv, (float)(j - R)), hm1, hm1 / 2.f);
      const float flx = floorf(ux), fly = floorf(uy);
      const bool act = j < RD;
      int mx = act ? (int)flx - j : 0x7fffffff, my = act ? (int)fly - j : 0x7fffffff;
#pragma unroll
      for (int o = 1; o < CC::G; o <<= 1) {
        mx = min(mx, __shfl_xor(mx, o));
        my = min(my, __shfl_xor(my, o));
      }
      const bool far = mx + CC::WD <= 0 || mx >= A.w || my + CC::WD <= 0 || my >= A.h;
      if (j == 0) org[qq] = far ? make_int2(FAR_ORIGIN, FAR_ORIGIN) : make_int2(mx, my);
      if (act) {
        const float fx = __fsub_rn(ux, flx), fy = __fsub_rn(uy, fly);
        const int col = far ? 0 : (int)flx - (mx & ~3);
        const int row = far ? 0 : ((int)fly - my) * RS;
        xs[j * QB + qq] = make_float4(__int_as_float(col), fx, __fsub_rn(1.f, fx), 0.f);
        ys[j * QB + qq] = make_float4(__int_as_float(row), fy, __fsub_rn(1.f, fy), 0.f);
      }
    }
  } else {
    wide_phase0<R, 512>(coords, g, A, b, l, q0, tid, xs, ys, org);
  }
  __syncthreads();
  const unsigned long long t1 = (XP & 256) ? __builtin_amdgcn_s_memrealtime() : 0ull;
  auto record = [&](unsigned long long t2, unsigned long long t3) {
    if constexpr ((XP & 256) != 0) {
      if (tid < 5) {
        const long long wg = ((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        const unsigned long long hw = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                                      ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11)) << 32);
        const unsigned long long v = tid == 0 ? t0 : tid == 1 ? t1 : tid == 2 ? t2 : tid == 3 ? t3 : hw;
        trace[wg * 5 + tid] = v;
      }
    }
  };
  if constexpr ((XP & 4) != 0) {
    if (xs[tid % (RD * QB)].y == 1234.5f) out[tid] = 0.f;
    record(t1, t1);
    return;
  }

  if constexpr ((XP & 1) == 0) {
    const PT* base = pyr + A.off + ((long long)b * A.qt + (q0 >> A.lqb)) * A.qstride;
    const int qb0 = q0 & ((1 << A.lqb) - 1);
    constexpr bool QM = (XP & 32) != 0;   // query-major slots on levels 2/3
    if (A.lth == 30)
      gather_windows<R, 512, 1, PT>(base, qb0, A, org, cells, q0, g.N, tid);
    else if (A.tw >= 8)
      gather_windows<R, 512, 4, PT>(base, qb0, A, org, cells, q0, g.N, tid);
    else if (A.tw == 4)
      gather_windows<R, 512, 4, PT, QM>(base, qb0, A, org, cells, q0, g.N, tid);
    else if (A.tw == 2)
      gather_windows<R, 512, 2, PT, QM>(base, qb0, A, org, cells, q0, g.N, tid);
    else
      gather_windows<R, 512, 1, PT>(base, qb0, A, org, cells, q0, g.N, tid);
  }
  __syncthreads();
  const unsigned long long t2 = (XP & 256) ? __builtin_amdgcn_s_memrealtime() : 0ull;
  if constexpr ((XP & 2) != 0) {
    if (cells[tid] == 1234.5f) out[tid] = 0.f;
    record(t2, t2);
    return;
  }

  if constexpr ((XP & 16) != 0) {
    // outputs of the thread's (query, class) slots in registers, then through
    // LDS as [k][QB] rows, stored as 16-byte write-through (sc1) vectors of 4
    // consecutive queries (N % 4 == 0, checked by the host)
    constexpr int NKT = (K + C::NCLS - 1) / C::NCLS;
    const int qq = tid % QB, cls = tid / QB;
    float rv[NKT];
    {
      const float* cq = cells + qq * C::QS;
#pragma unroll
      for (int i = 0; i < NKT; ++i) {
        const int k = cls + i * C::NCLS;
        rv[i] = 0.f;
        if (k < K) {
          const int ox = k / RD, oy = k - ox * RD;
          const float4 xd = xs[ox * QB + qq], yd = ys[oy * QB + qq];
          const float* p = cq + __float_as_int(yd.x) + __float_as_int(xd.x);
          const float v00 = p[0], v01 = p[1], v10 = p[RS], v11 = p[RS + 1];
          const float nw = __fmul_rn(yd.z, xd.z), ne = __fmul_rn(yd.z, xd.y);
          const float sw = __fmul_rn(yd.y, xd.z), se = __fmul_rn(yd.y, xd.y);
          float r = __fmul_rn(nw, v00);
          r = __builtin_fmaf(ne, v01, r);
          r = __builtin_fmaf(sw, v10, r);
          rv[i] = __builtin_fmaf(se, v11, r);
        }
      }
    }
    __syncthreads();   // cells are free
#pragma unroll
    for (int i = 0; i < NKT; ++i) {
      const int k = cls + i * C::NCLS;
      if (k < K) cells[k * QB + qq] = rv[i];
    }
    __syncthreads();
    float* ob0 = out + ((long long)b * g.cout + (long long)l * K) * g.N + q0;
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(ob0, (short)0, 0x7fffffff, 0x00020000);
    for (int s = tid; s < K * (QB / 4); s += C::NT) {
      const int k = s / (QB / 4), qa = 4 * (s % (QB / 4));
      const float4 v = *reinterpret_cast<const float4*>(cells + k * QB + qa);
      if (q0 + qa + 3 < g.N) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4 w = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                      __float_as_uint(v.w)};
        __builtin_amdgcn_raw_buffer_store_b128(w, ro, (unsigned)(k * g.N + qa) * 4u, 0, 16);
      }
    }
    if constexpr ((XP & 256) != 0) {
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      record(t2, __builtin_amdgcn_s_memrealtime());
    }
    return;
  }
  const int qq = tid % QB, cls = tid / QB;
  if (q0 + qq < g.N) {
    const float* cq = cells + qq * C::QS;
    float* ob = out + ((long long)b * g.cout + (long long)l * K) * g.N + q0 + qq;
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
      __hip_atomic_store(ob + (unsigned)(k * g.N), r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if constexpr ((XP & 256) != 0) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    record(t2, __builtin_amdgcn_s_memrealtime());
  }
}

template <int XP, typename PT>
int xp_launch(const PT* pyr, const float* coords, float* out, const LookupGeom& g, int B,
              unsigned long long* trace, hipStream_t stream) {
  using W = WideCfg<4>;
  const dim3 grid((unsigned)((g.N + W::QB - 1) / W::QB), (unsigned)g.levels, (unsigned)B);
  hipLaunchKernelGGL((xp_lookup_kernel<4, PT, XP>), grid, dim3(512), 0, stream, pyr, coords, out,
                     g, trace);
  return dxr::launch_status();
}

// The product kernel with another workgroup shape: NT threads x QB queries
// (the same 16 threads per query as the product's 512 x 32).
template <int NT, int QB, typename PT>
int xp_shape(const PT* pyr, const float* coords, float* out, const LookupGeom& g0, int B,
             hipStream_t stream, int out_nt = 0) {
  LookupGeom g = g0;
  g.out_nt = out_nt;
  const dim3 grid((unsigned)((g.N + QB - 1) / QB), (unsigned)g.levels, (unsigned)B);
  hipLaunchKernelGGL((corr_lookup_wide_kernel<4, PT, NT, QB>), grid, dim3(NT), 0, stream, pyr,
                     coords, out, g);
  return dxr::launch_status();
}

typedef __attribute__((address_space(3))) void xl_lds_void_t;

// Round 6: the wide kernel with its window gathers by
// LDS-DMA (buffer_load ... lds, 16 B per lane) on the f32 paged levels whose
// tile rows hold >= 4 cells and whose width is a multiple of 4 (no partial
// vectors): the per-query LDS block of QS = 180 floats is 45 16-B granules (44
// window vectors + the bank-skew granule), so granule g of the workgroup's
// staging area is (query g / 45, vector g % 45) and a wave instruction covers
// 64 consecutive granules, lane-linear as the DMA writes them; the skew granules
// get an out-of-range offset (zeros).  Off-level rows / vectors and far queries
// read as zero by the range check.  Other levels keep the register gather.
template <int R, typename PT, int NT_, int QB_>
__global__ __launch_bounds__(NT_) void xp_lookup_dma_kernel(const PT* __restrict__ pyr,
                                                           const float* __restrict__ coords,
                                                           float* __restrict__ out, LookupGeom g) {
  using C = WideCfg<R, NT_, QB_>;
  constexpr int RD = C::RD, RS = C::RS, K = C::K, QB = C::QB, NT = NT_;
  static_assert(C::QS == 4 * (C::WD * C::NQ + 1), "one skew granule per query");
  constexpr int GQ = C::QS / 4, NG = QB * GQ, GIT = (NG + NT - 1) / NT;
  // every lane of a DMA instruction writes its 16 B (zeros when out of range):
  // the staging area is padded to whole 64-granule wave instructions
  __shared__ __attribute__((aligned(16))) float cells[((NG + 63) / 64) * 64 * 4];
  __shared__ float4 xs[RD * QB];
  __shared__ float4 ys[RD * QB];
  __shared__ int2 org[QB];
  const int tid = threadIdx.x;
  const int l = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * QB;
  const LevelAddr A = g.lv[l];
  if constexpr (QB_ <= 16) {
    if (l == 0) __builtin_amdgcn_s_setprio(3);
    else if (l == 1) __builtin_amdgcn_s_setprio(2);
    else if (l == 2) __builtin_amdgcn_s_setprio(1);
  }
  wide_phase0<R, NT_, QB_>(coords, g, A, b, l, q0, tid, xs, ys, org);
  __syncthreads();
  {
    const PT* base = pyr + A.off + ((long long)b * A.qt + (q0 >> A.lqb)) * A.qstride;
    const int qb0 = q0 & ((1 << A.lqb) - 1);
    if (sizeof(PT) == 4 && A.lth != 30 && A.tw >= 4 && (A.w & 3) == 0) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<PT*>(base), (short)0, 0x7fffffff, 0x00020000);
      const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
#pragma unroll
      for (int i = 0; i < GIT; ++i) {
        const int gw = i * NT + wave * 64;            // the wave's first granule (uniform)
        if (gw >= NG) break;
        const int gi = gw + lane, qq = gi / GQ, rem = gi - qq * GQ;
        uint32_t voff = 0x80000000u;
        if (gi < NG && rem < GQ - 1 && q0 + qq < g.N) {
          const int2 o = org[qq];
          const int r = rem / C::NQ, k = rem - r * C::NQ;
          const int yy = o.y + r, x0 = (o.x & ~3) + 4 * k;
          if (o.x != FAR_ORIGIN && (unsigned)yy < (unsigned)A.h && x0 >= 0 && x0 < A.w) {
            const unsigned tl = __umul24((unsigned)(yy >> A.lth), (unsigned)A.tx) + (unsigned)(x0 >> A.ltw);
            const unsigned e = ((unsigned)(qb0 + qq) << A.lS) + (tl << A.lpS) +
                               ((unsigned)(yy & A.mh) << A.ltw) + (unsigned)(x0 & A.mw);
            voff = e * 4u;
          }
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (xl_lds_void_t*)(cells + gw * 4), 16, voff, 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (A.lth == 30) {
      gather_windows<R, NT_, 1, PT, false, QB_>(base, qb0, A, org, cells, q0, g.N, tid);
    } else if (A.tw >= 8) {
      gather_windows<R, NT_, 4, PT, false, QB_>(base, qb0, A, org, cells, q0, g.N, tid);
    } else if (A.tw == 4) {
      gather_windows<R, NT_, 4, PT, true, QB_>(base, qb0, A, org, cells, q0, g.N, tid);
    } else if (A.tw == 2) {
      gather_windows<R, NT_, 2, PT, true, QB_>(base, qb0, A, org, cells, q0, g.N, tid);
    } else {
      gather_windows<R, NT_, 1, PT, false, QB_>(base, qb0, A, org, cells, q0, g.N, tid);
    }
  }
  __syncthreads();
  const int qq = tid % QB, cls = tid / QB;
  if (q0 + qq >= g.N) return;
  const float* cq = cells + qq * C::QS;
  float* op = out + ((long long)b * g.cout + (long long)l * K + cls) * g.N + q0 + qq;
  const long long ostep = (long long)C::NCLS * g.N;
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
    if (g.out_nt) __builtin_nontemporal_store(r, op);
    else __hip_atomic_store(op, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    op += ostep;
  }
}

template <typename PT>
int xp_dma_launch(const PT* pyr, const float* coords, float* out, const LookupGeom& g0, int B,
                  hipStream_t stream) {
  // launch_lookup_r's shape and output policy
  using W = WideCfg<4>;
  LookupGeom g = g0;
  const long long wg32 = (long long)((g.N + W::QB - 1) / W::QB) * g.levels * B;
  const double pyr_bytes = (double)B * g.lv[0].qt * (double)g.lv[0].qstride * sizeof(PT) * (4.0 / 3.0);
  const bool big_misaligned = g.N % 32 != 0 && pyr_bytes >= 128.0 * (1 << 20);
  if (wg32 <= 1024 && !big_misaligned) {
    g.out_nt = g.N % 32 == 0 ? 1 : 0;
    const dim3 grid((unsigned)((g.N + 15) / 16), (unsigned)g.levels, (unsigned)B);
    hipLaunchKernelGGL((xp_lookup_dma_kernel<4, PT, 256, 16>), grid, dim3(256), 0, stream, pyr,
                       coords, out, g);
    return dxr::launch_status();
  }
  g.out_nt = 1;
  const dim3 grid((unsigned)((g.N + 31) / 32), (unsigned)g.levels, (unsigned)B);
  hipLaunchKernelGGL((xp_lookup_dma_kernel<4, PT, 512, 32>), grid, dim3(512), 0, stream, pyr,
                     coords, out, g);
  return dxr::launch_status();
}

template <typename PT>
int xp_dispatch(int xp, const PT* pyr, const float* coords, float* out, const LookupGeom& g, int B,
                unsigned long long* trace, hipStream_t stream) {
  switch (xp) {
    case 64: return xp_shape<256, 16>(pyr, coords, out, g, B, stream);
    case 65: return xp_shape<128, 8>(pyr, coords, out, g, B, stream);
    case 66: return xp_shape<512, 32>(pyr, coords, out, g, B, stream);   // the product's multi-round shape
    case 67: return xp_shape<512, 32>(pyr, coords, out, g, B, stream, 1);   // + non-temporal outputs
    case 68: return xp_shape<256, 16>(pyr, coords, out, g, B, stream, 1);
    case 69: return xp_shape<128, 8>(pyr, coords, out, g, B, stream, 1);
    case 70: return xp_shape<1024, 64>(pyr, coords, out, g, B, stream, 1);
    case 128: return xp_shape<1024, 64>(pyr, coords, out, g, B, stream);
    // round 6: query-minor staging (corr_lookup_qm_kernel) with the product's
    // shape / output policy; 91: 256 x 32 on one-round grids
    case 89: return launch_lookup_wide_r<4, PT>(pyr, coords, out, g, B, stream);   // the round-5 product
    case 90: return launch_lookup_r<4, PT, 16, 1, false, false>(pyr, coords, out, g, B, stream);
    case 91: return launch_lookup_r<4, PT, 32, 1, false, false>(pyr, coords, out, g, B, stream);
    case 92: return xp_dma_launch(pyr, coords, out, g, B, stream);   // LDS-DMA gathers
    case 93: return launch_lookup_r<4, PT, 16, 2, false, false>(pyr, coords, out, g, B, stream);  // phase 2 x2
    case 94: return launch_lookup_r<4, PT, 16, 1, true, true>(pyr, coords, out, g, B, stream);  // buffer loads
    // multi-round grids at 256 x 32 / 256 x 16 (the product: 512 x 32)
    case 95: return launch_lookup_r<4, PT, 16, 1, false, true, 0, 256, 32>(pyr, coords, out, g, B, stream);
    case 96: return launch_lookup_r<4, PT, 16, 1, false, true, 0, 256, 16>(pyr, coords, out, g, B, stream);
    // product shapes, timing ablations: no gathers / no output stores / phase 0 only
    case 97: return launch_lookup_r<4, PT, 16, 1, false, true, 1>(pyr, coords, out, g, B, stream);
    case 98: return launch_lookup_r<4, PT, 16, 1, false, true, 2>(pyr, coords, out, g, B, stream);
    case 99: return launch_lookup_r<4, PT, 16, 1, false, true, 4>(pyr, coords, out, g, B, stream);
    case 0: return xp_launch<0>(pyr, coords, out, g, B, trace, stream);
    case 1: return xp_launch<1>(pyr, coords, out, g, B, trace, stream);
    case 2: return xp_launch<2>(pyr, coords, out, g, B, trace, stream);
    case 4: return xp_launch<4>(pyr, coords, out, g, B, trace, stream);
    case 8: return xp_launch<8>(pyr, coords, out, g, B, trace, stream);
    case 12: return xp_launch<12>(pyr, coords, out, g, B, trace, stream);
    case 16: return xp_launch<16>(pyr, coords, out, g, B, trace, stream);
    case 256: return xp_launch<256>(pyr, coords, out, g, B, trace, stream);
    case 272: return xp_launch<272>(pyr, coords, out, g, B, trace, stream);
    case 264: return xp_launch<264>(pyr, coords, out, g, B, trace, stream);
    case 258: return xp_launch<258>(pyr, coords, out, g, B, trace, stream);
    case 260: return xp_launch<260>(pyr, coords, out, g, B, trace, stream);
    case 32: return xp_launch<32>(pyr, coords, out, g, B, trace, stream);
    case 288: return xp_launch<288>(pyr, coords, out, g, B, trace, stream);
    default: return DXR_EINVAL;
  }
}

}  // namespace

// Variant `xp` of the radius-4 lookup (see xp_lookup_kernel); trace: 5 x u64
// per workgroup when xp has bit 8.
extern "C" int dxr_xp_lookup(const void* pyramid, int pyr_dtype, int64_t B, int64_t H, int64_t W,
                             int num_levels, const float* coords, float* out, int xp,
                             unsigned long long* trace, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L) || num_levels > 4) return DXR_EINVAL;
  LookupGeom g;
  g.N = (int)(H * W);
  g.levels = num_levels;
  g.cout = num_levels * 81;
  for (int l = 0; l < L.n; ++l) g.lv[l] = level_addr(L.lay[l]);
  if (pyr_dtype == DXR_F32)
    return xp_dispatch(xp, static_cast<const float*>(pyramid), coords, out, g, (int)B, trace,
                       stream);
  return xp_dispatch(xp, static_cast<const uint16_t*>(pyramid), coords, out, g, (int)B, trace,
                     stream);
}
