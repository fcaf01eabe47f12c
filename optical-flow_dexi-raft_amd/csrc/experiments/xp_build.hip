// Experiments target only (libdexiraft_corr_exp.so, build.py --experiments):
// timing ablations and a per-workgroup timeline of the pre-split LDS-DMA f32
// build (csrc/corr_build.hip corr_build_dma_kernel).  Never loaded by the package.
// (The builds' pyramid store policy is chosen per launch, dma_stream_out; its
// A/Bs are profiles/r05/experiments/r5x_*, r6n_* and r6q_*.)
#include "../corr_build.hip"

namespace {

// The split pass as first written in round 3 (plain stores), for A/B (XP bit 5).
__global__ __launch_bounds__(1024) void xp_split_plain_kernel(const float* __restrict__ f1,
                                                              const float* __restrict__ f2,
                                                              uint4* __restrict__ sp1,
                                                              uint4* __restrict__ sp2,
                                                              int* __restrict__ e1,
                                                              int* __restrict__ e2, int D, int N) {
  __shared__ float red[16][65];
  const int tid = threadIdx.x;
  const int kb0 = tid >> 6, pl = tid & 63;
  const int p = blockIdx.x * 64 + pl;
  const bool live = p < N;
  const int b = blockIdx.y;
  const float* src = (blockIdx.z == 0 ? f1 : f2) + (long long)b * D * N;
  uint4* sp = (blockIdx.z == 0 ? sp1 : sp2) + (long long)b * (D / 16) * N * 4;
  int* ex = (blockIdx.z == 0 ? e1 : e2) + (long long)b * N;
  float x[16];
  float m = 0.f;
  if (live && kb0 < D / 16) {
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = src[(long long)(kb0 * 16 + i) * N + p];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float a = __builtin_fabsf(x[i]);
      m = (m < 0.f || !(a <= 3.40282347e38f)) ? -1.f : (a > m ? a : m);
    }
  }
  red[kb0][pl] = m;
  __syncthreads();
  float mm = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const float v = red[k][pl];
    mm = (mm < 0.f || v < 0.f) ? -1.f : (v > mm ? v : mm);
  }
  if (!live || kb0 >= D / 16) return;
  const int s = pixel_scale(mm < 0.f ? 0.f : mm, mm >= 0.f);
  if (kb0 == 0) ex[p] = s;
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = __builtin_ldexpf(x[i], s);
  uint32_t h[8], l[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h[e] = cvt_pk_f16(x[2 * e], x[2 * e + 1]);
    const f16x2_t hv = __builtin_bit_cast(f16x2_t, h[e]);
    f16x2_t lv;
    lv[0] = (_Float16)__builtin_fmaf((float)hv[0], -1.f, x[2 * e]);
    lv[1] = (_Float16)__builtin_fmaf((float)hv[1], -1.f, x[2 * e + 1]);
    l[e] = __builtin_bit_cast(uint32_t, lv);
  }
  uint4* dst = sp + ((long long)kb0 * N + p) * 4;
  dst[0] = make_uint4(h[0], h[1], h[2], h[3]);
  dst[1] = make_uint4(h[4], h[5], h[6], h[7]);
  dst[2] = make_uint4(l[0], l[1], l[2], l[3]);
  dst[3] = make_uint4(l[4], l[5], l[6], l[7]);
}

// XP bits: 0 skip the epilogue stores (K loop kept live), 1 skip the MFMAs,
// 5 the split pass with plain stores (A/B of the product's write-through stores),
// 2 no DMA after the first two ring stages (the loop reads those two stages
// again: same finite data, timing only), 3 no barrier in the K loop (timing
// only), 8 record per-workgroup s_memrealtime stamps {start, K loop done,
// epilogue stores done, hw id}.
// XP bit 9 (512): the second workgroup to start on a CU (per-CU arrival count,
// zeroed before the launch) sleeps `XP >> 12` x 100 ticks (1 us) first, so the
// two workgroups of a CU run out of phase from the first dispatch round on (one
// in its K loop while the other stores); later arrivals do not wait.
template <typename OT, bool DIV, int XP>
__global__ __launch_bounds__(2 * NT, 4) void xp_build_dma_kernel(
    const uint8_t* __restrict__ sp1, const uint8_t* __restrict__ sp2, const int* __restrict__ ex1,
    const int* __restrict__ ex2, OT* __restrict__ pyr, BuildGeom g,
    unsigned long long* __restrict__ trace, int* __restrict__ cu_arrivals) {
  if constexpr ((XP & 512) != 0) {
    __shared__ int order;
    if (threadIdx.x == 0) {
      const unsigned hw = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
      const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11)) & 7u;
      const unsigned cu = (hw >> 8) & 15u, sh = (hw >> 12) & 1u, se = (hw >> 13) & 7u;
      order = atomicAdd(cu_arrivals + (((xcc * 8u + se) * 2u + sh) * 16u + cu), 1);
    }
    __syncthreads();
    if (order == 1) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)(100 * (XP >> 12)))
        __builtin_amdgcn_s_sleep(8);
    }
  }
  const unsigned long long xt0 = (XP & 256) ? __builtin_amdgcn_s_memrealtime() : 0ull;
  constexpr int LDS_RING = DMA_RING * DMA_STAGE;
  constexpr int LDS_E = 2 * WAVES * 16 * P0 * 4;          // epilogue staging (8 waves)
  static_assert(LDS_E <= LDS_RING, "the epilogue staging aliases the ring");
  // one LDS array (cdna_hip_programming.md §5 item 4(a)): ring | target
  // exponents (128 int) | redo flag
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_RING + NTGT * 4 + 16];
  int* const sexp = reinterpret_cast<int*>(smem + LDS_RING);
  int* const redo = reinterpret_cast<int*>(smem + LDS_RING + NTGT * 4);

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
  const long long spstride = (long long)g.D * g.N * 4;   // SP bytes per pair

  // exponents: the lane's query, the tile's 128 targets (LDS, by tile pixel)
  const int qj = q0 + wave * 32 + j;
  const int sq = qj < g.N ? ex1[(long long)b * g.N + qj] : 0;
  if (tid < NTGT) {
    const int r = tid >> 4, c = tid & 15;
    const bool in = th0 + r < g.H && tw0 + c < g.W;
    sexp[tid] = in ? ex2[(long long)b * g.N + (th0 + r) * g.W + tw0 + c] : 0;
  }
  if (tid == 0) *redo = 0;

  const __amdgpu_buffer_rsrc_t rq =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp1 + b * spstride), (short)0,
                                        (int)spstride, 0x00020000);
  const __amdgpu_buffer_rsrc_t rt =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp2 + b * spstride), (short)0,
                                        (int)spstride, 0x00020000);
  // DMA source offsets (fixed over K; the step's offset ks * N * 64 in soffset).
  // Query instruction i of this wave: LDS rows 16 i + (lane >> 2) of the wave's
  // 2 KB region; target instruction: tile row r = wave.
  uint32_t vq[2], vt;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * i + (lane >> 2), ps = lane & 3;
    const int q = q0 + wave * 32 + row;
    const int cq = ps ^ ((row >> 2) & 3);
    vq[i] = q < g.N ? (uint32_t)(q * 64 + 16 * cq) : 0x80000000u;
  }
  {
    const int ps = lane & 3, r = wave, col = lane >> 2, trow = r * 16 + col;
    const int ct = ps ^ (((trow >> 2) & 1) | ((trow >> 3) & 2));
    const int hh = th0 + r, ww = tw0 + col;
    vt = (hh < g.H && ww < g.W) ? (uint32_t)((hh * g.W + ww) * 64 + 16 * ct) : 0x80000000u;
  }
  auto dma = [&](int ks) {
    unsigned char* st = smem + (ks % DMA_RING) * DMA_STAGE;
    const int so = ks * g.N * 64;
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
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // exponent loads and LDS writes above must not count against the ring's vmcnt
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int nk = g.D / BKS;
  // XP bit 10: the K loop at wave priority 1 (wins issue arbitration against the
  // co-resident workgroup's epilogue waves); bit 11: the epilogue at priority 1
  if constexpr ((XP & 1024) != 0) __builtin_amdgcn_s_setprio(1);
  dma(0);
  if (nk > 1) dma(1);
  for (int ks = 0; ks < nk; ++ks) {
    // this wave's 3 DMAs of step ks have landed (those of ks + 1 stay in flight);
    // the barrier publishes every wave's, and orders the ring slot's previous
    // readers (step ks - 1) before the refill below
    if constexpr ((XP & 4) == 0) {
      if (ks + 1 < nk) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (ks < 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr ((XP & 8) == 0) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((XP & 16) == 0)
      if (ks + 2 < nk && (XP & 4) == 0) dma(ks + 2);
    const unsigned char* st = smem + ((XP & 4) ? (ks & 1) : (ks % DMA_RING)) * DMA_STAGE;
    const h8v qh = *reinterpret_cast<const h8v*>(st + qh_off);
    const h8v ql = *reinterpret_cast<const h8v*>(st + ql_off);
    h8v thv[4], tlv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      thv[t] = *reinterpret_cast<const h8v*>(st + th_off + t * 2048);
      tlv[t] = *reinterpret_cast<const h8v*>(st + tl_off + t * 2048);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const h8v th = thv[t], tl = tlv[t];
      // small terms first
      if constexpr ((XP & 2) != 0) {
        acc[t][0] += (float)(th[0] + tl[1] + qh[2] + ql[3]);
      } else {
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, qh, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ql, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, qh, acc[t], 0, 0, 0);
      }
      // XP bit 4: the next DMAs issue behind the first tile's MFMAs (their issue
      // cost then overlaps the matrix pipe instead of delaying the fragment reads)
      if constexpr ((XP & 16) != 0)
        if (t == 0 && ks + 2 < nk && (XP & 4) == 0) {
          __builtin_amdgcn_sched_barrier(0);
          dma(ks + 2);
          __builtin_amdgcn_sched_barrier(0);
        }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // ring reads done: the LDS is free for reuse
  if constexpr ((XP & 1024) != 0) __builtin_amdgcn_s_setprio(0);
  if constexpr ((XP & 2048) != 0) __builtin_amdgcn_s_setprio(1);
  const unsigned long long xt1 = (XP & 256) ? __builtin_amdgcn_s_memrealtime() : 0ull;

  // vote: a non-finite sum means an operand pixel was not finite; the
  // workgroup's pages are then recomputed from the f32 operands
  bool bad = false;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) bad |= !(__builtin_fabsf(acc[t][r]) <= 3.40282347e38f);
  if (bad) *redo = 1;
  __syncthreads();
  const bool live = pc.qblk + half < g.qt;            // this half's query block exists
  const long long page = pc.page + (live ? (long long)half * g.tiles_h * g.tiles_w : 0);
  if (*redo) {
    // (timing experiments run finite data only)
  } else {
    // undo the pixel scales: acc[t][r] is query qj x tile pixel (row 2t + kh, col r)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int4* se = reinterpret_cast<const int4*>(sexp + (2 * t + kh) * 16);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int4 s4 = se[u];
        acc[t][4 * u + 0] = __builtin_ldexpf(acc[t][4 * u + 0], -(sq + s4.x));
        acc[t][4 * u + 1] = __builtin_ldexpf(acc[t][4 * u + 1], -(sq + s4.y));
        acc[t][4 * u + 2] = __builtin_ldexpf(acc[t][4 * u + 2], -(sq + s4.z));
        acc[t][4 * u + 3] = __builtin_ldexpf(acc[t][4 * u + 3], -(sq + s4.w));
      }
    }
    if (live) {   // a half past the last query block has no page (epilogue syncs per wave)
      scale_acc<DIV>(acc, g);
      if constexpr ((XP & 1) != 0) {
        float sum = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) sum += acc[t][r];
        if (sum == 1234.5f) pyr[tid] = to_out<OT>(sum);  // keeps the K loop live
      } else if constexpr ((XP & 64) != 0) {   // non-temporal instead of write-through stores
        paged_epilogue<OT, 1 | 2>(acc, reinterpret_cast<float*>(smem) + half * WAVES * 16 * P0,
                                  pyr, g, page, w4, lane);
      } else if constexpr ((XP & 128) != 0) {  // plain (write-back) stores
        paged_epilogue<OT, 1>(acc, reinterpret_cast<float*>(smem) + half * WAVES * 16 * P0,
                              pyr, g, page, w4, lane);
      } else {
        paged_epilogue<OT, 1 | 4>(acc, reinterpret_cast<float*>(smem) + half * WAVES * 16 * P0,
                                  pyr, g, page, w4, lane);
      }
    }
  }
  if constexpr ((XP & 256) != 0) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const unsigned long long xt2 = __builtin_amdgcn_s_memrealtime();
    if (tid < 4) {
      const long long wg = blockIdx.x;
      const unsigned long long hw = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                                    ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11)) << 32);
      trace[wg * 4 + tid] = tid == 0 ? xt0 : tid == 1 ? xt1 : tid == 2 ? xt2 : hw;
    }
  }
}

template <int XP>
int xp_dma(const float* f1, const float* f2, float* pyr, const BuildGeom& g, int B, void* ws,
           unsigned long long* trace, hipStream_t stream) {
  const long long N = g.N, spb = align256((long long)B * g.D * N * 4), eb = align256((long long)B * N * 4);
  uint8_t* w = static_cast<uint8_t*>(ws);
  int* e1 = reinterpret_cast<int*>(w + 2 * spb);
  int* e2 = reinterpret_cast<int*>(w + 2 * spb + eb);
  if (XP & 32)   // the r03 split pass with plain (write-back) stores
    hipLaunchKernelGGL((xp_split_plain_kernel), dim3((unsigned)((N + 63) / 64), (unsigned)B, 2),
                       dim3(1024), 0, stream, f1, f2, reinterpret_cast<uint4*>(w),
                       reinterpret_cast<uint4*>(w + spb), e1, e2, g.D, g.N);
  else
    hipLaunchKernelGGL((split_pairs_kernel<false>), dim3((unsigned)((N + 63) / 64), (unsigned)B, 2),
                       dim3(1024), 0, stream, f1, f2, reinterpret_cast<uint4*>(w),
                       reinterpret_cast<uint4*>(w + spb), e1, e2, g.D, g.N);
  static int* arrivals = nullptr;
  if (XP & 512) {
    if (!arrivals && hipMalloc(&arrivals, 2048 * sizeof(int)) != hipSuccess) return DXR_EHIP;
    if (hipMemsetAsync(arrivals, 0, 2048 * sizeof(int), stream) != hipSuccess) return DXR_EHIP;
  }
  hipLaunchKernelGGL((xp_build_dma_kernel<float, false, (XP & ~32)>), remap_grid(g, B, 2), dim3(2 * NT), 0,
                     stream, w, w + spb, e1, e2, pyr, g, trace, arrivals);
  return dxr::launch_status();
}


// Split-pass variants for A/B (NCHW, D == 256): PX pixels x 16 channel blocks
// per workgroup (PX * 16 threads), lane -> pixel fastest; per-lane write-through
// record stores (the product transposes through LDS for whole-line stores).
template <int PX>
__global__ __launch_bounds__(PX * 16) void xp_split_px_kernel(const float* __restrict__ f1,
                                                              const float* __restrict__ f2,
                                                              uint4* __restrict__ sp1,
                                                              uint4* __restrict__ sp2,
                                                              int* __restrict__ e1,
                                                              int* __restrict__ e2, int D, int N) {
  __shared__ float red[16][PX + 1];
  const int tid = threadIdx.x;
  const int kb0 = tid / PX, pl = tid % PX;
  const int p = blockIdx.x * PX + pl;
  const bool live = p < N;
  const int b = blockIdx.y;
  const float* src = (blockIdx.z == 0 ? f1 : f2) + (long long)b * D * N;
  uint4* sp = (blockIdx.z == 0 ? sp1 : sp2) + (long long)b * (D / 16) * N * 4;
  int* ex = (blockIdx.z == 0 ? e1 : e2) + (long long)b * N;
  float x[16];
  float m = 0.f;
  if (live) {
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = src[(long long)(kb0 * 16 + i) * N + p];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float a = __builtin_fabsf(x[i]);
      m = (m < 0.f || !(a <= 3.40282347e38f)) ? -1.f : (a > m ? a : m);
    }
  }
  red[kb0][pl] = m;
  __syncthreads();
  float mm = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const float v = red[k][pl];
    mm = (mm < 0.f || v < 0.f) ? -1.f : (v > mm ? v : mm);
  }
  if (!live) return;
  const int s = pixel_scale(mm < 0.f ? 0.f : mm, mm >= 0.f);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(sp, (short)0, 0x7fffffff, 0x00020000);
  if (kb0 == 0) {
    const __amdgpu_buffer_rsrc_t re =
        __builtin_amdgcn_make_buffer_rsrc(ex, (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)s, re, (unsigned)p * 4u, 0, 16);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = __builtin_ldexpf(x[i], s);
  uint4 rec[4];
  split_record<false>(x, rec);
  const unsigned off = (unsigned)((kb0 * N + p) * 64);
#pragma unroll
  for (int c = 0; c < 4; ++c)   // per-lane 64-B records: partial-line write-through stores
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, rec[c]), rs, off + 16 * c, 0, 16);
}

// Persistent form of the DMA build (round 4 experiment): gridDim.x workgroups
// (a multiple of 8) walk the units (two query blocks x one tile) of the linear
// order; XCD k's workgroups take XCD k's contiguous range of units, local slot
// i taking units i, i + G/8, ...  XP bit 1: workgroups of the upper half of each
// XCD's slots first sleep `stagger` real-time ticks (10 ns), so that the two
// workgroups of a CU run out of phase (one in its K loop while the other
// stores).  Bit 8: per-unit s_memrealtime stamps {start, K loop done, stores
// done, hw id} at trace[4 * unit].  Finite data only (no recompute path).
template <typename OT, int XP>
__global__ __launch_bounds__(2 * NT, 4) void xp_build_persist_kernel(
    const uint8_t* __restrict__ sp1, const uint8_t* __restrict__ sp2, const int* __restrict__ ex1,
    const int* __restrict__ ex2, OT* __restrict__ pyr, BuildGeom g, long long nunits, int stagger,
    unsigned long long* __restrict__ trace) {
  constexpr int LDS_RING = DMA_RING * DMA_STAGE;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_RING + NTGT * 4 + 16];
  int* const sexp = reinterpret_cast<int*>(smem + LDS_RING);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave >> 2, w4 = wave & 3;
  const int j = lane & 31, kh = lane >> 5;
  const long long spstride = (long long)g.D * g.N * 4;
  const int per_xcd = gridDim.x / 8, xcd = blockIdx.x % 8, local = blockIdx.x / 8;
  const long long q8 = nunits / 8, r8 = nunits % 8;
  const long long ustart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const long long ucount = q8 + (xcd < r8 ? 1 : 0);
  if constexpr ((XP & 2) != 0) {
    if (local >= per_xcd / 2) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)stagger)
        __builtin_amdgcn_s_sleep(8);
    }
  }
  const int kq = (j >> 2) & 3;
  const int qh_off = wave * 2048 + j * 64 + 16 * (kh ^ kq);
  const int ql_off = wave * 2048 + j * 64 + 16 * ((2 + kh) ^ kq);
  const int trow0 = ((j >> 2) & 1) * 16 + (j & 3) + 4 * (j >> 3);
  const int kt = ((trow0 >> 2) & 1) | ((trow0 >> 3) & 2);
  const int th_off = DMA_TILE + trow0 * 64 + 16 * (kh ^ kt);
  const int tl_off = DMA_TILE + trow0 * 64 + 16 * ((2 + kh) ^ kt);
  const int nk = g.D / BKS;

  for (long long u = local; u < ucount; u += per_xcd) {
    const long long wl = ustart + u;
    const unsigned long long xt0 = (XP & 256) ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const PageCoord pc = unit_coord<2>(g, wl);
    const int th0 = pc.tyi * TH, tw0 = pc.txi * TW;
    const int q0 = pc.qblk * BM;
    const int b = pc.b;
    __syncthreads();   // the previous unit's epilogue is done with the LDS
    const int qj = q0 + wave * 32 + j;
    const int sq = qj < g.N ? ex1[(long long)b * g.N + qj] : 0;
    if (tid < NTGT) {
      const int r = tid >> 4, c = tid & 15;
      const bool in = th0 + r < g.H && tw0 + c < g.W;
      sexp[tid] = in ? ex2[(long long)b * g.N + (th0 + r) * g.W + tw0 + c] : 0;
    }
    const __amdgpu_buffer_rsrc_t rq =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp1 + b * spstride), (short)0,
                                          (int)spstride, 0x00020000);
    const __amdgpu_buffer_rsrc_t rt =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp2 + b * spstride), (short)0,
                                          (int)spstride, 0x00020000);
    uint32_t vq[2], vt;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 16 * i + (lane >> 2), ps = lane & 3;
      const int q = q0 + wave * 32 + row;
      const int cq = ps ^ ((row >> 2) & 3);
      vq[i] = q < g.N ? (uint32_t)(q * 64 + 16 * cq) : 0x80000000u;
    }
    {
      const int ps = lane & 3, r = wave, col = lane >> 2, trow = r * 16 + col;
      const int ct = ps ^ (((trow >> 2) & 1) | ((trow >> 3) & 2));
      const int hh = th0 + r, ww = tw0 + col;
      vt = (hh < g.H && ww < g.W) ? (uint32_t)((hh * g.W + ww) * 64 + 16 * ct) : 0x80000000u;
    }
    auto dma = [&](int ks) {
      unsigned char* st = smem + (ks % DMA_RING) * DMA_STAGE;
      const int so = ks * g.N * 64;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rq, (lds_void_t*)(st + wave * 2048 + i * 1024), 16, vq[i], so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (lds_void_t*)(st + DMA_TILE + wave * 1024), 16,
                                               vt, so, 0, 0);
    };
    f32x16 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dma(0);
    if (nk > 1) dma(1);
    for (int ks = 0; ks < nk; ++ks) {
      if (ks + 1 < nk) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((XP & 16) == 0)
        if (ks + 2 < nk) dma(ks + 2);
      const unsigned char* st = smem + (ks % DMA_RING) * DMA_STAGE;
      const h8v qh = *reinterpret_cast<const h8v*>(st + qh_off);
      const h8v ql = *reinterpret_cast<const h8v*>(st + ql_off);
      h8v thv[4], tlv[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        thv[t] = *reinterpret_cast<const h8v*>(st + th_off + t * 2048);
        tlv[t] = *reinterpret_cast<const h8v*>(st + tl_off + t * 2048);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(tlv[t], qh, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(thv[t], ql, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(thv[t], qh, acc[t], 0, 0, 0);
        if constexpr ((XP & 16) != 0)
          if (t == 0 && ks + 2 < nk) {
            __builtin_amdgcn_sched_barrier(0);
            dma(ks + 2);
            __builtin_amdgcn_sched_barrier(0);
          }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned long long xt1 = (XP & 256) ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const bool live = pc.qblk + half < g.qt;
    const long long page = pc.page + (live ? (long long)half * g.tiles_h * g.tiles_w : 0);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int4* se = reinterpret_cast<const int4*>(sexp + (2 * t + kh) * 16);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int4 s4 = se[v];
        acc[t][4 * v + 0] = __builtin_ldexpf(acc[t][4 * v + 0], -(sq + s4.x));
        acc[t][4 * v + 1] = __builtin_ldexpf(acc[t][4 * v + 1], -(sq + s4.y));
        acc[t][4 * v + 2] = __builtin_ldexpf(acc[t][4 * v + 2], -(sq + s4.z));
        acc[t][4 * v + 3] = __builtin_ldexpf(acc[t][4 * v + 3], -(sq + s4.w));
      }
    }
    if (live) {
      scale_acc<false>(acc, g);
      paged_epilogue<OT, 1 | 4>(acc, reinterpret_cast<float*>(smem) + half * WAVES * 16 * P0, pyr,
                                g, page, w4, lane);
    }
    if constexpr ((XP & 256) != 0) {
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      const unsigned long long xt2 = __builtin_amdgcn_s_memrealtime();
      if (tid < 4) {
        const unsigned long long hw = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                                      ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11)) << 32);
        trace[wl * 4 + tid] = tid == 0 ? xt0 : tid == 1 ? xt1 : tid == 2 ? xt2 : hw;
      }
    }
  }
}

template <int XP>
int xp_persist(const float* f1, const float* f2, float* pyr, const BuildGeom& g, int B, void* ws,
               int nwg, int stagger, unsigned long long* trace, hipStream_t stream) {
  const long long N = g.N, spb = align256((long long)B * g.D * N * 4), eb = align256((long long)B * N * 4);
  uint8_t* w = static_cast<uint8_t*>(ws);
  int* e1 = reinterpret_cast<int*>(w + 2 * spb);
  int* e2 = reinterpret_cast<int*>(w + 2 * spb + eb);
  hipLaunchKernelGGL((split_pairs_kernel<false>), dim3((unsigned)((N + 63) / 64), (unsigned)B, 2),
                     dim3(1024), 0, stream, f1, f2, reinterpret_cast<uint4*>(w),
                     reinterpret_cast<uint4*>(w + spb), e1, e2, g.D, g.N);
  const long long nunits = (long long)B * ((g.qt + 1) / 2) * g.tiles_h * g.tiles_w;
  long long grid = std::min<long long>(nwg, nunits);
  grid = std::max<long long>(8, grid / 8 * 8);
  hipLaunchKernelGGL((xp_build_persist_kernel<float, XP>), dim3((unsigned)grid), dim3(2 * NT), 0,
                     stream, w, w + spb, e1, e2, pyr, g, nunits, stagger, trace);
  return dxr::launch_status();
}

// ---------------------------------------------------------------------------
// Software-pipelined DMA build (round 4 experiment; slower than the product:
// Sintel 151 vs 125 us, KITTI B=8 bf16 760 vs 551 us — two workgroups per CU at
// 4 waves/SIMD hide the K loop's latency better than this overlap gains): one persistent workgroup per CU walks
// its XCD's units (two query blocks x one target tile, the order of
// unit_coord) and writes unit i's pages WHILE it runs unit i+1's K loop: the
// epilogue is cut into three wave-private parts (level 0 queries 0-15, level 0
// queries 16-31, levels 1-3), each issued behind the barrier of one K step.
// In the one-unit-per-workgroup kernel the two workgroups of a CU ran their K
// loops (MFMA-bound) and then their epilogues (store-bound) in step, so the
// matrix cores idled through every epilogue (r03: K loop ~19 us + epilogue
// ~11 us per unit).  The previous unit's accumulators stay in registers
// (64 VGPRs more: 8 waves = 2 per SIMD, one workgroup per CU by LDS: ring 72 KB
// + epilogue staging 66 KB).  Every part issues a fixed number of stores —
// dropped by a zero-size buffer resource when there is nothing to write — so
// the K loop's counted vmcnt waits are compile-time constants.
// Same products, same order, same epilogue arithmetic: the pages of
// corr_build_dma_kernel bit for bit.
// ---------------------------------------------------------------------------
template <typename OT>
constexpr int pipe_part_stores(int part) {
  return sizeof(OT) == 4 ? (part < 2 ? 8 : 6) : 4;
}

// buffer store of V from a page-base resource (num_records 0: dropped)
template <int AUX, typename V>
__device__ __forceinline__ void pipe_put(__amdgpu_buffer_rsrc_t r, unsigned off, const V v) {
  if constexpr (sizeof(V) == 16)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), r, off, 0, AUX);
  else if constexpr (sizeof(V) == 8)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, v), r, off, 0, AUX);
  else if constexpr (sizeof(V) == 4)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, AUX);
  else
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, v), r, off, 0, AUX);
}

template <typename OT>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t page_rsrc(OT* base, int elems, bool en) {
  return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, en ? elems * (int)sizeof(OT) : 0,
                                           0x00020000);
}

// Part PART of paged_epilogue for one wave (same arithmetic and order):
// 0 / 1 level-0 queries 0-15 / 16-31 of the wave, 2 levels 1-3.  `wl` is the
// wave's private staging region (16 x P0 floats), `w4` its 32 queries' slot in
// the page.
template <typename OT, int AUX, int PART>
__device__ __forceinline__ void pipe_epilogue_part(const f32x16 (&acc)[4], float* wl, OT* pyr,
                                                   const BuildGeom& g, long long page, int w4,
                                                   int lane, bool en) {
  const int j = lane & 31, h = lane >> 5;
  if constexpr (PART < 2) {
    constexpr int r = PART;
    const __amdgpu_buffer_rsrc_t rs = page_rsrc(pyr + g.loff[0] + page * (BM * NTGT), BM * NTGT, en);
    if ((j >> 4) == r) {
      float* row = wl + (j & 15) * P0 + h * TW;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4)
          st4(row + 2 * t * TW + 4 * c4, acc[t][4 * c4], acc[t][4 * c4 + 1], acc[t][4 * c4 + 2],
              acc[t][4 * c4 + 3]);
    }
    epi_sync<1>();
    if constexpr (sizeof(OT) == 4) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int qq = 2 * k + (lane >> 5);
        const int off = (lane & 31) * 4;
        const float4 x = f4(wl + qq * P0 + off);
        pipe_put<AUX>(rs, (unsigned)(((w4 * 32 + r * 16 + qq) * NTGT + off) * 4),
                      f32x4v{x.x, x.y, x.z, x.w});
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int qq = 4 * k + (lane >> 4);
        const int off = (lane & 15) * 8;
        const float4 a = f4(wl + qq * P0 + off), c = f4(wl + qq * P0 + off + 4);
        u32x4v u;
        u.x = (uint32_t)to_out<OT>(a.x) | ((uint32_t)to_out<OT>(a.y) << 16);
        u.y = (uint32_t)to_out<OT>(a.z) | ((uint32_t)to_out<OT>(a.w) << 16);
        u.z = (uint32_t)to_out<OT>(c.x) | ((uint32_t)to_out<OT>(c.y) << 16);
        u.w = (uint32_t)to_out<OT>(c.z) | ((uint32_t)to_out<OT>(c.w) << 16);
        pipe_put<AUX>(rs, (unsigned)(((w4 * 32 + r * 16 + qq) * NTGT + off) * 2), u);
      }
    }
    epi_sync<1>();
  } else {
    float l2[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float l1[2][8];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int t = 2 * u + s;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const float o0 = acc[t][2 * m], o1 = acc[t][2 * m + 1];
          const float p0 = __shfl_xor(o0, 32), p1 = __shfl_xor(o1, 32);
          const float t0 = h ? p0 : o0, t1 = h ? p1 : o1;
          const float b0 = h ? o0 : p0, b1 = h ? o1 : p1;
          l1[s][m] = (((t0 + t1) + b0) + b1) * 0.25f;
        }
        st4(wl + j * P1 + t * 8 + 4 * h, l1[s][4 * h], l1[s][4 * h + 1], l1[s][4 * h + 2],
            l1[s][4 * h + 3]);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n)
        l2[u][n] = (((l1[0][2 * n] + l1[0][2 * n + 1]) + l1[1][2 * n]) + l1[1][2 * n + 1]) * 0.25f;
    }
    epi_sync<1>();
    {
      const __amdgpu_buffer_rsrc_t rs =
          page_rsrc(pyr + g.loff[1] + page * (BM * NTGT / 4), BM * NTGT / 4, en);
      if constexpr (sizeof(OT) == 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int qq = 8 * k + (lane >> 3);
          const int off = (lane & 7) * 4;
          const float4 x = f4(wl + qq * P1 + off);
          pipe_put<AUX>(rs, (unsigned)(((w4 * 32 + qq) * 32 + off) * 4), f32x4v{x.x, x.y, x.z, x.w});
        }
      } else {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int qq = 16 * k + (lane >> 2);
          const int off = (lane & 3) * 8;
          const float4 a = f4(wl + qq * P1 + off), c = f4(wl + qq * P1 + off + 4);
          u32x4v u;
          u.x = (uint32_t)to_out<OT>(a.x) | ((uint32_t)to_out<OT>(a.y) << 16);
          u.y = (uint32_t)to_out<OT>(a.z) | ((uint32_t)to_out<OT>(a.w) << 16);
          u.z = (uint32_t)to_out<OT>(c.x) | ((uint32_t)to_out<OT>(c.y) << 16);
          u.w = (uint32_t)to_out<OT>(c.z) | ((uint32_t)to_out<OT>(c.w) << 16);
          pipe_put<AUX>(rs, (unsigned)(((w4 * 32 + qq) * 32 + off) * 2), u);
        }
      }
    }
    {
      const __amdgpu_buffer_rsrc_t rs =
          page_rsrc(pyr + g.loff[2] + page * (BM * NTGT / 16), BM * NTGT / 16, en);
      const float r0 = h ? l2[1][0] : l2[0][0], r1 = h ? l2[1][1] : l2[0][1];
      const float r2 = h ? l2[1][2] : l2[0][2], r3 = h ? l2[1][3] : l2[0][3];
      const unsigned off = (unsigned)((w4 * 32 * 8 + j * 8 + 4 * h) * (int)sizeof(OT));
      if constexpr (sizeof(OT) == 4) {
        pipe_put<AUX>(rs, off, f32x4v{r0, r1, r2, r3});
      } else {
        u32x2v w;
        w.x = (uint32_t)to_out<OT>(r0) | ((uint32_t)to_out<OT>(r1) << 16);
        w.y = (uint32_t)to_out<OT>(r2) | ((uint32_t)to_out<OT>(r3) << 16);
        pipe_put<AUX>(rs, off, w);
      }
    }
    {
      float l3[2];
#pragma unroll
      for (int v = 0; v < 2; ++v)
        l3[v] = (((l2[0][2 * v] + l2[0][2 * v + 1]) + l2[1][2 * v]) + l2[1][2 * v + 1]) * 0.25f;
      const __amdgpu_buffer_rsrc_t rs = page_rsrc(pyr + g.loff[3] + page * (BM * 2), BM * 2, en);
      pipe_put<AUX>(rs, (unsigned)((w4 * 32 * 2 + j * 2 + h) * (int)sizeof(OT)),
                    to_out<OT>(h ? l3[1] : l3[0]));
    }
  }
}

// s_waitcnt immediate that waits for vmcnt <= n only (gfx9 encoding: vmcnt
// bits 3:0 and 15:14, expcnt 6:4 and lgkmcnt 11:8 left at their maxima).
constexpr int vmcnt_imm(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// K steps of the unit (D = 256: 16 f32 / 8 bf16 stages) and the steps whose
// barrier carries an epilogue part of the previous unit.
template <bool BF> constexpr int pipe_nk() { return BF ? 8 : 16; }
template <bool BF> constexpr int pipe_part_at(int ks) {
  return BF ? (ks == 1 ? 0 : ks == 3 ? 1 : ks == 5 ? 2 : -1)
            : (ks == 2 ? 0 : ks == 7 ? 1 : ks == 12 ? 2 : -1);
}
template <typename OT, bool BF> constexpr int pipe_stores_at(int ks) {
  return (ks < 0 || pipe_part_at<BF>(ks) < 0) ? 0 : pipe_part_stores<OT>(pipe_part_at<BF>(ks));
}

constexpr int PIPE_STAGE_BYTES = 2 * WAVES * 16 * P0 * 4;   // epilogue staging, 8 waves
constexpr int PIPE_LDS = DMA_RING * DMA_STAGE + PIPE_STAGE_BYTES + NTGT * 4 + 16;

template <typename OT, bool DIV, bool BF = false>
__global__ __launch_bounds__(2 * NT, 2) void corr_build_pipe_kernel(
    const uint8_t* __restrict__ sp1, const uint8_t* __restrict__ sp2, const int* __restrict__ ex1,
    const int* __restrict__ ex2, OT* __restrict__ pyr, const float* __restrict__ f1,
    const float* __restrict__ f2, int ps, int ks_f, int pstr, int kstr, BuildGeom g,
    long long nunits) {
  constexpr int LDS_RING = DMA_RING * DMA_STAGE;
  constexpr int NK = pipe_nk<BF>();
  constexpr int AUX = BF ? 2 : 16;        // bf16 pyramid: non-temporal; f32: write-through
  __shared__ __attribute__((aligned(16))) unsigned char smem[PIPE_LDS];
  float* const stage = reinterpret_cast<float*>(smem + LDS_RING);
  int* const sexp = reinterpret_cast<int*>(smem + LDS_RING + PIPE_STAGE_BYTES);
  int* const redo = sexp + NTGT;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave >> 2, w4 = wave & 3;
  const int j = lane & 31, kh = lane >> 5;
  const long long spstride = (long long)g.D * g.N * (BF ? 2 : 4);
  float* const wl = stage + (half * WAVES + w4) * 16 * P0;
  // this workgroup's units: XCD x (round-robin dispatch, speed only) takes the
  // x-th contiguous range of the unit order, its workgroups every per_xcd-th
  const int per_xcd = gridDim.x / 8, xcd = blockIdx.x % 8, local = blockIdx.x / 8;
  const long long q8 = nunits / 8, r8 = nunits % 8;
  const long long ustart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const long long ucount = q8 + (xcd < r8 ? 1 : 0);

  const int kq = (j >> 2) & 3;
  const int qh_off = wave * 2048 + j * 64 + 16 * (kh ^ kq);
  const int ql_off = wave * 2048 + j * 64 + 16 * ((2 + kh) ^ kq);
  const int trow0 = ((j >> 2) & 1) * 16 + (j & 3) + 4 * (j >> 3);
  const int kt = ((trow0 >> 2) & 1) | ((trow0 >> 3) & 2);
  const int th_off = DMA_TILE + trow0 * 64 + 16 * (kh ^ kt);
  const int tl_off = DMA_TILE + trow0 * 64 + 16 * ((2 + kh) ^ kt);

  f32x16 prev[4];                 // the previous unit's pages (unscaled, divided)
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) prev[t][r] = 0.f;
  long long prev_page = 0;
  bool prev_en = false;

  for (long long u = local; u < ucount; u += per_xcd) {
    const PageCoord pc = unit_coord<2>(g, ustart + u);
    const int th0 = pc.tyi * TH, tw0 = pc.txi * TW;
    const int q0 = pc.qblk * BM;
    const int b = pc.b;
    const int qj = q0 + wave * 32 + j;
    // the previous unit's ring reads, exponent reads and redo vote are done
    if (tid == 0) *redo = 0;
    __syncthreads();
    int sq = 0;
    if constexpr (!BF) {
      sq = qj < g.N ? ex1[(long long)b * g.N + qj] : 0;
      if (tid < NTGT) {
        const int r = tid >> 4, c = tid & 15;
        const bool in = th0 + r < g.H && tw0 + c < g.W;
        sexp[tid] = in ? ex2[(long long)b * g.N + (th0 + r) * g.W + tw0 + c] : 0;
      }
    }
    const __amdgpu_buffer_rsrc_t rq =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp1 + b * spstride), (short)0,
                                          (int)spstride, 0x00020000);
    const __amdgpu_buffer_rsrc_t rt =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp2 + b * spstride), (short)0,
                                          (int)spstride, 0x00020000);
    uint32_t vq[2], vt;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 16 * i + (lane >> 2), pp = lane & 3;
      const int q = q0 + wave * 32 + row;
      const int cq = pp ^ ((row >> 2) & 3);
      vq[i] = q < g.N ? (uint32_t)q * (uint32_t)pstr + 16u * cq : 0x80000000u;
    }
    {
      const int pp = lane & 3, r = wave, col = lane >> 2, trow = r * 16 + col;
      const int ct = pp ^ (((trow >> 2) & 1) | ((trow >> 3) & 2));
      const int hh = th0 + r, ww = tw0 + col;
      vt = (hh < g.H && ww < g.W) ? (uint32_t)(hh * g.W + ww) * (uint32_t)pstr + 16u * ct
                                  : 0x80000000u;
    }
    auto dma = [&](int ks) {
      unsigned char* st = smem + (ks % DMA_RING) * DMA_STAGE;
      const int so = ks * kstr;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rq, (lds_void_t*)(st + wave * 2048 + i * 1024), 16, vq[i], so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (lds_void_t*)(st + DMA_TILE + wave * 1024), 16,
                                               vt, so, 0, 0);
    };
    f32x16 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    // the exponent loads must not count against the ring's waits
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dma(0);
    dma(1);
    static_for<0, NK>([&](auto ksc) {
      constexpr int ks = decltype(ksc)::value;
      // DMA(ks) has landed: younger are the stores of steps ks-2, ks-1 and DMA(ks+1)
      constexpr int younger = pipe_stores_at<OT, BF>(ks - 2) + pipe_stores_at<OT, BF>(ks - 1) +
                              (ks + 1 < NK ? 3 : 0);
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(younger));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (ks + 2 < NK) dma(ks + 2);
      constexpr int part = pipe_part_at<BF>(ks);
      if constexpr (part >= 0) {
        __builtin_amdgcn_sched_barrier(0);
        pipe_epilogue_part<OT, AUX, part>(prev, wl, pyr, g, prev_page, w4, lane, prev_en);
        __builtin_amdgcn_sched_barrier(0);
      }
      const unsigned char* st = smem + (ks % DMA_RING) * DMA_STAGE;
      if constexpr (BF) {
        const bf8v q0v = *reinterpret_cast<const bf8v*>(st + qh_off);
        const bf8v q1v = *reinterpret_cast<const bf8v*>(st + ql_off);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf8v t0v = *reinterpret_cast<const bf8v*>(st + th_off + t * 2048);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t0v, q0v, acc[t], 0, 0, 0);
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
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, qh, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ql, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, qh, acc[t], 0, 0, 0);
        }
      }
    });
    const bool live = pc.qblk + half < g.qt;
    const long long page = pc.page + (live ? (long long)half * g.tiles_h * g.tiles_w : 0);
    if constexpr (!BF) {
      bool bad = false;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) bad |= !(__builtin_fabsf(acc[t][r]) <= 3.40282347e38f);
      if (bad) *redo = 1;
      __syncthreads();
      if (*redo) {
        // exact-f32 recompute of this unit (corr_build_dma_kernel's path):
        // no scales to undo
        int trw = trow0;
        asm volatile("" : "+v"(trw));
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
          to[t] = (hh < g.H && ww < g.W) ? (unsigned)(hh * g.W + ww) * (unsigned)ps * 4u
                                         : 0x80000000u;
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
        }
        const int kstep = ks_f * 4;
#pragma unroll 1
        for (int k = kh; k < g.D; k += 2) {
          const int ko = k * kstep;
          const float bq =
              __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r1, qo, ko, 0));
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const float at =
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r2, to[t], ko, 0));
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(at, bq, acc[t], 0, 0, 0);
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int4* se = reinterpret_cast<const int4*>(sexp + (2 * t + kh) * 16);
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int4 s4 = se[v];
            acc[t][4 * v + 0] = __builtin_ldexpf(acc[t][4 * v + 0], -(sq + s4.x));
            acc[t][4 * v + 1] = __builtin_ldexpf(acc[t][4 * v + 1], -(sq + s4.y));
            acc[t][4 * v + 2] = __builtin_ldexpf(acc[t][4 * v + 2], -(sq + s4.z));
            acc[t][4 * v + 3] = __builtin_ldexpf(acc[t][4 * v + 3], -(sq + s4.w));
          }
        }
      }
    }
    scale_acc<DIV>(acc, g);
#pragma unroll
    for (int t = 0; t < 4; ++t) prev[t] = acc[t];
    prev_page = page;
    prev_en = live;
  }
  // the last unit's pages
  pipe_epilogue_part<OT, AUX, 0>(prev, wl, pyr, g, prev_page, w4, lane, prev_en);
  pipe_epilogue_part<OT, AUX, 1>(prev, wl, pyr, g, prev_page, w4, lane, prev_en);
  pipe_epilogue_part<OT, AUX, 2>(prev, wl, pyr, g, prev_page, w4, lane, prev_en);
}

// Workgroups of the pipelined build: one per CU (its LDS takes the CU), whole
// XCDs' worth (a multiple of 8), never more than there are units.
int pipe_grid(long long nunits) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    cus = n;
  }
  long long g = std::min<long long>(cus, (nunits + 7) / 8 * 8);
  g = g / 8 * 8;
  return (int)std::max<long long>(8, g);
}

// The pre-split f32 build on the pipelined kernel (D = 256).
template <typename OT, bool NHWC>
int launch_pipe(const float* f1, const float* f2, OT* pyr, const BuildGeom& g, int B, void* ws,
                hipStream_t stream) {
  const long long N = g.N, spb = align256((long long)B * g.D * N * 4), eb = align256((long long)B * N * 4);
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint8_t* sp1 = w;
  uint8_t* sp2 = w + spb;
  int* e1 = reinterpret_cast<int*>(w + 2 * spb);
  int* e2 = reinterpret_cast<int*>(w + 2 * spb + eb);
  hipLaunchKernelGGL((split_pairs_kernel<NHWC>), dim3((unsigned)((N + 63) / 64), (unsigned)B, 2),
                     dim3(1024), 0, stream, f1, f2, reinterpret_cast<uint4*>(sp1),
                     reinterpret_cast<uint4*>(sp2), e1, e2, g.D, g.N);
  int st = dxr::launch_status();
  if (st != DXR_OK) return st;
  const long long nunits = (long long)B * ((g.qt + 1) / 2) * g.tiles_h * g.tiles_w;
  const int grid = pipe_grid(nunits);
  const int ps = NHWC ? g.D : 1, ks = NHWC ? 1 : g.N;   // fallback operand strides
  if (g.recip == 0.f)
    hipLaunchKernelGGL((corr_build_pipe_kernel<OT, true>), dim3(grid), dim3(2 * NT), 0, stream,
                       sp1, sp2, e1, e2, pyr, f1, f2, ps, ks, 64, g.N * 64, g, nunits);
  else
    hipLaunchKernelGGL((corr_build_pipe_kernel<OT, false>), dim3(grid), dim3(2 * NT), 0, stream,
                       sp1, sp2, e1, e2, pyr, f1, f2, ps, ks, 64, g.N * 64, g, nunits);
  return dxr::launch_status();
}

// The bf16 channels-last build on the pipelined kernel (D = 256).
template <typename OT>
int launch_pipe_bf16_nhwc(const uint16_t* f1, const uint16_t* f2, OT* pyr, const BuildGeom& g,
                          int B, hipStream_t stream) {
  const long long nunits = (long long)B * ((g.qt + 1) / 2) * g.tiles_h * g.tiles_w;
  const int grid = pipe_grid(nunits);
  const uint8_t* a = reinterpret_cast<const uint8_t*>(f1);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(f2);
  if (g.recip == 0.f)
    hipLaunchKernelGGL((corr_build_pipe_kernel<OT, true, true>), dim3(grid), dim3(2 * NT), 0,
                       stream, a, c, nullptr, nullptr, pyr, nullptr, nullptr, 0, 0, g.D * 2, 64,
                       g, nunits);
  else
    hipLaunchKernelGGL((corr_build_pipe_kernel<OT, false, true>), dim3(grid), dim3(2 * NT), 0,
                       stream, a, c, nullptr, nullptr, pyr, nullptr, nullptr, 0, 0, g.D * 2, 64,
                       g, nunits);
  return dxr::launch_status();
}

}  // namespace

// Variant xp of the pre-split build (f32 NCHW fmaps, W % 4 == 0, D % 16 == 0,
// sqrt(D) a power of two, 4 levels); ws as dxr_corr_pyramid_build_ws; trace:
// 4 x u64 per workgroup when xp has bit 8.
extern "C" int dxr_xp_build(const float* f1, const float* f2, int64_t B, int64_t D, int64_t H,
                            int64_t W, float* pyr, void* ws, int xp, unsigned long long* trace,
                            hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, 4, &L) || W % 4 || D % 16) return DXR_EINVAL;
  const BuildGeom g = make_geom(D, H, W, std::sqrt((float)D), L);
  if (g.recip == 0.f) return DXR_EINVAL;
  switch (xp) {
    case 0: return xp_dma<0>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 1: return xp_dma<1>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 2: return xp_dma<2>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 3: return xp_dma<3>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 4: return xp_dma<4>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 5: return xp_dma<5>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 12: return xp_dma<12>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 13: return xp_dma<13>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 8: return xp_dma<8>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 256: return xp_dma<256>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 257: return xp_dma<257>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 32: return xp_dma<32>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 33: return xp_dma<33>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 16: return xp_dma<16>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 64: return xp_dma<64>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 512 + (4 << 12): return xp_dma<512 + (4 << 12)>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 512 + (8 << 12): return xp_dma<512 + (8 << 12)>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 512 + (12 << 12): return xp_dma<512 + (12 << 12)>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 512 + (16 << 12): return xp_dma<512 + (16 << 12)>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 768 + (8 << 12): return xp_dma<768 + (8 << 12)>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 768 + (12 << 12): return xp_dma<768 + (12 << 12)>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 128: return xp_dma<128>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 1024: return xp_dma<1024>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 2048: return xp_dma<2048>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    case 272: return xp_dma<272>(f1, f2, pyr, g, (int)B, ws, trace, stream);
    default: return DXR_EINVAL;
  }
}

// Split pass alone (NCHW f32, D == 256), variant v: 0 product (64 px, 1024
// threads), 1 plain stores, 2 / 3 / 4: 16 / 32 / 128 pixels per workgroup.
extern "C" int dxr_xp_split(const float* f1, const float* f2, int64_t B, int64_t D, int64_t H,
                            int64_t W, void* ws, int v, hipStream_t stream) {
  if (D != 256) return DXR_EINVAL;
  const long long N = H * W, spb = align256(B * D * N * 4), eb = align256(B * N * 4);
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint4* s1 = reinterpret_cast<uint4*>(w);
  uint4* s2 = reinterpret_cast<uint4*>(w + spb);
  int* e1 = reinterpret_cast<int*>(w + 2 * spb);
  int* e2 = reinterpret_cast<int*>(w + 2 * spb + eb);
  auto grid = [&](int px) { return dim3((unsigned)((N + px - 1) / px), (unsigned)B, 2); };
  switch (v) {
    case 0: hipLaunchKernelGGL((split_pairs_kernel<false>), grid(64), dim3(1024), 0, stream, f1, f2, s1, s2, e1, e2, (int)D, (int)N); break;
    case 1: hipLaunchKernelGGL(xp_split_plain_kernel, grid(64), dim3(1024), 0, stream, f1, f2, s1, s2, e1, e2, (int)D, (int)N); break;
    case 2: hipLaunchKernelGGL((xp_split_px_kernel<16>), grid(16), dim3(256), 0, stream, f1, f2, s1, s2, e1, e2, (int)D, (int)N); break;
    case 3: hipLaunchKernelGGL((xp_split_px_kernel<32>), grid(32), dim3(512), 0, stream, f1, f2, s1, s2, e1, e2, (int)D, (int)N); break;
    case 4: hipLaunchKernelGGL((xp_split_px_kernel<64>), grid(64), dim3(1024), 0, stream, f1, f2, s1, s2, e1, e2, (int)D, (int)N); break;
    default: return DXR_EINVAL;
  }
  return dxr::launch_status();
}

// Persistent build variant xp (0 plain, 2 stagger, +256 trace) over nwg workgroups.
extern "C" int dxr_xp_build_persist(const float* f1, const float* f2, int64_t B, int64_t D,
                                    int64_t H, int64_t W, float* pyr, void* ws, int xp, int nwg,
                                    int stagger, unsigned long long* trace, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, 4, &L) || W % 4 || D % 16) return DXR_EINVAL;
  const BuildGeom g = make_geom(D, H, W, std::sqrt((float)D), L);
  if (g.recip == 0.f || nwg < 8) return DXR_EINVAL;
  switch (xp) {
    case 0: return xp_persist<0>(f1, f2, pyr, g, (int)B, ws, nwg, stagger, trace, stream);
    case 2: return xp_persist<2>(f1, f2, pyr, g, (int)B, ws, nwg, stagger, trace, stream);
    case 256: return xp_persist<256>(f1, f2, pyr, g, (int)B, ws, nwg, stagger, trace, stream);
    case 258: return xp_persist<258>(f1, f2, pyr, g, (int)B, ws, nwg, stagger, trace, stream);
    case 16: return xp_persist<16>(f1, f2, pyr, g, (int)B, ws, nwg, stagger, trace, stream);
    case 18: return xp_persist<18>(f1, f2, pyr, g, (int)B, ws, nwg, stagger, trace, stream);
    default: return DXR_EINVAL;
  }
}

// The product's DMA builds with another strip width of the XCD-banded page
// order (BuildGeom::strip, product 8): f32 NCHW (ws as dxr_corr_pyramid_build_ws)
// or bf16 channels-last (no workspace).  Same pages bit for bit.
extern "C" int dxr_xp_build_strip(const void* f1, const void* f2, int in_dtype, int64_t B,
                                  int64_t D, int64_t H, int64_t W, void* pyr, void* ws, int strip,
                                  hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, 4, &L) || strip < 1) return DXR_EINVAL;
  BuildGeom g = make_geom(D, H, W, std::sqrt((float)D), L);
  g.strip = strip;
  if (in_dtype == DXR_F32)
    return launch_dma<float, false>(static_cast<const float*>(f1), static_cast<const float*>(f2),
                                    static_cast<float*>(pyr), g, (int)B, ws, stream);
  return launch_dma_bf16_nhwc(static_cast<const uint16_t*>(f1), static_cast<const uint16_t*>(f2),
                              static_cast<uint16_t*>(pyr), g, (int)B, stream);
}

// The software-pipelined build (corr_build_pipe_kernel) for A/B against the
// product: f32 NCHW with its split pass (ws as dxr_corr_pyramid_build_ws) or
// bf16 channels-last (no workspace); D = 256.
extern "C" int dxr_xp_build_pipe(const void* f1, const void* f2, int in_dtype, int64_t B,
                                 int64_t D, int64_t H, int64_t W, void* pyr, void* ws,
                                 hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, 4, &L) || D != 256) return DXR_EINVAL;
  const BuildGeom g = make_geom(D, H, W, std::sqrt((float)D), L);
  if (in_dtype == DXR_F32)
    return launch_pipe<float, false>(static_cast<const float*>(f1), static_cast<const float*>(f2),
                                     static_cast<float*>(pyr), g, (int)B, ws, stream);
  return launch_pipe_bf16_nhwc(static_cast<const uint16_t*>(f1), static_cast<const uint16_t*>(f2),
                               static_cast<uint16_t*>(pyr), g, (int)B, stream);
}

// The product's DMA builds under another tail policy (dma_grid `tail`: split
// the last partial dispatch round into quarter units when 8 T <= tail x S; 0
// never, 8 always): f32 NCHW (ws as dxr_corr_pyramid_build_ws), bf16
// channels-last (no workspace) or bf16 NCHW (ws: the pack pass's records).
// Same pages bit for bit.
extern "C" int dxr_xp_build_tail(const void* f1, const void* f2, int in_dtype, int fmap_layout,
                                 int64_t B, int64_t D, int64_t H, int64_t W, void* pyr, void* ws,
                                 int tail, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, 4, &L) || tail < 0) return DXR_EINVAL;
  const BuildGeom g = make_geom(D, H, W, std::sqrt((float)D), L);
  if (in_dtype == DXR_F32)
    return launch_dma<float, false>(static_cast<const float*>(f1), static_cast<const float*>(f2),
                                    static_cast<float*>(pyr), g, (int)B, ws, stream, tail);
  if (fmap_layout == DXR_NHWC)
    return launch_dma_bf16_nhwc(static_cast<const uint16_t*>(f1), static_cast<const uint16_t*>(f2),
                                static_cast<uint16_t*>(pyr), g, (int)B, stream, tail);
  return launch_dma_bf16_nchw(static_cast<const uint16_t*>(f1), static_cast<const uint16_t*>(f2),
                              static_cast<uint16_t*>(pyr), g, (int)B, ws, stream, tail);
}

// ---------------------------------------------------------------------------
// Round 5 experiment ("cut the per-step LDS re-reads of the
// 8x16 target tile"): the product's unit, ring and DMA, but each wave computes
// 2 x 2 MFMA tiles — 64 queries (sub-blocks 2 qg, 2 qg + 1) x 64 targets (tile
// rows 4 tg .. 4 tg + 3) — instead of 32 queries x the whole tile: per k-step
// 8 ds_read_b128 per wave instead of 10 for the same 12 MFMAs.  The epilogue
// writes half of each query's level-0 and level-1 rows per wave, level 2 per
// wave row, and level 3 from the two target halves through LDS (the reference
// order ((v00 + v01) + v10) + v11).  Whole units only (no quarter tail), no
// non-finite recompute: a timing experiment on finite data, its pages checked
// bit-identical to the product's by scripts/ab_build.py.  Measured (r5u/r5v,
// against the product without its tail split): Sintel B=1 -1.6 %, B=8 +9.8 %,
// Chairs +2.3 %, 1080p +7.4 % with plain stores on levels 1-3 (each line
// completed by the two target halves in L2); written through, the half lines
// cost far more (B=8 +30 %).  Not adopted.
namespace {
template <bool DIV>
__global__ __launch_bounds__(2 * NT, 4) void xp_dma22_kernel(const uint8_t* __restrict__ sp1,
                                                              const uint8_t* __restrict__ sp2,
                                                              const int* __restrict__ ex1,
                                                              const int* __restrict__ ex2,
                                                              float* __restrict__ pyr, BuildGeom g) {
  constexpr int PQ22 = 4 * 16 + 4;   // staged level-0 half row per query (floats)
  __shared__ __attribute__((aligned(16))) unsigned char smem[DMA_LDS_BYTES + 8 * 32 * 2 * 4];
  static_assert(8 * 32 * PQ22 * 4 <= DMA_LDS_RING, "staging aliases the ring");
  int* const sexp = reinterpret_cast<int*>(smem + DMA_LDS_RING);
  float* const x3 = reinterpret_cast<float*>(smem + DMA_LDS_BYTES);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qg = wave & 3, tg = wave >> 2;
  const PageCoord pc = page_coord<true, 2>(g);
  const int th0 = pc.tyi * TH, tw0 = pc.txi * TW;
  const int q0 = pc.qblk * BM;
  const int b = pc.b;
  const int j = lane & 31, kh = lane >> 5;
  const long long spstride = (long long)g.D * g.N * 4;
  int sq[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int qj = q0 + (2 * qg + s) * 32 + j;
    sq[s] = qj < g.N ? ex1[(long long)b * g.N + qj] : 0;
  }
  if (tid < NTGT) {
    const int r = tid >> 4, c = tid & 15;
    const bool in = th0 + r < g.H && tw0 + c < g.W;
    sexp[tid] = in ? ex2[(long long)b * g.N + (th0 + r) * g.W + tw0 + c] : 0;
  }
  const __amdgpu_buffer_rsrc_t rq =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp1 + b * spstride), (short)0,
                                        (int)spstride, 0x00020000);
  const __amdgpu_buffer_rsrc_t rt =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sp2 + b * spstride), (short)0,
                                        (int)spstride, 0x00020000);
  const int pstr = 64, kstr = g.N * 64;
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
  const int kq = (j >> 2) & 3;
  const int trow0 = ((j >> 2) & 1) * 16 + (j & 3) + 4 * (j >> 3);
  const int kt = ((trow0 >> 2) & 1) | ((trow0 >> 3) & 2);
  const int qh_off = 2 * qg * 2048 + j * 64 + 16 * (kh ^ kq);
  const int ql_off = 2 * qg * 2048 + j * 64 + 16 * ((2 + kh) ^ kq);
  const int th_off = DMA_TILE + 2 * tg * 2048 + trow0 * 64 + 16 * (kh ^ kt);
  const int tl_off = DMA_TILE + 2 * tg * 2048 + trow0 * 64 + 16 * ((2 + kh) ^ kt);

  f32x16 acc[2][2];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int nk = g.D / BKS;
  dma(0);
  if (nk > 1) dma(1);
  auto kstep = [&](int kk, auto first_tag) {
    constexpr bool FIRST = decltype(first_tag)::value;
    if (kk + 1 < nk) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kk + 2 < nk) dma(kk + 2);
    const unsigned char* st = smem + (kk % DMA_RING) * DMA_STAGE;
    h8v qh[2], ql[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      qh[s] = *reinterpret_cast<const h8v*>(st + qh_off + s * 2048);
      ql[s] = *reinterpret_cast<const h8v*>(st + ql_off + s * 2048);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const h8v th = *reinterpret_cast<const h8v*>(st + th_off + u * 2048);
      const h8v tl = *reinterpret_cast<const h8v*>(st + tl_off + u * 2048);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        acc[s][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(tl, qh[s], FIRST ? f32x16{} : acc[s][u], 0, 0, 0);
        acc[s][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, ql[s], acc[s][u], 0, 0, 0);
        acc[s][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(th, qh[s], acc[s][u], 0, 0, 0);
      }
    }
  };
  kstep(0, std::true_type{});
  for (int kk = 1; kk < nk; ++kk) kstep(kk, std::false_type{});
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // ring reads done

  const int blk = qg >> 1;                          // both sub-blocks of the wave: one block
  const bool live = pc.qblk + blk < g.qt;
  const long long page = pc.page + (live ? (long long)blk * g.tiles_h * g.tiles_w : 0);
  int e2 = 0;
  if constexpr (!DIV) (void)__builtin_frexpf(g.recip, &e2);
  // unscale: ldexp by -(s_q + s_t) (+ log2 1/sqrt(D)), as the product
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int eq = -sq[s] + (DIV ? 0 : e2 - 1);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int* se = sexp + (2 * (2 * tg + u) + kh) * 16;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = __builtin_ldexpf(acc[s][u][r], eq - se[r]);
        if constexpr (DIV) v = v / g.divisor;
        acc[s][u][r] = v;
      }
    }
  }
  float* const wl = reinterpret_cast<float*>(smem) + wave * 32 * PQ22;
  float* const pb0 = pyr + g.loff[0] + page * (BM * NTGT);
  float* const pb1 = pyr + g.loff[1] + page * (BM * NTGT / 4);
  float* const pb2 = pyr + g.loff[2] + page * (BM * NTGT / 16);
  float* const pb3 = pyr + g.loff[3] + page * (BM * 2);
  float l2[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int qbase = ((2 * qg + s) & 3) * 32;
    // level 0: this wave's half rows (tile rows 4 tg .. 4 tg + 3) of 32 queries
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float* row = wl + j * PQ22 + (2 * u + kh) * 16;
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4)
        st4(row + 4 * c4, acc[s][u][4 * c4], acc[s][u][4 * c4 + 1], acc[s][u][4 * c4 + 2],
            acc[s][u][4 * c4 + 3]);
    }
    epi_sync<1>();
    if (live) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int q = 4 * k + (lane >> 4), pc16 = lane & 15;
        const float4 x = f4(wl + q * PQ22 + pc16 * 4);
        epi_put<4>(pb0, pb0 + (long long)(qbase + q) * NTGT + tg * 64 + pc16 * 4,
                   f32x4v{x.x, x.y, x.z, x.w});
      }
    }
    epi_sync<1>();
    // level 1: rows t = 2 tg + u, cols 4 kh .. 4 kh + 3 (pair-swap pooling)
    float l1[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float x[8], y[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[s][u][k]),
                                                        __float_as_uint(acc[s][u][8 + k]), false, false);
        x[k] = __uint_as_float(p[0]);
        y[k] = __uint_as_float(p[1]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        l1[u][i] = (((x[2 * i] + x[2 * i + 1]) + y[2 * i]) + y[2 * i + 1]) * 0.25f;
      if (live)   // plain stores: the two target halves complete each line in L2
        *reinterpret_cast<float4*>(pb1 + (long long)(qbase + j) * 32 + (2 * tg + u) * 8 + 4 * kh) =
            make_float4(l1[u][0], l1[u][1], l1[u][2], l1[u][3]);
    }
    // level 2: row tg, cols 2 kh, 2 kh + 1
#pragma unroll
    for (int i = 0; i < 2; ++i)
      l2[s][i] = (((l1[0][2 * i] + l1[0][2 * i + 1]) + l1[1][2 * i]) + l1[1][2 * i + 1]) * 0.25f;
    if (live)
      *reinterpret_cast<float2*>(pb2 + (long long)(qbase + j) * 8 + tg * 4 + 2 * kh) =
          make_float2(l2[s][0], l2[s][1]);
    if (tg == 0) x3[((qg * 2 + s) * 32 + j) * 2 + kh] = l2[s][0] + l2[s][1];
  }
  __syncthreads();   // level 3: row 0's pair sums from the tg = 0 waves
  if (tg == 1 && live) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int qbase = ((2 * qg + s) & 3) * 32;
      const float a = x3[((qg * 2 + s) * 32 + j) * 2 + kh];
      pb3[(long long)(qbase + j) * 2 + kh] = ((a + l2[s][0]) + l2[s][1]) * 0.25f;
    }
  }
}
}  // namespace

extern "C" int dxr_xp_build22(const float* f1, const float* f2, int64_t B, int64_t D, int64_t H,
                              int64_t W, float* pyr, void* ws, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, 4, &L) || D % 16 != 0) return DXR_EINVAL;
  BuildGeom g = make_geom(D, H, W, std::sqrt((float)D), L);
  const long long N = g.N, spb = align256(B * D * N * 4), eb = align256(B * N * 4);
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint8_t* sp1 = w;
  uint8_t* sp2 = w + spb;
  int* e1 = reinterpret_cast<int*>(w + 2 * spb);
  int* e2 = reinterpret_cast<int*>(w + 2 * spb + eb);
  hipLaunchKernelGGL((split_pairs_kernel<false, false, 32>), dim3((unsigned)((N + 31) / 32), (unsigned)B, 2),
                     dim3(512), 0, stream, f1, f2, reinterpret_cast<uint4*>(sp1),
                     reinterpret_cast<uint4*>(sp2), e1, e2, g.D, g.N);
  int st = dxr::launch_status();
  if (st != DXR_OK) return st;
  const dim3 rg = dma_grid(g, (int)B, stream, 0);   // whole units only
  if (g.recip == 0.f)
    hipLaunchKernelGGL((xp_dma22_kernel<true>), rg, dim3(2 * NT), 0, stream, sp1, sp2, e1, e2, pyr, g);
  else
    hipLaunchKernelGGL((xp_dma22_kernel<false>), rg, dim3(2 * NT), 0, stream, sp1, sp2, e1, e2, pyr, g);
  return dxr::launch_status();
}
