// Experiments target only (libdexiraft_corr_exp.so, build.py --experiments):
// variants of the ordered on-the-fly lookup (csrc/alt_corr.hip).  Never loaded
// by the package.
#include "../alt_corr.hip"

// variant 0: the ordered lookup with cell loads 1 k step ahead (3 workgroups per
// CU; the product keeps 4 ahead = variant 3); 1: cell vectors by LDS-DMA into per-wave swizzled buffers (2 per CU);
// 2 / 3 / 4 / 5: cell loads 2 / 4 / 6 / 8 k steps ahead (register ring); 6 / 7: variant 3
// with the level-by-XCD workgroup mapping off / on (3 = the product's choice); 8: variant 3
// without the cell vectors' f16 split (a timing ablation); 9: DMA with one-k-step stages, 4 deep.
// Radius 4, C % 32 == 0, 16-byte aligned NHWC fmaps; ws as dxr_alt_corr_lookup_ws.
extern "C" int dxr_xp_alt_lookup(const float* fmap1, const float* const* fmap2_levels,
                                 const float* coords, float* out, int64_t B, int64_t H,
                                 int64_t W, int64_t C, int num_levels, float divisor, void* ws,
                                 int variant, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, num_levels, &L) || C % 32 != 0 || C > 256 || !ws)
    return DXR_EINVAL;
  AltGeom g;
  g.N = (int)(H * W);
  g.C = (int)C;
  g.Nc = 1;
  g.cout = num_levels * 81;
  g.divisor = divisor;
  g.div_recip = pow2_recip(divisor);
  g.f1_bstride = H * W * C;
  g.coord_zstride = 2 * H * W;
  g.coord_cstride = H * W;
  g.coord_qstride = 1;
  for (int l = 0; l < num_levels; ++l)
    g.lv[l] = AltLevel{fmap2_levels[l], L.h[l], L.w[l], 1.f / (float)(1 << l), l * 81};
  if (variant == 0)
    return launch_alt_mfma_r<4, 1, 0, 1>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                          stream, ws);
  if (variant == 1)
    return launch_alt_mfma_r<4, 1, 1>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                         stream, ws);
  if (variant == 9)   // round 6: one-k-step DMA stages, 4-deep ring per wave
    return launch_alt_mfma_r<4, 1, 2>(fmap1, coords, out, g, num_levels, (int)B, (int)W, stream, ws);
  if (variant == 2)
    return launch_alt_mfma_r<4, 1, 0, 2>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                             stream, ws);
  if (variant == 3)
    return launch_alt_mfma_r<4, 1, 0, 4>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                             stream, ws);
  if (variant == 4)
    return launch_alt_mfma_r<4, 1, 0, 6>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                             stream, ws);
  if (variant == 5)
    return launch_alt_mfma_r<4, 1, 0, 8>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                             stream, ws);
  if (variant == 11)  // variant 3 without the output stores (timing ablation)
    return launch_alt_mfma_r<4, 1, 0, 4, 2>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                                stream, ws);
  if (variant == 8)   // variant 3 without the cell split (timing ablation)
    return launch_alt_mfma_r<4, 1, 0, 4, 1>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                                stream, ws);
  if (variant == 12)  // variant 3 with every lane loading one of 8 hot cells (ablation: the gather's cost)
    return launch_alt_mfma_r<4, 1, 0, 4, 4>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                                stream, ws);
  if (variant == 13)  // variant 3 without MFMAs (ablation)
    return launch_alt_mfma_r<4, 1, 0, 4, 8>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                                stream, ws);
  if (variant == 14)  // neither cell gathers nor MFMAs nor stores (ablation: the skeleton)
    return launch_alt_mfma_r<4, 1, 0, 4, 14>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                                 stream, ws);
  if (variant == 15)  // variant 3 with the round-5 S pitch (100: 4-way phase-2 conflicts)
    return launch_alt_mfma_r<4, 1, 0, 4, 16>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                                 stream, ws);
  if (variant == 6 || variant == 7)
    return launch_alt_mfma_r<4, 1, 0, 4>(fmap1, coords, out, g, num_levels, (int)B, (int)W,
                                             stream, ws, variant - 6);
  return DXR_EINVAL;
}

// The coarse-level volumes with every level by the FULL box kernel (round 6's
// first form; the product uses alt_volume_gemm_kernel for tiled levels).
extern "C" int dxr_xp_alt_coarse_volumes_full(const float* fmap1, const float* const* fmap2_levels,
                                              int64_t B, int64_t H, int64_t W, int64_t C,
                                              int num_levels, int first_level, float* volumes,
                                              hipStream_t stream) {
  return alt_coarse_volumes(fmap1, fmap2_levels, B, H, W, C, num_levels, first_level, volumes,
                            stream, true);
}

// One tiled level's volume by alt_volume_gemm_kernel with ablation bits xa (its XA):
// the volume buffer from `level` on (dxr_alt_volume_numel(B, H, W, level + 1, level));
// with a workspace (>= dxr_alt_coarse_volumes_ws_bytes(B, H, W, C, level + 1, level))
// the operands are split into f16 pair planes there first and the LDS-DMA form runs.
extern "C" int dxr_xp_alt_volume_gemm(const float* fmap1, const float* fmap2_level, float* vol,
                                      int64_t B, int64_t H, int64_t W, int64_t C, int level,
                                      int xa, void* ws, hipStream_t stream) {
  dxr::Levels L;
  if (!dxr::make_levels(B, H, W, level + 1, &L) || level >= dxr::TILED_LEVELS || C % 32 != 0)
    return DXR_EINVAL;
  dxr::LevelLayout vl = L.lay[level];
  vl.off = 0;
  const int N = (int)(H * W);
  _Float16 *p1 = nullptr, *p2 = nullptr;
  if (ws != nullptr) {
    long long loff[8] = {};
    alt_volume_planes_bytes(L, B, H, W, C, level + 1, level, loff);
    p1 = static_cast<_Float16*>(ws);
    p2 = reinterpret_cast<_Float16*>(static_cast<unsigned char*>(ws) + loff[level]);
    int st = launch_split_planes(fmap1, p1, B, H * W, (int)C, stream);
    if (st == DXR_OK)
      st = launch_split_planes(fmap2_level, p2, B, (long long)L.h[level] * L.w[level], (int)C, stream);
    if (st != DXR_OK) return st;
  }
  if (xa == 99) return DXR_EINVAL;   // the split passes alone (timing)
  switch (xa) {
    case 0: return launch_alt_volume_gemm<0>(fmap1, fmap2_level, vol, vl, (int)B, N, (int)C, stream, p1, p2);
    case 1: return launch_alt_volume_gemm<1>(fmap1, fmap2_level, vol, vl, (int)B, N, (int)C, stream, p1, p2);
    case 2: return launch_alt_volume_gemm<2>(fmap1, fmap2_level, vol, vl, (int)B, N, (int)C, stream, p1, p2);
    case 4: return launch_alt_volume_gemm<4>(fmap1, fmap2_level, vol, vl, (int)B, N, (int)C, stream, p1, p2);
    case 6: return launch_alt_volume_gemm<6>(fmap1, fmap2_level, vol, vl, (int)B, N, (int)C, stream, p1, p2);
    case 7: return launch_alt_volume_gemm<7>(fmap1, fmap2_level, vol, vl, (int)B, N, (int)C, stream, p1, p2);
    default: return DXR_EINVAL;
  }
}
