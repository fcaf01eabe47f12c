/*
 * dexiraft_corr.h — C-ABI of the MI355X-native RAFT correlation subsystem.
 *
 * This is the drop-in boundary for the hot path named in BASELINE.json
 * (`north_star`): RAFT's correlation block as used by Dexi+RAFT.  Every entry
 * point takes plain device pointers, int64 sizes and a hipStream_t; none
 * allocates, none throws, and each returns a status code (0 = ok, >0 = invalid
 * argument / unsupported, <0 = HIP launch error).  Outputs and workspaces are
 * allocated by the caller (the Python shell allocates them from torch's caching
 * allocator).  Functions are reentrant and thread-safe per stream.
 *
 * Reference interfaces replaced (paths relative to the reference repository):
 *   dxr_corr_pyramid_build   core/corr.py:13-27  CorrBlock.__init__ (matmul,
 *                            / sqrt(D), 3x F.avg_pool2d); NCHW or channels-last
 *                            fmaps (core/extractor.py:166-192 -> core/raft.py:139-148)
 *   dxr_corr_volume          core/corr.py:52-60  CorrBlock.corr (static)
 *   dxr_pyramid_unpack/pack  core/corr.py:16,24,27 the corr_pyramid attribute
 *                            (reference layout <-> paged storage)
 *   dxr_corr_lookup          core/corr.py:29-50  CorrBlock.__call__ together with
 *                            core/utils/utils.py:57-71 bilinear_sampler
 *                            (F.grid_sample, align_corners=True, zero padding)
 *   dxr_corr_lookup_backward core/utils/utils.py:65 grid_sample backward
 *                            (autograd of CorrBlock.__call__, train.py:175-178);
 *                            _multi: several lookups' backwards in one launch
 *   dxr_pyramid_backward     core/corr.py:25-27,58-60 avg_pool2d + division
 *                            backward (autograd of CorrBlock.__init__)
 *   dxr_fmap_grads           core/corr.py:13-27,52-60 the whole CorrBlock.__init__
 *                            backward (pooling + division + matmul) to d fmap1/2
 *   dxr_avg_pool2x2          core/corr.py:69-71  F.avg_pool2d(fmap, 2, stride=2)
 *                            in AlternateCorrBlock.__init__
 *   dxr_avg_pool2x2_nhwc     core/corr.py:70-71 the same pool on channels-last fmaps
 *   dxr_transpose            core/corr.py:82-83 fmap.permute(0, 2, 3, 1).contiguous()
 *                            (NCHW <-> NHWC)
 *   dxr_alt_corr_forward     alt_cuda_corr/correlation.cpp:23-33 `forward`
 *                            (alt_cuda_corr/correlation_kernel.cu:260-286)
 *   dxr_alt_corr_backward    alt_cuda_corr/correlation.cpp:36-48 `backward`
 *                            (alt_cuda_corr/correlation_kernel.cu:288-320)
 *   dxr_alt_corr_lookup      core/corr.py:74-91  AlternateCorrBlock.__call__
 *   dxr_alt_corr_lookup_ws   the same, queries ordered by window position first
 *                            (all levels in one launch, / sqrt(D) fused)
 *   dxr_corr_lookup_conv1x1  core/corr.py:29-50 CorrBlock.__call__ followed by
 *                            core/update.py:90 F.relu(self.convc1(corr))
 *                            (BasicMotionEncoder; :71 SmallMotionEncoder)
 *   dxr_conv1x1_pack_weight  core/update.py:83 / :66 the convc1 weight,
 *                            rearranged once into the fused kernel's operand layout
 *
 * Layouts (all row-major, C-contiguous):
 *   fmap (CorrBlock)        [B, D, H, W]               (NCHW, as core/raft.py:139-142)
 *                           or [B, H, W, D] (DXR_NHWC)
 *   pyramid                 PAGED storage (opaque to callers; sizes and level
 *                           offsets from dxr_pyramid_numel/_level_offset).  Level l
 *                           has H_l = floor(H_{l-1}/2) rows, as F.avg_pool2d.  Levels
 *                           0..3 are split into pages of 128 query pixels x one
 *                           (8x16 >> l) tile of image-2 cells, each page contiguous
 *                           and written by one build workgroup; levels >= 4 are
 *                           row-major.  dxr_pyramid_unpack converts a level to the
 *                           reference's corr_pyramid[l] layout [B*H*W, H_l, W_l].
 *   coords                  [B, 2, H, W] float32       channel 0 = x, 1 = y
 *                           (core/utils/utils.py:74-77)
 *   lookup output           [B, L*(2r+1)^2, H, W] float32, channel
 *                           l*(2r+1)^2 + ix*(2r+1) + iy, x offset = ix - r
 *                           (x-major, core/corr.py:37-46)
 *   alt fmaps               [B, H, W, C]               (NHWC, core/corr.py:82-83)
 *   alt coords              [B, Nc, H1, W1, 2]
 *   alt output              [B, Nc, (2r+1)^2, H1, W1]  channel iy + (2r+1)*ix
 *                           (alt_cuda_corr/correlation_kernel.cu:92-95)
 */
#ifndef DEXIRAFT_CORR_H
#define DEXIRAFT_CORR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* HIP's own definition; repeating an identical typedef is legal in C11/C++. */
typedef struct ihipStream_t* hipStream_t;

#define DXR_ABI_VERSION 10

enum dxr_status {
  DXR_OK = 0,
  DXR_EINVAL = 1,        /* bad pointer / shape / radius / level count   */
  DXR_EUNSUPPORTED = 2,  /* valid request this build does not implement  */
  DXR_EHIP = -1          /* a HIP launch failed; see dxr_last_hip_error() */
};

enum dxr_dtype {
  DXR_F32 = 0,
  DXR_BF16 = 1          /* storage as IEEE bfloat16 bit patterns (uint16) */
};

enum dxr_layout {
  DXR_NCHW = 0,         /* fmaps [B, D, H, W] (core/raft.py:139-142)              */
  DXR_NHWC = 1          /* fmaps [B, H, W, D] (channels-last encoders, §8(f) row 4) */
};

enum dxr_build_algo {
  DXR_BUILD_AUTO = 0,       /* f32 fmaps: split build where its layout allows  */
  DXR_BUILD_EXACT_F32 = 1   /* f32 fmaps: exact-f32 MFMA build (v_mfma_f32_32x32x2_f32) */
};

/* ABI version of the loaded library (== DXR_ABI_VERSION it was built with). */
int dxr_abi_version(void);

/* Human-readable name of a dxr_status value. */
const char* dxr_status_string(int status);

/* hipError_t of the most recent failed launch on the calling thread. */
int dxr_last_hip_error(void);

/* Elements (not bytes) of a num_levels pyramid for B pairs of H x W fmaps. */
int64_t dxr_pyramid_numel(int64_t B, int64_t H, int64_t W, int num_levels);

/* Element offset of level `level` inside that pyramid buffer. */
int64_t dxr_pyramid_level_offset(int64_t B, int64_t H, int64_t W, int level);

/*
 * Stage (a)+(b): all-pairs correlation fmap1^T . fmap2 / divisor and its
 * avg-pool pyramid, written in one pass (pooling fused into the MFMA epilogue).
 *   fmap1, fmap2 : [B, D, H, W] (fmap_layout DXR_NCHW) or [B, H, W, D]
 *                  (DXR_NHWC), dtype in_dtype (DXR_F32 or DXR_BF16)
 *   divisor      : the reference divides by sqrt(D) (core/corr.py:60)
 *   pyramid      : dxr_pyramid_numel(B,H,W,num_levels) elements of pyr_dtype
 *                  (levels beyond 4 need pyr_dtype DXR_F32)
 *   num_levels   : >= 1; every level must be at least 1 x 1
 *   algo         : DXR_BUILD_AUTO, or DXR_BUILD_EXACT_F32 (f32 fmaps only)
 * DXR_F32 inputs compute in f32 class: every f32 operand is split into an f16
 * pair x = hi + 2^-11 lo and three f16 x f16 MFMA products per f32 product are
 * accumulated in two f32 accumulators (the lo*lo term, <= 2^-22 |x y|, dropped);
 * a page whose sums are not finite (an operand beyond the f16 range, or inf/NaN)
 * is recomputed on an exact three-way bf16 split (six products).  The pair is
 * unscaled here: where |x| < 2^-14, hi falls on f16's subnormal grid and the
 * pair's error stays ~2^-36 absolute, so relative accuracy drops for tiny fmaps
 * (~1e-4 at |x| ~ 1e-7); dxr_corr_pyramid_build_ws (per-pixel power-of-two
 * scaling, what CorrBlock calls) has no such bound.  With
 * D % 16 != 0, odd W or DXR_BUILD_EXACT_F32 the exact-f32 MFMA
 * v_mfma_f32_32x32x2_f32 is used.  Pyramid stores are write-through (sc1).
 * DXR_BF16 inputs use bf16 MFMA with f32 accumulation.  NHWC and NCHW inputs
 * of the same values give bit-identical pyramids.
 *
 * Kernels by request (both build entry points; tests/test_gpu_parity.py
 * test_build_kernel_by_request runs each one by name against the oracle):
 *   f32, workspace, AUTO, D % 16 == 0   split_pairs_kernel + corr_build_dma_kernel
 *                                        (CorrBlock's path; NCHW or NHWC)
 *   f32, no workspace, AUTO, D % 16 == 0, even W
 *                                        corr_build_split_kernel (round-2 register
 *                                        split; the documented fallback for callers
 *                                        that cannot provide a workspace)
 *   f32, EXACT_F32 or D % 16 != 0 (or odd W without a workspace)
 *                                        corr_build_f32_kernel (exact-f32 MFMA)
 *   bf16 NCHW, workspace, D % 32 == 0   pack_bf16_kernel + corr_build_dma_kernel
 *   bf16 NHWC, D % 32 == 0              corr_build_dma_kernel (rows read in place)
 *   bf16 NCHW, no workspace, W % 4 == 0 corr_build_bf16_q2_kernel
 *   bf16 otherwise                      corr_build_bf16_kernel (one query block)
 */
int dxr_corr_pyramid_build(const void* fmap1, const void* fmap2, int in_dtype,
                           int fmap_layout, int64_t B, int64_t D, int64_t H,
                           int64_t W, int num_levels, float divisor,
                           void* pyramid, int pyr_dtype, int algo,
                           hipStream_t stream);

/*
 * Bytes of device workspace dxr_corr_pyramid_build_ws uses for B pairs of
 * D x H x W fmaps of in_dtype (0: that request needs none; -1: bad geometry):
 * f32 with D % 16 == 0 the pre-split operands, bf16 with D % 32 == 0 the pack
 * pass's blocked copies of NCHW fmaps (channels-last bf16 fmaps need none).
 * ABI 6.
 */
int64_t dxr_build_workspace_bytes(int in_dtype, int64_t B, int64_t D, int64_t H,
                                  int64_t W);

/*
 * dxr_corr_pyramid_build with a caller-owned workspace (16-byte aligned, at
 * least dxr_build_workspace_bytes; contents need no initialisation and are
 * dead after the build).  Same arguments, same result contract; with DXR_F32
 * fmaps, algo DXR_BUILD_AUTO and D % 16 == 0 it runs the pre-split build:
 * one pass scales every pixel's channel vector by a power of two 2^s
 * (|x 2^s| < 2^14) and splits it into an f16 pair x 2^s = hi + lo
 * (lo = RNE_f16(x 2^s - hi)) in the workspace, then the build's K loop moves
 * those pairs by LDS-DMA and runs three f16 MFMA products per f32 product
 * (lo.hi + hi.lo + hi.hi into one f32 accumulator), undoing both scales
 * exactly in its epilogue — f32-class error (the pair holds each element to
 * <= 2^-23 |x| unless it is more than 2^16 below its pixel's max) at any fmap
 * scale, bit-identical for NCHW and NHWC fmaps and exactly linear in
 * power-of-two scalings of either fmap.  A workgroup whose sums are not
 * finite (an inf/NaN operand) rewrites its pages from the f32 operands on the
 * exact-f32 MFMA (IEEE inf/NaN semantics).  NHWC fmaps need 16-byte aligned
 * pixel rows.  With DXR_BF16 NCHW fmaps (D % 32 == 0) a pack pass copies the
 * operands into 64-byte records of 32 channels per pixel and the bf16 build
 * runs the same LDS-DMA K loop on them — the workspace-less bf16 build's
 * pyramid bit for bit.  A NULL or short workspace runs dxr_corr_pyramid_build.
 * Replaces the same reference lines: core/corr.py:52-60 + :21-27.  ABI 6.
 */
int dxr_corr_pyramid_build_ws(const void* fmap1, const void* fmap2, int in_dtype,
                              int fmap_layout, int64_t B, int64_t D, int64_t H,
                              int64_t W, int num_levels, float divisor,
                              void* pyramid, int pyr_dtype, int algo,
                              void* workspace, int64_t workspace_bytes,
                              hipStream_t stream);

/*
 * CorrBlock.corr: the level-0 volume alone, row-major [B, H, W, 1, H, W]
 * (= [B*H*W, H, W]) float32, divided by `divisor`.
 */
int dxr_corr_volume(const void* fmap1, const void* fmap2, int in_dtype,
                    int64_t B, int64_t D, int64_t H, int64_t W, float divisor,
                    float* out, hipStream_t stream);

/*
 * Convert one level between the paged pyramid and the reference layout
 * [B*H*W, H_l, W_l] float32 (core/corr.py:22-27).  Padding cells of the paged
 * storage are neither read nor written.
 */
int dxr_pyramid_unpack(const void* pyramid, int pyr_dtype, int64_t B, int64_t H,
                       int64_t W, int num_levels, int level, float* out,
                       hipStream_t stream);
int dxr_pyramid_pack(const float* level_data, int64_t B, int64_t H, int64_t W,
                     int num_levels, int level, void* pyramid, int pyr_dtype,
                     hipStream_t stream);

/*
 * Stage (c): radius-r bilinear lookup of every level around coords / 2^l.
 *   pyramid : as produced by dxr_corr_pyramid_build
 *   coords  : [B, 2, H, W] float32
 *   out     : [B, num_levels*(2r+1)^2, H, W] float32
 * A level with H_l == 1 or W_l == 1 yields NaN, as the reference does
 * (bilinear_sampler divides by H_l-1 / W_l-1, core/utils/utils.py:61-62).
 */
int dxr_corr_lookup(const void* pyramid, int pyr_dtype,
                    int64_t B, int64_t H, int64_t W, int num_levels, int radius,
                    const float* coords, float* out, hipStream_t stream);

/*
 * Backward of stage (c) (training: core/utils/utils.py:65 grid_sample under
 * autograd, train.py:175-178): ADDS d loss / d pyramid of one lookup to
 * grad_pyramid, a float32 buffer with the pyramid's paged layout and size
 * (dxr_pyramid_numel; the caller zero-fills it once and may accumulate several
 * lookups into it).  grad_out: [B, num_levels*(2r+1)^2, H, W] float32.  No
 * coordinate gradient (the reference detaches coords, core/raft.py:170).
 */
int dxr_corr_lookup_backward(const float* coords, const float* grad_out,
                             int64_t B, int64_t H, int64_t W, int num_levels,
                             int radius, void* grad_pyramid, int grad_dtype,
                             hipStream_t stream);

/*
 * The same for n_sets lookups of one block at once (coords[i], grad_out[i]),
 * added in the order given — the result equals n_sets single calls in that
 * order bit for bit — in one launch, so each workgroup's window lines stay in
 * L2 across the sets.  n_sets <= 16 (more: DXR_EUNSUPPORTED).  ABI 7.
 */
int dxr_corr_lookup_backward_multi(const float* const* coords, const float* const* grad_out,
                                   int n_sets, int64_t B, int64_t H, int64_t W,
                                   int num_levels, int radius, void* grad_pyramid,
                                   int grad_dtype, hipStream_t stream);

/*
 * dxr_corr_lookup_backward_multi that also records a magnitude bound of the
 * gradient pyramid for dxr_fmap_grads_bounded: every workgroup adds to its own
 * element of bound_slots (a float32 array of dxr_lookup_backward_bound_slots(B,
 * H, W, num_levels, radius) elements that the caller zero-fills with the
 * gradient pyramid) 9 x the largest |grad_out| it reads per set (a cell hears
 * from at most 3 x 3 samples, tap weights <= 1; non-finite values count as
 * +inf), so after any number of calls max(bound_slots) >= max |grad_pyramid|.
 * The gradient pyramid is the one dxr_corr_lookup_backward_multi writes, bit
 * for bit.  ABI 8.
 */
int64_t dxr_lookup_backward_bound_slots(int64_t B, int64_t H, int64_t W, int num_levels,
                                        int radius);
int dxr_corr_lookup_backward_multi_bound(const float* const* coords,
                                         const float* const* grad_out, int n_sets,
                                         int64_t B, int64_t H, int64_t W, int num_levels,
                                         int radius, void* grad_pyramid, int grad_dtype,
                                         float* bound_slots, hipStream_t stream);

/*
 * Stage (c) fused with the motion encoder's 1x1 convolution (SURVEY.md §8(f)
 * row 2; inference):
 *   out[b,o,h,w] = act(bias[o] + sum_c weight[o,c] * lookup(coords)[b,c,h,w])
 * lookup() is dxr_corr_lookup (bit-identical samples), the contraction runs in
 * f32 class (f16 pair split of both operands, x = hi + 2^-11 lo, three MFMA
 * products, f32 accumulation; workgroups whose sums are not finite re-run it on
 * the exact three-way bf16 split).
 *   weight_packed : dxr_conv1x1_pack_weight of the [cout, cin] float32 weight,
 *                   cin = num_levels*(2r+1)^2 (dxr_conv1x1_packed_bytes bytes:
 *                   float32 [ceil(cin/16)*2][cout][8], zero padded, followed by
 *                   the same layout as f16 pairs, 8 hi then 8 lo per 32 bytes)
 *   bias          : [cout] float32 or NULL;  relu: 1 = F.relu, 0 = none
 *   out           : [B, cout, H, W] float32
 * Supported: radius 3 or 4, num_levels <= 4, cout a multiple of 32 (<= 4096);
 * other valid requests return DXR_EUNSUPPORTED.
 */
int64_t dxr_conv1x1_packed_bytes(int64_t cout, int64_t cin);
int dxr_conv1x1_pack_weight(const float* weight, int64_t cout, int64_t cin,
                            void* packed, hipStream_t stream);
int dxr_corr_lookup_conv1x1(const void* pyramid, int pyr_dtype,
                            int64_t B, int64_t H, int64_t W, int num_levels,
                            int radius, const float* coords,
                            const void* weight_packed, const float* bias,
                            int64_t cout, int relu, float* out,
                            hipStream_t stream);

/*
 * Backward of stages (a)+(b) down to the volume: folds the gradient of every
 * level down the avg-pool chain (core/corr.py:25-27) and divides by `divisor`
 * (core/corr.py:60), writing d loss / d (fmap1^T fmap2) as row-major
 * [B*H*W, H, W] float32.  The fmap gradients are then two plain GEMMs:
 * dfmap1 = fmap2 . dV^T, dfmap2 = fmap1 . dV (per pair, [D, H*W]).
 */
int dxr_pyramid_backward(const void* grad_pyramid, int grad_dtype,
                         int64_t B, int64_t H, int64_t W, int num_levels,
                         float divisor, float* grad_volume, hipStream_t stream);

/*
 * Backward of stages (a)+(b) straight to the fmap gradients, without the
 * [B, H*W, H*W] volume gradient (core/corr.py:13-27,52-60 under autograd,
 * train.py:175-178): the gradient pyramid is folded down the pooling chain
 * inside the two GEMMs' operand loads,
 *   grad_fmap1 = fmap2 . dV^T,  grad_fmap2 = fmap1 . dV   (dV as above),
 * on MFMA with a three-way bf16 split of both operands (six products, f32
 * accumulation: f32-class).  Deterministic (fixed summation order).
 * Range: every finite operand stays finite in the split (one beyond
 * bfloat16's largest finite value, |x| > 3.3895e38, keeps its truncation as the
 * high part instead of rounding it to +-inf); inf and NaN operands propagate as
 * in an f32 GEMM.
 *   grad_pyramid : float32, the paged layout of dxr_corr_pyramid_build
 *   fmap1, fmap2 : [B, D, H, W] float32, NCHW contiguous
 *   grad_fmap1/2 : [B, D, H, W] float32 outputs, either may be NULL (skipped)
 *   workspace    : >= dxr_fmap_grads_workspace_bytes(B, D, H, W, num_levels)
 * Supported: D a multiple of 32, num_levels <= 4 (other valid requests return
 * DXR_EUNSUPPORTED; dxr_pyramid_backward + two GEMMs covers them).
 * dxr_fmap_grads_workspace_bytes returns -1 for unsupported shapes.  ABI 7.
 */
int64_t dxr_fmap_grads_workspace_bytes(int64_t B, int64_t D, int64_t H, int64_t W,
                                       int num_levels);
int dxr_fmap_grads(const void* grad_pyramid, int grad_dtype, const float* fmap1,
                   const float* fmap2, int64_t B, int64_t D, int64_t H, int64_t W,
                   int num_levels, float divisor, float* grad_fmap1, float* grad_fmap2,
                   void* workspace, int64_t workspace_bytes, hipStream_t stream);

/*
 * dxr_fmap_grads given a bound on the gradient pyramid: bound_slots[0..n_slots)
 * (device float32, e.g. dxr_corr_lookup_backward_multi_bound's slots) hold
 * values whose maximum is >= max |grad_pyramid|.  Both operands then run as
 * power-of-two-scaled f16 pairs (x 2^s = hi + lo, |x 2^s| < 2^14; one scale per
 * fmap channel, one for the folded dV) with three f16 MFMA products and f32
 * accumulation — half the MFMA work of the six-product split, f32-class:
 * per-operand error <= 2^-22 |x| + 2^-39 of its scale's bound.  A pair whose
 * fmap holds inf/NaN, or a non-finite bound, runs the six-product arithmetic of
 * dxr_fmap_grads (same IEEE propagation).  A bound below the true maximum gives
 * wrong (overflowed) results.  workspace: >= dxr_fmap_grads_bounded_workspace_bytes
 * (<= dxr_fmap_grads_workspace_bytes, which covers both forms).  Same outputs'
 * layout, deterministic.  ABI 8.
 */
int64_t dxr_fmap_grads_bounded_workspace_bytes(int64_t B, int64_t D, int64_t H, int64_t W,
                                               int num_levels);
int dxr_fmap_grads_bounded(const void* grad_pyramid, int grad_dtype, const float* fmap1,
                           const float* fmap2, int64_t B, int64_t D, int64_t H, int64_t W,
                           int num_levels, float divisor, const float* bound_slots,
                           int64_t n_slots, float* grad_fmap1, float* grad_fmap2,
                           void* workspace, int64_t workspace_bytes, hipStream_t stream);

/*
 * 2x2 / stride-2 average pool, floor mode, of [planes, H, W] float32 into
 * [planes, H/2, W/2] (F.avg_pool2d(x, 2, stride=2), core/corr.py:26,70-71).
 */
int dxr_avg_pool2x2(const float* in, float* out, int64_t planes,
                    int64_t H, int64_t W, hipStream_t stream);

/*
 * Channels-last fmaps.
 *
 * dxr_transpose: batched [B, rows, cols] -> [B, cols, rows] of float32
 * (dtype DXR_F32) or bfloat16 (DXR_BF16) elements; NCHW -> NHWC is rows = C,
 * cols = H*W (core/corr.py:82-83 `permute(0, 2, 3, 1).contiguous()`), NHWC ->
 * NCHW the reverse.  Bit-exact.
 *
 * dxr_avg_pool2x2_nhwc: F.avg_pool2d(x, 2, stride=2) (core/corr.py:70-71) of a
 * channels-last [B, H, W, C] float32 tensor into [B, H/2, W/2, C]; bit-identical
 * to dxr_avg_pool2x2 on the NCHW tensor (same four values, same summation order).
 */
int dxr_transpose(const void* in, void* out, int dtype, int64_t B, int64_t rows,
                  int64_t cols, hipStream_t stream);
int dxr_avg_pool2x2_nhwc(const float* in, float* out, int64_t B, int64_t H,
                         int64_t W, int64_t C, hipStream_t stream);

/*
 * Stage (d), reference-FFI form: alt_cuda_corr.forward(fmap1, fmap2, coords,
 * radius) with the reference's layouts (see the header comment).  `corr` is
 * fully overwritten (the reference zero-fills then accumulates).
 */
int dxr_alt_corr_forward(const float* fmap1, const float* fmap2,
                         const float* coords, float* corr,
                         int64_t B, int64_t H1, int64_t W1, int64_t H2,
                         int64_t W2, int64_t C, int64_t Nc, int radius,
                         hipStream_t stream);

/*
 * Stage (d), reference-FFI backward: alt_cuda_corr.backward(fmap1, fmap2, coords,
 * corr_grad, radius) (correlation.cpp:36-48, correlation_kernel.cu:122-256,288-320).
 *   corr_grad  : [B, Nc, (2r+1)^2, H1, W1] float32 (the forward's output layout)
 *   fmap1_grad : [B, H1, W1, C]  fully overwritten
 *   fmap2_grad : [B, H2, W2, C]  zero-filled on `stream`, then accumulated with
 *                atomics (summation order, hence the last bits, is not fixed —
 *                as in the reference)
 * The reference's third output, coords_grad, is identically zero; the caller
 * allocates it.  Radius 0..6.
 */
int dxr_alt_corr_backward(const float* fmap1, const float* fmap2,
                          const float* coords, const float* corr_grad,
                          float* fmap1_grad, float* fmap2_grad,
                          int64_t B, int64_t H1, int64_t W1, int64_t H2,
                          int64_t W2, int64_t C, int64_t Nc, int radius,
                          hipStream_t stream);

/*
 * Stage (d), fused form used by AlternateCorrBlock.__call__: every level in one
 * launch, output already divided by `divisor`, written in CorrBlock's layout.
 *   fmap1        : [B, H, W, C] full resolution (NHWC)
 *   fmap2_levels : num_levels pointers; level l is [B, H_l, W_l, C] (NHWC),
 *                  H_l = floor(H_{l-1}/2)
 *   coords       : [B, 2, H, W] float32 (CorrBlock convention)
 *   out          : [B, num_levels*(2r+1)^2, H, W] float32
 */
int dxr_alt_corr_lookup(const float* fmap1, const float* const* fmap2_levels,
                        const float* coords, float* out,
                        int64_t B, int64_t H, int64_t W, int64_t C,
                        int num_levels, int radius, float divisor,
                        hipStream_t stream);

/*
 * Bytes of device workspace dxr_alt_corr_lookup_ws uses for B coordinate sets
 * of H x W queries over num_levels levels (per level and set: the ordered list,
 * 16 B per query slot of every 4 x 8 query tile, 4-B bin ids, 64 blocks'
 * histograms of up to 4097 bins; -1: bad geometry).  ABI 6.
 */
int64_t dxr_alt_workspace_bytes(int64_t B, int64_t H, int64_t W, int num_levels);

/*
 * dxr_alt_corr_lookup with a caller-owned workspace (16-byte aligned, at least
 * dxr_alt_workspace_bytes; no initialisation needed).  Three small launches
 * (count, scan, scatter) order each level's queries before the lookup: grouped
 * by window position (bins of ~32 queries) when the 4 x 8 query tiles' union
 * boxes would be larger than 1.5x a bin group's (flows that vary pixel to
 * pixel), else in tile order.  The scan always walks the fixed 64 x 4097-bin
 * histogram, so the three launches cost a few microseconds even for small
 * maps.  The outputs are the workspace-less call's, bit for bit.  Falls back to
 * dxr_alt_corr_lookup when the workspace is NULL or short.  Replaces
 * core/corr.py:74-91 as above.  ABI 6.
 */
int dxr_alt_corr_lookup_ws(const float* fmap1, const float* const* fmap2_levels,
                           const float* coords, float* out,
                           int64_t B, int64_t H, int64_t W, int64_t C,
                           int num_levels, int radius, float divisor,
                           void* workspace, int64_t workspace_bytes,
                           hipStream_t stream);

/*
 * dxr_alt_corr_lookup_ws for levels [0, n_levels) only of a num_levels-level
 * output (channels of the other levels untouched): the alternate block's
 * on-the-fly part when its coarse levels come from dxr_alt_volume_lookup.
 * Workspace: dxr_alt_workspace_bytes(B, H, W, n_levels).  Replaces
 * core/corr.py:74-91 for those levels.  ABI 9.
 */
int dxr_alt_corr_lookup_levels_ws(const float* fmap1, const float* const* fmap2_levels,
                                  const float* coords, float* out,
                                  int64_t B, int64_t H, int64_t W, int64_t C,
                                  int num_levels, int n_levels, int radius, float divisor,
                                  void* workspace, int64_t workspace_bytes,
                                  hipStream_t stream);

/*
 * Coarse-level volumes of the alternate block (round 6).  An on-the-fly
 * lookup recomputes each level's window dot products on every call; for a
 * coarse level the whole volume (every fmap1 pixel against every cell of the
 * pooled fmap2 level) costs less than one lookup, once per block.
 *   dxr_alt_volume_numel    floats of the volumes of levels
 *                           [first_level, num_levels) (-1: bad geometry);
 *   dxr_alt_coarse_volumes  computes them: raw dot products <fmap1[q],
 *                           fmap2_levels[l][cell]> (not divided), the same
 *                           f16-pair MFMA products as dxr_alt_corr_lookup's,
 *                           stored in the paged layout of those pyramid levels
 *                           (the tail of a num_levels-level pyramid buffer);
 *                           fmap1 / fmap2_levels as dxr_alt_corr_lookup
 *                           (NHWC, 16-byte aligned), C % 16 == 0, C <= 256;
 *   dxr_alt_volume_lookup   reads the windows of levels [first_level,
 *                           num_levels) from them with correlation_kernel.cu's
 *                           arithmetic (origin floor(c / 2^l) - r, bilinear
 *                           weights of the fraction, :92-114's order, divided
 *                           by divisor) into those levels' channels of `out`
 *                           ([B, num_levels*(2r+1)^2, H, W]); r <= 8.
 * With finite operands inside the f16 pair's range the outputs are
 * dxr_alt_corr_lookup's bit for bit.  Replaces core/corr.py:74-91 (levels
 * >= first_level) with the reference's alt_cuda_corr semantics.  ABI 9.
 *   dxr_alt_coarse_volumes_ws_bytes / dxr_alt_coarse_volumes_ws (ABI 10): the
 *                           same volumes, bit for bit, with a caller workspace
 *                           for the f16 pair planes of fmap1 and of the levels
 *                           (C % 32 == 0, levels 0-3), which the volume GEMM
 *                           then stages by LDS-DMA; a null or short workspace
 *                           falls back to dxr_alt_coarse_volumes.  0 bytes when
 *                           no level takes the GEMM; -1: bad geometry.
 */
int64_t dxr_alt_volume_numel(int64_t B, int64_t H, int64_t W, int num_levels, int first_level);
int dxr_alt_coarse_volumes(const float* fmap1, const float* const* fmap2_levels,
                           int64_t B, int64_t H, int64_t W, int64_t C,
                           int num_levels, int first_level, float* volumes,
                           hipStream_t stream);
int64_t dxr_alt_coarse_volumes_ws_bytes(int64_t B, int64_t H, int64_t W, int64_t C,
                                        int num_levels, int first_level);
int dxr_alt_coarse_volumes_ws(const float* fmap1, const float* const* fmap2_levels,
                              int64_t B, int64_t H, int64_t W, int64_t C,
                              int num_levels, int first_level, float* volumes,
                              void* workspace, int64_t workspace_bytes, hipStream_t stream);
int dxr_alt_volume_lookup(const float* volumes, const float* coords, float* out,
                          int64_t B, int64_t H, int64_t W, int num_levels, int first_level,
                          int radius, float divisor, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* DEXIRAFT_CORR_H */
