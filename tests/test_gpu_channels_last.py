"""Channels-last (NHWC) fmaps, through the C-ABI on an MI355X.

The encoders (core/extractor.py:168-192) may emit channels-last fmaps.  The
blocks take them without torch's strided copies: ``dxr_transpose`` for the NCHW
build operands, a free view for AlternateCorrBlock's NHWC operands, and
``dxr_avg_pool2x2_nhwc`` for its pooled levels.  Every result must be
bit-identical to the same block fed the NCHW-contiguous fmaps, and the pools
bit-identical to the oracle's F.avg_pool2d restatement (oracle/corr_oracle.py:42,
pinned to the reference's pyramids by tests/test_oracle_golden.py).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import datagen as dg
import oracle

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def dx():
    import dexiraft_amd
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dexiraft_amd.load_native()
    return dexiraft_amd


def _t(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _cl(t: torch.Tensor) -> torch.Tensor:
    out = t.contiguous(memory_format=torch.channels_last)
    assert not out.is_contiguous()
    return out


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(1, 64, 64), (2, 37, 130), (3, 256, 7040), (1, 5, 1)])
def test_transpose_bit_exact(dx, dtype, shape):
    B, R, C = shape
    x = _t(dg.normal(11, B * R * C).reshape(B, R, C).astype(np.float32)).to(dtype)
    out = torch.empty((B, C, R), dtype=dtype, device=DEV)
    code = 0 if dtype == torch.float32 else 1
    lib = dx._native.load()
    assert lib.dxr_transpose(x.data_ptr(), out.data_ptr(), code, B, R, C, _stream()) == 0
    torch.cuda.synchronize()
    assert torch.equal(out, x.transpose(1, 2))


@pytest.mark.parametrize("shape", [(1, 9, 13, 64), (2, 55, 128, 256), (1, 6, 7, 3)])
def test_avg_pool_nhwc_matches_oracle_bit_exact(dx, shape):
    B, H, W, C = shape
    x = dg.normal(21, B * H * W * C).reshape(B, H, W, C).astype(np.float32)
    out = torch.empty((B, H // 2, W // 2, C), dtype=torch.float32, device=DEV)
    lib = dx._native.load()
    assert lib.dxr_avg_pool2x2_nhwc(_t(x).data_ptr(), out.data_ptr(), B, H, W, C, _stream()) == 0
    ref = oracle.avg_pool2x2(x.transpose(0, 3, 1, 2)).transpose(0, 2, 3, 1)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_alternate_block_channels_last_bit_identical(dx):
    B, D, H, W, r = 2, 64, 33, 47, 4
    f1 = _t(dg.fmap(31, B, D, H, W, "fnet"))
    f2 = _t(dg.fmap(32, B, D, H, W, "fnet"))
    c = _t(dg.coords(33, B, H, W, "normal", 4.0))
    with torch.no_grad():
        a = dx.AlternateCorrBlock(f1, f2, radius=r)
        b = dx.AlternateCorrBlock(_cl(f1), _cl(f2), radius=r)
        # the channels-last block reads the caller's storage: no copy of fmap1
        assert b._f1_nhwc.data_ptr() == b._fmaps[0].data_ptr()
        assert torch.equal(a(c), b(c))
        assert len(b.pyramid) == 5
        for lvl in range(5):
            for k in range(2):
                pa, pb = a.pyramid[lvl][k], b.pyramid[lvl][k]
                assert tuple(pa.shape) == tuple(pb.shape) == (B, D, H >> lvl, W >> lvl)
                assert torch.equal(pa, pb)
    # the pooled entries are F.avg_pool2d of the previous one (oracle restatement)
    f1n = f1.cpu().numpy()
    for lvl in range(1, 5):
        f1n = oracle.avg_pool2x2(f1n)
        np.testing.assert_array_equal(b.pyramid[lvl][0].cpu().numpy(), f1n)


def test_alternate_block_channels_last_matches_oracle(dx):
    B, D, H, W, r = 1, 128, 24, 40, 3
    f1 = dg.fmap(41, B, D, H, W)
    f2 = dg.fmap(42, B, D, H, W)
    c = dg.coords(43, B, H, W, "uniform", 9.0)
    ref = oracle.alt_corr_block(f1, f2, c, 4, r, np.float64)
    with torch.no_grad():
        got = dx.AlternateCorrBlock(_cl(_t(f1)), _cl(_t(f2)), radius=r)(_t(c)).cpu().numpy()
    scale = np.abs(ref).max()
    assert np.abs(got - ref).max() <= 1e-4 * scale


@pytest.mark.parametrize("shape", [(2, 256, 23, 31), (2, 256, 23, 32), (1, 256, 46, 62),
                                   (1, 64, 55, 128)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_corr_block_channels_last_bit_identical(dx, dtype, shape):
    """Channels-last fmaps give the NCHW block's bits: f32 with even W takes the
    split build's NHWC operand loads, bf16 with D % 32 == 0 the two-block bf16
    build's (no layout pass); other cases one transpose."""
    B, D, H, W = shape
    f1 = _t(dg.fmap(51, B, D, H, W, "fnet")).to(dtype)
    f2 = _t(dg.fmap(52, B, D, H, W, "fnet")).to(dtype)
    c = _t(dg.coords(53, B, H, W, "normal", 4.0))
    with torch.no_grad():
        a = dx.CorrBlock(f1, f2)
        b = dx.CorrBlock(_cl(f1), _cl(f2))
        for lvl in range(4):   # valid cells (page padding is never read)
            assert torch.equal(a.corr_pyramid[lvl], b.corr_pyramid[lvl])
        assert torch.equal(a(c), b(c))
        if dtype == torch.float32:
            assert torch.equal(dx.CorrBlock.corr(f1, f2), dx.CorrBlock.corr(_cl(f1), _cl(f2)))


def test_corr_block_channels_last_under_grad_keeps_autograd(dx):
    """With grad, the build's operands stay on torch's tracked copy: the fmap
    gradients of a channels-last input equal those of the NCHW input."""
    B, D, H, W = 1, 64, 12, 16
    base1 = _t(dg.fmap(61, B, D, H, W))
    base2 = _t(dg.fmap(62, B, D, H, W))
    c = _t(dg.coords(63, B, H, W, "normal", 3.0))
    grads = []
    for conv in (lambda t: t, _cl):
        f1 = conv(base1.clone()).requires_grad_(True)
        f2 = conv(base2.clone()).requires_grad_(True)
        out = dx.CorrBlock(f1, f2)(c)
        out.square().sum().backward()
        grads.append((f1.grad.contiguous(), f2.grad.contiguous()))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])


def test_nhwc_build_entry_point(dx):
    """dxr_corr_pyramid_build with DXR_NHWC reads channels-last operands in place
    (f32, D % 16 == 0, even W) and writes the NCHW build's pyramid bit for bit;
    other layouts of the request are DXR_EUNSUPPORTED (the shell transposes)."""
    from dexiraft_amd import _native as nat
    lib = nat.load()
    B, D, H, W = 2, 128, 21, 40
    f1 = _t(dg.fmap(71, B, D, H, W, "fnet"))
    f2 = _t(dg.fmap(72, B, D, H, W, "fnet"))
    n = lib.dxr_pyramid_numel(B, H, W, 4)
    bufs = []
    for layout, a, b in ((nat.DXR_NCHW, f1, f2), (nat.DXR_NHWC, _cl(f1), _cl(f2))):
        buf = torch.full((n,), float("nan"), device=DEV)
        st = lib.dxr_corr_pyramid_build(a.data_ptr(), b.data_ptr(), nat.DXR_F32, layout, B, D, H,
                                        W, 4, float(np.sqrt(np.float32(D))), buf.data_ptr(),
                                        nat.DXR_F32, nat.DXR_BUILD_AUTO, nat.stream_of(a))
        assert st == 0
        bufs.append(buf)
    assert torch.equal(bufs[0], bufs[1])          # pages, padding included
    g1, g2 = _cl(f1[:, :, :, :39].contiguous()), _cl(f2[:, :, :, :39].contiguous())
    st = lib.dxr_corr_pyramid_build(g1.data_ptr(), g2.data_ptr(), nat.DXR_F32, nat.DXR_NHWC, B, D,
                                    H, 39, 4, 11.3137, bufs[0].data_ptr(), nat.DXR_F32,
                                    nat.DXR_BUILD_AUTO, nat.stream_of(g1))
    assert st == nat.DXR_EUNSUPPORTED             # odd W: the NCHW build is exact-f32 there


@pytest.mark.parametrize("W", [40, 39])
@pytest.mark.parametrize("pyr_dt", ["f32", "bf16"])
def test_nhwc_bf16_build_entry_point(dx, W, pyr_dt):
    """dxr_corr_pyramid_build with bf16 DXR_NHWC operands (the bf16 mode's
    channels-last encoders, core/extractor.py:168-192) reads them in place (the
    bf16 LDS-DMA build) and writes the workspace-less NCHW bf16 build's pyramid
    bit for bit, page padding included — also for W % 4 != 0, where the NCHW
    build is the one-block kernel; so does the NCHW build with a workspace
    (pack pass + the LDS-DMA build).  D % 32 != 0 is DXR_EUNSUPPORTED (the
    shell transposes)."""
    from dexiraft_amd import _native as nat
    lib = nat.load()
    B, D, H = 2, 128, 21
    f1 = _t(dg.fmap(81, B, D, H, W, "fnet")).bfloat16()
    f2 = _t(dg.fmap(82, B, D, H, W, "fnet")).bfloat16()
    n = lib.dxr_pyramid_numel(B, H, W, 4)
    tdt, code = (torch.float32, nat.DXR_F32) if pyr_dt == "f32" else (torch.bfloat16, nat.DXR_BF16)
    bufs = []
    for layout, a, b in ((nat.DXR_NCHW, f1, f2), (nat.DXR_NHWC, _cl(f1), _cl(f2))):
        buf = torch.full((n,), float("nan"), device=DEV, dtype=tdt)
        st = lib.dxr_corr_pyramid_build(a.data_ptr(), b.data_ptr(), nat.DXR_BF16, layout, B, D, H,
                                        W, 4, float(np.sqrt(np.float32(D))), buf.data_ptr(),
                                        code, nat.DXR_BUILD_AUTO, nat.stream_of(a))
        assert st == 0
        bufs.append(buf)
    # NCHW with a workspace: the pack pass + the bf16 LDS-DMA build (scalar pack
    # loads for W = 39: N = 819 is not a multiple of 4)
    ws = torch.empty(lib.dxr_build_workspace_bytes(nat.DXR_BF16, B, D, H, W), dtype=torch.uint8,
                     device=DEV)
    buf = torch.full((n,), float("nan"), device=DEV, dtype=tdt)
    st = lib.dxr_corr_pyramid_build_ws(f1.data_ptr(), f2.data_ptr(), nat.DXR_BF16, nat.DXR_NCHW,
                                       B, D, H, W, 4, float(np.sqrt(np.float32(D))), buf.data_ptr(),
                                       code, nat.DXR_BUILD_AUTO, ws.data_ptr(), ws.numel(),
                                       nat.stream_of(f1))
    assert st == 0
    bufs.append(buf)
    torch.cuda.synchronize()
    assert not torch.isnan(bufs[1].float()).any()   # every page written
    assert torch.equal(bufs[0], bufs[1])
    assert torch.equal(bufs[0], bufs[2])
    g1 = _cl(_t(dg.fmap(83, B, 48, H, W)).bfloat16())
    st = lib.dxr_corr_pyramid_build(g1.data_ptr(), g1.data_ptr(), nat.DXR_BF16, nat.DXR_NHWC, B,
                                    48, H, W, 4, 6.9282, bufs[0].data_ptr(), code,
                                    nat.DXR_BUILD_AUTO, nat.stream_of(g1))
    assert st == nat.DXR_EUNSUPPORTED


def test_kitti_b8_bf16_channels_last_bit_identical(dx, monkeypatch):
    """C3 at full size (KITTI 375x1242 -> fmap 47x156, B = 8, D = 256, bf16):
    channels-last fmaps are read in place by the bf16 build (no dxr_transpose)
    and give the NCHW block's pyramid and lookups bit for bit."""
    B, D, H, W = 8, 256, 47, 156
    g = torch.Generator(device=DEV)
    g.manual_seed(2024)
    f1 = torch.randn((B, D, H, W), generator=g, device=DEV).bfloat16()
    f2 = torch.randn((B, D, H, W), generator=g, device=DEV).bfloat16()
    c = _t(dg.coords(93, B, H, W, "normal", 4.0))
    with torch.no_grad():
        a = dx.CorrBlock(f1, f2)
        ga = a(c)
        buf_a = a._buf
        del a
        import sys
        corr_mod = sys.modules[dx.CorrBlock.__module__]

        def no_transpose(t):
            raise AssertionError("channels-last bf16 fmaps must not be transposed")
        monkeypatch.setattr(corr_mod, "_nchw", no_transpose)
        b = dx.CorrBlock(_cl(f1), _cl(f2))
        assert torch.equal(buf_a, b._buf)             # every page, padding included
        del buf_a
        assert torch.equal(ga, b(c))
