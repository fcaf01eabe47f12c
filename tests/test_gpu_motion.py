"""GPU parity of the lookup fused with the motion encoder's convc1
(``CorrBlock.lookup_conv1x1`` -> ``dxr_corr_lookup_conv1x1``; SURVEY.md §8(f)
row 2): ``F.relu(convc1(corr_fn(coords)))`` of core/raft.py:172 +
core/update.py:90 (BasicMotionEncoder) / :71 (SmallMotionEncoder).

Tolerance (f32, as the north star): |ours - ref| <= 1e-4 * max|ref|, against
the reference encoder's golden output, and against a float64 product of the
fused kernel's own lookup samples at full benchmark size.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import datagen as dg
import oracle
from conftest import MOTION_CASES, load_motion, tolerance_check

pytestmark = pytest.mark.gpu

RTOL = 1e-4
DEV = "cuda:0"


@pytest.fixture(scope="module")
def dx():
    import dexiraft_amd
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dexiraft_amd.load_native()
    return dexiraft_amd


def _t(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _ref64(corr: torch.Tensor, w: torch.Tensor, b, relu=True) -> np.ndarray:
    return oracle.motion_conv1x1(corr.cpu().numpy(), w.cpu().numpy(),
                                 None if b is None else b.cpu().numpy(), relu)


@pytest.mark.parametrize("name", MOTION_CASES)
def test_fused_matches_reference_encoder(dx, name):
    d = load_motion(name)
    cb = dx.CorrBlock(_t(d["fmap1"]), _t(d["fmap2"]), radius=d["radius"])
    w4 = _t(d["weight"]).reshape(d["cout"], d["cin"], 1, 1)   # nn.Conv2d weight layout
    out = cb.lookup_conv1x1(_t(d["coords"]), w4, _t(d["bias"]))
    assert out.shape == (d["B"], d["cout"], d["H"], d["W"])
    assert out.dtype == torch.float32 and out.is_contiguous()
    tolerance_check(out.cpu().numpy(), d["out"], RTOL)


@pytest.mark.parametrize("workload,H,W", [("sintel", 55, 128), ("chairs", 46, 62)])
def test_fused_full_size_against_float64(dx, workload, H, W):
    """Benchmark sizes: the fused output vs a float64 product of the unfused
    lookup (whose samples the fused kernel reproduces bit for bit)."""
    g = torch.Generator(device=DEV).manual_seed(7)
    f1 = torch.randn((1, 256, H, W), generator=g, device=DEV)
    f2 = torch.randn((1, 256, H, W), generator=g, device=DEV)
    ys, xs = torch.meshgrid(torch.arange(H, device=DEV, dtype=torch.float32),
                            torch.arange(W, device=DEV, dtype=torch.float32), indexing="ij")
    coords = (torch.stack((xs, ys))[None] + 4 * torch.randn((1, 2, H, W), generator=g,
                                                           device=DEV)).contiguous()
    w = torch.randn((256, 324), generator=g, device=DEV) / 18.0
    b = 0.5 * torch.randn((256,), generator=g, device=DEV)
    cb = dx.CorrBlock(f1, f2)
    got = cb.lookup_conv1x1(coords, w, b).cpu().numpy()
    err = tolerance_check(got, _ref64(cb(coords), w, b).astype(np.float32), RTOL)
    assert err < 1e-5   # f32 class: ~1e-7 expected


def test_fused_options_and_radius3(dx):
    """No bias / no ReLU, Cout 96 at radius 3 (SmallMotionEncoder), batch of 3,
    a ragged query count (17 x 23 = 391 pixels)."""
    B, D, H, W = 3, 64, 17, 23
    f1, f2 = _t(dg.fmap(11, B, D, H, W, "fnet")), _t(dg.fmap(12, B, D, H, W, "fnet"))
    c = _t(dg.coords(13, B, H, W, "uniform", 8.0))
    for r, cout in ((3, 96), (4, 256), (4, 32)):
        cin = 4 * (2 * r + 1) ** 2
        w = _t(dg.fmap(14, 1, 1, cout, cin)[0, 0] / np.float32(np.sqrt(cin)))
        b = _t(dg.fmap(15, 1, 1, 1, cout)[0, 0, 0])
        cb = dx.CorrBlock(f1, f2, radius=r)
        corr = cb(c)
        for bias, relu in ((b, True), (None, True), (b, False), (None, False)):
            got = cb.lookup_conv1x1(c, w, bias, relu=relu).cpu().numpy()
            tolerance_check(got, _ref64(corr, w, bias, relu).astype(np.float32), RTOL)


def test_fused_batch_independence_and_determinism(dx):
    """Both Dexi+RAFT volumes in one batch-2 block (core/raft.py:146-148, 172-173)
    give bit-identical results to two blocks; repeated calls are bit-identical."""
    D, H, W = 128, 20, 36
    fa = [_t(dg.fmap(20 + k, 1, D, H, W, "fnet")) for k in range(4)]
    ca = [_t(dg.coords(30 + k, 1, H, W, "normal", 4.0)) for k in range(2)]
    w = _t(dg.fmap(40, 1, 1, 256, 324)[0, 0] / np.float32(18.0))
    b = _t(dg.fmap(41, 1, 1, 1, 256)[0, 0, 0])
    one = [dx.CorrBlock(fa[2 * k], fa[2 * k + 1]).lookup_conv1x1(ca[k], w, b) for k in range(2)]
    both = dx.CorrBlock(torch.cat([fa[0], fa[2]]), torch.cat([fa[1], fa[3]]))
    out = both.lookup_conv1x1(torch.cat(ca), w, b)
    assert torch.equal(out, torch.cat(one))
    assert torch.equal(out, both.lookup_conv1x1(torch.cat(ca), w, b))


def test_fused_bf16_pyramid(dx):
    """bf16 mode: the fused kernel reads the bf16 pyramid like the lookup does;
    the contraction stays f32 class (tolerance vs its own lookup: 1e-4)."""
    B, D, H, W = 2, 256, 24, 40
    f1 = _t(dg.fmap(50, B, D, H, W, "fnet")).bfloat16()
    f2 = _t(dg.fmap(51, B, D, H, W, "fnet")).bfloat16()
    c = _t(dg.coords(52, B, H, W, "normal", 4.0))
    w = _t(dg.fmap(53, 1, 1, 256, 324)[0, 0] / np.float32(18.0))
    cb = dx.CorrBlock(f1, f2)
    got = cb.lookup_conv1x1(c, w, None).cpu().numpy()
    tolerance_check(got, _ref64(cb(c), w, None).astype(np.float32), RTOL)


def test_fused_weight_planes_follow_weight_updates(dx):
    """The split weight is cached per (storage, version): an in-place update of
    the weight is seen by the next call."""
    B, D, H, W = 1, 64, 16, 16
    cb = dx.CorrBlock(_t(dg.fmap(60, B, D, H, W)), _t(dg.fmap(61, B, D, H, W)))
    c = _t(dg.coords(62, B, H, W, "normal", 2.0))
    w = _t(dg.fmap(63, 1, 1, 256, 324)[0, 0] / np.float32(18.0))
    a = cb.lookup_conv1x1(c, w, None, relu=False)
    with torch.no_grad():
        w.mul_(2.0)
    bb = cb.lookup_conv1x1(c, w, None, relu=False)
    torch.testing.assert_close(bb, 2.0 * a, rtol=1e-6, atol=1e-6)


def test_fused_unsupported_and_grad_raise(dx):
    B, D, H, W = 1, 64, 16, 16
    f1, f2 = _t(dg.fmap(70, B, D, H, W)), _t(dg.fmap(71, B, D, H, W))
    c = _t(dg.coords(72, B, H, W, "normal", 2.0))
    with pytest.raises(NotImplementedError):
        dx.CorrBlock(f1, f2, radius=2).lookup_conv1x1(c, torch.zeros(256, 100, device=DEV))
    cb = dx.CorrBlock(f1, f2)
    with pytest.raises(NotImplementedError):
        cb.lookup_conv1x1(c, torch.zeros(100, 324, device=DEV))   # Cout % 32
    with pytest.raises(RuntimeError):
        cb.lookup_conv1x1(c, torch.zeros(256, 300, device=DEV))   # wrong Cin
    with pytest.raises(RuntimeError):
        cb.lookup_conv1x1(c, torch.zeros(256, 324))               # host weight
    w = torch.zeros(256, 324, device=DEV, requires_grad=True)
    with pytest.raises(NotImplementedError):
        cb.lookup_conv1x1(c, w)
    with torch.no_grad():
        assert cb.lookup_conv1x1(c, w).shape == (1, 256, 16, 16)


@pytest.mark.parametrize("levels,r", [(1, 4), (2, 4), (3, 3)])
def test_fused_fewer_levels(dx, levels, r):
    """num_levels < 4 (Cin = L*(2r+1)^2 padded to whole k steps inside the kernel)."""
    B, D, H, W = 2, 64, 19, 27
    f1, f2 = _t(dg.fmap(80, B, D, H, W, "fnet")), _t(dg.fmap(81, B, D, H, W, "fnet"))
    c = _t(dg.coords(82, B, H, W, "normal", 3.0))
    cin = levels * (2 * r + 1) ** 2
    w = _t(dg.fmap(83, 1, 1, 64, cin)[0, 0] / np.float32(np.sqrt(cin)))
    b = _t(dg.fmap(84, 1, 1, 1, 64)[0, 0, 0])
    cb = dx.CorrBlock(f1, f2, num_levels=levels, radius=r)
    got = cb.lookup_conv1x1(c, w, b).cpu().numpy()
    tolerance_check(got, _ref64(cb(c), w, b).astype(np.float32), RTOL)


def test_fused_weight_above_bf16_max_stays_finite(dx):
    """A finite weight that rounds to inf in bf16 (3.4e38 > ~3.396e38) keeps a
    finite hi/mid/lo split (hi = its truncation), so the contraction matches the
    float64 product instead of turning into inf (dxr_common.h split8)."""
    B, D, H, W = 1, 64, 16, 16
    f1 = _t(dg.fmap(100, B, D, H, W) * np.float32(1e-3))
    f2 = _t(dg.fmap(101, B, D, H, W) * np.float32(1e-3))
    c = _t(dg.coords(102, B, H, W, "normal", 2.0))
    w = _t(dg.fmap(103, 1, 1, 32, 324)[0, 0] / np.float32(18.0))
    w[:, 7] = 3.4e38
    w[::2, 7] = -3.4e38
    cb = dx.CorrBlock(f1, f2)
    got = cb.lookup_conv1x1(c, w, None, relu=False).cpu().numpy()
    assert np.isfinite(got).all()
    tolerance_check(got, _ref64(cb(c), w, None, relu=False).astype(np.float32), RTOL)


def test_fused_far_and_nan_coords(dx):
    """Far coordinates give zero samples (bias only); a NaN coordinate makes that
    pixel's samples NaN, so its outputs are NaN exactly where the unfused path's are."""
    B, D, H, W = 1, 64, 16, 24
    f1, f2 = _t(dg.fmap(90, B, D, H, W)), _t(dg.fmap(91, B, D, H, W))
    c = dg.coords(92, B, H, W, "normal", 2.0)
    c[0, 0, 3, 5] = 1e6           # far
    c[0, 1, 7, 9] = np.nan        # non-finite
    c = _t(c)
    w = _t(dg.fmap(93, 1, 1, 256, 324)[0, 0] / np.float32(18.0))
    b = _t(dg.fmap(94, 1, 1, 1, 256)[0, 0, 0])
    cb = dx.CorrBlock(f1, f2)
    corr = cb(c)
    got = cb.lookup_conv1x1(c, w, b, relu=False).cpu().numpy()
    ref = _ref64(corr, w, b, relu=False).astype(np.float32)
    tolerance_check(got, ref, RTOL)       # identical NaN pattern, finite entries within 1e-4
    np.testing.assert_allclose(got[0, :, 3, 5], b.cpu().numpy(), rtol=0, atol=1e-6)
    assert np.isnan(got[0, :, 7, 9]).all()
