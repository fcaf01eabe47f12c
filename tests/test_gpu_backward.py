"""GPU parity of the fused fmap-gradient backward (``dxr_fmap_grads``).

The reference trains through matmul -> / sqrt(D) -> avg_pool2d -> grid_sample
(train.py:175-178, core/corr.py:13-27,52-60).  Given a gradient pyramid G (what
the lookups' backwards leave), d fmap1 = F2 dV^T and d fmap2 = F1 dV with dV the
pooling-chain fold of G / sqrt(D).  The check: ``dxr_fmap_grads`` (dV folded
inside the MFMA operand loads, never stored) against ``dxr_pyramid_backward``
(dV in HBM, itself pinned by the reference autograd goldens) followed by float64
GEMMs, and against the same dV through float32 rocBLAS (the round-2 path): the
fused GEMMs must be at least as close to float64 as float32 BLAS is (f32 class),
and within 1e-5 of max|grad|.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import datagen as dg

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def dx():
    import dexiraft_amd
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dexiraft_amd.load_native()
    return dexiraft_amd


def _nat():
    from dexiraft_amd import _native
    return _native


def _grad_pyramid(nat, B, H, W, L, seed, nan_at=None):
    """A paged gradient pyramid with N(0, 1) cells on every level (zero padding)."""
    lib = nat.load()
    numel = lib.dxr_pyramid_numel(B, H, W, L)
    gp = torch.zeros(numel, dtype=torch.float32, device=DEV)
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    h, w = H, W
    for lvl in range(L):
        if lvl:
            h, w = h // 2, w // 2
        ref = torch.randn((B * H * W, h, w), generator=g, device=DEV)
        if lvl == 0 and nan_at is not None:
            ref[nan_at] = float("nan")
        st = lib.dxr_pyramid_pack(ref.data_ptr(), B, H, W, L, lvl, gp.data_ptr(), nat.DXR_F32,
                                  nat.stream_of(ref))
        nat.check(st, "pack")
    return gp


def _fused(nat, gp, f1, f2, L, div, want=(True, True)):
    lib = nat.load()
    B, D, H, W = f1.shape
    wsb = lib.dxr_fmap_grads_workspace_bytes(B, D, H, W, L)
    assert wsb > 0
    ws = torch.empty(wsb, dtype=torch.uint8, device=DEV)
    df1 = torch.full_like(f1, float("nan")) if want[0] else None
    df2 = torch.full_like(f2, float("nan")) if want[1] else None
    st = lib.dxr_fmap_grads(gp.data_ptr(), nat.DXR_F32, f1.data_ptr(), f2.data_ptr(), B, D, H, W,
                            L, div, nat.ptr(df1), nat.ptr(df2), ws.data_ptr(), wsb,
                            nat.stream_of(f1))
    nat.check(st, "dxr_fmap_grads")
    return df1, df2


def _volume_grad(nat, gp, B, H, W, L, div):
    lib = nat.load()
    dv = torch.empty((B, H * W, H * W), dtype=torch.float32, device=DEV)
    st = lib.dxr_pyramid_backward(gp.data_ptr(), nat.DXR_F32, B, H, W, L, div, dv.data_ptr(),
                                  nat.stream_of(dv))
    nat.check(st, "dxr_pyramid_backward")
    return dv


SHAPES = [
    (1, 256, 55, 128, 4),   # Sintel (C2): K split in 4 chunks
    (1, 256, 46, 62, 4),    # Chairs (C1): ragged tiles and query block
    (2, 64, 23, 37, 3),
    (1, 32, 9, 17, 1),      # one level, one ragged tile
    (3, 96, 16, 16, 2),
    (1, 512, 20, 30, 4),    # two 256-channel slabs
    (6, 256, 55, 128, 4),   # 330 n blocks: no K split
]


@pytest.mark.parametrize("shape", SHAPES)
def test_fmap_grads_match_volume_gradient_gemms(dx, shape):
    nat = _nat()
    B, D, H, W, L = shape
    f1 = torch.from_numpy(dg.fmap(900 + D, B, D, H, W, "fnet")).to(DEV)
    f2 = torch.from_numpy(dg.fmap(901 + D, B, D, H, W, "fnet")).to(DEV)
    div = float(np.sqrt(np.float32(D), dtype=np.float32))
    gp = _grad_pyramid(nat, B, H, W, L, seed=B * 1000 + H)
    g1, g2 = _fused(nat, gp, f1, f2, L, div)
    dv = _volume_grad(nat, gp, B, H, W, L, div)
    N = H * W
    r1 = torch.bmm(f2.reshape(B, D, N).double(), dv.double().transpose(1, 2)).reshape(B, D, H, W)
    r2 = torch.bmm(f1.reshape(B, D, N).double(), dv.double()).reshape(B, D, H, W)
    b1 = torch.bmm(f2.reshape(B, D, N), dv.transpose(1, 2)).reshape(B, D, H, W)
    b2 = torch.bmm(f1.reshape(B, D, N), dv).reshape(B, D, H, W)
    del dv
    for name, got, ref, blas in (("dfmap1", g1, r1, b1), ("dfmap2", g2, r2, b2)):
        assert torch.isfinite(got).all(), name
        scale = ref.abs().max().item()
        err = (got.double() - ref).abs().max().item()
        err_blas = (blas.double() - ref).abs().max().item()
        print(f"{shape} {name}: max|err| {err:.3e} (f32 BLAS {err_blas:.3e}) of max {scale:.3e}")
        assert err <= 1e-5 * scale
        assert err <= 2 * err_blas + 1e-7 * scale


def test_fmap_grads_deterministic_and_one_sided(dx):
    """Same inputs -> bit-identical gradients; a NULL output is skipped and the
    other is unchanged by it."""
    nat = _nat()
    B, D, H, W, L = 1, 128, 30, 44, 4
    f1 = torch.from_numpy(dg.fmap(911, B, D, H, W)).to(DEV)
    f2 = torch.from_numpy(dg.fmap(912, B, D, H, W)).to(DEV)
    gp = _grad_pyramid(nat, B, H, W, L, seed=913)
    a1, a2 = _fused(nat, gp, f1, f2, L, 11.3137)
    b1, b2 = _fused(nat, gp, f1, f2, L, 11.3137)
    assert torch.equal(a1, b1) and torch.equal(a2, b2)
    c1, none2 = _fused(nat, gp, f1, f2, L, 11.3137, want=(True, False))
    none1, c2 = _fused(nat, gp, f1, f2, L, 11.3137, want=(False, True))
    assert none1 is None and none2 is None
    assert torch.equal(a1, c1) and torch.equal(a2, c2)


def test_fmap_grads_propagate_nan_like_the_gemms(dx):
    """A NaN gradient cell poisons exactly the query's dfmap1 column and the
    target's dfmap2 column, as the dense GEMMs do."""
    nat = _nat()
    B, D, H, W, L = 1, 64, 24, 40, 4
    f1 = torch.from_numpy(dg.fmap(921, B, D, H, W)).to(DEV)
    f2 = torch.from_numpy(dg.fmap(922, B, D, H, W)).to(DEV)
    q, ty, tx = 37, 5, 17
    gp = _grad_pyramid(nat, B, H, W, L, seed=923, nan_at=(q, ty, tx))
    g1, g2 = _fused(nat, gp, f1, f2, L, 8.0)
    dv = _volume_grad(nat, gp, B, H, W, L, 8.0)
    r1 = torch.bmm(f2.reshape(B, D, -1), dv.transpose(1, 2)).reshape(B, D, H, W)
    r2 = torch.bmm(f1.reshape(B, D, -1), dv).reshape(B, D, H, W)
    assert torch.equal(torch.isnan(g1), torch.isnan(r1))
    assert torch.equal(torch.isnan(g2), torch.isnan(r2))
    assert torch.isnan(g1[0, :, q // W, q % W]).all() and torch.isnan(g2[0, :, ty, tx]).all()
    assert torch.isnan(g1).sum().item() == D and torch.isnan(g2).sum().item() == D


@pytest.mark.parametrize("D", [48, 64])
def test_corr_block_backward_fused_and_fallback_agree_with_torch(dx, D):
    """D = 64 takes dxr_fmap_grads, D = 48 the dV + rocBLAS fallback; both match
    torch autograd of the PyTorch restatement (tests/torch_ref.py)."""
    from torch_ref import TorchCorrBlock
    B, H, W = 1, 20, 36
    f1 = torch.from_numpy(dg.fmap(931, B, D, H, W, "fnet")).to(DEV)
    f2 = torch.from_numpy(dg.fmap(932, B, D, H, W, "fnet")).to(DEV)
    cs = [torch.from_numpy(dg.coords(933 + k, B, H, W, "normal", 3.0)).to(DEV) for k in range(4)]
    ws = [torch.from_numpy(dg.fmap(940 + k, B, 4 * 81, H, W)).to(DEV) for k in range(4)]

    def run(cls):
        a1, a2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
        cb = cls(a1, a2)
        sum((cb(c) * w).sum() for c, w in zip(cs, ws)).backward()
        return a1.grad, a2.grad

    for got, ref in zip(run(dx.CorrBlock), run(TorchCorrBlock)):
        assert (got - ref).abs().max().item() <= 1e-4 * ref.abs().max().item()


@pytest.mark.parametrize("r", [4, 3, 6, 8])
def test_lookup_backward_multi_equals_sequential_calls(dx, r):
    """dxr_corr_lookup_backward_multi over n coordinate sets == n single calls
    in the same order, bit for bit (what the deferred autograd path relies on)."""
    import ctypes
    nat = _nat()
    lib = nat.load()
    B, H, W, L = 2, 30, 44, 4
    n = 5
    K = L * (2 * r + 1) ** 2
    cs = [torch.from_numpy(dg.coords(960 + k, B, H, W, "normal", 3.0 + k)).to(DEV) for k in range(n)]
    gs = [torch.from_numpy(dg.fmap(970 + k, B, K, H, W)).to(DEV) for k in range(n)]
    numel = lib.dxr_pyramid_numel(B, H, W, L)
    seq = torch.zeros(numel, device=DEV)
    s = nat.stream_of(seq)
    for c, g in zip(cs, gs):
        assert lib.dxr_corr_lookup_backward(c.data_ptr(), g.data_ptr(), B, H, W, L, r,
                                            seq.data_ptr(), nat.DXR_F32, s) == 0
    multi = torch.zeros(numel, device=DEV)
    cp = (ctypes.c_void_p * n)(*[c.data_ptr() for c in cs])
    gp = (ctypes.c_void_p * n)(*[g.data_ptr() for g in gs])
    assert lib.dxr_corr_lookup_backward_multi(cp, gp, n, B, H, W, L, r, multi.data_ptr(),
                                              nat.DXR_F32, s) == 0
    torch.cuda.synchronize()
    assert seq.abs().sum().item() > 0
    assert torch.equal(seq, multi)


def test_deferred_lookup_backwards_flush_per_backward_pass(dx):
    """Six lookups (one batch of four, then the last two at the build's backward),
    backpropagated twice through a retained graph: the second pass starts from a
    fresh gradient pyramid, so the fmap gradients exactly double."""
    B, D, H, W = 1, 64, 24, 40
    f1 = torch.from_numpy(dg.fmap(981, B, D, H, W, "fnet")).to(DEV)
    f2 = torch.from_numpy(dg.fmap(982, B, D, H, W, "fnet")).to(DEV)
    cs = [torch.from_numpy(dg.coords(983 + k, B, H, W, "normal", 3.0)).to(DEV) for k in range(6)]
    ws = [torch.from_numpy(dg.fmap(990 + k, B, 4 * 81, H, W)).to(DEV) for k in range(6)]
    a1, a2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
    cb = dx.CorrBlock(a1, a2)
    loss = sum((cb(c) * w).sum() for c, w in zip(cs, ws))
    loss.backward(retain_graph=True)
    g1, g2 = a1.grad.clone(), a2.grad.clone()
    assert cb._gs.pending == [] and cb._gs.grad_pyr is None
    loss.backward()
    assert torch.equal(a1.grad, 2 * g1) and torch.equal(a2.grad, 2 * g2)


def test_partial_backward_pass_does_not_leak(dx):
    """A backward pass that stops before the build (autograd.grad with respect to
    the build's token) leaves pending lookup gradients behind; the
    end-of-pass callback drops them, so a following full pass gives exactly the
    gradients of a fresh block."""
    B, D, H, W = 1, 64, 24, 40
    f1 = torch.from_numpy(dg.fmap(1081, B, D, H, W, "fnet")).to(DEV)
    f2 = torch.from_numpy(dg.fmap(1082, B, D, H, W, "fnet")).to(DEV)
    cs = [torch.from_numpy(dg.coords(1083 + k, B, H, W, "normal", 3.0)).to(DEV) for k in range(3)]
    ws = [torch.from_numpy(dg.fmap(1090 + k, B, 4 * 81, H, W)).to(DEV) for k in range(3)]

    def run(partial):
        a1, a2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
        cb = dx.CorrBlock(a1, a2)
        loss = sum((cb(c) * w).sum() for c, w in zip(cs, ws))
        if partial:
            # a pass that runs the lookups' backward nodes but not the build's:
            # gradients with respect to the build's token only
            outs = [cb(c) for c in cs]
            l2 = sum((o * w).sum() for o, w in zip(outs, ws))
            torch.autograd.grad(l2, [cb._token], retain_graph=True, allow_unused=True)
            assert cb._gs.pending == [] and cb._gs.grad_pyr is None
        loss.backward()
        return a1.grad.clone(), a2.grad.clone()

    g1, g2 = run(False)
    p1, p2 = run(True)
    assert torch.equal(g1, p1) and torch.equal(g2, p2)


# ---------------------------------------------------------------------------
# Bounded form (dxr_fmap_grads_bounded): f16 pair operands scaled by a bound on
# |G|, three MFMA products; the six-product arithmetic for non-finite inputs.

def _bounded(nat, gp, f1, f2, L, div, slots, want=(True, True)):
    lib = nat.load()
    B, D, H, W = f1.shape
    wsb = lib.dxr_fmap_grads_bounded_workspace_bytes(B, D, H, W, L)
    ws = torch.empty(wsb, dtype=torch.uint8, device=DEV)
    df1 = torch.full_like(f1, float("nan")) if want[0] else None
    df2 = torch.full_like(f2, float("nan")) if want[1] else None
    st = lib.dxr_fmap_grads_bounded(gp.data_ptr(), nat.DXR_F32, f1.data_ptr(), f2.data_ptr(), B, D,
                                    H, W, L, div, slots.data_ptr(), slots.numel(), nat.ptr(df1),
                                    nat.ptr(df2), ws.data_ptr(), wsb, nat.stream_of(f1))
    nat.check(st, "dxr_fmap_grads_bounded")
    return df1, df2


def _slots(gp, factor=1.0, n=7):
    """n bound slots whose max is factor * max|gp| (the rest smaller)."""
    m = gp.abs().max().float() * factor
    return torch.stack([m * (0.5 ** k) for k in range(n)][::-1]).contiguous()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("factor", [1.0, 3000.0])
def test_fmap_grads_bounded_match_volume_gradient_gemms(dx, shape, factor):
    """f32 class: within 1e-5 of max|grad| of float64 and within 4x of what float32
    BLAS on the same dV gets, for a tight bound and a 3000x loose one."""
    nat = _nat()
    B, D, H, W, L = shape
    f1 = torch.from_numpy(dg.fmap(900 + D, B, D, H, W, "fnet")).to(DEV)
    f2 = torch.from_numpy(dg.fmap(901 + D, B, D, H, W, "fnet")).to(DEV)
    div = float(np.sqrt(np.float32(D), dtype=np.float32))
    gp = _grad_pyramid(nat, B, H, W, L, seed=B * 1000 + H)
    g1, g2 = _bounded(nat, gp, f1, f2, L, div, _slots(gp, factor))
    dv = _volume_grad(nat, gp, B, H, W, L, div)
    N = H * W
    r1 = torch.bmm(f2.reshape(B, D, N).double(), dv.double().transpose(1, 2)).reshape(B, D, H, W)
    r2 = torch.bmm(f1.reshape(B, D, N).double(), dv.double()).reshape(B, D, H, W)
    b1 = torch.bmm(f2.reshape(B, D, N), dv.transpose(1, 2)).reshape(B, D, H, W)
    b2 = torch.bmm(f1.reshape(B, D, N), dv).reshape(B, D, H, W)
    del dv
    for name, got, ref, blas in (("dfmap1", g1, r1, b1), ("dfmap2", g2, r2, b2)):
        assert torch.isfinite(got).all(), name
        scale = ref.abs().max().item()
        err = (got.double() - ref).abs().max().item()
        err_blas = (blas.double() - ref).abs().max().item()
        print(f"{shape} x{factor} {name}: max|err| {err:.3e} (f32 BLAS {err_blas:.3e}) of max {scale:.3e}")
        assert err <= 1e-5 * scale
        assert err <= 4 * err_blas + 1e-7 * scale


def test_fmap_grads_bounded_deterministic_and_one_sided(dx):
    nat = _nat()
    B, D, H, W, L = 1, 128, 30, 44, 4
    f1 = torch.from_numpy(dg.fmap(911, B, D, H, W)).to(DEV)
    f2 = torch.from_numpy(dg.fmap(912, B, D, H, W)).to(DEV)
    gp = _grad_pyramid(nat, B, H, W, L, seed=913)
    sl = _slots(gp)
    a1, a2 = _bounded(nat, gp, f1, f2, L, 11.3137, sl)
    b1, b2 = _bounded(nat, gp, f1, f2, L, 11.3137, sl)
    assert torch.equal(a1, b1) and torch.equal(a2, b2)
    c1, none2 = _bounded(nat, gp, f1, f2, L, 11.3137, sl, want=(True, False))
    none1, c2 = _bounded(nat, gp, f1, f2, L, 11.3137, sl, want=(False, True))
    assert none1 is None and none2 is None
    assert torch.equal(a1, c1) and torch.equal(a2, c2)


def test_fmap_grads_bounded_non_finite_takes_the_six_product_path(dx):
    """A NaN gradient cell makes the bound NaN: the whole call runs the
    six-product arithmetic, so the outputs equal dxr_fmap_grads' bit for bit
    (NaN exactly in the query's and the target's columns).  An inf in one pair's
    fmap sends only that pair there; the other pair keeps the f16 form."""
    nat = _nat()
    B, D, H, W, L = 1, 64, 24, 40, 4
    f1 = torch.from_numpy(dg.fmap(921, B, D, H, W)).to(DEV)
    f2 = torch.from_numpy(dg.fmap(922, B, D, H, W)).to(DEV)
    q, ty, tx = 37, 5, 17
    gp = _grad_pyramid(nat, B, H, W, L, seed=923, nan_at=(q, ty, tx))
    sl = torch.full((3,), float("nan"), device=DEV)
    g1, g2 = _bounded(nat, gp, f1, f2, L, 8.0, sl)
    u1, u2 = _fused(nat, gp, f1, f2, L, 8.0)
    assert torch.equal(torch.isnan(g1), torch.isnan(u1)) and torch.equal(torch.isnan(g2), torch.isnan(u2))
    assert torch.isnan(g1).sum().item() == D and torch.isnan(g2).sum().item() == D
    fin = ~torch.isnan(u1)
    assert torch.equal(g1[fin], u1[fin]) and torch.equal(g2[~torch.isnan(u2)], u2[~torch.isnan(u2)])

    B = 2
    f1 = torch.from_numpy(dg.fmap(924, B, D, H, W)).to(DEV)
    f2 = torch.from_numpy(dg.fmap(925, B, D, H, W)).to(DEV)
    f2[1, 3, 4, 5] = float("inf")
    gp = _grad_pyramid(nat, B, H, W, L, seed=926)
    g1, _ = _bounded(nat, gp, f1, f2, L, 8.0, _slots(gp), want=(True, False))
    u1, _ = _fused(nat, gp, f1, f2, L, 8.0, want=(True, False))
    assert torch.equal(torch.isnan(g1[1]), torch.isnan(u1[1]))
    assert torch.equal(torch.isinf(g1[1]), torch.isinf(u1[1]))
    same = torch.isfinite(u1[1])
    assert torch.equal(g1[1][same], u1[1][same])          # pair 1: six-product path
    assert torch.isfinite(g1[0]).all() and not torch.equal(g1[0], u1[0])   # pair 0: f16 pairs
    assert (g1[0] - u1[0]).abs().max().item() <= 1e-5 * u1[0].abs().max().item()


@pytest.mark.parametrize("r", [4, 3])
def test_lookup_backward_multi_bound_slots(dx, r):
    """The bound form writes the same gradient pyramid bit for bit, and its slots'
    maximum bounds max|G|: each workgroup adds 9 x its largest |grad_out| per set."""
    import ctypes
    nat = _nat()
    lib = nat.load()
    B, H, W, L = 2, 30, 44, 4
    n = 6
    K = L * (2 * r + 1) ** 2
    cs = [torch.from_numpy(dg.coords(1260 + k, B, H, W, "normal", 3.0 + k)).to(DEV) for k in range(n)]
    gs = [torch.from_numpy(dg.fmap(1270 + k, B, K, H, W)).to(DEV) for k in range(n)]
    numel = lib.dxr_pyramid_numel(B, H, W, L)
    nsl = lib.dxr_lookup_backward_bound_slots(B, H, W, L, r)
    ref = torch.zeros(numel, device=DEV)
    got = torch.zeros(numel + nsl, device=DEV)
    s = nat.stream_of(ref)
    for lo, hi in ((0, 4), (4, 6)):
        cp = (ctypes.c_void_p * (hi - lo))(*[c.data_ptr() for c in cs[lo:hi]])
        gp = (ctypes.c_void_p * (hi - lo))(*[g.data_ptr() for g in gs[lo:hi]])
        assert lib.dxr_corr_lookup_backward_multi(cp, gp, hi - lo, B, H, W, L, r, ref.data_ptr(),
                                                  nat.DXR_F32, s) == 0
        assert lib.dxr_corr_lookup_backward_multi_bound(cp, gp, hi - lo, B, H, W, L, r,
                                                        got.data_ptr(), nat.DXR_F32,
                                                        got.data_ptr() + 4 * numel, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(got[:numel], ref)
    m = ref.abs().max().item()
    bound = got[numel:].max().item()
    top = 9 * sum(g.abs().max().item() for g in gs)
    assert m > 0 and m <= bound <= top * (1 + 1e-6)
    assert (got[numel:] >= 0).all()


def test_corr_block_backward_bounded_path_matches_six_products_on_nan(dx):
    """Training through CorrBlock takes the bounded path; a NaN in one lookup's
    output gradient makes its bound NaN, so the step falls back to the six-product
    arithmetic: the fmap gradients equal dxr_fmap_grads' on the same gradient
    pyramid bit for bit (NaN pattern included)."""
    import ctypes
    nat = _nat()
    lib = nat.load()
    B, D, H, W, L, r = 1, 64, 24, 40, 4, 4
    f1 = torch.from_numpy(dg.fmap(1181, B, D, H, W, "fnet")).to(DEV)
    f2 = torch.from_numpy(dg.fmap(1182, B, D, H, W, "fnet")).to(DEV)
    cs = [torch.from_numpy(dg.coords(1183 + k, B, H, W, "normal", 3.0)).to(DEV) for k in range(3)]
    ws = [torch.from_numpy(dg.fmap(1190 + k, B, L * 81, H, W)).to(DEV) for k in range(3)]
    ws[1][0, 5, 7, 9] = float("nan")
    a1, a2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
    cb = dx.CorrBlock(a1, a2)
    sum((cb(c) * w).sum() for c, w in zip(cs, ws)).backward()
    # the same gradient pyramid by hand, then the unbounded (six-product) form
    numel = lib.dxr_pyramid_numel(B, H, W, L)
    gp = torch.zeros(numel, device=DEV)
    # autograd delivers the lookups' backwards last-created first
    cp = (ctypes.c_void_p * 3)(*[c.data_ptr() for c in cs[::-1]])
    gq = (ctypes.c_void_p * 3)(*[w.data_ptr() for w in ws[::-1]])
    assert lib.dxr_corr_lookup_backward_multi(cp, gq, 3, B, H, W, L, r, gp.data_ptr(), nat.DXR_F32,
                                              nat.stream_of(gp)) == 0
    u1, u2 = _fused(nat, gp, f1, f2, L, float(np.sqrt(np.float32(D))))
    for got, ref in ((a1.grad, u1), (a2.grad, u2)):
        assert torch.isnan(ref).any()
        assert torch.equal(torch.isnan(got), torch.isnan(ref))
        fin = ~torch.isnan(ref)
        assert torch.equal(got[fin], ref[fin])


@pytest.mark.parametrize("levels,radius,D", [(5, 4, 64), (6, 3, 32), (3, 2, 64)])
def test_corr_block_backward_other_levels_agree_with_torch(dx, levels, radius, D):
    """Lookup backwards on row-major levels (>= 4: one-cell column pass) and on
    fewer tiled levels, through CorrBlock (L > 4 takes the dV + GEMM fallback,
    L <= 4 the bounded fused GEMMs): against torch autograd of the PyTorch
    restatement (tests/torch_ref.py)."""
    from torch_ref import TorchCorrBlock
    B, H, W = 1, 36, 52
    f1 = torch.from_numpy(dg.fmap(1331, B, D, H, W, "fnet")).to(DEV)
    f2 = torch.from_numpy(dg.fmap(1332, B, D, H, W, "fnet")).to(DEV)
    cs = [torch.from_numpy(dg.coords(1333 + k, B, H, W, "normal", 3.0)).to(DEV) for k in range(5)]
    K = levels * (2 * radius + 1) ** 2
    ws = [torch.from_numpy(dg.fmap(1340 + k, B, K, H, W)).to(DEV) for k in range(5)]

    def run(cls):
        a1, a2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
        cb = cls(a1, a2, num_levels=levels, radius=radius)
        sum((cb(c) * w).sum() for c, w in zip(cs, ws)).backward()
        return a1.grad, a2.grad

    for got, ref in zip(run(dx.CorrBlock), run(TorchCorrBlock)):
        assert torch.isfinite(got).all()
        assert (got - ref).abs().max().item() <= 1e-4 * ref.abs().max().item()
