"""Drop-in for the reference's pybind module ``alt_cuda_corr``.

Mirrors alt_cuda_corr/correlation.cpp:23-54: ``forward(fmap1, fmap2, coords,
radius) -> [corr]`` and ``backward(fmap1, fmap2, coords, corr_grad, radius) ->
[fmap1_grad, fmap2_grad, coords_grad]`` with fmap1 ``[B, H1, W1, C]``, fmap2 ``[B, H2, W2, C]``,
coords ``[B, N, H1, W1, 2]`` (all float32, contiguous, on the device) and
``corr`` ``[B, N, (2r+1)^2, H1, W1]``, channel ``iy + (2r+1)*ix``.  Argument
errors raise ``RuntimeError`` like the reference's ``TORCH_CHECK``
(correlation.cpp:19-21).  Unlike the reference, the kernel runs on torch's
current stream rather than the legacy default stream (correlation_kernel.cu:278).
"""
from __future__ import annotations

import torch

from . import _native as nat

__all__ = ["forward", "backward"]


def _check_input(t: torch.Tensor, name: str) -> None:
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (the reference kernel is float-only)")


def forward(fmap1: torch.Tensor, fmap2: torch.Tensor, coords: torch.Tensor, radius: int):
    """alt_cuda_corr.forward (correlation.cpp:23-33, correlation_kernel.cu:260-286)."""
    for t, n in ((fmap1, "fmap1"), (fmap2, "fmap2"), (coords, "coords")):
        _check_input(t, n)
    if fmap1.dim() != 4 or fmap2.dim() != 4 or coords.dim() != 5 or coords.shape[-1] != 2:
        raise RuntimeError("expected fmap1 [B,H1,W1,C], fmap2 [B,H2,W2,C], coords [B,N,H1,W1,2]")
    B, H1, W1, C = (int(s) for s in fmap1.shape)
    B2, H2, W2, C2 = (int(s) for s in fmap2.shape)
    Bc, N, Hc, Wc, _ = (int(s) for s in coords.shape)
    if B2 != B or C2 != C or Bc != B or (Hc, Wc) != (H1, W1):
        raise RuntimeError("fmap1 / fmap2 / coords shapes are inconsistent")
    rd = 2 * int(radius) + 1
    corr = torch.empty((B, N, rd * rd, H1, W1), dtype=torch.float32, device=fmap1.device)
    lib = nat.load()
    with torch.cuda.device(fmap1.device):
        st = lib.dxr_alt_corr_forward(fmap1.data_ptr(), fmap2.data_ptr(), coords.data_ptr(),
                                      corr.data_ptr(), B, H1, W1, H2, W2, C, N, int(radius),
                                      nat.stream_of(fmap1))
    nat.check(st, "alt_cuda_corr.forward (dxr_alt_corr_forward)")
    return [corr]


def backward(fmap1: torch.Tensor, fmap2: torch.Tensor, coords: torch.Tensor,
             corr_grad: torch.Tensor, radius: int):
    """alt_cuda_corr.backward (correlation.cpp:36-48, correlation_kernel.cu:122-256,288-320).

    Returns ``[fmap1_grad, fmap2_grad, coords_grad]``; coords_grad is zero, as in
    the reference (correlation_kernel.cu:307).  fmap2_grad is accumulated with
    atomics, so its last bits depend on the summation order (also as in the
    reference).  The reference's core/corr.py never calls it (AlternateCorrBlock
    wraps no autograd.Function); this is the FFI surface only.
    """
    for t, n in ((fmap1, "fmap1"), (fmap2, "fmap2"), (coords, "coords"),
                 (corr_grad, "corr_grad")):
        _check_input(t, n)
    if fmap1.dim() != 4 or fmap2.dim() != 4 or coords.dim() != 5 or coords.shape[-1] != 2:
        raise RuntimeError("expected fmap1 [B,H1,W1,C], fmap2 [B,H2,W2,C], coords [B,N,H1,W1,2]")
    B, H1, W1, C = (int(s) for s in fmap1.shape)
    B2, H2, W2, C2 = (int(s) for s in fmap2.shape)
    Bc, N, Hc, Wc, _ = (int(s) for s in coords.shape)
    if B2 != B or C2 != C or Bc != B or (Hc, Wc) != (H1, W1):
        raise RuntimeError("fmap1 / fmap2 / coords shapes are inconsistent")
    rd = 2 * int(radius) + 1
    if tuple(corr_grad.shape) != (B, N, rd * rd, H1, W1):
        raise RuntimeError(f"corr_grad must be [B, N, (2r+1)^2, H1, W1] = "
                           f"{[B, N, rd * rd, H1, W1]}, got {list(corr_grad.shape)}")
    fmap1_grad = torch.empty_like(fmap1)
    fmap2_grad = torch.empty_like(fmap2)
    coords_grad = torch.zeros_like(coords)
    lib = nat.load()
    with torch.cuda.device(fmap1.device):
        st = lib.dxr_alt_corr_backward(fmap1.data_ptr(), fmap2.data_ptr(), coords.data_ptr(),
                                       corr_grad.data_ptr(), fmap1_grad.data_ptr(),
                                       fmap2_grad.data_ptr(), B, H1, W1, H2, W2, C, N,
                                       int(radius), nat.stream_of(fmap1))
    nat.check(st, "alt_cuda_corr.backward (dxr_alt_corr_backward)")
    return [fmap1_grad, fmap2_grad, coords_grad]
