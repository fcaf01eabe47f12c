"""MI355X-native drop-in for the reference ``core/corr.py``.

``CorrBlock`` and ``AlternateCorrBlock`` keep the reference constructors and
``__call__(coords)`` signatures (core/corr.py:12-91), so ``core/raft*.py`` and
``core/update.py`` run unchanged on top of them.  All arithmetic happens in the
HIP kernels of ``libdexiraft_corr.so``; the Python side only validates,
allocates (from torch's caching allocator) and launches on torch's current
stream.  There is no CPU path: host tensors raise.

Training: with float32 fmaps that require grad (under grad mode), the block is
differentiable with respect to the fmaps, as the reference is through matmul /
avg_pool2d / grid_sample (train.py:175-178).  Each lookup's backward adds its
bilinear transpose into one gradient pyramid owned by the block
(``dxr_corr_lookup_backward_multi``, a few lookups per launch); the build's
backward runs once after all of them and takes the fmap gradients as two MFMA GEMMs that fold that pyramid down
the pooling chain in their operand loads (``dxr_fmap_grads``: no [B, N, N]
volume gradient).  Shapes it does not cover (D % 32 != 0, more than 4 levels)
form dV (``dxr_pyramid_backward``) and run two torch.bmm (rocBLAS).

Differences from the reference, all loud:
  * host (CPU) tensors raise ``RuntimeError`` instead of running on the CPU;
  * coords that require grad raise ``NotImplementedError`` (the reference
    detaches them, core/raft.py:170; no grid gradient is implemented), as do
    bfloat16 fmaps that require grad and AlternateCorrBlock inputs that require
    grad (the reference's alt_cuda_corr output carries no autograd graph).
"""
from __future__ import annotations

import ctypes
from functools import lru_cache

import numpy as np
import torch

from . import _native as nat

__all__ = ["CorrBlock", "AlternateCorrBlock"]


@lru_cache(maxsize=None)
def _sqrt_dim(dim: int) -> float:
    # torch.sqrt(torch.tensor(dim).float()) (core/corr.py:60,91): f32 IEEE sqrt.
    return float(np.sqrt(np.float32(dim), dtype=np.float32))


def _require_device(t: torch.Tensor, name: str) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor, got {type(t).__name__}")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{name} is on {t.device}; dexiraft_amd runs only on HIP devices (no CPU path)")


def _require_no_grad(*ts: torch.Tensor, what: str = "these inputs") -> None:
    if torch.is_grad_enabled() and any(t.requires_grad for t in ts):
        raise NotImplementedError(
            f"dexiraft_amd: no gradient is implemented for {what} (wrap the call in "
            "torch.no_grad() or detach the inputs)")


def _wants_grad(*ts: torch.Tensor) -> bool:
    return torch.is_grad_enabled() and any(t.requires_grad for t in ts)


def _volume_grads(ctx_needs, f1: torch.Tensor, f2: torch.Tensor, dv: torch.Tensor):
    """d/d fmap of corr = f1^T f2 given dV = d loss / d corr ([B, N, N], already
    divided by sqrt(D)): dF1 = F2 dV^T, dF2 = F1 dV (plain GEMMs, rocBLAS)."""
    B, D, H, W = f1.shape
    N = H * W
    df1 = df2 = None
    if ctx_needs[0]:
        df1 = torch.bmm(f2.reshape(B, D, N), dv.transpose(1, 2)).reshape(B, D, H, W)
    if ctx_needs[1]:
        df2 = torch.bmm(f1.reshape(B, D, N), dv).reshape(B, D, H, W)
    return df1, df2


class _GradState:
    """What the backward of a differentiable CorrBlock needs: its geometry and
    the gradient pyramid the lookups' backwards add into.  Held by the block
    and by the autograd nodes, it references neither the block nor the graph,
    so no reference cycle keeps the pyramid (``block._buf``) or the gradient
    pyramid alive after the step: both are freed by refcount."""

    __slots__ = ("geom", "num_levels", "radius", "device", "numel", "nslots", "grad_pyr",
                 "zero_ev", "pending", "end_hook")

    def __init__(self, geom, num_levels, radius, device, numel):
        self.geom, self.num_levels, self.radius = geom, num_levels, radius
        self.device, self.numel = device, numel
        B, _, H, W = geom
        # the lookup backwards' magnitude bound (one float per workgroup), kept
        # after the gradient pyramid in the same zero-filled buffer
        self.nslots = max(int(nat.load().dxr_lookup_backward_bound_slots(B, H, W, num_levels,
                                                                          radius)), 0)
        self.grad_pyr = None
        self.zero_ev = None   # the side-stream zero fill of grad_pyr, until a launch waits on it
        self.pending = []   # (coords, grad_out) of lookups whose backward is not applied yet
        self.end_hook = False   # an end-of-backward-pass callback is queued

    def flush(self):
        """Add the pending lookups' backwards into the gradient pyramid, in the
        order autograd delivered them, with one launch per _BW_SETS lookups
        (dxr_corr_lookup_backward_multi: bit-identical to one launch each)."""
        if not self.pending:
            return
        if self.grad_pyr is None:
            self.grad_pyr = torch.zeros(self.numel + self.nslots, dtype=torch.float32,
                                        device=self.device)
        if self.zero_ev is not None:
            torch.cuda.current_stream(self.device).wait_event(self.zero_ev)
            self.zero_ev = None
        B, D, H, W = self.geom
        n = len(self.pending)
        cs = (ctypes.c_void_p * n)(*[c.data_ptr() for c, _ in self.pending])
        gs = (ctypes.c_void_p * n)(*[g.data_ptr() for _, g in self.pending])
        lib = nat.load()
        try:
            with _Launch(self.device):
                st = lib.dxr_corr_lookup_backward_multi_bound(
                    cs, gs, n, B, H, W, self.num_levels, self.radius, self.grad_pyr.data_ptr(),
                    nat.DXR_F32, self.slots_ptr(), nat.stream_of(self.grad_pyr))
        finally:
            # never carry (coords, grad_out) entries into another flush, even if
            # the launch failed: a stale entry would be added twice
            self.pending = []
        nat.check(st, "CorrBlock lookup backward (dxr_corr_lookup_backward_multi_bound)")

    def prefill(self):
        """At a pass's first lookup backward: allocate the gradient pyramid and
        zero it on a side stream, so the fill (~270 MB at Sintel) overlaps the
        backward work that runs before the first flush instead of preceding it."""
        if self.grad_pyr is not None:
            return
        main = torch.cuda.current_stream(self.device)
        buf = torch.empty(self.numel + self.nslots, dtype=torch.float32, device=self.device)
        side = _side_stream(self.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            buf.zero_()
        buf.record_stream(side)
        ev = torch.cuda.Event()
        ev.record(side)
        self.grad_pyr, self.zero_ev = buf, ev

    def slots_ptr(self):
        """Device address of the bound slots behind the gradient pyramid."""
        return self.grad_pyr.data_ptr() + 4 * self.numel

    def reset(self):
        """Drop pending lookups and the partial gradient pyramid (a backward pass
        that ended before the build's backward ran, e.g. an exception part-way or
        ``autograd.grad`` with inputs that stop before the build)."""
        self.pending = []
        self.grad_pyr = None
        self.zero_ev = None
        # a pass that failed elsewhere never runs its queued _end: re-arm
        # (a second queued _end is harmless, it is idempotent)
        self.end_hook = False

    def arm_end_of_pass(self):
        """Queue (once per backward pass) a callback that runs when autograd's
        pass ends: whatever the build's backward did not consume by then belongs
        to a partial pass and is dropped, so it cannot leak into the next one."""
        if self.end_hook:
            return
        self.end_hook = True

        def _end():
            self.end_hook = False
            if self.pending or self.grad_pyr is not None:
                self.reset()
        torch.autograd.Variable._execution_engine.queue_callback(_end)


_SIDE_STREAMS: dict = {}


def _side_stream(device):
    """One side stream per device for the gradient pyramid's zero fill."""
    key = torch.device(device).index
    st = _SIDE_STREAMS.get(key)
    if st is None:
        st = _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return st


# Lookup backwards applied per launch: their window lines stay in L2 across the
# sets; the pending grad_out tensors ([B, L*(2r+1)^2, H, W] each) live until then.
# Round 6 (profiles/r06/experiments/r6y_r6z_backward_sets.jsonl, medians of six
# alternated runs): two per launch 1.299 / 1.335 ms per Sintel training step (cloned
# inputs + mul-sum loss / persistent leaves + vdot), four 1.353 / 1.340 — the eager
# step is host-paced, and earlier flushes start the GPU sooner; peak memory alike.
_BW_SETS = 2


class _BuildGrad(torch.autograd.Function):
    """Graph node of CorrBlock.__init__: returns a scalar token every lookup
    consumes, so autograd runs this backward once, after every lookup's
    backward has added into the gradient pyramid."""

    @staticmethod
    def forward(ctx, fmap1, fmap2, gs):
        ctx.gs = gs
        ctx.save_for_backward(fmap1, fmap2)
        return fmap1.new_zeros(())

    @staticmethod
    def backward(ctx, _gtoken):
        gs = ctx.gs
        try:
            gs.flush()
        except BaseException:
            gs.reset()
            raise
        # the state is consumed here: a later pass (retain_graph) arms its own
        # end-of-pass cleanup
        gs.end_hook = False
        if gs.grad_pyr is None:
            return None, None, None
        slots = gs.slots_ptr()
        gp, gs.grad_pyr = gs.grad_pyr, None
        f1, f2 = ctx.saved_tensors
        B, D, H, W = gs.geom
        lib = nat.load()
        wsb = lib.dxr_fmap_grads_bounded_workspace_bytes(B, D, H, W, gs.num_levels)
        if wsb >= 0:   # the fused MFMA backward: no [B, N, N] dV
            need1, need2 = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
            c1 = f1.contiguous() if need2 else None
            c2 = f2.contiguous() if need1 else None
            df1 = torch.empty((B, D, H, W), dtype=torch.float32, device=f1.device) if need1 else None
            df2 = torch.empty((B, D, H, W), dtype=torch.float32, device=f1.device) if need2 else None
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=f1.device)
            with _Launch(gs.device):
                # f16 pair GEMMs scaled by the lookups' bound (three MFMA products)
                st = lib.dxr_fmap_grads_bounded(gp.data_ptr(), nat.DXR_F32, nat.ptr(c1),
                                                nat.ptr(c2), B, D, H, W, gs.num_levels,
                                                _sqrt_dim(D), slots, gs.nslots, nat.ptr(df1),
                                                nat.ptr(df2), ws.data_ptr(), wsb,
                                                nat.stream_of(ws))
            nat.check(st, "CorrBlock backward (dxr_fmap_grads_bounded)")
            return df1, df2, None
        # D % 32 != 0 or more than 4 levels: dV, then two GEMMs
        dv = torch.empty((B, H * W, H * W), dtype=torch.float32, device=f1.device)
        with _Launch(gs.device):
            st = lib.dxr_pyramid_backward(gp.data_ptr(), nat.DXR_F32, B, H, W, gs.num_levels,
                                          _sqrt_dim(D), dv.data_ptr(), nat.stream_of(dv))
        nat.check(st, "CorrBlock backward (dxr_pyramid_backward)")
        del gp
        df1, df2 = _volume_grads(ctx.needs_input_grad, f1, f2, dv)
        return df1, df2, None


class _LookupGrad(torch.autograd.Function):
    """Graph node of CorrBlock.__call__ (differentiable in the pyramid only)."""

    @staticmethod
    def forward(ctx, token, coords, block):
        ctx.gs = block._gs
        ctx.save_for_backward(coords)
        return block._lookup(coords)

    @staticmethod
    def backward(ctx, gout):
        gs = ctx.gs
        (coords,) = ctx.saved_tensors
        gs.arm_end_of_pass()
        gs.prefill()
        gs.pending.append((coords, gout.contiguous().float()))
        if len(gs.pending) >= _BW_SETS:
            gs.flush()
        # no gradient for the token: autograd still runs the build's backward
        # after every lookup's (it waits on the edge, and materialises one zero)
        # without a fill per lookup and the adds that would sum them
        return None, None, None


class _VolumeGrad(torch.autograd.Function):
    """CorrBlock.corr with autograd: backward = dV / sqrt(D), two GEMMs."""

    @staticmethod
    def forward(ctx, fmap1, fmap2):
        ctx.save_for_backward(fmap1, fmap2)
        return CorrBlock._volume(fmap1, fmap2)

    @staticmethod
    def backward(ctx, gout):
        f1, f2 = ctx.saved_tensors
        B, D, H, W = f1.shape
        dv = gout.reshape(B, H * W, H * W).float() / _sqrt_dim(D)
        df1, df2 = _volume_grads(ctx.needs_input_grad, f1, f2, dv)
        return df1, df2


def _fmap_geometry(fmap1: torch.Tensor, fmap2: torch.Tensor) -> tuple[int, int, int, int]:
    _require_device(fmap1, "fmap1")
    _require_device(fmap2, "fmap2")
    if fmap1.dim() != 4 or fmap2.dim() != 4:
        raise RuntimeError(f"fmaps must be [B, D, H, W]; got {tuple(fmap1.shape)} and "
                           f"{tuple(fmap2.shape)}")
    if fmap1.shape != fmap2.shape:
        raise RuntimeError(f"fmap1 {tuple(fmap1.shape)} and fmap2 {tuple(fmap2.shape)} differ")
    if fmap1.device != fmap2.device:
        raise RuntimeError("fmap1 and fmap2 are on different devices")
    if fmap1.dtype != fmap2.dtype:
        raise RuntimeError(f"fmap dtypes differ: {fmap1.dtype} vs {fmap2.dtype}")
    B, D, H, W = (int(s) for s in fmap1.shape)
    return B, D, H, W


def _level_sizes(H: int, W: int, num_levels: int) -> list[tuple[int, int]]:
    sizes = [(H, W)]
    for _ in range(num_levels - 1):
        h, w = sizes[-1]
        if h < 2 or w < 2:
            # F.avg_pool2d raises here in the reference (core/corr.py:26).
            raise RuntimeError(
                f"pyramid level {len(sizes)} of a {H}x{W} fmap would be empty "
                f"(avg_pool2d of {h}x{w}); num_levels={num_levels} is too many")
        sizes.append((h // 2, w // 2))
    return sizes


def _channels_last(t: torch.Tensor) -> bool:
    """A channels-last (NHWC-strided) 4-D fmap that is not also NCHW-contiguous."""
    return t.is_contiguous(memory_format=torch.channels_last) and not t.is_contiguous()


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return nat.DXR_F32
    if t.dtype == torch.bfloat16:
        return nat.DXR_BF16
    raise RuntimeError(f"fmaps must be float32 or bfloat16, got {t.dtype}")


def _nchw(t: torch.Tensor) -> torch.Tensor:
    """NCHW-contiguous fmap (no autograd graph: callers use it only without grad).

    Channels-last fmaps (encoders emitting NHWC) go through
    one native tiled transpose (``dxr_transpose``); other layouts through
    ``.contiguous()`` (a no-op for the reference's own NCHW fmaps).
    """
    if not _channels_last(t):
        return t.contiguous()
    B, D, H, W = (int(s) for s in t.shape)
    out = torch.empty((B, D, H, W), dtype=t.dtype, device=t.device)
    with _Launch(t.device):
        st = nat.load().dxr_transpose(t.data_ptr(), out.data_ptr(), _dtype_code(t), B, H * W, D,
                                      nat.stream_of(t))
    nat.check(st, "NHWC -> NCHW fmap (dxr_transpose)")
    return out


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    """``t.permute(0, 2, 3, 1).contiguous()`` (core/corr.py:82-83): a free view of a
    channels-last fmap, one native tiled transpose (``dxr_transpose``) otherwise."""
    if _channels_last(t):
        return t.permute(0, 2, 3, 1)
    t = t.contiguous()
    B, D, H, W = (int(s) for s in t.shape)
    out = torch.empty((B, H, W, D), dtype=t.dtype, device=t.device)
    with _Launch(t.device):
        st = nat.load().dxr_transpose(t.data_ptr(), out.data_ptr(), _dtype_code(t), B, D, H * W,
                                      nat.stream_of(t))
    nat.check(st, "NCHW -> NHWC fmap (dxr_transpose)")
    return out


def _pool_nhwc(t: torch.Tensor) -> torch.Tensor:
    """F.avg_pool2d(x, 2, stride=2) of a channels-last fmap held as [B, H, W, C]."""
    B, H, W, C = (int(s) for s in t.shape)
    out = torch.empty((B, H // 2, W // 2, C), dtype=t.dtype, device=t.device)
    with _Launch(t.device):
        st = nat.load().dxr_avg_pool2x2_nhwc(t.data_ptr(), out.data_ptr(), B, H, W, C,
                                             nat.stream_of(t))
    nat.check(st, "AlternateCorrBlock pooling (dxr_avg_pool2x2_nhwc)")
    return out


class _Launch:
    """Runs a native call with fmap's device current (multi-GPU processes)."""

    def __init__(self, device: torch.device):
        self.device = device
        self._ctx = None

    def __enter__(self):
        # torch._C._cuda_getDevice: torch.cuda.current_device() without its
        # lazy-init check (a block exists only on an initialised device)
        if self.device.index is not None and self.device.index != torch._C._cuda_getDevice():
            self._ctx = torch.cuda.device(self.device)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self._ctx is not None:
            self._ctx.__exit__(*exc)
        return False


def _check_coords(coords: torch.Tensor, B: int, H: int, W: int, device: torch.device) -> torch.Tensor:
    _require_device(coords, "coords")
    if coords.dim() != 4 or tuple(coords.shape) != (B, 2, H, W):
        raise RuntimeError(f"coords must be [B, 2, H, W] = {(B, 2, H, W)}, got {tuple(coords.shape)}")
    if coords.device != device:
        raise RuntimeError(f"coords on {coords.device}, correlation block on {device}")
    if coords.dtype != torch.float32:
        coords = coords.float()
    return coords.contiguous()


_PACKED_CACHE: dict = {}


def _packed_weight(weight: torch.Tensor, device: torch.device) -> torch.Tensor:
    """A [Cout, Cin] conv weight in the fused kernel's operand layout
    (dxr_conv1x1_pack_weight), cached per (storage, version, shape) so the 12 GRU
    iterations pack it once."""
    key = (weight.data_ptr(), weight._version, tuple(weight.shape), weight.dtype, str(device))
    hit = _PACKED_CACHE.get(key)
    if hit is not None:
        return hit[1]
    cout, cin = (int(s) for s in weight.shape)
    w = weight.detach().float().contiguous()
    lib = nat.load()
    planes = torch.empty(lib.dxr_conv1x1_packed_bytes(cout, cin), dtype=torch.uint8, device=device)
    with _Launch(device):
        st = lib.dxr_conv1x1_pack_weight(w.data_ptr(), cout, cin, planes.data_ptr(),
                                          nat.stream_of(w))
    nat.check(st, "conv1x1 weight packing (dxr_conv1x1_pack_weight)")
    if len(_PACKED_CACHE) > 16:
        _PACKED_CACHE.clear()
    _PACKED_CACHE[key] = (weight, planes)   # keeps the weight alive: its pointer stays unique
    return planes


class CorrBlock:
    """All-pairs correlation pyramid + radius-r lookup (reference core/corr.py:12-60).

    ``CorrBlock(fmap1, fmap2, num_levels=4, radius=4)`` builds the pyramid of
    ``fmap1^T fmap2 / sqrt(D)`` with its avg-pool levels fused into the GEMM's
    epilogue (``dxr_corr_pyramid_build_ws``, with a workspace from torch's
    caching allocator); each ``__call__(coords)`` is one lookup launch
    (``dxr_corr_lookup``) returning a new contiguous float32
    ``[B, num_levels*(2r+1)^2, H, W]`` tensor in the reference's channel order.

    fp32 fmaps (the reference's dtype, core/raft.py:139-142) compute in f32
    class: a split pass scales every pixel's channel vector by a power of two
    and stores it as an f16 pair hi + lo, then the LDS-DMA build runs three f16
    MFMA products per f32 product (lo*hi, hi*lo, hi*hi) into one f32
    accumulator and undoes the scales exactly in the epilogue.  A workgroup
    whose sums are not finite (inf/NaN operands) recomputes its pages on the
    exact-f32 MFMA.  The pyramid is stored in f32; bf16 fmaps build a bf16
    pyramid on bf16 MFMA.  It lives in one paged buffer (``_buf``);
    ``corr_pyramid`` gives the reference-layout levels on demand.
    """

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        self.num_levels = num_levels
        self.radius = radius
        B, D, H, W = _fmap_geometry(fmap1, fmap2)
        self._token = None
        self._gs = None
        if not isinstance(num_levels, int) or num_levels < 1:
            raise ValueError(f"num_levels must be a positive int, got {num_levels!r}")
        if not isinstance(radius, int) or radius < 0:
            raise ValueError(f"radius must be a non-negative int, got {radius!r}")
        sizes = _level_sizes(H, W, num_levels)
        if fmap1.dtype == torch.float32:
            in_dt, pyr_dt, pyr_torch = nat.DXR_F32, nat.DXR_F32, torch.float32
        elif fmap1.dtype == torch.bfloat16:
            in_dt, pyr_dt, pyr_torch = nat.DXR_BF16, nat.DXR_BF16, torch.bfloat16
        else:
            raise RuntimeError(f"fmaps must be float32 or bfloat16, got {fmap1.dtype}")
        if pyr_dt != nat.DXR_F32:
            _require_no_grad(fmap1, fmap2, what="bfloat16 fmaps")
        self._geom = (B, D, H, W)
        self._pyr_dt = pyr_dt
        self._device = fmap1.device
        lib = nat.load()
        numel = lib.dxr_pyramid_numel(B, H, W, num_levels)
        self._buf = torch.empty(numel, dtype=pyr_torch, device=fmap1.device)
        grad = _wants_grad(fmap1, fmap2)
        self._in_dt = in_dt
        f1, f2, st = self._launch_build(fmap1, fmap2, grad)
        nat.check(st, "CorrBlock build (dxr_corr_pyramid_build_ws)")
        self._level_sizes = sizes
        self._ref_pyramid = None
        if grad:
            self._gs = _GradState(self._geom, num_levels, radius, self._device, numel)
            self._token = _BuildGrad.apply(f1, f2, self._gs)

    def _launch_build(self, fmap1, fmap2, grad=False):
        """One build launch into this block's pyramid buffer.  Returns the operand
        tensors the kernel read and the status.

        f32 fmaps get a workspace from torch's caching allocator (freed when the
        build's stream work is done) for the pre-split build
        (``dxr_corr_pyramid_build_ws``: operands scaled and split into f16 pairs
        once, then moved by LDS-DMA)."""
        B, D, H, W = self._geom
        lib = nat.load()
        nbytes = max(lib.dxr_build_workspace_bytes(self._in_dt, B, D, H, W), 0)

        def launch(f1, f2, layout, with_ws=True):
            ws = torch.empty(nbytes, dtype=torch.uint8, device=self._device) \
                if with_ws and nbytes > 0 else None
            with _Launch(self._device):
                return lib.dxr_corr_pyramid_build_ws(
                    f1.data_ptr(), f2.data_ptr(), self._in_dt, layout, B, D, H, W,
                    self.num_levels, _sqrt_dim(D), self._buf.data_ptr(), self._pyr_dt,
                    nat.DXR_BUILD_AUTO, nat.ptr(ws), nbytes if ws is not None else 0,
                    nat.stream_of(f1))

        st = nat.DXR_EUNSUPPORTED
        if not grad and _channels_last(fmap1) and _channels_last(fmap2):
            # channels-last fmaps: read in place by the
            # build's NHWC operand loads (f32: the pre-split pass, into the
            # workspace; bf16: the DMA build reads the rows directly and needs no
            # workspace), no layout pass
            f1, f2 = fmap1, fmap2
            st = launch(f1, f2, nat.DXR_NHWC, with_ws=self._in_dt != nat.DXR_BF16)
        if st == nat.DXR_EUNSUPPORTED:
            if grad:
                f1, f2 = fmap1.contiguous(), fmap2.contiguous()   # tracked by autograd
            else:
                f1, f2 = _nchw(fmap1), _nchw(fmap2)
            st = launch(f1, f2, nat.DXR_NCHW)
        return f1, f2, st

    @property
    def corr_pyramid(self):
        """Reference-layout levels ``[B*H*W, 1, H_l, W_l]`` (core/corr.py:16-27).

        The native pyramid is stored paged (one contiguous page per build
        workgroup, include/dexiraft_corr.h); this list is materialised on first
        access by ``dxr_pyramid_unpack`` and cached.  Values are float32 (bf16
        pyramids are widened).  The lookup never needs it.
        """
        if self._ref_pyramid is None:
            B, D, H, W = self._geom
            lib = nat.load()
            levels = []
            with _Launch(self._device):
                for lvl, (h, w) in enumerate(self._level_sizes):
                    t = torch.empty((B * H * W, 1, h, w), dtype=torch.float32, device=self._device)
                    st = lib.dxr_pyramid_unpack(self._buf.data_ptr(), self._pyr_dt, B, H, W,
                                                self.num_levels, lvl, t.data_ptr(),
                                                nat.stream_of(t))
                    nat.check(st, "CorrBlock.corr_pyramid (dxr_pyramid_unpack)")
                    levels.append(t)
            self._ref_pyramid = levels
        return self._ref_pyramid

    def __call__(self, coords):
        B, D, H, W = self._geom
        _require_no_grad(coords, what="coords (the reference detaches them, core/raft.py:170)")
        c = _check_coords(coords, B, H, W, self._device)
        if self._token is not None and torch.is_grad_enabled():
            return _LookupGrad.apply(self._token, c, self)
        return self._lookup(c)

    def _lookup(self, c):
        B, D, H, W = self._geom
        rd = 2 * self.radius + 1
        out = torch.empty((B, self.num_levels * rd * rd, H, W), dtype=torch.float32,
                          device=self._device)
        lib = nat.load()
        with _Launch(self._device):
            st = lib.dxr_corr_lookup(self._buf.data_ptr(), self._pyr_dt, B, H, W,
                                     self.num_levels, self.radius, c.data_ptr(),
                                     out.data_ptr(), nat.stream_of(c))
        nat.check(st, "CorrBlock lookup (dxr_corr_lookup)")
        return out

    def lookup_conv1x1(self, coords, weight, bias=None, relu=True):
        """Lookup fused with the motion encoder's first 1x1 convolution:
        ``F.relu(F.conv2d(self(coords), weight, bias))`` in one launch
        (``dxr_corr_lookup_conv1x1``).

        Replaces ``corr = corr_fn(coords1)`` (core/raft.py:172) followed by
        ``cor = F.relu(self.convc1(corr))`` in BasicMotionEncoder.forward
        (core/update.py:90; SmallMotionEncoder :71): pass ``convc1.weight`` and
        ``convc1.bias``.  Returns a new contiguous float32 ``[B, Cout, H, W]``.
        The samples are bit-identical to ``__call__``'s; the contraction runs in
        f32 class on the matrix cores.  Inference only (raises under grad for
        inputs that require grad).  Supported: radius 3/4, num_levels <= 4,
        Cout a multiple of 32 (the reference's 256 and 96).
        """
        B, D, H, W = self._geom
        _require_no_grad(coords, weight, *(() if bias is None else (bias,)),
                         what="CorrBlock.lookup_conv1x1 (inference fusion)")
        if self._token is not None and torch.is_grad_enabled():
            raise NotImplementedError("CorrBlock.lookup_conv1x1 is inference-only; call the "
                                      "block and convc1 separately to train through them")
        c = _check_coords(coords, B, H, W, self._device)
        rd = 2 * self.radius + 1
        cin = self.num_levels * rd * rd
        _require_device(weight, "weight")
        if weight.dim() == 4 and tuple(weight.shape[2:]) == (1, 1):
            weight = weight.reshape(weight.shape[0], weight.shape[1])
        if weight.dim() != 2 or int(weight.shape[1]) != cin:
            raise RuntimeError(f"weight must be [Cout, {cin}, 1, 1] (or [Cout, {cin}]), "
                               f"got {tuple(weight.shape)}")
        cout = int(weight.shape[0])
        if bias is not None:
            _require_device(bias, "bias")
            if tuple(bias.shape) != (cout,):
                raise RuntimeError(f"bias must be [{cout}], got {tuple(bias.shape)}")
            bias = bias.detach().float().contiguous()
        planes = _packed_weight(weight, self._device)
        out = torch.empty((B, cout, H, W), dtype=torch.float32, device=self._device)
        lib = nat.load()
        with _Launch(self._device):
            st = lib.dxr_corr_lookup_conv1x1(self._buf.data_ptr(), self._pyr_dt, B, H, W,
                                             self.num_levels, self.radius, c.data_ptr(),
                                             planes.data_ptr(), nat.ptr(bias), cout, int(bool(relu)),
                                             out.data_ptr(), nat.stream_of(c))
        nat.check(st, "CorrBlock.lookup_conv1x1 (dxr_corr_lookup_conv1x1)")
        return out

    @staticmethod
    def corr(fmap1, fmap2):
        """``[B, H, W, 1, H, W]`` volume ``fmap1^T fmap2 / sqrt(D)`` (core/corr.py:52-60);
        differentiable in the fmaps under grad mode."""
        _fmap_geometry(fmap1, fmap2)
        if _wants_grad(fmap1, fmap2) and fmap1.dtype == torch.float32:
            return _VolumeGrad.apply(fmap1.contiguous(), fmap2.contiguous())
        return CorrBlock._volume(fmap1, fmap2)

    @staticmethod
    def _volume(fmap1, fmap2):
        B, D, H, W = _fmap_geometry(fmap1, fmap2)
        if fmap1.dtype != torch.float32:
            raise RuntimeError(f"CorrBlock.corr expects float32 fmaps, got {fmap1.dtype}")
        out = torch.empty((B, H, W, 1, H, W), dtype=torch.float32, device=fmap1.device)
        f1, f2 = _nchw(fmap1), _nchw(fmap2)
        lib = nat.load()
        with _Launch(fmap1.device):
            st = lib.dxr_corr_volume(f1.data_ptr(), f2.data_ptr(), nat.DXR_F32, B, D, H, W,
                                     _sqrt_dim(D), out.data_ptr(), nat.stream_of(f1))
        nat.check(st, "CorrBlock.corr (dxr_corr_volume)")
        return out


class AlternateCorrBlock:
    """On-the-fly correlation lookup (reference core/corr.py:63-91 + alt_cuda_corr).

    Memory is O(H*W*D) at the fine levels instead of O((H*W)^2): only pooled fmaps
    are kept and each ``__call__`` computes the (2r+2)^2 window dot products of
    those levels in one launch (``dxr_alt_corr_lookup_levels_ws``), divided by
    sqrt(D).  Round 6: on large maps (``COARSE_MIN_QUERIES``) the coarse levels —
    from the first level of at most ``COARSE_LEVEL_MAX_CELLS`` cells on, within
    ``COARSE_VOLUME_MAX_BYTES`` — are computed once per block as whole volumes of the
    same dot products (``dxr_alt_coarse_volumes``, one tiled GEMM per level) and read
    by ``dxr_alt_volume_lookup``: an on-the-fly lookup pays each level's box GEMMs
    again on every call (~15-26 us per coarse level at 1080p), while a coarse
    level's whole volume costs about one or two calls (1080p: levels 2-3).
    With finite operands in the f16 pair's range the outputs are the all-on-the-
    fly form's bit for bit (``coarse_first_level`` None: no volumes).  As in the
    reference, the constructor pools ``num_levels`` times, so fmaps smaller than
    2^num_levels in either dimension raise (core/corr.py:69-71).
    """

    # Which levels are precomputed (round 6, bench.py --block alt, profiles/r06/experiments/
    # r6n_*): at 1080p (32,640 queries) levels 2-3 (2,040 + 510 cells) as volumes take the
    # lookup from 164.1 to 127.2 us for ~200 us per block (tiled GEMM: level 2 149 us, level 3
    # 42 us): 498.9 -> 568.0 pairs/s (+13.9 %; level 3 alone 536.8); at Sintel (7,040
    # queries) the on-the-fly coarse levels cost ~2-4 us per lookup and volumes lose 3-4 %.
    COARSE_LEVEL_MAX_CELLS = 2048          # a level of at most this many cells is precomputed
    COARSE_MIN_QUERIES = 16384             # on maps of at least this many query pixels
    COARSE_VOLUME_MAX_BYTES = 1 << 30      # and all precomputed volumes fit in this
    # The volume GEMM's LDS-DMA form on pre-split f16 pair planes (dxr_alt_coarse_volumes_ws):
    # bit-identical, 6 % faster isolated, but 1.2 % slower in the 1080p step (r6u: 563 vs 570
    # pairs/s, two rounds each on one box), so off.
    COARSE_VOLUME_PLANES = False

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        self.num_levels = num_levels
        self.radius = radius
        B, D, H, W = _fmap_geometry(fmap1, fmap2)
        _require_no_grad(fmap1, fmap2, what="AlternateCorrBlock (the reference's alt_cuda_corr "
                                            "output carries no autograd graph, core/corr.py:85-88)")
        if fmap1.dtype == torch.bfloat16:
            # The reference computes in float32 (core/raft.py:139-142 casts the
            # fmaps; alt_cuda_corr is float-only): bf16 encoder outputs are widened
            # exactly, keeping their memory format (channels-last stays a free view).
            fmap1, fmap2 = fmap1.float(), fmap2.float()
        elif fmap1.dtype != torch.float32:
            raise RuntimeError(f"AlternateCorrBlock expects float32 or bfloat16 fmaps, got "
                               f"{fmap1.dtype}")
        if not isinstance(num_levels, int) or num_levels < 1:
            raise ValueError(f"num_levels must be a positive int, got {num_levels!r}")
        if not isinstance(radius, int) or radius < 0:
            raise ValueError(f"radius must be a non-negative int, got {radius!r}")
        _level_sizes(H, W, num_levels + 1)  # the reference pools num_levels times
        self._geom = (B, D, H, W)
        self._device = fmap1.device
        # NHWC operands (core/corr.py:82-83 permutes on every call; here once per
        # block): a free view of channels-last fmaps, one tiled transpose otherwise.
        # Only full-res fmap1 and the pooled fmap2 levels are used (core/corr.py:82-83),
        # so only those are pooled; ``pyramid`` materialises the rest on demand.
        self._fmaps = (fmap1, fmap2)
        self._pyramid = None
        self._f1_nhwc = _nhwc(fmap1)
        self._f2_nhwc = [_nhwc(fmap2)]
        for _ in range(1, num_levels):
            self._f2_nhwc.append(_pool_nhwc(self._f2_nhwc[-1]))
        self._f2_ptrs = (ctypes.c_void_p * num_levels)(*[t.data_ptr() for t in self._f2_nhwc])
        self.coarse_first_level = None
        self._volumes = None
        if D % 16 == 0 and D <= 256 and radius <= 6 and B > 0 and H * W >= self.COARSE_MIN_QUERIES:
            self._make_volumes(B, D, H, W)

    def _make_volumes(self, B, D, H, W):
        lib = nat.load()
        sizes = _level_sizes(H, W, self.num_levels)
        first = next((lvl for lvl in range(1, self.num_levels)
                      if sizes[lvl][0] * sizes[lvl][1] <= self.COARSE_LEVEL_MAX_CELLS), None)
        while first is not None and first < self.num_levels:
            n = lib.dxr_alt_volume_numel(B, H, W, self.num_levels, first)
            if 0 < n * 4 <= self.COARSE_VOLUME_MAX_BYTES:
                break
            first += 1
        if first is None or first >= self.num_levels:
            return
        vol = torch.empty((n,), dtype=torch.float32, device=self._device)
        # with COARSE_VOLUME_PLANES, the f16 pair planes of the operands (the volume GEMM's
        # LDS-DMA form), from torch's caching allocator: freed once the launches that read
        # them have run; 0 bytes: the register form
        nbytes = (lib.dxr_alt_coarse_volumes_ws_bytes(B, H, W, D, self.num_levels, first)
                  if self.COARSE_VOLUME_PLANES else 0)
        ws = torch.empty(max(nbytes, 0), dtype=torch.uint8, device=self._device)
        with _Launch(self._device):
            st = lib.dxr_alt_coarse_volumes_ws(self._f1_nhwc.data_ptr(), self._f2_ptrs, B, H, W, D,
                                               self.num_levels, first, vol.data_ptr(), nat.ptr(ws),
                                               max(nbytes, 0), nat.stream_of(vol))
        nat.check(st, "AlternateCorrBlock coarse volumes (dxr_alt_coarse_volumes_ws)")
        self.coarse_first_level = first
        self._volumes = vol

    @property
    def pyramid(self):
        """The reference's ``pyramid`` (core/corr.py:66-72): ``num_levels + 1`` pairs
        ``(fmap1_i, fmap2_i)`` of 2x2-pooled fmaps, ``[B, D, H_i, W_i]`` float32.

        Entry 0 is the caller's fmaps; the pooled entries are channels-last
        tensors (values bit-identical to F.avg_pool2d), materialised on first access
        — the lookup needs only full-res fmap1 and fmap2's first num_levels levels.
        """
        if self._pyramid is None:
            p1 = [self._f1_nhwc]
            p2 = list(self._f2_nhwc)
            while len(p1) < self.num_levels + 1:
                p1.append(_pool_nhwc(p1[-1]))
            while len(p2) < self.num_levels + 1:
                p2.append(_pool_nhwc(p2[-1]))
            pyr = [self._fmaps]
            pyr += [(a.permute(0, 3, 1, 2), b.permute(0, 3, 1, 2)) for a, b in zip(p1[1:], p2[1:])]
            self._pyramid = pyr
        return self._pyramid

    def __call__(self, coords):
        B, D, H, W = self._geom
        _require_no_grad(coords, what="coords (the reference detaches them, core/raft.py:170)")
        c = _check_coords(coords, B, H, W, self._device)
        return self._lookup(c)

    def _lookup(self, c):
        B, D, H, W = self._geom
        rd = 2 * self.radius + 1
        out = torch.empty((B, self.num_levels * rd * rd, H, W), dtype=torch.float32,
                          device=self._device)
        lib = nat.load()
        first = self.coarse_first_level
        if first is None:
            # query-order workspace (dxr_alt_corr_lookup_ws), from torch's caching
            # allocator: freed once the launches that use it have run
            nbytes = lib.dxr_alt_workspace_bytes(B, H, W, self.num_levels)
            ws = torch.empty(max(nbytes, 0), dtype=torch.uint8, device=self._device)
            with _Launch(self._device):
                st = lib.dxr_alt_corr_lookup_ws(self._f1_nhwc.data_ptr(), self._f2_ptrs,
                                                c.data_ptr(), out.data_ptr(), B, H, W, D,
                                                self.num_levels, self.radius, _sqrt_dim(D),
                                                nat.ptr(ws), max(nbytes, 0), nat.stream_of(c))
            nat.check(st, "AlternateCorrBlock lookup (dxr_alt_corr_lookup_ws)")
            return out
        with _Launch(self._device):
            if first > 0:   # the fine levels on the fly
                nbytes = lib.dxr_alt_workspace_bytes(B, H, W, first)
                ws = torch.empty(max(nbytes, 0), dtype=torch.uint8, device=self._device)
                st = lib.dxr_alt_corr_lookup_levels_ws(self._f1_nhwc.data_ptr(), self._f2_ptrs,
                                                       c.data_ptr(), out.data_ptr(), B, H, W, D,
                                                       self.num_levels, first, self.radius,
                                                       _sqrt_dim(D), nat.ptr(ws), max(nbytes, 0),
                                                       nat.stream_of(c))
                nat.check(st, "AlternateCorrBlock lookup (dxr_alt_corr_lookup_levels_ws)")
            st = lib.dxr_alt_volume_lookup(self._volumes.data_ptr(), c.data_ptr(), out.data_ptr(),
                                           B, H, W, self.num_levels, first, self.radius,
                                           _sqrt_dim(D), nat.stream_of(c))
        nat.check(st, "AlternateCorrBlock lookup (dxr_alt_volume_lookup)")
        return out
