"""numpy restatement of the reference correlation path (TEST INFRASTRUCTURE ONLY).

Each function cites the reference lines it restates (paths relative to the
reference repository).  ``dtype`` selects the accumulation precision: float64
(default) gives an independent high-precision check; float32 mirrors the
reference's own rounding (used to pin the restatement against golden vectors).

Coordinate arithmetic is always float32, exactly as the reference performs it:
``bilinear_sampler`` normalises pixel coordinates to [-1, 1] in float32
(core/utils/utils.py:61-62) and ATen's grid sampler maps them back with
``(g + 1) * ((size - 1) / 2)`` before flooring.  That round trip moves samples by
a few ulps, so it is part of the semantics being restated.

Parity status: pinned — tests/test_oracle_golden.py checks every function here
against fixtures generated from the reference itself (tests/golden/).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def corr_volume(fmap1: np.ndarray, fmap2: np.ndarray, dtype=np.float64) -> np.ndarray:
    """All-pairs correlation, core/corr.py:52-60.

    ``fmap1, fmap2``: [B, D, H, W].  Returns [B*H*W, H, W] (the reference's
    ``corr.reshape(batch*h1*w1, dim, h2, w2)`` of core/corr.py:21-22 with dim=1
    dropped): ``matmul(f1^T, f2) / sqrt(D)`` where sqrt(D) is taken in float32
    (``torch.sqrt(torch.tensor(dim).float())``) and the division comes after the
    product.
    """
    B, D, H, W = fmap1.shape
    f1 = fmap1.reshape(B, D, H * W).astype(dtype)
    f2 = fmap2.reshape(B, D, H * W).astype(dtype)
    corr = np.matmul(f1.transpose(0, 2, 1), f2)
    sq = np.sqrt(F32(D), dtype=F32)
    corr = corr / corr.dtype.type(sq)
    return corr.reshape(B * H * W, H, W)


def avg_pool2x2(x: np.ndarray) -> np.ndarray:
    """F.avg_pool2d(x, 2, stride=2) over the last two dims, floor mode (core/corr.py:26).

    Window sum order ((x00 + x01) + x10) + x11, then / 4, as ATen's CPU kernel.
    """
    H, W = x.shape[-2:]
    Ho, Wo = H // 2, W // 2
    if Ho < 1 or Wo < 1:
        raise RuntimeError(f"avg_pool2d: output size of a {H}x{W} input is empty")
    x = x[..., :2 * Ho, :2 * Wo]
    s = ((x[..., 0::2, 0::2] + x[..., 0::2, 1::2]) + x[..., 1::2, 0::2]) + x[..., 1::2, 1::2]
    return s / x.dtype.type(4)


def corr_pyramid(fmap1, fmap2, num_levels: int = 4, dtype=np.float64) -> list[np.ndarray]:
    """CorrBlock.__init__, core/corr.py:13-27: level 0 + (num_levels-1) poolings.

    Level l has shape [B*H*W, H_l, W_l] (the reference keeps a singleton channel
    dim, [B*H*W, 1, H_l, W_l]).
    """
    pyr = [corr_volume(fmap1, fmap2, dtype)]
    for _ in range(num_levels - 1):
        pyr.append(avg_pool2x2(pyr[-1]))
    return pyr


def corr_rows_pyramid(fmap1, fmap2, queries, num_levels: int = 4,
                      dtype=np.float64) -> list[np.ndarray]:
    """corr_pyramid of ONE pair restricted to some query rows (core/corr.py:13-27,
    52-60): every level of a query row depends only on that row, since the
    pooling runs over the image-2 dims.  ``fmap1, fmap2``: [D, H, W];
    ``queries``: flat query indices.  Level l: [len(queries), H_l, W_l].  Lets
    full-size configurations (C4 Sintel B=64, C5 1080p) be checked on sampled
    rows without the O(N^2) volume."""
    D, H, W = fmap1.shape
    q = np.asarray(queries, dtype=np.int64)
    f1 = fmap1.reshape(D, H * W)[:, q].astype(dtype)
    f2 = fmap2.reshape(D, H * W).astype(dtype)
    rows = f1.T @ f2
    rows = rows / rows.dtype.type(np.sqrt(F32(D), dtype=F32))
    pyr = [rows.reshape(len(q), H, W)]
    for _ in range(num_levels - 1):
        pyr.append(avg_pool2x2(pyr[-1]))
    return pyr


def corr_lookup_rows(rows_pyramid: list[np.ndarray], coords_q: np.ndarray,
                     radius: int) -> np.ndarray:
    """corr_lookup for the query rows of corr_rows_pyramid: ``coords_q`` [Q, 2]
    (x, y) of those queries.  Returns [Q, L*(2r+1)^2] in the reference's channel
    order (core/corr.py:29-50)."""
    Q = coords_q.shape[0]
    c = np.asarray(coords_q, dtype=F32).T.reshape(1, 2, 1, Q)
    return corr_lookup(rows_pyramid, c, radius)[0, :, 0, :].T


def alt_corr_block_queries(fmap1: np.ndarray, fmap2: np.ndarray, coords: np.ndarray, queries,
                           num_levels: int = 4, radius: int = 4,
                           dtype=np.float64) -> np.ndarray:
    """alt_corr_block (core/corr.py:63-91) of ONE pair restricted to some query
    pixels.  ``fmap1, fmap2``: [D, H, W]; ``coords``: [2, H, W]; ``queries``: flat
    indices.  Returns [len(queries), L*(2r+1)^2] (already / sqrt(D))."""
    D, H, W = fmap1.shape
    q = np.asarray(queries, dtype=np.int64)
    f1q = fmap1.reshape(D, H * W)[:, q].T[:, None, None, :]          # [Q, 1, 1, D]
    cq = np.asarray(coords, dtype=F32).reshape(2, H * W)[:, q].T      # [Q, 2]
    f2 = fmap2
    outs = []
    for i in range(num_levels):
        if i:
            f2 = avg_pool2x2(f2)
        f2i = f2.transpose(1, 2, 0)                                  # [H_i, W_i, D]
        ci = (cq / F32(2 ** i)).reshape(len(q), 1, 1, 1, 2)
        # each query as its own 1x1 "image" with the level's fmap2 (the kernel's
        # semantics do not depend on the query's own position)
        o = alt_corr_forward(f1q, np.broadcast_to(f2i, (len(q),) + f2i.shape), ci, radius, dtype)
        outs.append(o[:, 0, :, 0, 0])
    out = np.concatenate(outs, axis=1)
    return out / out.dtype.type(np.sqrt(F32(D), dtype=F32))


def sample_coord(c: np.ndarray, size: int) -> np.ndarray:
    """Pixel coordinate -> grid_sample sampling position, all in float32.

    core/utils/utils.py:61-62 (``2*x/(W-1) - 1``) followed by ATen's
    align_corners=True unnormalise ``(g + 1) * ((size - 1) / 2)``.  size == 1
    divides by zero: the result is NaN/inf, as in the reference.
    """
    c = np.asarray(c, dtype=F32)
    s = F32(size - 1)
    with np.errstate(divide="ignore", invalid="ignore"):
        g = (F32(2) * c) / s - F32(1)
        return (g + F32(1)) * (s / F32(2))


def bilinear_sample(img: np.ndarray, x: np.ndarray, y: np.ndarray) -> np.ndarray:
    """bilinear_sampler(img, coords) with mask=False, core/utils/utils.py:57-71.

    ``img``: [P, H, W]; ``x``, ``y``: [P, K] float32 pixel coordinates, sample k
    of plane p reads plane p.  F.grid_sample semantics: bilinear, zero padding
    (taps outside [0, W-1] x [0, H-1] contribute 0), align_corners=True.
    Weights and tap sum follow ATen's CPU grid sampler:
      w = u - floor(u), e = 1 - w; nw = s*e, ne = s*w, sw = n*e, se = n*w;
      out = nw*v_nw + ne*v_ne + sw*v_sw + se*v_se,
    which the reference's compiled CPU kernel evaluates as the fused chain
    fma(se, v_se, fma(sw, v_sw, fma(ne, v_ne, nw*v_nw))) — for float32 ``img``
    this function reproduces that chain (bit-exact against the golden vectors);
    for float64 ``img`` it sums in float64.  Weights are always float32.
    """
    P, H, W = img.shape
    ix = sample_coord(x, W)
    iy = sample_coord(y, H)
    with np.errstate(invalid="ignore"):
        x0 = np.floor(ix)
        y0 = np.floor(iy)
        w = ix - x0
        e = F32(1) - w
        n = iy - y0
        s = F32(1) - n
        nw, ne, sw, se = s * e, s * w, n * e, n * w
    dt = img.dtype
    plane = np.arange(P)[:, None]
    flat = img.reshape(P, H * W)

    def tap(yy: np.ndarray, xx: np.ndarray) -> np.ndarray:
        ok = np.isfinite(yy) & np.isfinite(xx)
        ok &= (yy >= 0) & (yy <= H - 1) & (xx >= 0) & (xx <= W - 1)
        yi = np.where(ok, yy, 0).astype(np.int64)
        xi = np.where(ok, xx, 0).astype(np.int64)
        v = flat[np.broadcast_to(plane, yi.shape), yi * W + xi]
        return np.where(ok, v, dt.type(0))

    with np.errstate(invalid="ignore", over="ignore"):
        v_nw, v_ne = tap(y0, x0), tap(y0, x0 + 1)
        v_sw, v_se = tap(y0 + 1, x0), tap(y0 + 1, x0 + 1)
        if dt == np.float32:
            out = _fma32(se, v_se, _fma32(sw, v_sw, _fma32(ne, v_ne, nw * v_nw)))
        else:
            out = ((nw.astype(dt) * v_nw + ne.astype(dt) * v_ne) + sw.astype(dt) * v_sw) + \
                se.astype(dt) * v_se
    return out


def _fma32(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """float32 fused multiply-add: the f32 x f32 product is exact in float64."""
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F32)


def corr_lookup(pyramid: list[np.ndarray], coords: np.ndarray, radius: int) -> np.ndarray:
    """CorrBlock.__call__, core/corr.py:29-50.

    ``coords``: [B, 2, H, W] float32 (channel 0 = x).  Returns
    [B, L*(2r+1)^2, H, W] with channel l*(2r+1)^2 + ix*(2r+1) + iy, x offset
    ix - r: the meshgrid(dy, dx) delta grid adds its FIRST index to x
    (core/corr.py:37-43).  Per level, centre = coords / 2^l in float32.
    """
    B, _, H, W = coords.shape
    rd = 2 * radius + 1
    c = np.asarray(coords, dtype=F32).transpose(0, 2, 3, 1).reshape(B * H * W, 2)
    offs = np.arange(-radius, radius + 1, dtype=F32)
    outs = []
    for lvl, img in enumerate(pyramid):
        cen = c / F32(2 ** lvl)
        xs = np.broadcast_to(cen[:, 0, None, None] + offs[None, :, None], (B * H * W, rd, rd))
        ys = np.broadcast_to(cen[:, 1, None, None] + offs[None, None, :], (B * H * W, rd, rd))
        v = bilinear_sample(img, xs.reshape(-1, rd * rd), ys.reshape(-1, rd * rd))
        outs.append(v.reshape(B, H, W, rd * rd))
    out = np.concatenate(outs, axis=-1)
    return np.ascontiguousarray(out.transpose(0, 3, 1, 2))


def alt_corr_forward(fmap1: np.ndarray, fmap2: np.ndarray, coords: np.ndarray, radius: int,
                     dtype=np.float64) -> np.ndarray:
    """alt_cuda_corr.forward, alt_cuda_corr/correlation_kernel.cu:18-119 + :260-286.

    ``fmap1``: [B, H1, W1, C], ``fmap2``: [B, H2, W2, C], ``coords``:
    [B, N, H1, W1, 2].  Returns [B, N, (2r+1)^2, H1, W1], channel oy + (2r+1)*ox.
    For each query, x0 = floor(x), dx = x - x0; the (2r+2)^2 cells
    (y0 - r + iy, x0 - r + ix) get <fmap1[q], fmap2[cell]> (0 outside, :80-83) and
    each is scattered to up to four outputs with weights dy*dx, dy*(1-dx),
    (1-dy)*dx, (1-dy)*(1-dx) (:92-114).  No 1/sqrt(D) here.
    """
    B, H1, W1, C = fmap1.shape
    _, H2, W2, _ = fmap2.shape
    N = coords.shape[1]
    rd = 2 * radius + 1
    f1 = fmap1.astype(dtype).reshape(B, 1, H1 * W1, C)
    f2 = fmap2.astype(dtype)
    c = np.asarray(coords, dtype=F32).reshape(B, N, H1 * W1, 2)
    x, y = c[..., 0], c[..., 1]
    x0, y0 = np.floor(x), np.floor(y)
    dx, dy = (x - x0).astype(dtype), (y - y0).astype(dtype)
    x0i, y0i = x0.astype(np.int64), y0.astype(np.int64)
    bidx = np.arange(B)[:, None, None]
    s = np.zeros((rd + 1, rd + 1) + x.shape, dtype=dtype)
    for iy in range(rd + 1):
        for ix in range(rd + 1):
            h2 = y0i - radius + iy
            w2 = x0i - radius + ix
            ok = (h2 >= 0) & (h2 < H2) & (w2 >= 0) & (w2 < W2)
            v = f2[bidx, np.where(ok, h2, 0), np.where(ok, w2, 0)]  # [B, N, Q, C]
            s[iy, ix] = np.where(ok, np.einsum("bnqc,bnqc->bnq", np.broadcast_to(f1, v.shape), v), 0)
    out = np.zeros((B, N, rd * rd, H1 * W1), dtype=dtype)
    for ox in range(rd):
        for oy in range(rd):
            out[:, :, oy + rd * ox] = (s[oy, ox] * (1 - dy) * (1 - dx) + s[oy, ox + 1] * (1 - dy) * dx
                                       + s[oy + 1, ox] * dy * (1 - dx) + s[oy + 1, ox + 1] * dy * dx)
    return out.reshape(B, N, rd * rd, H1, W1)


def alt_corr_backward(fmap1: np.ndarray, fmap2: np.ndarray, coords: np.ndarray,
                      corr_grad: np.ndarray, radius: int, dtype=np.float64):
    """alt_cuda_corr.backward, alt_cuda_corr/correlation_kernel.cu:122-256 + :288-320.

    ``corr_grad``: [B, N, (2r+1)^2, H1, W1].  Returns (fmap1_grad [B, H1, W1, C],
    fmap2_grad [B, H2, W2, C], coords_grad = zeros [B, N, H1, W1, 2] (:307)).
    Cell (iy, ix) of a query's (2r+2)^2 window gets g = the corr_grad taps of the
    up-to-four outputs it feeds, weighted dy*dx, dy*(1-dx), (1-dy)*dx,
    (1-dy)*(1-dx) (:197-216, output index oy + rd*ox); in-bounds cells add
    g*fmap2[cell] to fmap1_grad[q] and g*fmap1[q] to fmap2_grad[cell] (:218-233).
    It is the adjoint of alt_corr_forward in fmap1 and in fmap2
    (tests/test_oracle_golden.py checks that identity).
    """
    B, H1, W1, C = fmap1.shape
    _, H2, W2, _ = fmap2.shape
    N = coords.shape[1]
    Q = H1 * W1
    rd = 2 * radius + 1
    f1 = fmap1.astype(dtype).reshape(B, Q, C)
    f2 = fmap2.astype(dtype)
    G = np.asarray(corr_grad).astype(dtype).reshape(B, N, rd * rd, Q)
    c = np.asarray(coords, dtype=F32).reshape(B, N, Q, 2)
    x0, y0 = np.floor(c[..., 0]), np.floor(c[..., 1])
    dx, dy = (c[..., 0] - x0).astype(dtype), (c[..., 1] - y0).astype(dtype)
    x0i, y0i = x0.astype(np.int64), y0.astype(np.int64)
    bidx = np.arange(B)[:, None, None]
    f1g = np.zeros((B, Q, C), dtype=dtype)
    f2g = np.zeros((B, H2, W2, C), dtype=dtype)
    for iy in range(rd + 1):
        for ix in range(rd + 1):
            g = np.zeros((B, N, Q), dtype=dtype)
            if iy > 0 and ix > 0:
                g += G[:, :, (iy - 1) + rd * (ix - 1)] * dy * dx
            if iy > 0 and ix < rd:
                g += G[:, :, (iy - 1) + rd * ix] * dy * (1 - dx)
            if iy < rd and ix > 0:
                g += G[:, :, iy + rd * (ix - 1)] * (1 - dy) * dx
            if iy < rd and ix < rd:
                g += G[:, :, iy + rd * ix] * (1 - dy) * (1 - dx)
            h2 = y0i - radius + iy
            w2 = x0i - radius + ix
            ok = (h2 >= 0) & (h2 < H2) & (w2 >= 0) & (w2 < W2)
            g = np.where(ok, g, 0)
            h2, w2 = np.where(ok, h2, 0), np.where(ok, w2, 0)
            f1g += np.einsum("bnq,bnqc->bqc", g, f2[bidx, h2, w2])
            for b in range(B):
                np.add.at(f2g[b], (h2[b].ravel(), w2[b].ravel()),
                          (g[b][..., None] * f1[b][None]).reshape(-1, C))
    return (f1g.reshape(B, H1, W1, C), f2g,
            np.zeros((B, N, H1, W1, 2), dtype=dtype))


def alt_corr_block(fmap1: np.ndarray, fmap2: np.ndarray, coords: np.ndarray, num_levels: int = 4,
                   radius: int = 4, dtype=np.float64) -> np.ndarray:
    """AlternateCorrBlock(fmap1, fmap2)(coords), core/corr.py:63-91.

    ``fmap1, fmap2``: [B, D, H, W]; ``coords``: [B, 2, H, W].  Pools both fmaps
    ``num_levels`` times (:68-72; raises for fmaps below 2^num_levels), then per
    level runs alt_corr_forward on full-res fmap1 and level-i fmap2 with
    coords / 2^i (:80-87), stacks, and divides by sqrt(D) after sampling (:89-91).
    """
    B, D, H, W = fmap1.shape
    pyr = [(fmap1, fmap2)]
    for _ in range(num_levels):
        p1, p2 = pyr[-1]
        pyr.append((avg_pool2x2(p1), avg_pool2x2(p2)))
    c = np.asarray(coords, dtype=F32).transpose(0, 2, 3, 1)  # [B, H, W, 2]
    f1 = fmap1.transpose(0, 2, 3, 1)
    outs = []
    for i in range(num_levels):
        f2 = pyr[i][1].transpose(0, 2, 3, 1)
        ci = (c / F32(2 ** i)).reshape(B, 1, H, W, 2)
        outs.append(alt_corr_forward(f1, f2, ci, radius, dtype)[:, 0])
    out = np.stack(outs, axis=1).reshape(B, -1, H, W)
    return out / out.dtype.type(np.sqrt(F32(D), dtype=F32))


# --------------------------------------------------------------------------- backward
# Gradients of the reference CorrBlock with respect to its fmaps (training,
# train.py:175-178 backpropagates through core/corr.py).  coords are detached
# by the reference (core/raft.py:170), so no coordinate gradient is restated.


def bilinear_sample_backward(grad: np.ndarray, shape: tuple[int, int, int], x: np.ndarray,
                             y: np.ndarray) -> np.ndarray:
    """Gradient of ``bilinear_sample`` w.r.t. ``img`` (F.grid_sample backward,
    zero padding, align_corners=True, core/utils/utils.py:65): every in-bounds
    tap of sample k receives grad[p, k] times its weight.  float64 accumulation."""
    P, H, W = shape
    ix = sample_coord(x, W)
    iy = sample_coord(y, H)
    with np.errstate(invalid="ignore"):
        x0 = np.floor(ix)
        y0 = np.floor(iy)
        w = ix - x0
        e = F32(1) - w
        n = iy - y0
        s = F32(1) - n
        wts = {(0, 0): s * e, (0, 1): s * w, (1, 0): n * e, (1, 1): n * w}
    g = grad.astype(np.float64)
    out = np.zeros((P, H * W), dtype=np.float64)
    plane = np.broadcast_to(np.arange(P)[:, None], g.shape)
    for (dy_, dx_), wt in wts.items():
        yy, xx = y0 + dy_, x0 + dx_
        with np.errstate(invalid="ignore"):
            ok = np.isfinite(yy) & np.isfinite(xx) & (yy >= 0) & (yy <= H - 1) & (xx >= 0) & \
                (xx <= W - 1)
        idx = np.where(ok, yy, 0).astype(np.int64) * W + np.where(ok, xx, 0).astype(np.int64)
        np.add.at(out, (plane[ok], idx[ok]), (g * wt.astype(np.float64))[ok])
    return out.reshape(P, H, W)


def corr_lookup_backward(level_shapes: list[tuple[int, int]], coords: np.ndarray, radius: int,
                         grad_out: np.ndarray) -> list[np.ndarray]:
    """Gradient of ``corr_lookup`` (core/corr.py:29-50) w.r.t. each pyramid level:
    the channel split / permute inverted, then one grid_sample backward per level.
    Returns float64 levels [B*H*W, H_l, W_l]."""
    B, _, H, W = coords.shape
    rd = 2 * radius + 1
    c = np.asarray(coords, dtype=F32).transpose(0, 2, 3, 1).reshape(B * H * W, 2)
    offs = np.arange(-radius, radius + 1, dtype=F32)
    g = np.asarray(grad_out).transpose(0, 2, 3, 1).reshape(B * H * W, len(level_shapes), rd * rd)
    grads = []
    for lvl, (hl, wl) in enumerate(level_shapes):
        cen = c / F32(2 ** lvl)
        xs = np.broadcast_to(cen[:, 0, None, None] + offs[None, :, None], (B * H * W, rd, rd))
        ys = np.broadcast_to(cen[:, 1, None, None] + offs[None, None, :], (B * H * W, rd, rd))
        grads.append(bilinear_sample_backward(g[:, lvl], (B * H * W, hl, wl),
                                              xs.reshape(-1, rd * rd), ys.reshape(-1, rd * rd)))
    return grads


def avg_pool2x2_backward(dy: np.ndarray, in_shape: tuple[int, int]) -> np.ndarray:
    """F.avg_pool2d(2, stride=2) backward: each covered input cell gets dy / 4;
    the floor-mode remainder row / column gets 0."""
    H, W = in_shape
    Ho, Wo = dy.shape[-2:]
    dx = np.zeros(dy.shape[:-2] + (H, W), dtype=dy.dtype)
    q = dy / dy.dtype.type(4)
    for a in range(2):
        for b in range(2):
            dx[..., a:2 * Ho:2, b:2 * Wo:2] = q
    return dx


def corr_pyramid_backward(fmap1: np.ndarray, fmap2: np.ndarray,
                          dlevels: list[np.ndarray]) -> tuple[np.ndarray, np.ndarray]:
    """Gradient of CorrBlock.__init__ (core/corr.py:13-27, 52-60) w.r.t. the fmaps,
    given the gradient of every pyramid level: the pooling chain backward
    (level l receives level l+1's total gradient / 4), then / sqrt(D), then the
    two matmul gradients dF1 = F2 dV^T, dF2 = F1 dV.  float64."""
    B, D, H, W = fmap1.shape
    N = H * W
    tot = dlevels[-1].astype(np.float64)
    for lvl in range(len(dlevels) - 2, -1, -1):
        hl, wl = dlevels[lvl].shape[-2:]
        tot = dlevels[lvl].astype(np.float64) + avg_pool2x2_backward(tot, (hl, wl))
    dv = tot.reshape(B, N, N) / np.float64(np.sqrt(F32(D), dtype=F32))
    f1 = fmap1.reshape(B, D, N).astype(np.float64)
    f2 = fmap2.reshape(B, D, N).astype(np.float64)
    df1 = np.matmul(f2, dv.transpose(0, 2, 1))
    df2 = np.matmul(f1, dv)
    return df1.reshape(B, D, H, W), df2.reshape(B, D, H, W)


def motion_conv1x1(corr: np.ndarray, weight: np.ndarray, bias: np.ndarray | None = None,
                   relu: bool = True, dtype=np.float64) -> np.ndarray:
    """First layer of the motion encoder on the lookup output:
    ``F.relu(self.convc1(corr))`` (core/update.py:90 BasicMotionEncoder, :71
    SmallMotionEncoder; ``convc1 = nn.Conv2d(cor_planes, Cout, 1, padding=0)``,
    :83 / :66).  A 1x1 convolution is a per-pixel matrix product:
    ``out[b, o, h, w] = bias[o] + sum_c weight[o, c] * corr[b, c, h, w]``.

    ``corr``: [B, Cin, H, W]; ``weight``: [Cout, Cin] or [Cout, Cin, 1, 1].
    """
    B, C, H, W = corr.shape
    w = weight.reshape(weight.shape[0], -1).astype(dtype)
    assert w.shape[1] == C
    out = np.einsum("oc,bcn->bon", w, corr.reshape(B, C, H * W).astype(dtype))
    if bias is not None:
        out = out + bias.astype(dtype)[None, :, None]
    if relu:
        out = np.where(out < 0, out.dtype.type(0), out)   # NaN stays NaN (torch.relu)
    return out.reshape(B, -1, H, W)
