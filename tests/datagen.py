"""Deterministic, portable synthetic inputs for parity tests and golden fixtures.

splitmix64 -> 53-bit uniforms -> Box-Muller normals, all in numpy integer and
float64 arithmetic, so the GPU box regenerates bit-identical inputs from a seed
(no large tensors need to be committed).  Shapes follow SURVEY.md §8(c)/(d):
fmaps [B, D, H, W], coords [B, 2, H, W] = coords_grid + displacement.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n outputs of the splitmix64 stream started at ``seed``."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + np.arange(1, n + 1, dtype=np.uint64) * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, n: int) -> np.ndarray:
    """float64 in [0, 1)."""
    return (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def normal(seed: int, n: int) -> np.ndarray:
    """Standard normals (float64) by Box-Muller on paired uniforms."""
    m = (n + 1) // 2
    u = uniform(seed, 2 * m)
    u1 = 1.0 - u[:m]            # (0, 1]
    u2 = u[m:]
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.concatenate([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)])
    return z[:n]


def fmap(seed: int, B: int, D: int, H: int, W: int, dist: str = "normal") -> np.ndarray:
    """Synthetic feature map [B, D, H, W] float32.

    ``normal``: N(0, 1).  ``fnet``: N(1.1, 1.45^2), the mean/std measured on
    random-weight fnet/efnet outputs; gives large, positively
    biased correlations (max ~40-60) like the real encoders.
    """
    z = normal(seed, B * D * H * W).reshape(B, D, H, W)
    if dist == "fnet":
        z = 1.1 + 1.45 * z
    elif dist != "normal":
        raise ValueError(dist)
    return z.astype(np.float32)


def coords(seed: int, B: int, H: int, W: int, mode: str = "normal", scale: float = 4.0) -> np.ndarray:
    """coords_grid(B, H, W) + displacement, float32 [B, 2, H, W].

    modes: ``normal`` (N(0, scale^2) per pixel, the benchmark's flow model),
    ``uniform`` (U(-scale, scale): many taps off the map), ``integer`` (integer
    displacements in [-scale, scale]: exact-integer sample positions),
    ``identity`` (the grid itself), ``far`` (shifted ~3 maps away: all taps
    outside, output 0).
    """
    ys, xs = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64),
                         indexing="ij")
    grid = np.broadcast_to(np.stack([xs, ys])[None], (B, 2, H, W))
    n = B * 2 * H * W
    if mode == "normal":
        d = scale * normal(seed, n)
    elif mode == "uniform":
        d = scale * (2.0 * uniform(seed, n) - 1.0)
    elif mode == "integer":
        d = np.floor((2 * scale + 1) * uniform(seed, n)) - scale
    elif mode == "identity":
        d = np.zeros(n)
    elif mode == "far":
        d = np.full(n, 3.0 * max(H, W)) * np.where(uniform(seed, n) < 0.5, -1.0, 1.0)
    else:
        raise ValueError(mode)
    return (grid + d.reshape(B, 2, H, W)).astype(np.float32)


def conv1x1_weights(i: int, cout: int, cin: int):
    """Motion-encoder convc1 weight [cout, cin] ~ N(0, 1/cin) and bias [cout] ~
    N(0, 0.25) for fixture case i (tests/golden/make_motion_golden.py)."""
    w = fmap(5000 + 10 * i, 1, 1, cout, cin, "normal")[0, 0] / np.float32(np.sqrt(cin))
    b = fmap(5001 + 10 * i, 1, 1, 1, cout, "normal")[0, 0, 0] * np.float32(0.5)
    return w.astype(np.float32), b.astype(np.float32)
