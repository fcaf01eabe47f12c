#!/usr/bin/env python3
"""Line model of the lookup's window gathers under two pyramid page layouts
(the layout-imposed cap).  For Sintel's fmap (55 x 128),
radius 4, 4 levels, it counts the distinct 128-byte lines (f32 cells) holding
every query's 10 x 10 tap cells per level (clipped to the level):
  paged   — the product's pages (§3.3): a query's 8x16 tile (>> level) is
            contiguous, so a line holds cells of one query;
  qminor  — a query-minor page: element ((tile * S + cell) * 128 + q % 128), so
            a line holds one cell of 32 consecutive queries;
for i.i.d. N(0, 4^2) flow (the bench's model) and a flow correlated over ~16 px
with the same per-pixel spread.  Prints lines / window-cell bytes per layout.
CPU only; no GPU, no reference code."""
import numpy as np
from scipy.ndimage import zoom

H, W, R = 55, 128, 4


def coords(rng, smooth):
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    if smooth:
        c = rng.standard_normal((2, H // 16 + 2, W // 16 + 2))
        f = np.stack([zoom(c[i], 16, order=3)[:H, :W] for i in range(2)])
        f = f / f.std(axis=(1, 2), keepdims=True) * 4
        return xs + f[0], ys + f[1]
    return xs + 4 * rng.standard_normal((H, W)), ys + 4 * rng.standard_normal((H, W))


def line_bytes(cx, cy, layout):
    x, y = cx.reshape(-1), cy.reshape(-1)
    q = np.arange(H * W)
    offs = np.arange(2 * R + 2)
    tx = -(-W // 16)
    tot = 0
    for lvl in range(4):
        h, w, th, tw = H >> lvl, W >> lvl, 8 >> lvl, 16 >> lvl
        ccx = np.floor(x / 2 ** lvl)[:, None] - R + offs
        ccy = np.floor(y / 2 ** lvl)[:, None] - R + offs
        ok = ((ccy >= 0) & (ccy < h))[:, :, None] & ((ccx >= 0) & (ccx < w))[:, None, :]
        tile = (ccy // th)[:, :, None] * tx + (ccx // tw)[:, None, :]
        cell = ((ccy % th) * tw)[:, :, None] + (ccx % tw)[:, None, :]
        S = th * tw
        if layout == "paged":
            elem = (q[:, None, None] % 128) * S + tile * (128 * S) + cell
        else:
            elem = (tile * S + cell) * 128 + (q[:, None, None] % 128)
        key = np.where(ok, (q[:, None, None] // 128) * 10 ** 9 + elem * 4 // 128, -1).reshape(-1)
        tot += np.unique(key[key >= 0]).size
    return tot * 128


def main():
    rng = np.random.default_rng(1)
    win = sum(min(10, H >> l) * min(10, W >> l) for l in range(4)) * 4 * H * W
    for smooth in (False, True):
        cx, cy = coords(rng, smooth)
        for lay in ("paged", "qminor"):
            b = line_bytes(cx, cy, lay)
            print(f"{'smooth' if smooth else 'iid':6s} {lay:6s} lines {b / 1e6:6.2f} MB, window cells "
                  f"{win / 1e6:.2f} MB, ratio {b / win:.2f}")


if __name__ == "__main__":
    main()
