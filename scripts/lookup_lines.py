#!/usr/bin/env python3
"""Line-granular HBM floor of the lookup (CPU analysis, no GPU).

For the bench's coordinates (grid + N(0, 4^2) px) this counts, per query and
level, the 128-byte lines of the paged pyramid that hold the
cells the reference's bilinear taps read (the window of 2r+2 = 10 cells per axis
clipped to the level, or 11 where the coordinate round trip floors a sample to
the neighbouring cell), and the lines the kernel's staging loads touch
(corr_lookup.hip gather_load: WD = 11 rows x four 4-cell vectors from the origin
rounded down to a multiple of 4).  Compares them with the compulsory window bytes
SURVEY §8(d) prices the lookup at.  Any layout of a per-query map in 128-byte
lines must touch at least ceil-covering lines of each window; this prints the
layout's figure and the 4x8-cell-block alternative's.

Usage: python scripts/lookup_lines.py [--workload sintel|kitti] [--dtype f32|bf16]
"""
from __future__ import annotations

import argparse
import json

import numpy as np

LINE = 128
R = 4


def level_sizes(H, W, L=4):
    s = [(H, W)]
    for _ in range(L - 1):
        s.append((s[-1][0] // 2, s[-1][1] // 2))
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="sintel", choices=["sintel", "kitti", "chairs"])
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--queries", type=int, default=4096, help="sampled query pixels")
    a = ap.parse_args()
    H, W = {"sintel": (55, 128), "kitti": (47, 156), "chairs": (46, 62)}[a.workload]
    es = 4 if a.dtype == "f32" else 2
    rng = np.random.default_rng(0)
    n = min(a.queries, H * W)
    q = rng.choice(H * W, n, replace=False)
    qy, qx = q // W, q % W
    cx = qx + 4.0 * rng.standard_normal(n)
    cy = qy + 4.0 * rng.standard_normal(n)
    res = {"workload": a.workload, "dtype": a.dtype, "levels": []}
    tot = {"compulsory": 0, "tap_lines": 0, "staged_lines": 0, "block48_lines": 0}
    for lvl, (h, w) in enumerate(level_sizes(H, W)):
        th, tw = 8 >> lvl, 16 >> lvl
        row_major = th < 1 or tw < 1
        comp = tap = staged = blk = 0
        for i in range(n):
            x, y = cx[i] / 2 ** lvl, cy[i] / 2 ** lvl
            x0, y0 = int(np.floor(x)) - R, int(np.floor(y)) - R
            xs = [c for c in range(x0, x0 + 2 * R + 2) if 0 <= c < w]
            ys = [r for r in range(y0, y0 + 2 * R + 2) if 0 <= r < h]
            comp += len(xs) * len(ys) * es

            def line_of(r, c):
                # element offset inside this query's map: tile-major, row-major in a tile
                if row_major:
                    return (r * w + c) * es // LINE
                t = (r // th) * ((w + tw - 1) // tw) + c // tw
                return (t * th * tw + (r % th) * tw + c % tw) * es // LINE

            tap += len({line_of(r, c) for r in ys for c in xs})
            blk += len({(r // 4, c // 8) for r in ys for c in xs}) if es == 4 else \
                len({(r // 8, c // 8) for r in ys for c in xs})
            sx = (x0 & ~3)
            sset = set()
            for r in range(y0, y0 + 2 * R + 3):
                if not 0 <= r < h:
                    continue
                for k in range(4):
                    for c in range(sx + 4 * k, sx + 4 * k + 4):
                        if 0 <= c < w:
                            sset.add(line_of(r, c))
            staged += len(sset)
        s = n / (H * W)
        lv = {"level": lvl, "compulsory_bytes": comp / s, "tap_line_bytes": tap * LINE / s,
              "staged_line_bytes": staged * LINE / s, "block_line_bytes": blk * LINE / s}
        res["levels"].append({k: round(v) if isinstance(v, float) else v for k, v in lv.items()})
        tot["compulsory"] += comp / s
        tot["tap_lines"] += tap * LINE / s
        tot["staged_lines"] += staged * LINE / s
        tot["block48_lines"] += blk * LINE / s
    res["per_pair_bytes"] = {k: round(v) for k, v in tot.items()}
    res["ratios"] = {"tap_lines/compulsory": round(tot["tap_lines"] / tot["compulsory"], 3),
                     "staged_lines/compulsory": round(tot["staged_lines"] / tot["compulsory"], 3),
                     "block_lines/compulsory": round(tot["block48_lines"] / tot["compulsory"], 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
