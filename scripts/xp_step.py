#!/usr/bin/env python3
"""Full-step A/B of split-build variants (experiments target, never shipped).

One step = ``dxr_xp_build`` variant + 12 ``dxr_corr_lookup`` calls (the bench's
step, Sintel B=1 by default), captured in one HIP graph per variant and
replayed; rounds interleave the variants so they share the clock/thermal
history.  A second graph per variant holds only the 12 lookups, replayed right
after a build replay, so the lookup time includes whatever the build left in
the caches (e.g. non-temporal pyramid stores that bypass them).

Usage: python scripts/xp_step.py [--xp 1003,2032,2096] [--B 1 --H 55 --W 128]
A variant "X:Y" runs build variant X with ``dxr_xp_lookup`` variant Y instead of
the product lookup (e.g. 1003:16384, sc1 lookup stores).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--H", type=int, default=55)
    ap.add_argument("--W", type=int, default=128)
    ap.add_argument("--xp", default="1003,2032,2096")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"],
                    help="bf16: dxr_xp_build_bf16 variants, bf16 fmaps and pyramid")
    a = ap.parse_args()
    import dexiraft_amd
    nat = dexiraft_amd._native
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.dxr_xp_build.restype = ctypes.c_int
    lib.dxr_xp_build.argtypes = [vp, vp, i64, i64, i64, i64, vp, ctypes.c_int, vp]
    lib.dxr_xp_build_bf16.restype = ctypes.c_int
    lib.dxr_xp_build_bf16.argtypes = [vp, vp, i64, i64, i64, i64, vp, ctypes.c_int, vp]
    bf = a.dtype == "bf16"
    xbuild = lib.dxr_xp_build_bf16 if bf else lib.dxr_xp_build
    lib.dxr_corr_lookup.restype = ctypes.c_int
    lib.dxr_corr_lookup.argtypes = [vp, ctypes.c_int, i64, i64, i64, ctypes.c_int, ctypes.c_int, vp,
                                    vp, vp]
    lib.dxr_xp_lookup.restype = ctypes.c_int
    lib.dxr_xp_lookup.argtypes = [vp, ctypes.c_int, i64, i64, i64, vp, vp, ctypes.c_int, vp]
    dev = torch.device("cuda", 0)
    B, D, H, W = a.B, 256, a.H, a.W
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    if bf:
        f1, f2 = f1.bfloat16(), f2.bfloat16()
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack([xs, ys])[None].repeat(B, 1, 1, 1)
    coords = [grid + 4.0 * torch.randn(grid.shape, generator=g, device=dev) for _ in range(12)]
    pyr = torch.empty(nat.load().dxr_pyramid_numel(B, H, W, 4), device=dev,
                      dtype=torch.bfloat16 if bf else torch.float32)
    out = torch.empty((B, 324, H, W), device=dev)
    xps = a.xp.split(",")
    side = torch.cuda.Stream()

    def build(xp, s):
        st = xbuild(f1.data_ptr(), f2.data_ptr(), B, D, H, W, pyr.data_ptr(), int(xp.split(":")[0]), s)
        assert st == 0, (xp, st)

    def lookups(s, xp="0"):
        lx = int(xp.split(":")[1]) if ":" in xp else None
        for c in coords:
            if lx is None:
                st = lib.dxr_corr_lookup(pyr.data_ptr(), 1 if bf else 0, B, H, W, 4, 4, c.data_ptr(),
                                         out.data_ptr(), s)
            else:
                st = lib.dxr_xp_lookup(pyr.data_ptr(), 1 if bf else 0, B, H, W, c.data_ptr(),
                                       out.data_ptr(), lx, s)
            assert st == 0, st

    graphs = {}
    with torch.cuda.stream(side):
        for xp in xps:
            s = side.cuda_stream
            build(xp, s)
            lookups(s, xp)
            side.synchronize()
            gs, gl = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(gs, stream=side):
                build(xp, torch.cuda.current_stream().cuda_stream)
                lookups(torch.cuda.current_stream().cuda_stream, xp)
            with torch.cuda.graph(gl, stream=side):
                lookups(torch.cuda.current_stream().cuda_stream, xp)
            graphs[xp] = (gs, gl)
    torch.cuda.synchronize()
    for _ in range(100):         # clock warm-up
        for xp in xps:
            graphs[xp][0].replay()
    torch.cuda.synchronize()
    step = {xp: [] for xp in xps}
    look = {xp: [] for xp in xps}
    for _ in range(a.rounds):
        for xp in xps:
            gs, gl = graphs[xp]
            gs.replay()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            for _ in range(a.steps):
                gs.replay()
            e[1].record()
            for _ in range(a.steps):
                gs.replay()
                gl.replay()
            e[2].record()
            torch.cuda.synchronize()
            t_step = e[0].elapsed_time(e[1]) / a.steps
            t_both = e[1].elapsed_time(e[2]) / a.steps
            step[xp].append(t_step * 1e3)
            look[xp].append((t_both - t_step) / 12 * 1e3)
    for xp in xps:
        ms = float(np.median(step[xp]))
        print(json.dumps({"xp": xp, "step_us": round(ms, 2), "pairs_per_s": round(B * 1e6 / ms, 1),
                          "lookup_us_after_build": round(float(np.median(look[xp])), 2),
                          "build_us_est": round(ms - 12 * float(np.median(look[xp])), 2)}),
              flush=True)


if __name__ == "__main__":
    main()
