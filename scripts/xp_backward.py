#!/usr/bin/env python3
"""Time dxr_fmap_grads from one or more builds of the library (ablation A/B).

Each argument is a path to a libdexiraft_corr.so build; every build gets the same
random gradient pyramid and fmaps (Sintel shape by default) and is timed with
HIP events: both gradients, dfmap1 only, dfmap2 only (median of --reps).

Usage: python scripts/xp_backward.py lib_a.so [lib_b.so ...] [--shape B D H W L]
"""
from __future__ import annotations

import argparse
import ctypes
import json

import numpy as np
import torch

_vp, _i64, _int, _f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float


def bind(path):
    lib = ctypes.CDLL(path)
    lib.dxr_pyramid_numel.restype = _i64
    lib.dxr_pyramid_numel.argtypes = [_i64, _i64, _i64, _int]
    lib.dxr_pyramid_pack.argtypes = [_vp, _i64, _i64, _i64, _int, _int, _vp, _int, _vp]
    lib.dxr_fmap_grads_workspace_bytes.restype = _i64
    lib.dxr_fmap_grads_workspace_bytes.argtypes = [_i64, _i64, _i64, _i64, _int]
    lib.dxr_fmap_grads.argtypes = [_vp, _int, _vp, _vp, _i64, _i64, _i64, _i64, _int, _f32, _vp,
                                   _vp, _vp, _i64, _vp]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--shape", type=int, nargs=5, default=[1, 256, 55, 128, 4])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    B, D, H, W, L = a.shape
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    levels = []
    h, w = H, W
    for lvl in range(L):
        if lvl:
            h, w = h // 2, w // 2
        levels.append(torch.randn((B * H * W, h, w), generator=g, device=dev))
    s = torch.cuda.current_stream().cuda_stream
    ref = None
    for path in a.libs:
        lib = bind(path)
        gp = torch.zeros(lib.dxr_pyramid_numel(B, H, W, L), device=dev)
        for lvl, t in enumerate(levels):
            assert lib.dxr_pyramid_pack(t.data_ptr(), B, H, W, L, lvl, gp.data_ptr(), 0, s) == 0
        wsb = lib.dxr_fmap_grads_workspace_bytes(B, D, H, W, L)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        d1, d2 = torch.empty_like(f1), torch.empty_like(f2)

        def run(p1, p2):
            assert lib.dxr_fmap_grads(gp.data_ptr(), 0, f1.data_ptr(), f2.data_ptr(), B, D, H, W, L,
                                      float(np.sqrt(D)), p1, p2, ws.data_ptr(), wsb, s) == 0

        res = {"lib": path}
        for name, p1, p2 in (("both", d1.data_ptr(), d2.data_ptr()), ("df1", d1.data_ptr(), None),
                             ("df2", None, d2.data_ptr())):
            run(p1, p2)
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(p1, p2)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            res[name + "_us"] = round(float(np.median(ts)), 1)
        run(d1.data_ptr(), d2.data_ptr())
        torch.cuda.synchronize()
        if ref is None:
            ref = (d1.clone(), d2.clone())
        else:
            res["max_diff_vs_first"] = max((d1 - ref[0]).abs().max().item(),
                                           (d2 - ref[1]).abs().max().item())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
