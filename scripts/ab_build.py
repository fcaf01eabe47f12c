#!/usr/bin/env python3
"""Same-process A/B of the f32 builds through the C-ABI (build only, no lookups).

  ws   : dxr_corr_pyramid_build_ws (pre-split pass + LDS-DMA build, round 3)
  nows : dxr_corr_pyramid_build    (register-split build, round 2)
  exact: DXR_BUILD_EXACT_F32       (exact-f32 MFMA build)
  prev : dxr_corr_pyramid_build_ws of an earlier product library (--prev-lib)
  tailN: the product's DMA build under tail policy N (dxr_xp_build_tail of the
         experiments library: split the last partial dispatch round into
         quarter units when 8 T <= N x slots; tail0 never, tail8 always)
  x22  : dxr_xp_build22 (experiments): each wave 2 x 2 MFMA tiles (64 queries x
         64 targets), whole units only — compare with tail0

Each variant is captured as a HIP graph of --reps back-to-back builds and the
graphs are replayed in interleaved rounds after a clock warm-up (HIP events;
a build plus its same-stream boundary).  Run it under
``rocprofv3 --kernel-trace --stats`` for per-kernel durations.
Usage: python scripts/ab_build.py [--shapes 1x55x128 8x55x128 1x46x62]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=["1x55x128", "8x55x128", "1x46x62"])
    ap.add_argument("--variants", nargs="+", default=["ws", "nows"])
    ap.add_argument("--layout", default="nchw", choices=["nchw", "nhwc"])
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"],
                    help="bf16: bf16 fmaps -> bf16 pyramid (variants ws / prev)")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--prev-lib", default=str(REPO / "scripts" / "libdexiraft_corr_r04.so"))
    a = ap.parse_args()
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    lib = dexiraft_amd.load_native()
    prev = None
    if "prev" in a.variants:
        import ctypes
        prev = ctypes.CDLL(a.prev_lib)
        for name, (res, args) in nat.SIGNATURES.items():
            if hasattr(prev, name):
                getattr(prev, name).restype = res
                getattr(prev, name).argtypes = args
    xlib = None
    if any(v.startswith("tail") or v == "x22" for v in a.variants):
        import ctypes
        xlib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        xlib.dxr_xp_build_tail.restype = i32
        xlib.dxr_xp_build_tail.argtypes = [vp, vp, i32, i32, i64, i64, i64, i64, vp, vp, i32, vp]
        xlib.dxr_xp_build22.restype = i32
        xlib.dxr_xp_build22.argtypes = [vp, vp, i64, i64, i64, i64, vp, vp, vp]
    dev = torch.device("cuda", 0)
    D = 256
    stream = torch.cuda.Stream(device=dev)
    for shp in a.shapes:
        B, H, W = (int(v) for v in shp.split("x"))
        g = torch.Generator(device=dev)
        g.manual_seed(7)
        f1 = torch.randn((B, D, H, W), generator=g, device=dev)
        f2 = torch.randn((B, D, H, W), generator=g, device=dev)
        dt = nat.DXR_F32
        if a.dtype == "bf16":
            f1, f2, dt = f1.bfloat16(), f2.bfloat16(), nat.DXR_BF16
        layout = nat.DXR_NCHW
        if a.layout == "nhwc":
            f1 = f1.contiguous(memory_format=torch.channels_last)
            f2 = f2.contiguous(memory_format=torch.channels_last)
            layout = nat.DXR_NHWC
        n = lib.dxr_pyramid_numel(B, H, W, 4)
        pyr = torch.empty(n, device=dev, dtype=torch.float32 if dt == nat.DXR_F32 else torch.bfloat16)
        wsb = lib.dxr_build_workspace_bytes(dt, B, D, H, W)
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=dev)
        div = float(np.sqrt(np.float32(D)))

        def build(v):
            s = stream.cuda_stream
            if v == "x22":
                st = xlib.dxr_xp_build22(f1.data_ptr(), f2.data_ptr(), B, D, H, W, pyr.data_ptr(),
                                         ws.data_ptr(), s)
            elif v.startswith("tail"):
                st = xlib.dxr_xp_build_tail(f1.data_ptr(), f2.data_ptr(), dt, layout, B, D, H, W,
                                            pyr.data_ptr(), ws.data_ptr(), int(v[4:]), s)
            elif v in ("ws", "prev"):
                fn = lib if v == "ws" else prev
                st = fn.dxr_corr_pyramid_build_ws(f1.data_ptr(), f2.data_ptr(), dt,
                                                   layout, B, D, H, W, 4, div, pyr.data_ptr(),
                                                   dt, nat.DXR_BUILD_AUTO, ws.data_ptr(),
                                                   max(wsb, 0), s)
            else:
                algo = nat.DXR_BUILD_EXACT_F32 if v == "exact" else nat.DXR_BUILD_AUTO
                st = lib.dxr_corr_pyramid_build(f1.data_ptr(), f2.data_ptr(), nat.DXR_F32, layout,
                                                B, D, H, W, 4, div, pyr.data_ptr(), nat.DXR_F32,
                                                algo, s)
            assert st == 0, (v, st)

        graphs = {}
        ref = None
        with torch.cuda.stream(stream):
            for v in a.variants:
                build(v)
                torch.cuda.synchronize()
                if v in ("ws", "prev", "x22") or v.startswith("tail"):
                    if ref is None:
                        ref = pyr.clone()
                    same = torch.equal(torch.nan_to_num(pyr.float(), nan=3.0),
                                       torch.nan_to_num(ref.float(), nan=3.0))
                    assert same, v
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=stream):
                    for _ in range(a.reps):
                        build(v)
                graphs[v] = gr
            for _ in range(10):
                for v in a.variants:
                    graphs[v].replay()
            torch.cuda.synchronize()
            res = {v: [] for v in a.variants}
            for _ in range(a.rounds):
                for v in a.variants:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    graphs[v].replay()
                    e1.record(stream)
                    torch.cuda.synchronize()
                    res[v].append(e0.elapsed_time(e1) * 1e3 / a.reps)
        print(json.dumps({"shape": [B, D, H, W], "layout": a.layout, "dtype": a.dtype,
                          "us_per_build_min_med": {v: [round(min(x), 1), round(float(np.median(x)), 1)]
                                                   for v, x in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
