#!/usr/bin/env python3
"""Software-pipelined build A/B (experiments target: dxr_xp_build_pipe).

  prod : the product build (dxr_corr_pyramid_build_ws; split pass + DMA build, or
         the bf16 channels-last DMA build)
  pipe : corr_build_pipe_kernel (one persistent workgroup per CU, the previous
         unit's epilogue interleaved into the next unit's K loop)
Pages are checked bit-identical; then graphs of --reps builds (and, with
--step, of build + 12 lookups as in bench.py) are timed in interleaved rounds
with HIP events.
Usage: python scripts/xp_pipe.py [--shape 1x55x128] [--dtype f32|bf16] [--step]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="1x55x128")
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--step", action="store_true", help="also time build + 12 lookups")
    a = ap.parse_args()
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    plib = dexiraft_amd.load_native()
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.dxr_xp_build_pipe.restype = i32
    lib.dxr_xp_build_pipe.argtypes = [vp, vp, i32, i64, i64, i64, i64, vp, vp, vp]
    dev = torch.device("cuda", 0)
    B, H, W = (int(v) for v in a.shape.split("x"))
    D = 256
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    dt, layout = nat.DXR_F32, nat.DXR_NCHW
    if a.dtype == "bf16":
        f1 = f1.bfloat16().contiguous(memory_format=torch.channels_last)
        f2 = f2.bfloat16().contiguous(memory_format=torch.channels_last)
        dt, layout = nat.DXR_BF16, nat.DXR_NHWC
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack((xs, ys))[None].expand(B, 2, H, W)
    coords = [(grid + 4.0 * torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous()
              for _ in range(12)]
    ref = dexiraft_amd.CorrBlock(f1, f2)._buf.clone()
    pyr = torch.empty_like(ref)
    nb = max(plib.dxr_build_workspace_bytes(dt, B, D, H, W), 0)
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
    outs = [torch.empty((B, 324, H, W), device=dev) for _ in range(12)]
    stream = torch.cuda.Stream(device=dev)
    div = float(np.sqrt(np.float32(D)))

    def build(v):
        s = stream.cuda_stream
        if v == "prod":
            st = plib.dxr_corr_pyramid_build_ws(f1.data_ptr(), f2.data_ptr(), dt, layout, B, D, H, W,
                                                4, div, pyr.data_ptr(), dt, nat.DXR_BUILD_AUTO,
                                                ws.data_ptr() if nb else None, nb, s)
        else:
            st = lib.dxr_xp_build_pipe(f1.data_ptr(), f2.data_ptr(), dt, B, D, H, W, pyr.data_ptr(),
                                       ws.data_ptr(), s)
        assert st == 0, (v, st)

    def step(v):
        build(v)
        for c, o in zip(coords, outs):
            assert plib.dxr_corr_lookup(pyr.data_ptr(), dt, B, H, W, 4, 4, c.data_ptr(),
                                        o.data_ptr(), stream.cuda_stream) == 0

    variants = ["prod", "pipe"]
    graphs = {}
    with torch.cuda.stream(stream):
        for v in variants:
            pyr.fill_(float("nan")) if a.dtype == "f32" else pyr.zero_()
            build(v)
            torch.cuda.synchronize()
            same = torch.equal(pyr, ref) if a.dtype == "bf16" else \
                torch.equal(torch.nan_to_num(pyr, nan=7.0), torch.nan_to_num(ref, nan=7.0))
            assert same, f"{v} differs from the product build"
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=stream):
                for _ in range(a.reps):
                    build(v)
            graphs[("build", v)] = gr
            if a.step:
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=stream):
                    step(v)
                graphs[("step", v)] = gr
        t_end = time.perf_counter() + 0.5
        while time.perf_counter() < t_end:
            for gr in graphs.values():
                gr.replay()
            torch.cuda.synchronize()
        res = {k: [] for k in graphs}
        for _ in range(a.rounds):
            for k, gr in graphs.items():
                n = 1 if k[0] == "build" else 20
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(n):
                    gr.replay()
                e1.record(stream)
                torch.cuda.synchronize()
                per = a.reps if k[0] == "build" else n
                res[k].append(e0.elapsed_time(e1) * 1e3 / per)
    print(json.dumps({"shape": [B, D, H, W], "dtype": a.dtype,
                      "us_min_med": {f"{k[0]}:{k[1]}": [round(min(x), 1), round(float(np.median(x)), 1)]
                                     for k, x in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
