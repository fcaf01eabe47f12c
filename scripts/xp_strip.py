#!/usr/bin/env python3
"""Strip width of the builds' XCD-banded page order (experiments target).

dxr_xp_build_strip runs the product's DMA build (f32 NCHW with its split pass,
or bf16 channels-last) with another BuildGeom::strip (product: 8 target tiles).
Graphs of --reps builds per width, interleaved rounds, HIP events; pages checked
bit-identical to the product build.  Run it under rocprofv3 --pmc FETCH_SIZE for
the operand re-fetch.
Usage: python scripts/xp_strip.py [--shape 8x47x156 --dtype bf16] [--strips 8 16 30]
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
    ap.add_argument("--shape", default="1x55x128")
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--strips", type=int, nargs="+", default=[8, 16, 28])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    plib = dexiraft_amd.load_native()
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.dxr_xp_build_strip.restype = i32
    lib.dxr_xp_build_strip.argtypes = [vp, vp, i32, i64, i64, i64, i64, vp, vp, i32, vp]
    dev = torch.device("cuda", 0)
    B, H, W = (int(v) for v in a.shape.split("x"))
    D = 256
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    dt = nat.DXR_F32
    if a.dtype == "bf16":
        f1 = f1.bfloat16().contiguous(memory_format=torch.channels_last)
        f2 = f2.bfloat16().contiguous(memory_format=torch.channels_last)
        dt = nat.DXR_BF16
    ref = dexiraft_amd.CorrBlock(f1, f2)._buf.clone()
    pyr = torch.empty_like(ref)
    nbytes = plib.dxr_build_workspace_bytes(dt, B, D, H, W)
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)

    def launch(sw):
        st = lib.dxr_xp_build_strip(f1.data_ptr(), f2.data_ptr(), dt, B, D, H, W, pyr.data_ptr(),
                                    ws.data_ptr(), sw, stream.cuda_stream)
        assert st == 0, (sw, st)

    graphs = {}
    with torch.cuda.stream(stream):
        for sw in a.strips:
            pyr.zero_()
            launch(sw)
            torch.cuda.synchronize()
            assert torch.equal(pyr, ref), f"strip {sw} differs from the product build"
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=stream):
                for _ in range(a.reps):
                    launch(sw)
            graphs[sw] = gr
        for _ in range(3):
            for sw in a.strips:
                graphs[sw].replay()
        torch.cuda.synchronize()
        res = {sw: [] for sw in a.strips}
        for _ in range(a.rounds):
            for sw in a.strips:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                graphs[sw].replay()
                e1.record(stream)
                torch.cuda.synchronize()
                res[sw].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    print(json.dumps({"shape": [B, D, H, W], "dtype": a.dtype,
                      "us_per_build_min_med": {sw: [round(min(x), 1), round(float(np.median(x)), 1)]
                                               for sw, x in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
