#!/usr/bin/env python3
"""A/B of the fused lookup + convc1 kernels (experiments target, never shipped).

Builds a CorrBlock with the product library, packs a random 256 x 324 convc1
weight (dxr_conv1x1_pack_weight: f32 copy + f16-pair copy), then times
``dxr_xp_lookup_conv1x1`` of libdexiraft_corr_exp.so per kernel (0: r01 form,
1: round-2 form, 512 threads, 2: round-2 form at 1024 threads) as HIP graphs of
12 calls, and checks each against relu(conv1x1(lookup)) in float64.

Usage: python scripts/xp_motion.py [--B 1] [--H 55 --W 128] [--xp 0,1,2]
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
    ap.add_argument("--xp", default="0,1,2")
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    import dexiraft_amd
    nat = dexiraft_amd._native
    plib = nat.load()
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    fn = lib.dxr_xp_lookup_conv1x1
    fn.restype = ctypes.c_int
    fn.argtypes = [vp, i64, i64, i64, vp, vp, vp, i64, vp, ctypes.c_int, vp]
    dev = torch.device("cuda", 0)
    B, D, H, W, Cout = a.B, 256, a.H, a.W, 256
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    with torch.no_grad():
        cb = dexiraft_amd.CorrBlock(f1, f2)
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack([xs, ys])[None].repeat(B, 1, 1, 1)
    cs = [(grid + 4.0 * torch.randn(grid.shape, generator=g, device=dev)).contiguous()
          for _ in range(12)]
    wt = 0.05 * torch.randn((Cout, 324), generator=g, device=dev)
    bias = 0.1 * torch.randn((Cout,), generator=g, device=dev)
    packed = torch.empty(plib.dxr_conv1x1_packed_bytes(Cout, 324), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    assert plib.dxr_conv1x1_pack_weight(wt.data_ptr(), Cout, 324, packed.data_ptr(), s) == 0
    outs = [torch.empty((B, Cout, H, W), device=dev) for _ in range(12)]
    xps = [int(x) for x in a.xp.split(",")]

    def run(xp, k, stream):
        st = fn(cb._buf.data_ptr(), B, H, W, cs[k].data_ptr(), packed.data_ptr(), bias.data_ptr(),
                Cout, outs[k].data_ptr(), xp, stream)
        assert st == 0, (xp, st)

    with torch.no_grad():
        look = cb(cs[0]).double()
        ref = torch.relu(torch.einsum("oc,bchw->bohw", wt.double(), look) +
                         bias.double()[None, :, None, None])
    scale = ref.abs().max().item()
    for xp in xps:
        outs[0].fill_(float("nan"))
        run(xp, 0, s)
        torch.cuda.synchronize()
        err = (outs[0].double() - ref).abs().max().item() / scale
        print(json.dumps({"xp": xp, "max_err_rel_to_max": err}), flush=True)
    graphs = {}
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for xp in xps:
            run(xp, 0, side.cuda_stream)
            side.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=side):
                for k in range(12):
                    run(xp, k, torch.cuda.current_stream().cuda_stream)
            graphs[xp] = gr
    torch.cuda.synchronize()
    times = {xp: [] for xp in xps}
    for _ in range(a.rounds):
        for xp in xps:
            graphs[xp].replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                graphs[xp].replay()
            e1.record()
            torch.cuda.synchronize()
            times[xp].append(e0.elapsed_time(e1) / 60 * 1e3)
    for xp in xps:
        print(json.dumps({"xp": xp, "us_per_call": round(float(np.median(times[xp])), 2),
                          "shape": [B, H, W]}), flush=True)


if __name__ == "__main__":
    main()
