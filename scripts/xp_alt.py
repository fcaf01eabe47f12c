#!/usr/bin/env python3
"""Timing of on-the-fly (AlternateCorrBlock) lookup kernels (experiments target).

Builds an AlternateCorrBlock with the product library (its NHWC fmap and pooled
fmap2 levels), then times ``dxr_xp_alt`` of libdexiraft_corr_exp.so per kernel
(0: 4x8-box 32x32x16 form, 1/2: grouped 16x16x32 form) over 12 coordinate sets,
rounds interleaved, and reports each variant's max deviation from variant 0
relative to max|out| (different MFMA shapes sum in different orders).

Usage: python scripts/xp_alt.py [--H 136 --W 240] [--xp 0,1,2]
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
    ap.add_argument("--H", type=int, default=136)
    ap.add_argument("--W", type=int, default=240)
    ap.add_argument("--xp", default="0,1,2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--smooth", type=int, default=0,
                    help="flow correlation length in pixels (0: i.i.d. N(0, 4^2) per pixel, the "
                         "bench's model; S > 0: a N(0, 4^2) field on an S-pixel grid, bilinearly "
                         "upsampled — spatially smooth like real optical flow)")
    a = ap.parse_args()
    import dexiraft_amd
    nat = dexiraft_amd._native
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    fn = lib.dxr_xp_alt
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                   ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    B, H, W, D = a.B, a.H, a.W, 256
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    with torch.no_grad():
        ab = dexiraft_amd.AlternateCorrBlock(f1, f2)
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack((xs, ys))[None].expand(B, 2, H, W)
    def flow():
        if a.smooth <= 0:
            return 4.0 * torch.randn((B, 2, H, W), generator=g, device=dev)
        hs, ws = max(2, H // a.smooth + 1), max(2, W // a.smooth + 1)
        coarse = 4.0 * torch.randn((B, 2, hs, ws), generator=g, device=dev)
        return torch.nn.functional.interpolate(coarse, size=(H, W), mode="bilinear",
                                               align_corners=True)

    cs = [(grid + flow()).contiguous() for _ in range(12)]
    outs = [torch.empty((B, 324, H, W), device=dev) for _ in range(12)]
    s = torch.cuda.current_stream().cuda_stream
    xps = [int(x) for x in a.xp.split(",")]

    def run(xp, k):
        st = fn(ab._f1_nhwc.data_ptr(), ab._f2_ptrs, cs[k].data_ptr(), outs[k].data_ptr(), B, H, W,
                D, 4, 16.0, xp, s)
        if st != 0:
            raise RuntimeError(f"xp {xp}: status {st}")

    run(0, 0)
    torch.cuda.synchronize()
    ref = outs[0].clone()
    with torch.no_grad():
        prod = ab(cs[0])
    print(json.dumps({"xp0_vs_product_bit_identical": bool(torch.equal(prod, ref))}), flush=True)
    for xp in xps:
        outs[0].fill_(float("nan"))
        run(xp, 0)
        torch.cuda.synchronize()
        dev_rel = ((outs[0] - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps({"xp": xp, "max_rel_dev_vs_xp0": dev_rel}), flush=True)
    if 50 in xps:   # the binned form's per-level order choice (spatial box cost, flag)
        run(50, 0)
        run(55, 0)
        torch.cuda.synchronize()
        print(json.dumps({"bin_decisions": outs[0].flatten()[:8].tolist()}), flush=True)
    times = {xp: [] for xp in xps}
    for _ in range(a.rounds):
        for xp in xps:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(12):
                run(xp, k)
            e1.record()
            torch.cuda.synchronize()
            times[xp].append(e0.elapsed_time(e1) / 12 * 1e3)
    flops = 2.0 * B * H * W * 4 * 100 * D
    for xp in xps:
        med = float(np.median(times[xp]))
        print(json.dumps({"xp": xp, "us_median": round(med, 2), "us_min": round(min(times[xp]), 2),
                          "alg_tflops": round(flops / med / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
