#!/usr/bin/env python3
"""Timing ablations of the split build (experiments target, never shipped).

Loads optical-flow_dexi-raft_amd/libdexiraft_corr_exp.so (build.py --experiments)
and times ``dxr_xp_build`` per ablation mask (csrc/corr_build.hip
corr_build_split_kernel XP bits: 1 no epilogue stores, 2 no MFMAs, 4 no in-loop
global loads, 8 no operand split, 16 no in-loop barrier) with HIP events over
K back-to-back launches into one pyramid buffer, rounds interleaved so every
variant sees the same clock/thermal history.  Prints one JSON line per variant.

Usage: python scripts/xp_build.py [--B 1] [--H 55 --W 128] [--xp 0,1,2,...]
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
    ap.add_argument("--D", type=int, default=256)
    ap.add_argument("--xp", default="0,1,2,3,4,5,8,16,19")
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--check", default="", help="variants whose pyramid must equal --ref's bit for bit")
    ap.add_argument("--ref", type=int, default=0, help="reference variant of --check")
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"],
                    help="bf16: the bf16 build (dxr_xp_build_bf16) instead of the split build")
    a = ap.parse_args()
    import dexiraft_amd
    nat = dexiraft_amd._native
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    fn = lib.dxr_xp_build_bf16 if a.dtype == "bf16" else lib.dxr_xp_build
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                   ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    B, D, H, W = a.B, a.D, a.H, a.W
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    if a.dtype == "bf16":
        f1, f2 = f1.bfloat16(), f2.bfloat16()
    pyr = torch.empty(nat.load().dxr_pyramid_numel(B, H, W, 4), device=dev,
                      dtype=torch.bfloat16 if a.dtype == "bf16" else torch.float32)
    s = torch.cuda.current_stream().cuda_stream
    xps = [int(x) for x in a.xp.split(",")]

    def launch(xp):
        st = fn(f1.data_ptr(), f2.data_ptr(), B, D, H, W, pyr.data_ptr(), xp, s)
        if st != 0:
            raise RuntimeError(f"xp {xp}: status {st}")

    ref = None
    if a.check:
        pyr.fill_(float("nan"))
        launch(a.ref)
        torch.cuda.synchronize()
        ref = pyr.clone()
        for xp in (int(x) for x in a.check.split(",")):
            pyr.fill_(float("nan"))
            launch(xp)
            torch.cuda.synchronize()
            same = torch.equal(pyr, ref)
            diff = (pyr - ref).abs().nan_to_num(nan=float("inf")).max().item()
            print(json.dumps({"xp": xp, "ref": a.ref, "bit_identical_to_ref": same, "max_abs_diff": diff}),
                  flush=True)
    for xp in xps:
        launch(xp)
    torch.cuda.synchronize()
    times = {xp: [] for xp in xps}
    for _ in range(a.rounds):
        for xp in xps:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            launch(xp)
            e0.record()
            for _ in range(a.launches):
                launch(xp)
            e1.record()
            torch.cuda.synchronize()
            times[xp].append(e0.elapsed_time(e1) / a.launches * 1e3)
    flops = 2.0 * B * (H * W) ** 2 * D
    for xp in xps:
        med = float(np.median(times[xp]))
        print(json.dumps({"xp": xp, "us_median": round(med, 2),
                          "us_min": round(min(times[xp]), 2),
                          "f32eq_tflops": round(flops / med / 1e6, 1),
                          "shape": [B, D, H, W]}), flush=True)


if __name__ == "__main__":
    main()
