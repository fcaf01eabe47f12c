#!/usr/bin/env python3
"""Timing ablations / variants of the lookup (experiments target, never shipped).

Builds one pyramid with the product library, then times ``dxr_xp_lookup`` of
libdexiraft_corr_exp.so per variant (csrc/corr_lookup.hip XP bits: 1 no window
gathers, 2 no output stores, 4 phase 0 only; variants >= 100 are alternative
kernels) with HIP events over K back-to-back launches (12 coordinate sets),
rounds interleaved.  ``--check`` variants must equal variant 0 bit for bit.

Usage: python scripts/xp_lookup.py [--B 8] [--H 55 --W 128] [--dtype f32|bf16] [--xp 0,1,2]
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
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--xp", default="0,1,2,3,4")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--check", default="")
    a = ap.parse_args()
    import dexiraft_amd
    nat = dexiraft_amd._native
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    fn = lib.dxr_xp_lookup
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    B, H, W, D = a.B, a.H, a.W, 256
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    if a.dtype == "bf16":
        f1, f2 = f1.bfloat16(), f2.bfloat16()
    with torch.no_grad():
        cb = dexiraft_amd.CorrBlock(f1, f2)
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack((xs, ys))[None].expand(B, 2, H, W)
    cs = [(grid + 4.0 * torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous()
          for _ in range(12)]
    outs = [torch.empty((B, 324, H, W), device=dev) for _ in range(12)]
    s = torch.cuda.current_stream().cuda_stream
    pdt = nat.DXR_BF16 if a.dtype == "bf16" else nat.DXR_F32
    xps = [int(x) for x in a.xp.split(",")]

    def run(xp, k):
        st = fn(cb._buf.data_ptr(), pdt, B, H, W, cs[k].data_ptr(), outs[k].data_ptr(), xp, s)
        if st != 0:
            raise RuntimeError(f"xp {xp}: status {st}")

    if a.check:
        run(0, 0)
        torch.cuda.synchronize()
        ref = outs[0].clone()
        for xp in (int(x) for x in a.check.split(",")):
            outs[0].fill_(float("nan"))
            run(xp, 0)
            torch.cuda.synchronize()
            print(json.dumps({"xp": xp, "bit_identical_to_xp0": bool(torch.equal(outs[0], ref))}),
                  flush=True)
    times = {xp: [] for xp in xps}
    for _ in range(25):          # clock warm-up (~0.1-0.5 s of launches)
        for xp in xps:
            for k in range(12):
                run(xp, k)
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for xp in xps:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(12):
                run(xp, k)
            e1.record()
            torch.cuda.synchronize()
            times[xp].append(e0.elapsed_time(e1) / 12 * 1e3)
    rd = 9
    s_pyr = 2 if a.dtype == "bf16" else 4
    lv = [(H, W)]
    for _ in range(3):
        lv.append((lv[-1][0] // 2, lv[-1][1] // 2))
    win = sum(min(rd + 1, h) * min(rd + 1, w) for h, w in lv)
    nbytes = B * H * W * (win * s_pyr + 8 + 4 * rd * rd * 4)
    for xp in xps:
        med = float(np.median(times[xp]))
        print(json.dumps({"xp": xp, "us_median": round(med, 2), "us_min": round(min(times[xp]), 2),
                          "alg_TBps": round(nbytes / med / 1e6, 3), "B": B, "dtype": a.dtype}),
              flush=True)


if __name__ == "__main__":
    main()
