#!/usr/bin/env python3
"""Lookup timing ablations and timeline (experiments target, never shipped).

Builds a Sintel-shape pyramid with the product CorrBlock, then times variants of
the lookup from libdexiraft_corr_exp.so (csrc/experiments/xp_lookup.hip,
``dxr_xp_lookup``) in interleaved rounds of back-to-back launches (HIP events,
one launch plus its same-stream boundary), and optionally records a per-
workgroup timeline (s_memrealtime, 100 MHz) of one launch.

Usage: python scripts/xp_lookup.py [--batch 8] [--xp 0 4 1 2 8] [--trace]
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
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--hw", type=int, nargs=2, default=[55, 128])
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--xp", type=int, nargs="+", default=[0, 32, 64, 128, 4, 1])
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--trace", action="store_true")
    a = ap.parse_args()

    import dexiraft_amd
    from dexiraft_amd import _native as nat
    dexiraft_amd.load_native()
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.dxr_xp_lookup.restype = i32
    lib.dxr_xp_lookup.argtypes = [vp, i32, i64, i64, i64, i32, vp, vp, i32, vp, vp]

    dev = torch.device("cuda", 0)
    B, (H, W), D = a.batch, a.hw, 256
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    if a.dtype == "bf16":
        f1, f2 = f1.bfloat16(), f2.bfloat16()
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack((xs, ys))[None].expand(B, 2, H, W)
    coords = (grid + 4.0 * torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous()
    cb = dexiraft_amd.CorrBlock(f1, f2)
    ref = cb(coords)
    out = torch.empty_like(ref)
    nwg = ((H * W + 31) // 32) * 4 * B
    trace = torch.zeros(nwg * 5, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    pdt = 0 if a.dtype == "f32" else 1

    def launch(xp):
        st = lib.dxr_xp_lookup(cb._buf.data_ptr(), pdt, B, H, W, 4, coords.data_ptr(),
                               out.data_ptr(), xp, trace.data_ptr(), stream)
        assert st == 0, st

    for x in (0, 16, 32, 64, 128):
        out.zero_()
        launch(x)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), f"variant {x} must equal the product lookup"
    # clock warm-up
    for _ in range(2000):
        launch(0)
    torch.cuda.synchronize()
    res = {x: [] for x in a.xp}
    for _ in range(a.rounds):
        for x in a.xp:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                launch(x)
            e1.record()
            torch.cuda.synchronize()
            res[x].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    print(json.dumps({"shape": [B, H, W], "dtype": a.dtype,
                      "us_per_launch": {x: [round(min(v), 2), round(float(np.median(v)), 2)]
                                        for x, v in res.items()}}))
    if a.trace:
        for x in (256, 260, 258):
            for _ in range(50):
                launch(0)
            launch(x)
            torch.cuda.synchronize()
            t = trace.view(nwg, 5).cpu().numpy().astype(np.int64)
            t0 = t[:, 0].min()
            s = (t[:, :4] - t0) * 10.0 / 1e3          # 100 MHz ticks -> us
            lvl = (np.arange(nwg) // ((H * W + 31) // 32)) % 4
            summ = {"variant": x, "span_us": round(float(s[:, 3].max()), 2),
                    "start_p50_p100": [round(float(np.percentile(s[:, 0], q)), 2) for q in (50, 100)],
                    "phase0_p50_p90": [round(float(np.percentile(s[:, 1] - s[:, 0], q)), 2) for q in (50, 90)],
                    "gather_p50_p90": [round(float(np.percentile(s[:, 2] - s[:, 1], q)), 2) for q in (50, 90)],
                    "phase2_p50_p90": [round(float(np.percentile(s[:, 3] - s[:, 2], q)), 2) for q in (50, 90)],
                    "end_by_level": [round(float(s[lvl == k, 3].max()), 2) for k in range(4)]}
            print(json.dumps(summ))


if __name__ == "__main__":
    main()
