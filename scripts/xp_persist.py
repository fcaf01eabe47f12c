#!/usr/bin/env python3
"""Persistent f32 build A/B (experiments target, csrc/experiments/xp_build.hip).

Variants, each = split pass + build, captured as graphs of --reps launches and
timed in interleaved rounds (HIP events), outputs checked bit-identical to the
product build:
  prod            dxr_xp_build variant 0 (the product kernel, one workgroup per unit)
  p<nwg>          persistent, nwg workgroups
  p<nwg>s<ticks>  persistent with the upper half of each XCD's slots delayed
                  by <ticks> x 10 ns
  ...L            (prodL, p<nwg>L...) the next DMAs issued behind the first tile's
                  MFMAs instead of before the fragment reads
Then a per-unit timeline (s_memrealtime) of the fastest persistent variant.
Usage: python scripts/xp_persist.py [--shape 1x55x128] [--variants prod p512 p512s800]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import re
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="1x55x128")
    ap.add_argument("--variants", nargs="+",
                    default=["prod", "prodL", "p512", "p512L", "p512s500", "p512s1000",
                             "p512s1500", "p512Ls1000"])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--trace", default="p512")
    a = ap.parse_args()
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    plib = dexiraft_amd.load_native()
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.dxr_xp_build.restype = i32
    lib.dxr_xp_build.argtypes = [vp, vp, i64, i64, i64, i64, vp, vp, i32, vp, vp]
    lib.dxr_xp_build_persist.restype = i32
    lib.dxr_xp_build_persist.argtypes = [vp, vp, i64, i64, i64, i64, vp, vp, i32, i32, i32, vp, vp]
    dev = torch.device("cuda", 0)
    B, H, W = (int(v) for v in a.shape.split("x"))
    D = 256
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    pyr = torch.empty(plib.dxr_pyramid_numel(B, H, W, 4), device=dev)
    ws = torch.empty(plib.dxr_build_workspace_bytes(nat.DXR_F32, B, D, H, W), dtype=torch.uint8,
                     device=dev)
    qt, tiles = (H * W + 127) // 128, ((H + 7) // 8) * ((W + 15) // 16)
    nunits = B * ((qt + 1) // 2) * tiles
    trace = torch.zeros(nunits * 4, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)

    def parse(v):
        m = re.fullmatch(r"p(\d+)(L?)(?:s(\d+))?", v)
        return int(m.group(1)), int(m.group(3) or 0), bool(m.group(2))

    def launch(v, tr=False):
        s = stream.cuda_stream
        if v in ("prod", "prodL"):
            st = lib.dxr_xp_build(f1.data_ptr(), f2.data_ptr(), B, D, H, W, pyr.data_ptr(),
                                  ws.data_ptr(), 16 if v == "prodL" else 0, None, s)
        else:
            nwg, stag, late = parse(v)
            xp = (2 if stag else 0) | (256 if tr else 0) | (16 if late else 0)
            st = lib.dxr_xp_build_persist(f1.data_ptr(), f2.data_ptr(), B, D, H, W, pyr.data_ptr(),
                                          ws.data_ptr(), xp, nwg, stag, trace.data_ptr(), s)
        assert st == 0, (v, st)

    ref = dexiraft_amd.CorrBlock(f1, f2)._buf.clone()
    graphs = {}
    with torch.cuda.stream(stream):
        for v in a.variants:
            pyr.fill_(float("nan"))
            launch(v)
            torch.cuda.synchronize()
            assert torch.equal(pyr, ref), f"{v} differs from the product build"
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=stream):
                for _ in range(a.reps):
                    launch(v)
            graphs[v] = gr
        t_end = __import__("time").perf_counter() + 0.5
        while __import__("time").perf_counter() < t_end:
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
        print(json.dumps({"shape": [B, D, H, W], "units": nunits,
                          "us_per_build_incl_split_min_med":
                              {v: [round(min(x), 1), round(float(np.median(x)), 1)]
                               for v, x in res.items()}}), flush=True)
        if a.trace:
            for tv in [a.trace] + ([a.trace + "s1000"] if "s" not in a.trace else []):
                for _ in range(3):
                    graphs[a.variants[0]].replay()
                trace.zero_()
                launch(tv, tr=True)
                torch.cuda.synchronize()
                t = trace.view(nunits, 4).cpu().numpy().astype(np.int64)
                t0 = t[:, 0].min()
                s = (t[:, :3] - t0) * 10.0 / 1e3
                kl, ep = s[:, 1] - s[:, 0], s[:, 2] - s[:, 1]
                ends = np.sort(s[:, 2])
                print(json.dumps({
                    "trace_variant": tv, "span_us": round(float(ends[-1]), 2),
                    "end_p50_p90_p99": [round(float(np.percentile(ends, q)), 2) for q in (50, 90, 99)],
                    "kloop_p10_p50_p90": [round(float(np.percentile(kl, q)), 2) for q in (10, 50, 90)],
                    "epilogue_p10_p50_p90": [round(float(np.percentile(ep, q)), 2) for q in (10, 50, 90)],
                    "units_ending_after_90pct_span": int((ends > 0.9 * ends[-1]).sum()),
                }), flush=True)


if __name__ == "__main__":
    main()
