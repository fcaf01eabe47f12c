#!/usr/bin/env python3
"""Pre-split f32 build: timing ablations and per-page timeline (experiments target).

Variants of csrc/experiments/xp_build.hip (``dxr_xp_build``; each launch = the
split pass + the build): 0 product, 1 no epilogue stores, 2 no MFMAs, 3 both,
32 the split pass with plain stores; 256 / 257 record {start, K loop done, stores done} per
workgroup (two pages; s_memrealtime, 100 MHz).  Interleaved rounds of graphs of --reps
launches, HIP events.
Usage: python scripts/xp_build.py [--shape 1x55x128] [--xp 0 1 2 4 5]
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
    ap.add_argument("--xp", type=int, nargs="+", default=[0, 32, 1, 2, 3, 4, 5])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--split", type=int, nargs="*", default=[0, 1, 2, 3, 4],
                    help="split-pass variants timed alone (dxr_xp_split)")
    ap.add_argument("--trace-xp", type=int, nargs="*", default=[256, 257],
                    help="traced variants (bit 8 set): per-workgroup timeline summary")
    a = ap.parse_args()
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    plib = dexiraft_amd.load_native()
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.dxr_xp_build.restype = i32
    lib.dxr_xp_build.argtypes = [vp, vp, i64, i64, i64, i64, vp, vp, i32, vp, vp]
    lib.dxr_xp_split.restype = i32
    lib.dxr_xp_split.argtypes = [vp, vp, i64, i64, i64, i64, vp, i32, vp]
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
    npages = B * ((qt + 1) // 2) * tiles          # workgroups: two query blocks each
    trace = torch.zeros(npages * 4, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)

    def launch(x):
        st = lib.dxr_xp_build(f1.data_ptr(), f2.data_ptr(), B, D, H, W, pyr.data_ptr(),
                              ws.data_ptr(), x, trace.data_ptr(), stream.cuda_stream)
        assert st == 0, (x, st)

    # variant 0 must reproduce the product build
    ref = torch.empty_like(pyr)
    cb = dexiraft_amd.CorrBlock(f1, f2)
    ref.copy_(cb._buf)
    with torch.cuda.stream(stream):
        launch(0)
    torch.cuda.synchronize()
    assert torch.equal(pyr, ref), "variant 0 differs from the product build"
    graphs = {}
    with torch.cuda.stream(stream):
        for x in a.xp:
            launch(x)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=stream):
                for _ in range(a.reps):
                    launch(x)
            graphs[x] = gr
        for _ in range(10):
            for x in a.xp:
                graphs[x].replay()
        torch.cuda.synchronize()
        res = {x: [] for x in a.xp}
        for _ in range(a.rounds):
            for x in a.xp:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                graphs[x].replay()
                e1.record(stream)
                torch.cuda.synchronize()
                res[x].append(e0.elapsed_time(e1) * 1e3 / a.reps)
        print(json.dumps({"shape": [B, D, H, W], "us_per_launch_min_med":
                          {x: [round(min(v), 1), round(float(np.median(v)), 1)] for x, v in res.items()}}),
              flush=True)
        if a.split:
            ref_ws = None
            sg = {}
            for v in a.split:
                assert lib.dxr_xp_split(f1.data_ptr(), f2.data_ptr(), B, D, H, W, ws.data_ptr(), v,
                                        stream.cuda_stream) == 0
                torch.cuda.synchronize()
                if ref_ws is None:
                    ref_ws = ws.clone()
                assert torch.equal(ws, ref_ws), f"split variant {v} differs"
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=stream):
                    for _ in range(a.reps):
                        lib.dxr_xp_split(f1.data_ptr(), f2.data_ptr(), B, D, H, W, ws.data_ptr(), v,
                                         stream.cuda_stream)
                sg[v] = gr
            sres = {v: [] for v in a.split}
            for _ in range(a.rounds):
                for v in a.split:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    sg[v].replay()
                    e1.record(stream)
                    torch.cuda.synchronize()
                    sres[v].append(e0.elapsed_time(e1) * 1e3 / a.reps)
            print(json.dumps({"split_us_min_med": {v: [round(min(t), 2), round(float(np.median(t)), 2)]
                                                   for v, t in sres.items()}}), flush=True)
        for x in a.trace_xp:
            for _ in range(3):
                graphs[a.xp[0]].replay()
            launch(x)
            torch.cuda.synchronize()
            t = trace.view(npages, 4).cpu().numpy().astype(np.int64)
            t0 = t[:, 0].min()
            s = (t[:, :3] - t0) * 10.0 / 1e3
            kl, ep = s[:, 1] - s[:, 0], s[:, 2] - s[:, 1]
            cu = (t[:, 3] & 0xFFFFFFFF)
            print(json.dumps({
                "variant": x, "span_us": round(float(s[:, 2].max()), 2),
                "kloop_p10_p50_p90": [round(float(np.percentile(kl, q)), 2) for q in (10, 50, 90)],
                "epilogue_p10_p50_p90": [round(float(np.percentile(ep, q)), 2) for q in (10, 50, 90)],
                "first_round_end_p50": round(float(np.percentile(s[:512, 2], 50)), 2),
                "distinct_hw_ids": int(len(np.unique(cu)))}), flush=True)
            # co-residence of the first dispatch round: workgroups that started
            # within 2 us of the first, grouped by CU (xcc, se, sh, cu of HW_ID)
            hw = t[:, 3]
            key = ((hw >> 32) & 7) * 4096 + ((hw >> 8) & 0xFF)
            first = np.where(s[:, 0] < 2.0)[0]
            groups = {}
            for wg in first:
                groups.setdefault(int(key[wg]), []).append(int(wg))
            d = [g2[1] - g2[0] for g2 in groups.values() if len(g2) == 2]
            print(json.dumps({"variant": x, "first_round_wgs": int(len(first)),
                              "cus": len(groups),
                              "pair_blockidx_delta_hist": {str(k): int(v) for k, v in
                                                           zip(*np.unique(d, return_counts=True))}
                              if d else {}}), flush=True)


if __name__ == "__main__":
    main()
