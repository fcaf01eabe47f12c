#!/usr/bin/env python3
"""A/B of the two fmap-gradient arithmetics in one process: dxr_fmap_grads
(six bf16 products) vs dxr_fmap_grads_bounded (f16 pairs, three products), same
random gradient pyramid and fmaps, graphs of --reps calls replayed in
interleaved rounds, timed with HIP events.  Also prints both results' max error
against a float64 reference of dfmap1 (volume gradient + GEMM).
With --prev-lib, the same two entry points of an earlier product library run
beside them ("six_prev", "f16_prev") and their outputs must equal this
library's bit for bit.
Usage: python scripts/ab_fmap_grads.py [--shape B D H W L] [--reps 10] [--rounds 7] [--prev-lib X.so]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=5, default=[1, 256, 55, 128, 4])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--prev-lib", default=None)
    a = ap.parse_args()
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    dexiraft_amd.load_native()
    lib = nat.load()
    import ctypes
    prev = None
    if a.prev_lib:
        prev = ctypes.CDLL(a.prev_lib)
        for name, (res, args) in nat.SIGNATURES.items():
            if hasattr(prev, name):
                getattr(prev, name).restype = res
                getattr(prev, name).argtypes = args
    B, D, H, W, L = a.shape
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    numel = lib.dxr_pyramid_numel(B, H, W, L)
    gp = torch.zeros(numel, device=dev)
    h, w = H, W
    for lvl in range(L):
        if lvl:
            h, w = h // 2, w // 2
        ref = torch.randn((B * H * W, h, w), generator=g, device=dev) * 1e-3
        nat.check(lib.dxr_pyramid_pack(ref.data_ptr(), B, H, W, L, lvl, gp.data_ptr(), nat.DXR_F32,
                                       nat.stream_of(ref)), "pack")
    slots = gp.abs().max().reshape(1).contiguous()
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    div = float(np.sqrt(np.float32(D)))
    wsb = lib.dxr_fmap_grads_workspace_bytes(B, D, H, W, L)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    names = ("six", "f16") + (("six_prev", "f16_prev") if prev else ())
    outs = {v: (torch.empty_like(f1), torch.empty_like(f2)) for v in names}
    stream = torch.cuda.Stream(device=dev)

    def call(v):
        d1, d2 = outs[v]
        s = stream.cuda_stream
        L_ = prev if v.endswith("_prev") else lib
        if v.startswith("six"):
            st = L_.dxr_fmap_grads(gp.data_ptr(), nat.DXR_F32, f1.data_ptr(), f2.data_ptr(), B, D, H,
                                    W, L, div, d1.data_ptr(), d2.data_ptr(), ws.data_ptr(), wsb, s)
        else:
            st = L_.dxr_fmap_grads_bounded(gp.data_ptr(), nat.DXR_F32, f1.data_ptr(), f2.data_ptr(),
                                            B, D, H, W, L, div, slots.data_ptr(), 1, d1.data_ptr(),
                                            d2.data_ptr(), ws.data_ptr(), wsb, s)
        assert st == 0, (v, st)

    graphs = {}
    with torch.cuda.stream(stream):
        for v in outs:
            call(v)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=stream):
                for _ in range(a.reps):
                    call(v)
            graphs[v] = gr
        for _ in range(3):
            for gr in graphs.values():
                gr.replay()
        torch.cuda.synchronize()
        res = {v: [] for v in graphs}
        for _ in range(a.rounds):
            for v, gr in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                gr.replay()
                e1.record(stream)
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    if prev:
        for v in ("six", "f16"):
            for x, y in zip(outs[v], outs[v + "_prev"]):
                assert torch.equal(x, y), f"{v}: not bit-identical to --prev-lib"
    # accuracy of dfmap1 against float64 (pair 0)
    dv = torch.empty((B, H * W, H * W), device=dev)
    nat.check(lib.dxr_pyramid_backward(gp.data_ptr(), nat.DXR_F32, B, H, W, L, div, dv.data_ptr(),
                                       nat.stream_of(dv)), "pyramid_backward")
    r1 = torch.mm(f2[0].reshape(D, -1).double(), dv[0].double().t())
    err = {v: (outs[v][0][0].reshape(D, -1).double() - r1).abs().max().item() for v in outs}
    print(json.dumps({"shape": a.shape, "us_min_med": {v: [round(min(x), 1), round(float(np.median(x)), 1)]
                                                       for v, x in res.items()},
                      "dfmap1_maxerr": {v: float(f"{e:.3e}") for v, e in err.items()},
                      "dfmap1_max": float(f"{r1.abs().max().item():.3e}")}), flush=True)


if __name__ == "__main__":
    main()
