#!/usr/bin/env python3
"""Same-process A/B of the lookup backward (four coordinate sets per launch, as
the training path issues them): the previous product library's
dxr_corr_lookup_backward_multi vs this build's multi and multi_bound, and the
experiments build's multi_bound (6 waves per SIMD instead of 8).  Same
inputs; gradient pyramids checked bit-identical; graphs of --reps launches timed
with HIP events in interleaved rounds.
Usage: python scripts/ab_lookup_bw.py [--shape B H W] [--prev-lib path]
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
    ap.add_argument("--shape", type=int, nargs=3, default=[1, 55, 128])
    ap.add_argument("--radius", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--prev-lib", default=str(REPO / "scripts" / "libdexiraft_corr_prev.so"))
    a = ap.parse_args()
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    dexiraft_amd.load_native()
    lib = nat.load()
    _vp, _i64, _int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    xp = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    xp.dxr_corr_lookup_backward_multi_bound.restype = _int
    xp.dxr_corr_lookup_backward_multi_bound.argtypes = list(
        nat.SIGNATURES["dxr_corr_lookup_backward_multi_bound"][1])
    prev = ctypes.CDLL(a.prev_lib)
    prev.dxr_corr_lookup_backward_multi.restype = _int
    prev.dxr_corr_lookup_backward_multi.argtypes = list(
        nat.SIGNATURES["dxr_corr_lookup_backward_multi"][1])
    B, H, W = a.shape
    L, r = 4, a.radius
    K = L * (2 * r + 1) ** 2
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack((xs, ys))[None].expand(B, 2, H, W)
    n = 4
    cs = [(grid + 4.0 * torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous()
          for _ in range(n)]
    gs = [torch.randn((B, K, H, W), generator=g, device=dev) for _ in range(n)]
    cp = (ctypes.c_void_p * n)(*[c.data_ptr() for c in cs])
    gp = (ctypes.c_void_p * n)(*[x.data_ptr() for x in gs])
    numel = lib.dxr_pyramid_numel(B, H, W, L)
    nsl = lib.dxr_lookup_backward_bound_slots(B, H, W, L, r)
    bufs = {v: torch.zeros(numel + nsl, device=dev) for v in ("prev", "new", "bound", "bound6")}
    stream = torch.cuda.Stream(device=dev)

    def call(v):
        buf, s = bufs[v], stream.cuda_stream
        if v == "prev":
            st = prev.dxr_corr_lookup_backward_multi(cp, gp, n, B, H, W, L, r, buf.data_ptr(), 0, s)
        elif v == "new":
            st = lib.dxr_corr_lookup_backward_multi(cp, gp, n, B, H, W, L, r, buf.data_ptr(), 0, s)
        else:   # bound: this product; bound6: the experiments build (6 waves per SIMD)
            fn = lib if v == "bound" else xp
            st = fn.dxr_corr_lookup_backward_multi_bound(cp, gp, n, B, H, W, L, r, buf.data_ptr(), 0,
                                                         buf.data_ptr() + 4 * numel, s)
        assert st == 0, (v, st)

    with torch.cuda.stream(stream):
        for v in bufs:
            call(v)
        torch.cuda.synchronize()
        ref = bufs["prev"][:numel]
        for v in ("new", "bound", "bound6"):
            assert torch.equal(bufs[v][:numel], ref), v
        m = ref.abs().max().item()
        for v in ("bound", "bound6"):   # the slots bound max|G| (9 x max|grad_out| per set)
            assert bufs[v][numel:].max().item() >= m, v
        assert torch.equal(bufs["bound"][numel:], bufs["bound6"][numel:])
        graphs = {}
        for v in bufs:
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
    print(json.dumps({"shape": [B, H, W], "radius": r, "sets_per_launch": n,
                      "us_per_launch_min_med": {v: [round(min(x), 1), round(float(np.median(x)), 1)]
                                                for v, x in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
