#!/usr/bin/env python3
"""Per-level cost of the ordered on-the-fly lookup (profiles only).

Times 12 ordered on-the-fly lookups (dxr_alt_corr_lookup_ws, the product's form,
the bench's i.i.d. N(0, 4^2) coordinates) as one HIP graph with num_levels =
1 .. 4 (levels 0 .. L-1 of the same pooled fmap2), interleaved rounds, HIP
events — T(L) - T(L-1) is what level L-1 adds per 12 lookups: its ordering
launches' share, its query loads and splits, its box GEMMs and its stores.
Usage: python scripts/probe_alt_levels.py [--workload 1080p] [--rounds 7]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

SHAPES = {"sintel": (55, 128), "1080p": (136, 240)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="1080p", choices=sorted(SHAPES))
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import dexiraft_amd
    lib = dexiraft_amd.load_native()
    dev = torch.device("cuda", 0)
    B, (H, W), D = 1, SHAPES[a.workload], 256
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack((xs, ys))[None].expand(B, 2, H, W)
    coords = [(grid + 4.0 * torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous()
              for _ in range(12)]
    stream = torch.cuda.Stream(device=dev)
    res, graphs = {}, {}
    with torch.no_grad(), torch.cuda.stream(stream):
        ab = dexiraft_amd.AlternateCorrBlock(f1, f2)
        for L in (1, 2, 3, 4):
            nws = lib.dxr_alt_workspace_bytes(B, H, W, L)
            ws = torch.empty(nws, dtype=torch.uint8, device=dev)
            outs = [torch.empty((B, L * 81, H, W), device=dev) for _ in coords]

            def run(L=L, ws=ws, nws=nws, outs=outs):
                for c, o in zip(coords, outs):
                    st = lib.dxr_alt_corr_lookup_ws(ab._f1_nhwc.data_ptr(), ab._f2_ptrs,
                                                    c.data_ptr(), o.data_ptr(), B, H, W, D, L, 4,
                                                    16.0, ws.data_ptr(), nws, stream.cuda_stream)
                    assert st == 0
            run()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=stream):
                run()
            graphs[L] = (gr, ws, outs)
            res[L] = []
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            for gr, _, _ in graphs.values():
                gr.replay()
            torch.cuda.synchronize()
        for _ in range(a.rounds):
            for L, (gr, _, _) in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    gr.replay()
                e1.record(stream)
                torch.cuda.synchronize()
                res[L].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    med = {L: round(float(np.median(v)), 1) for L, v in res.items()}
    print(json.dumps({"workload": a.workload, "us_per_12_lookups_median_by_levels": med,
                      "us_added_per_lookup_by_level": {
                          l: round((med[l + 1] - (med[l] if l else 0.0)) / 12, 1)
                          for l in range(4)}}), flush=True)


if __name__ == "__main__":
    main()
