#!/usr/bin/env python3
"""Host cost per CorrBlock call (profiles only): how long the Python + C-ABI
path takes to enqueue one lookup, against the kernel's own time.

Eager training (scripts/time_backward.py) launches every lookup from Python;
when the host needs longer per call than the GPU per kernel, the step is
host-bound.  Times, per call, with the GPU kept busy by a long queue (no sync
inside the timed loop; the queue is drained before and after):
  empty          torch.empty of one lookup output
  stream         torch.cuda.current_stream(dev).cuda_stream
  ctypes         dxr_corr_lookup through ctypes alone (the kernel enqueue)
  lookup_nograd  CorrBlock.__call__ under no_grad
  lookup_grad    CorrBlock.__call__ with a differentiable block (autograd node)
Usage: python scripts/probe_host_overhead.py [--calls 2000]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    a = ap.parse_args()
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    lib = dexiraft_amd.load_native()
    dev = torch.device("cuda", 0)
    B, D, H, W = 1, 256, 55, 128
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    c = (torch.stack((xs, ys))[None] + 4.0 * torch.randn((B, 2, H, W), generator=g,
                                                         device=dev)).contiguous()
    with torch.no_grad():
        cb = dexiraft_amd.CorrBlock(f1, f2)
    a1, a2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
    cbg = dexiraft_amd.CorrBlock(a1, a2)
    out = torch.empty((B, 324, H, W), device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    n = a.calls

    def per_call(fn, kernel):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        host = (time.perf_counter() - t0) / n * 1e6
        e1.record()
        torch.cuda.synchronize()
        gpu = e0.elapsed_time(e1) * 1e3 / n if kernel else None
        return {"host_us_per_call": round(host, 2),
                "gpu_us_per_call": None if gpu is None else round(gpu, 2)}

    res = {}
    res["empty"] = per_call(lambda: torch.empty((B, 324, H, W), device=dev), False)
    res["stream"] = per_call(lambda: torch.cuda.current_stream(dev).cuda_stream, False)
    res["ctypes"] = per_call(lambda: lib.dxr_corr_lookup(cb._buf.data_ptr(), nat.DXR_F32, B, H, W,
                                                         4, 4, c.data_ptr(), out.data_ptr(), st),
                             True)
    with torch.no_grad():
        res["lookup_nograd"] = per_call(lambda: cb(c), True)
    outs = []

    def grad_call():
        outs.append(cbg(c))
        if len(outs) > 64:
            outs.clear()
    res["lookup_grad"] = per_call(grad_call, True)
    print(json.dumps({"what": "host and GPU time per call, Sintel B=1 lookups enqueued back to back",
                      **res}), flush=True)


if __name__ == "__main__":
    main()
