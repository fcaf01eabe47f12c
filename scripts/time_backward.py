#!/usr/bin/env python3
"""Training-path timing of the correlation block.

One training step of the correlation path = CorrBlock(fmap1, fmap2) with fmaps
that require grad + 12 lookups + backward of sum_k <w_k, lookup_k> (train.py:175-178
backpropagates through the same ops).  Times the forward, the whole step, and the
backward's pieces (12 dxr_corr_lookup_backward, then dxr_fmap_grads: two fused
fmap GEMMs that fold the gradient pyramid in their operand loads) with HIP events,
and reports the peak memory of the step.

Usage: python scripts/time_backward.py [--workload sintel|chairs] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="sintel", choices=["sintel", "chairs"])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--loss", default="vdot", choices=["vdot", "mulsum"])
    ap.add_argument("--clone-inputs", action="store_true")
    ap.add_argument("--bw-sets", type=int, default=None,
                    help="lookup backwards per launch (corr._BW_SETS; the pending output "
                         "gradients of that many lookups are held until their launch)")
    ap.add_argument("--no-breakdown", action="store_true",
                    help="skip the torch-profiler kernel breakdown (under rocprofv3)")
    a = ap.parse_args()
    import dexiraft_amd
    if a.bw_sets is not None:
        sys.modules["dexiraft_amd.corr"]._BW_SETS = a.bw_sets
    dev = torch.device("cuda", 0)
    H, W = {"sintel": (55, 128), "chairs": (46, 62)}[a.workload]
    B, D = 1, 256
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack([xs, ys])[None]
    coords = [grid + 4.0 * torch.randn(grid.shape, generator=g, device=dev) for _ in range(12)]
    wts = [torch.randn((B, 324, H, W), generator=g, device=dev) for _ in range(12)]

    def forward_loss(a1, a2):
        # the block is a local of the forward pass, as corr_fn in RAFT.forward
        # (core/raft.py:101,147): it is gone when loss.backward() runs
        cb = dexiraft_amd.CorrBlock(a1, a2)
        loss = 0.0
        for c, w in zip(coords, wts):
            out = cb(c)
            # the stand-in for the update block: <w_k, lookup_k>.  --loss mulsum
            # (rounds 1-4) as a multiply, a sum and their backwards; vdot one
            # fused reduction whose backward is w_k * grad (the same gradients)
            loss = loss + ((out * w).sum() if a.loss == "mulsum" else
                           torch.vdot(out.reshape(-1), w.reshape(-1)))
        return loss

    # the fmaps are the encoders' outputs (core/raft.py:139-142), allocated before
    # the correlation path runs: leaves that persist across steps, so the peak
    # below is the path's own extra memory (--clone-inputs: rounds 1-4, a fresh
    # clone of both per step inside the measured window, 13.8 MB at Sintel)
    a1p, a2p = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)

    def step(backward=True):
        if a.clone_inputs:
            a1, a2 = f1.clone().requires_grad_(True), f2.clone().requires_grad_(True)
        else:
            a1, a2 = a1p, a2p
            a1.grad = a2.grad = None      # the gradients are this step's outputs
        loss = forward_loss(a1, a2)
        if backward:
            loss.backward()
        return a1, a2

    for _ in range(2):
        step()
    a1p.grad = a2p.grad = None          # the fmap gradients count as the step's memory
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()

    def timed(fn):
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    t_fwd = timed(lambda: step(False))
    t_step = timed(step)
    peak = torch.cuda.max_memory_allocated() - base
    # kernel breakdown of one step from the profiler
    kern = {}
    events = []
    if not a.no_breakdown:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            step()
            torch.cuda.synchronize()
        events = prof.key_averages()
    for ev in events:
        name = ev.key
        for key in ("corr_lookup_backward", "pyramid_backward", "fmap_grad", "fmap_split",
                    "chunk_sum", "corr_build", "split_pairs", "corr_lookup_wide", "corr_lookup_qm", "Cijk", "gemm",
                    "elementwise", "reduce", "fill"):
            if key in name:
                t = getattr(ev, "device_time_total", None)
                if t is None:
                    t = getattr(ev, "cuda_time_total", 0.0)
                kern[key] = round(kern.get(key, 0.0) + t / 1e3, 3)
    print(json.dumps({"workload": a.workload, "fmap": [H, W], "loss": a.loss,
                      "bw_sets": sys.modules["dexiraft_amd.corr"]._BW_SETS,
                      "inputs": "cloned per step" if a.clone_inputs else "persistent leaves",
                      "forward_ms": round(t_fwd, 3),
                      "train_step_ms": round(t_step, 3), "backward_ms": round(t_step - t_fwd, 3),
                      "peak_extra_MB": round(peak / 2 ** 20, 1),
                      "dV_MB": round(B * (H * W) ** 2 * 4 / 2 ** 20, 1),
                      "kernel_ms_one_step": kern}), flush=True)


if __name__ == "__main__":
    main()
