#!/usr/bin/env python3
"""Where the step's idle time goes: the HIP graph replay boundary (profiles only).

The rocprofv3 kernel trace of bench.py (scripts/trace_gaps.py, profiles/r05)
puts all of the step's idle time at the boundary between two replays of the
step graph (last lookup -> next split pass); inside the graph the kernels run
back to back.  This measures that boundary directly, same process, HIP events
around back-to-back replays:
  one_step   the bench's step graph (build + 12 lookups), per replay;
  two_steps  a graph holding the same step twice, per step;
  tiny       a graph of one tiny kernel (torch fill of 1 element), per replay;
  tiny_x14   a graph of 14 such kernels (the step's kernel count), per replay;
  four_steps a graph holding the step four times, per step;
  alt_execs  two separately captured one-step graphs replayed alternately, per
             step (does the boundary come from relaunching the same graph exec?).
one_step - two_steps is the per-replay boundary cost; tiny bounds the runtime's
graph-launch floor.
Usage: python scripts/probe_graph_boundary.py [--workload sintel] [--reps 200]
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

SHAPES = {"sintel": (55, 128), "chairs": (46, 62)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="sintel", choices=sorted(SHAPES))
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    import dexiraft_amd
    dev = torch.device("cuda", 0)
    (H, W), B, D = SHAPES[a.workload], 1, 256
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack((xs, ys))[None].expand(B, 2, H, W)
    coords = [(grid + 4.0 * torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous()
              for _ in range(12)]
    small = torch.zeros(1, device=dev)
    stream = torch.cuda.Stream(device=dev)

    def step():
        cb = dexiraft_amd.CorrBlock(f1, f2)
        return [cb(c) for c in coords]

    bodies = {"one_step": (lambda: step(), 1), "two_steps": (lambda: (step(), step()), 2),
              "four_steps": (lambda: [step() for _ in range(4)], 4),
              "alt_a": (lambda: step(), 1), "alt_b": (lambda: step(), 1),
              "tiny": (lambda: small.fill_(1.0), 1),
              "tiny_x14": (lambda: [small.fill_(float(i)) for i in range(14)], 1)}
    graphs = {}
    with torch.no_grad(), torch.cuda.stream(stream):
        for name, (fn, _) in bodies.items():
            fn()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=stream):
                fn()
            graphs[name] = gr
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            graphs["one_step"].replay()
            torch.cuda.synchronize()
        res = {n: [] for n in graphs if n != "alt_b"}
        for _ in range(a.rounds):
            for n, gr in graphs.items():
                if n == "alt_b":
                    continue
                reps = a.reps if n.startswith("tiny") else max(20, a.reps // 4)
                if n == "alt_a":   # alternate the two execs: 2 * reps replays
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(reps):
                        gr.replay()
                        graphs["alt_b"].replay()
                    e1.record(stream)
                    torch.cuda.synchronize()
                    res[n].append(e0.elapsed_time(e1) * 1e3 / (2 * reps))
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(reps):
                    gr.replay()
                e1.record(stream)
                torch.cuda.synchronize()
                res[n].append(e0.elapsed_time(e1) * 1e3 / reps / bodies[n][1])
    med = {("alt_execs" if n == "alt_a" else n): round(float(np.median(v)), 2)
           for n, v in res.items()}
    print(json.dumps({"workload": a.workload, "us_per_step_or_replay_median": med,
                      "boundary_us_estimate": round(med["one_step"] - med["two_steps"], 2) * 2,
                      "what": "one_step - two_steps = half a replay boundary per step; x2 = "
                              "the boundary per replay"}), flush=True)


if __name__ == "__main__":
    main()
