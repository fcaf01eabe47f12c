#!/usr/bin/env python3
"""Can the bench time the build inside its own step graph?  (Profiles only.)

Captures the bench's step (CorrBlock build + 12 lookups, Sintel B=1) twice: as
bench.py does, and with timing events recorded inside the capture
(torch.cuda.Event(enable_timing=True, external=True): event-record graph nodes)
before the build, after the build and after the last lookup.  Replays both
interleaved and reports, per variant, the step time from events outside the
graph, and for the probed graph the in-graph build and lookup spans of the last
replay of each round — so one sees whether the probe nodes cost time and whether
their split agrees with the back-to-back build / lookup graphs of bench.py.
Usage: python scripts/probe_graph_events.py [--workload sintel] [--rounds 9]
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
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--reps", type=int, default=50)
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
    stream = torch.cuda.Stream(device=dev)
    ev = [torch.cuda.Event(enable_timing=True, external=True) for _ in range(3)]
    out = {"workload": a.workload}
    with torch.no_grad(), torch.cuda.stream(stream):
        def step(probe):
            if probe:
                ev[0].record(stream)
            cb = dexiraft_amd.CorrBlock(f1, f2)
            if probe:
                ev[1].record(stream)
            r = [cb(c) for c in coords]
            if probe:
                ev[2].record(stream)
            return r

        graphs = {}
        for probe in (False, True):
            step(probe)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(gr, stream=stream):
                    step(probe)
            except Exception as e:   # noqa: BLE001 - report what the runtime refused
                out["probe_capture_error"] = repr(e)
                print(json.dumps(out), flush=True)
                return
            graphs[probe] = gr
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            for gr in graphs.values():
                gr.replay()
            torch.cuda.synchronize()
        res = {False: [], True: []}
        inner = {"build": [], "lookups": []}
        for _ in range(a.rounds):
            for probe, gr in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    gr.replay()
                e1.record(stream)
                torch.cuda.synchronize()
                res[probe].append(e0.elapsed_time(e1) * 1e3 / a.reps)
                if probe:
                    try:
                        inner["build"].append(ev[0].elapsed_time(ev[1]) * 1e3)
                        inner["lookups"].append(ev[1].elapsed_time(ev[2]) * 1e3 / 12)
                    except Exception as e:   # noqa: BLE001
                        out["probe_elapsed_error"] = repr(e)
    med = lambda v: round(float(np.median(v)), 2) if v else None  # noqa: E731
    out.update({"step_us_plain": med(res[False]), "step_us_probed": med(res[True]),
                "in_graph_build_us": med(inner["build"]),
                "in_graph_lookup_us": med(inner["lookups"])})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
