#!/usr/bin/env python3
"""Same-process A/B timing of lookup kernel variants (DXR_LOOKUP_VARIANT, read
by the launcher on every call): a HIP graph of the 12 lookups per variant,
replayed in interleaved rounds.  Variants other than the 9x ablations are
checked bit-identical to the first.  Prints one JSON line.

Usage: python scripts/ab_lookup.py [--workload sintel] [--variants 0,91,92,93]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import dexiraft_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="sintel", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--variants", default="0,91,92,93")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    (_, _), (H, W), _, _ = bench.WORKLOADS[a.workload]
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.make_inputs(a.batch, H, W, a.dtype, 7, dev)
    variants = [int(v) for v in a.variants.split(",")]
    stream = torch.cuda.Stream(device=dev)
    graphs, ref = {}, None
    with torch.no_grad(), torch.cuda.stream(stream):
        cb = dexiraft_amd.CorrBlock(f1, f2)
        for v in variants:
            os.environ["DXR_LOOKUP_VARIANT"] = str(v)
            outs = [cb(c) for c in coords]
            if v < 90:
                if ref is None:
                    ref = outs
                assert all(torch.equal(x, y) for x, y in zip(outs, ref)), f"variant {v} differs"
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                [cb(c) for c in coords]
            graphs[v] = g
        torch.cuda.synchronize()
        times = {v: [] for v in variants}
        for _ in range(a.rounds):
            for v in variants:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    graphs[v].replay()
                e1.record(stream)
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.reps / len(coords) * 1e3)
    lb = bench.lookup_bytes(a.batch, H, W, s_pyr=2 if a.dtype == "bf16" else 4)
    res = {"workload": a.workload, "batch": a.batch, "dtype": a.dtype,
           "lookup_us": {v: {"median": float(np.median(t)), "min": float(np.min(t))}
                         for v, t in times.items()},
           "lookup_gbs_median": {v: lb / (np.median(t) * 1e-6) / 1e9 for v, t in times.items()}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
