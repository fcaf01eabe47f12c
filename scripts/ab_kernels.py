#!/usr/bin/env python3
"""Same-process A/B timing of kernel variants (MI355X_MICROARCH / §5.4 rule 24:
interleaved rounds in ONE process).  Build variants are selected through
DXR_BUILD_VARIANT (read by the launcher on every call).  Prints one JSON line.

Usage: python scripts/ab_kernels.py [--workload sintel] [--variants 0,1,2,3] [--rounds 5]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402  (workload table, algorithmic byte/flop formulas)
import dexiraft_amd  # noqa: E402

SPLIT_VARIANTS = {0, 7, 8, 9, 11, 12, 13, 40}  # f32 builds on bf16 MFMA (exact operand split); D % 16 == 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="sintel", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--ablations", default="", help="timing-only variants (outputs not checked)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--interleave", action="store_true",
                    help="run the 12 lookups between builds (as bench.py does) and time builds only")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--side-stream", action="store_true", help="launch on a non-default stream")
    a = ap.parse_args()
    (_, _), (H, W), _, _ = bench.WORKLOADS[a.workload]
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.make_inputs(a.batch, H, W, a.dtype, a.seed, dev)
    variants = [int(v) for v in a.variants.split(",")]
    ablations = [int(v) for v in a.ablations.split(",") if v]
    times = {v: [] for v in variants + ablations}
    side = torch.cuda.Stream(device=dev) if a.side_stream else torch.cuda.current_stream(dev)
    with torch.no_grad(), torch.cuda.stream(side):
        ref = {}
        for v in variants:  # correctness: variants of one family are bit-identical
            os.environ["DXR_BUILD_VARIANT"] = str(v)
            cb = dexiraft_amd.CorrBlock(f1, f2)      # valid cells only (padding is never read)
            fam = "split" if v in SPLIT_VARIANTS and a.dtype == "f32" else "mfma"
            if fam not in ref:
                ref[fam] = (v, cb.corr_pyramid)
            assert all(torch.equal(x, y) for x, y in zip(cb.corr_pyramid, ref[fam][1])), \
                f"variant {v} differs from variant {ref[fam][0]}"
        for _ in range(a.rounds):
            for v in variants + ablations:
                os.environ["DXR_BUILD_VARIANT"] = str(v)
                if a.interleave:
                    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                           for _ in range(a.reps)]
                    for e0, e1 in evs:
                        e0.record()
                        cb = dexiraft_amd.CorrBlock(f1, f2)
                        e1.record()
                        for c in coords:
                            cb(c)
                    torch.cuda.synchronize()
                    times[v].append(float(np.mean([x.elapsed_time(y) for x, y in evs])) * 1e3)
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    dexiraft_amd.CorrBlock(f1, f2)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.reps * 1e3)
        os.environ["DXR_BUILD_VARIANT"] = str(variants[0])
        cb = dexiraft_amd.CorrBlock(f1, f2)
        for _ in range(3):
            for c in coords:
                cb(c)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            outs = [cb(c) for c in coords]
        lk = []
        for _ in range(a.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            lk.append(e0.elapsed_time(e1) / a.reps / len(coords) * 1e3)
    flops = bench.build_flops(a.batch, H, W)
    res = {"workload": a.workload, "batch": a.batch, "dtype": a.dtype, "seed": a.seed,
           "interleave": a.interleave, "side_stream": a.side_stream,
           "build_us": {v: {"median": float(np.median(t)), "min": float(np.min(t))}
                        for v, t in times.items()},
           "build_tflops_median": {v: flops / (np.median(t) * 1e-6) / 1e12 for v, t in times.items()},
           "lookup_us_median": float(np.median(lk)),
           "lookup_gbs": bench.lookup_bytes(a.batch, H, W) / (np.median(lk) * 1e-6) / 1e9}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
