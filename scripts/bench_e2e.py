#!/usr/bin/env python3
"""End-to-end pairs/s of the Dexi+RAFT refinement loop around the HIP blocks
(reference evaluate.py:102-122 -> core/raft.py:143-193
minus the encoders, which are out of scope).

One "pair" = driver.InputPadder-sized image pair at config 1 (368x496, fmap
46x62) or Sintel (440x1024, fmap 55x128): TWO correlation blocks (image and
edge fmaps, core/raft.py:147-148) + 12 iterations of two lookups and two
BasicUpdateBlock passes (torch convs, MIOpen) + the convex upsampling
(tests/e2e_flow.py restates them).  Timed as one HIP graph per pair, K replays.
Prints one JSON line; ``corr_share`` is the part of the step spent in this
repository's kernels (the same step with the update block removed).

Usage: python scripts/bench_e2e.py [--workload chairs|sintel] [--block corr|alt]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "tests")]

import e2e_flow as ef  # noqa: E402

SHAPES = {"chairs": (46, 62), "sintel": (55, 128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="chairs", choices=sorted(SHAPES))
    ap.add_argument("--block", default="corr", choices=["corr", "alt"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    import dexiraft_amd
    dexiraft_amd.load_native()
    dev = torch.device("cuda", 0)
    H, W = SHAPES[args.workload]
    block_cls = dexiraft_amd.CorrBlock if args.block == "corr" else dexiraft_amd.AlternateCorrBlock
    x = ef.e2e_inputs(H=H, W=W)
    t = {k: torch.from_numpy(v).to(dev) for k, v in x.items()}
    Wt = ef.torch_weights(ef.update_weights(), dev)
    state = {}

    def step(update=True):
        cf = block_cls(t["fmap1"], t["fmap2"])
        ce = block_cls(t["fem1"], t["fem2"])
        if update:
            state["flows"], state["up"], _ = ef.refine(cf, ce, Wt, t)
        else:   # correlation work alone: 2 builds + 24 lookups at the loop's coords
            c = ef.coords_grid(1, H, W, dev)
            state["c"] = [(cf(c), ce(c)) for _ in range(ef.E2E["iters"])]

    stream = torch.cuda.Stream(device=dev)
    res = {}
    with torch.no_grad(), torch.cuda.stream(stream):
        for update in (True, False):
            for _ in range(args.warmup):
                step(update)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                step(update)
            for _ in range(args.warmup):
                g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                g.replay()
            torch.cuda.synchronize()
            res[update] = (time.perf_counter() - t0) / args.steps
    ms = res[True] * 1e3
    print(json.dumps({
        "metric": "Dexi+RAFT refinement loop pairs/s (2 correlation blocks + 12 iterations, "
                  "encoders excluded)",
        "value": round(1.0 / res[True], 2), "unit": "pairs/s", "ms_per_pair": round(ms, 3),
        "corr_ms_per_pair": round(res[False] * 1e3, 3),
        "corr_share": round(res[False] / res[True], 3),
        "workload": f"{args.workload} fmap {H}x{W}, D=256, r=4, L=4, B=1, f32, "
                    f"{'CorrBlock' if args.block == 'corr' else 'AlternateCorrBlock'}",
        "timing": "one HIP graph per pair, mean over replays",
        "data": "synthetic encoder outputs and name-keyed update weights (tests/e2e_flow.py)",
    }), flush=True)


if __name__ == "__main__":
    main()
