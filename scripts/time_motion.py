"""Time the lookup fused with convc1 against the unfused reference sequence
(SURVEY.md §8(f) row 2): per call, on one GPU, inputs resident in HBM.

  unfused : corr = block(coords); F.relu(F.conv2d(corr, convc1.weight, convc1.bias))
            (core/raft.py:172 + core/update.py:90: our lookup, torch conv + relu)
  fused   : block.lookup_conv1x1(coords, convc1.weight, convc1.bias)

Both are captured into HIP graphs of 12 calls (12 GRU iterations) and replayed;
HIP events around each replay.  Prints one JSON line per (workload, batch).
Usage: python scripts/time_motion.py [--reps 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import dexiraft_amd  # noqa: E402

DEV = "cuda:0"


def graph_of(fn, n):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn(0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(n):
            fn(k)
    return g


def time_graph(g, reps):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    st.record()
    for _ in range(reps):
        g.replay()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps * 1e3   # us per replay


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--variants", default="0", help="DXR_MOTION_VARIANT values to A/B")
    a = ap.parse_args()
    torch.backends.cudnn.allow_tf32 = False
    for name, H, W, B in (("sintel", 55, 128, 1), ("sintel", 55, 128, 2), ("kitti", 47, 156, 8)):
        g = torch.Generator(device=DEV).manual_seed(0)
        f1 = torch.randn((B, 256, H, W), generator=g, device=DEV)
        f2 = torch.randn((B, 256, H, W), generator=g, device=DEV)
        ys, xs = torch.meshgrid(torch.arange(H, device=DEV, dtype=torch.float32),
                                torch.arange(W, device=DEV, dtype=torch.float32), indexing="ij")
        coords = [(torch.stack((xs, ys))[None] + 4 * torch.randn((B, 2, H, W), generator=g,
                                                                device=DEV)).contiguous()
                  for _ in range(12)]
        w = torch.randn((256, 324, 1, 1), generator=g, device=DEV) / 18.0
        b = 0.5 * torch.randn((256,), generator=g, device=DEV)
        cb = dexiraft_amd.CorrBlock(f1, f2)
        outs = {}
        with torch.no_grad():
            g_look = graph_of(lambda k: outs.__setitem__("l", cb(coords[k])), 12)
            g_unf = graph_of(lambda k: outs.__setitem__(
                "u", F.relu(F.conv2d(cb(coords[k]), w, b))), 12)
            t_look = time_graph(g_look, a.reps) / 12
            t_unf = time_graph(g_unf, a.reps) / 12
            var_us = {}
            for var in a.variants.split(","):
                os.environ["DXR_MOTION_VARIANT"] = var
                g_fus = graph_of(lambda k: outs.__setitem__(
                    "f", cb.lookup_conv1x1(coords[k], w, b)), 12)
                var_us[var] = round(time_graph(g_fus, a.reps) / 12, 2)
                os.environ.pop("DXR_MOTION_VARIANT")
                if var == a.variants.split(",")[0]:   # ablation variants' outputs are invalid
                    err = ((outs["f"] - outs["u"]).abs().max() / outs["u"].abs().max()).item()
            t_fus = var_us[a.variants.split(",")[0]]
        n = B * H * W
        # compulsory bytes of the fused call: lookup windows + coords + conv output
        win = sum(min(10, h) * min(10, ww) for h, ww in
                  ((H, W), (H // 2, W // 2), (H // 4, W // 4), (H // 8, W // 8)))
        fbytes = n * (win * 4 + 8 + 256 * 4)
        flops = 2.0 * n * 324 * 256
        print(json.dumps({
            "workload": name, "pairs": B, "fmap": [H, W],
            "lookup_us": round(t_look, 2), "lookup_conv_relu_unfused_us": round(t_unf, 2),
            "fused_us": round(t_fus, 2), "fused_us_by_variant": var_us, "speedup": round(t_unf / t_fus, 3),
            "fused_vs_unfused_max_rel_err": err,
            "fused_algorithmic_bytes": fbytes,
            "fused_hbm_frac": round(fbytes / (t_fus * 1e-6) / 8e12, 4),
            "conv_f32_tflops_in_fused": round(flops / (t_fus * 1e-6) / 1e12, 2)}), flush=True)
        del g_look, g_unf, g_fus


if __name__ == "__main__":
    main()
