#!/usr/bin/env python3
"""Numerics diagnostic of the build variants at a benchmark shape: error of the
level-0 volume against a float64 GPU matmul (max, RMS, mean = bias) and the
level sums against the reference golden checksums.  Prints one JSON line."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "tests")]
import datagen as dg  # noqa: E402
from conftest import load_large  # noqa: E402
import dexiraft_amd  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "sintel"
variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "10"]
d = load_large(name)
B, D, H, W = d["B"], d["D"], d["H"], d["W"]
f1 = torch.from_numpy(dg.fmap(d["fmap_seeds"][0], B, D, H, W, d["dist"])).cuda()
f2 = torch.from_numpy(dg.fmap(d["fmap_seeds"][1], B, D, H, W, d["dist"])).cuda()
ref = torch.matmul(f1.double().view(B, D, -1).transpose(1, 2), f2.double().view(B, D, -1)) / 16.0
ref = ref.reshape(-1)
res = {"case": name}
with torch.no_grad():
    for v in variants:
        os.environ["DXR_BUILD_VARIANT"] = v
        cb = dexiraft_amd.CorrBlock(f1, f2)
        a = cb.corr_pyramid[0].reshape(-1).double()
        e = a - ref
        r = {"max_abs": e.abs().max().item(), "rms": e.pow(2).mean().sqrt().item(),
             "mean": e.mean().item(), "mean_rel_signed": (e * ref.sign()).mean().item(),
             "sum_vs_f64": (a.sum() - ref.sum()).item()}
        for lvl in range(4):
            s = cb.corr_pyramid[lvl].double().sum().item()
            r[f"lvl{lvl}_sum_minus_golden"] = s - float(d[f"pyr{lvl}_sum"][0])
        res["v" + v] = r
res["f64_sum_minus_golden"] = ref.sum().item() - float(d["pyr0_sum"][0])
print(json.dumps(res))
