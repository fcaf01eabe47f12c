"""Golden vectors for the lookup fused with the motion encoder's convc1, from the
REFERENCE core/corr.py + core/update.py on CPU.

Run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_motion_golden.py
For each case: fmaps from tests/datagen.py, the reference CorrBlock, one lookup,
and the reference encoder's ``F.relu(self.convc1(corr))`` (core/update.py:90 for
BasicMotionEncoder, :71 for SmallMotionEncoder) with convc1's weight and bias set
from datagen seeds.  Inputs are regenerated from the seeds at test time; the
recorded output is the fixture.
"""
from __future__ import annotations

import sys
import types
import warnings
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
REFERENCE = Path("/root/reference/core")

import datagen as dg  # noqa: E402

# name: (encoder, B, D, H, W, radius, fmap dist, coord mode, coord scale)
CASES = {
    "motion_basic": ("BasicMotionEncoder", 1, 64, 16, 20, 4, "fnet", "normal", 3.0),
    "motion_small_b2": ("SmallMotionEncoder", 2, 32, 17, 23, 3, "normal", "uniform", 10.0),
}


def main() -> None:
    warnings.filterwarnings("ignore")
    sys.path.insert(0, str(REFERENCE))
    import torch
    import torch.nn.functional as F
    import update
    from corr import CorrBlock  # the reference's own class
    torch.set_num_threads(8)
    for i, (name, (enc_name, B, D, H, W, r, dist, mode, scale)) in enumerate(CASES.items()):
        args = types.SimpleNamespace(corr_levels=4, corr_radius=r)
        enc = getattr(update, enc_name)(args)
        conv = enc.convc1
        cout, cin = conv.weight.shape[:2]
        w, b = dg.conv1x1_weights(i, cout, cin)
        with torch.no_grad():
            conv.weight.copy_(torch.from_numpy(w).reshape(cout, cin, 1, 1))
            conv.bias.copy_(torch.from_numpy(b))
            f1 = dg.fmap(6000 + 10 * i, B, D, H, W, dist)
            f2 = dg.fmap(6001 + 10 * i, B, D, H, W, dist)
            c = dg.coords(6002 + 10 * i, B, H, W, mode, scale)
            corr = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), radius=r)(
                torch.from_numpy(c))
            cor = F.relu(conv(corr))   # core/update.py:90 / :71
        np.savez_compressed(
            HERE / f"{name}.npz",
            case=np.array([B, D, H, W, r, cout, cin, i]), dist=np.array(dist),
            coord=np.array([mode, str(scale)]),
            fmap_checksum=np.array([f1.astype(np.float64).sum(), f2.astype(np.float64).sum()]),
            corr_checksum=np.array([corr.double().sum().item(), (corr.double() ** 2).sum().item()]),
            out=cor.numpy().astype(np.float32))
        print(name, tuple(cor.shape), float(cor.abs().max()))


if __name__ == "__main__":
    main()
