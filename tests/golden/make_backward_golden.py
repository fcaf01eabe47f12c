"""Golden vectors for the CorrBlock BACKWARD, from the REFERENCE core/corr.py on CPU.

Run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_backward_golden.py
The reference trains through CorrBlock (train.py:175-178: matmul, avg_pool2d,
grid_sample under autograd).  For each case: fmaps from tests/datagen.py with
requires_grad, one CorrBlock, three lookups (coords detached, as
core/raft.py:170), loss = sum_k <out_k, R_k> with R_k = datagen normals, and
the reference autograd's d loss / d fmap1, d fmap2 are recorded.
"""
from __future__ import annotations

import sys
import warnings
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
REFERENCE = Path("/root/reference/core")

import datagen as dg  # noqa: E402

# name: (B, D, H, W, radius, num_levels, fmap dist, [(coord mode, scale, seed), ...])
CASES = {
    "bw_basic": (1, 64, 16, 20, 4, 4, "normal", [("normal", 3.0, 201), ("uniform", 10.0, 202),
                                                 ("integer", 4.0, 203)]),
    "bw_batch2_r3": (2, 32, 17, 23, 3, 4, "fnet", [("normal", 4.0, 211), ("identity", 0.0, 212),
                                                    ("far", 1.0, 213)]),
    "bw_d256": (1, 256, 16, 16, 4, 4, "fnet", [("normal", 2.0, 221), ("uniform", 6.0, 222),
                                               ("normal", 5.0, 223)]),
}


def main() -> None:
    warnings.filterwarnings("ignore")
    sys.path.insert(0, str(REFERENCE))
    import torch
    from corr import CorrBlock  # the reference's own class
    torch.set_num_threads(8)
    for i, (name, (B, D, H, W, r, L, dist, sets)) in enumerate(CASES.items()):
        s1, s2 = 3000 + 10 * i, 3001 + 10 * i
        f1 = dg.fmap(s1, B, D, H, W, dist)
        f2 = dg.fmap(s2, B, D, H, W, dist)
        t1 = torch.from_numpy(f1).requires_grad_(True)
        t2 = torch.from_numpy(f2).requires_grad_(True)
        cb = CorrBlock(t1, t2, num_levels=L, radius=r)
        rd = 2 * r + 1
        loss = 0.0
        # inputs are regenerated from the seeds at test time; checksums pin them
        out = {"fmap_seeds": np.array([s1, s2]), "dist": np.array(dist),
               "fmap_checksum": np.array([f1.astype(np.float64).sum(), f2.astype(np.float64).sum()]),
               "coord_sets": np.array([[mode, str(scale), str(seed)] for mode, scale, seed in sets]),
               "weight_seeds": np.array([4000 + 10 * i + k for k in range(len(sets))])}
        for k, (mode, scale, seed) in enumerate(sets):
            c = dg.coords(seed, B, H, W, mode, scale)
            rk = dg.fmap(4000 + 10 * i + k, B, L * rd * rd, H, W, "normal")
            o = cb(torch.from_numpy(c))
            loss = loss + (o * torch.from_numpy(rk)).sum()
        loss.backward()
        out["dfmap1"] = t1.grad.numpy()
        out["dfmap2"] = t2.grad.numpy()
        out["meta"] = np.array([B, D, H, W, r, L])
        np.savez_compressed(HERE / f"{name}.npz", **out)
        print(name, {k: v.shape for k, v in out.items()}, float(loss))


if __name__ == "__main__":
    main()
