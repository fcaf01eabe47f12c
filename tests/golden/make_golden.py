"""Generate golden vectors by running the REFERENCE core/corr.py on CPU.

Run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
It imports the reference's own ``CorrBlock`` (core/corr.py:12-60, with
core/utils/utils.py:57-77) and records its outputs for inputs made by
tests/datagen.py.  Nothing here runs at test time: tests read the ``.npz``
fixtures only (the reference does not travel to the GPU box).

Fixtures:
  tiny_<name>.npz   full tensors: fmaps, coords sets, every pyramid level
                    (all query rows, or the ``pyr_rows`` subset for the larger
                    cases), every lookup output.
  large_<name>.npz  benchmark shapes: input seeds and
                    input checksums, per-level float64 sum / sum of squares,
                    4096 sampled pyramid entries per level, per-channel sums and
                    4096 sampled entries of each lookup output.
  manifest.json     case parameters.

The reference alt_cuda_corr cannot be built here (CUDA only);
its golden is CorrBlock's output, which it equals by linearity of pooling.
"""
from __future__ import annotations

import json
import sys
import warnings
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
REFERENCE = Path("/root/reference/core")

import datagen as dg  # noqa: E402

# name: (B, D, H, W, radius, num_levels, fmap dist, [(coord mode, scale, seed), ...])
TINY = {
    "nanlevel": (1, 64, 12, 16, 4, 4, "normal", [("normal", 3.0, 11), ("uniform", 12.0, 12),
                                                  ("integer", 4.0, 13)]),
    "fnet": (1, 256, 17, 23, 4, 4, "fnet", [("normal", 4.0, 21), ("uniform", 12.0, 22),
                                             ("identity", 0.0, 23)]),
    "small_r3": (1, 128, 17, 23, 3, 4, "normal", [("integer", 6.0, 31), ("far", 1.0, 32),
                                                   ("normal", 2.0, 33)]),
    "batch2_alt": (2, 64, 16, 20, 4, 4, "normal", [("normal", 4.0, 41), ("uniform", 8.0, 42)]),
    "ragged": (1, 96, 19, 37, 4, 4, "normal", [("normal", 4.0, 51), ("uniform", 10.0, 52)]),
    "min8": (1, 256, 8, 8, 4, 4, "normal", [("normal", 2.0, 61)]),
    "levels5": (1, 16, 32, 34, 2, 5, "normal", [("normal", 6.0, 71), ("uniform", 30.0, 72)]),
    "levels2_r1": (2, 16, 9, 11, 1, 2, "fnet", [("normal", 2.0, 81)]),
}

# name: (B, D, H, W, radius, fmap dist, [(coord mode, scale, seed), ...])
LARGE = {
    "chairs": (1, 256, 46, 62, 4, "normal", [("normal", 4.0, 101), ("normal", 4.0, 102)]),
    "sintel": (1, 256, 55, 128, 4, "normal", [("normal", 4.0, 101), ("uniform", 12.0, 112)]),
    "kitti": (1, 256, 47, 156, 4, "fnet", [("normal", 4.0, 101)]),
    # C5 1080p (1088x1920 padded -> 136x240 fmaps): pins both the full pyramid
    # and, by linearity, the on-the-fly AlternateCorrBlock at that size
    "hd": (1, 256, 136, 240, 4, "fnet", [("normal", 4.0, 101), ("uniform", 12.0, 112)]),
}
NSAMPLE = 4096
PYR_FULL_MAX = 200_000   # tiny cases above this many level-0 elements keep PYR_ROWS query rows
PYR_ROWS = 128


def _reference_corrblock():
    sys.path.insert(0, str(REFERENCE))
    import torch
    from corr import CorrBlock  # the reference's own class
    torch.set_num_threads(8)
    return torch, CorrBlock


def main() -> None:
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", default=None, help="regenerate only this benchmark-shape case")
    only = ap.parse_args().large
    warnings.filterwarnings("ignore")
    torch, CorrBlock = _reference_corrblock()
    manifest = {"tiny": {}, "large": {}, "nsample": NSAMPLE}
    if only is not None:
        manifest = json.loads((HERE / "manifest.json").read_text())

    for i, (name, (B, D, H, W, r, L, dist, sets)) in enumerate(TINY.items()):
        if only is not None:
            break
        s1, s2 = 1000 + 10 * i, 1001 + 10 * i
        f1 = dg.fmap(s1, B, D, H, W, dist)
        f2 = dg.fmap(s2, B, D, H, W, dist)
        cb = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=L, radius=r)
        out = {"fmap1": f1, "fmap2": f2}
        nq = B * H * W
        rows = np.arange(nq)
        if nq * H * W > PYR_FULL_MAX:
            rows = np.sort(np.random.default_rng(i).choice(nq, PYR_ROWS, replace=False))
        out["pyr_rows"] = rows
        for lvl, p in enumerate(cb.corr_pyramid):
            out[f"pyr{lvl}"] = p[rows, 0].numpy()
        for k, (mode, scale, seed) in enumerate(sets):
            c = dg.coords(seed, B, H, W, mode, scale)
            out[f"coords{k}"] = c
            out[f"out{k}"] = cb(torch.from_numpy(c)).numpy()
        np.savez_compressed(HERE / f"tiny_{name}.npz", **out)
        manifest["tiny"][name] = dict(B=B, D=D, H=H, W=W, radius=r, num_levels=L, dist=dist,
                                      fmap_seeds=[s1, s2], coords=[list(s) for s in sets])
        print("tiny", name, {k: v.shape for k, v in out.items()})

    for name, (B, D, H, W, r, dist, sets) in LARGE.items():
        if only is not None and name != only:
            continue
        s1, s2 = 7, 8
        f1 = dg.fmap(s1, B, D, H, W, dist)
        f2 = dg.fmap(s2, B, D, H, W, dist)
        cb = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=4, radius=r)
        out = {"fmap_checksum": np.array([f1.astype(np.float64).sum(), f2.astype(np.float64).sum()])}
        rng = np.random.default_rng(12345)
        for lvl in range(4):
            a = cb.corr_pyramid[lvl][:, 0].numpy()
            flat = a.reshape(-1)
            idx = rng.integers(0, flat.size, NSAMPLE)
            out[f"pyr{lvl}_sum"] = np.array([a.astype(np.float64).sum(),
                                            np.square(a.astype(np.float64)).sum()])
            out[f"pyr{lvl}_idx"] = idx
            out[f"pyr{lvl}_val"] = flat[idx]
            out[f"pyr{lvl}_maxabs"] = np.array(np.abs(a).max())
        for k, (mode, scale, seed) in enumerate(sets):
            c = dg.coords(seed, B, H, W, mode, scale)
            o = cb(torch.from_numpy(c)).numpy()
            flat = o.reshape(-1)
            idx = rng.integers(0, flat.size, NSAMPLE)
            out[f"coords{k}_checksum"] = np.array(c.astype(np.float64).sum())
            out[f"out{k}_chsum"] = o.astype(np.float64).sum(axis=(0, 2, 3))
            out[f"out{k}_idx"] = idx
            out[f"out{k}_val"] = flat[idx]
            out[f"out{k}_maxabs"] = np.array(np.abs(o).max())
        np.savez_compressed(HERE / f"large_{name}.npz", **out)
        manifest["large"][name] = dict(B=B, D=D, H=H, W=W, radius=r, num_levels=4, dist=dist,
                                       fmap_seeds=[s1, s2], coords=[list(s) for s in sets])
        print("large", name)

    (HERE / "manifest.json").write_text(json.dumps(manifest, indent=1) + "\n")


if __name__ == "__main__":
    main()
