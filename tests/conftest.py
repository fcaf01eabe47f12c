"""Shared test setup: markers, import paths, golden-fixture loading.

``-m "not gpu"`` runs here without a GPU: oracle vs golden vectors, the C-ABI
library's exports and host-side validation, the CPU-side error behaviour of the
Python shell, and the gloo multi-process path.  ``-m gpu`` tests are the parity
tests proper: they run the HIP kernels through the C-ABI on an MI355X.
"""
from __future__ import annotations

import json
import sys
from functools import lru_cache
from pathlib import Path

import numpy as np
import pytest

TESTS = Path(__file__).resolve().parent
REPO = TESTS.parent
GOLDEN = TESTS / "golden"
for p in (str(REPO), str(TESTS)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built library")


@lru_cache(maxsize=None)
def manifest() -> dict:
    return json.loads((GOLDEN / "manifest.json").read_text())


def tiny_cases() -> list[str]:
    return list(manifest()["tiny"].keys())


def large_cases() -> list[str]:
    return list(manifest()["large"].keys())


@lru_cache(maxsize=None)
def load_tiny(name: str) -> dict:
    with np.load(GOLDEN / f"tiny_{name}.npz") as z:
        d = {k: z[k] for k in z.files}
    d.update(manifest()["tiny"][name])
    d["n_coords"] = sum(1 for k in d if k.startswith("coords") and k[6:].isdigit())
    return d


@lru_cache(maxsize=None)
def load_large(name: str) -> dict:
    with np.load(GOLDEN / f"large_{name}.npz") as z:
        d = {k: z[k] for k in z.files}
    d.update(manifest()["large"][name])
    return d


def tolerance_check(got: np.ndarray, ref: np.ndarray, rtol_of_max: float) -> float:
    """North-star tolerance: |got - ref| <= rtol * max|ref| (finite entries),
    and identical NaN patterns.  Returns the achieved max error / max|ref|."""
    assert got.shape == ref.shape, (got.shape, ref.shape)
    nan_ref = np.isnan(ref)
    assert np.array_equal(np.isnan(got), nan_ref), "NaN pattern differs from the reference"
    fin = ~nan_ref
    if not fin.any():
        return 0.0
    scale = float(np.abs(ref[fin]).max()) or 1.0
    err = float(np.abs(got[fin].astype(np.float64) - ref[fin].astype(np.float64)).max())
    assert err <= rtol_of_max * scale, f"max err {err:.3e} > {rtol_of_max:.1e} * {scale:.3e}"
    return err / scale


BACKWARD_CASES = ["bw_basic", "bw_batch2_r3", "bw_d256"]


def load_backward(name: str) -> dict:
    """A backward golden (tests/golden/make_backward_golden.py) with its inputs
    regenerated from the recorded seeds: fmaps, coord sets, loss weights."""
    import datagen as dg
    with np.load(GOLDEN / f"{name}.npz") as z:
        d = {k: z[k] for k in z.files}
    B, D, H, W, r, L = (int(v) for v in d["meta"])
    dist = str(d["dist"])
    d.update(B=B, D=D, H=H, W=W, radius=r, num_levels=L)
    d["fmap1"] = dg.fmap(int(d["fmap_seeds"][0]), B, D, H, W, dist)
    d["fmap2"] = dg.fmap(int(d["fmap_seeds"][1]), B, D, H, W, dist)
    np.testing.assert_allclose([d["fmap1"].astype(np.float64).sum(),
                                d["fmap2"].astype(np.float64).sum()], d["fmap_checksum"],
                               rtol=0, atol=1e-6)
    rd = 2 * r + 1
    d["coords"] = [dg.coords(int(seed), B, H, W, str(mode), float(scale))
                   for mode, scale, seed in d["coord_sets"]]
    d["weights"] = [dg.fmap(int(s), B, L * rd * rd, H, W, "normal") for s in d["weight_seeds"]]
    return d


MOTION_CASES = ["motion_basic", "motion_small_b2"]


def load_motion(name: str) -> dict:
    """A lookup + convc1 golden (tests/golden/make_motion_golden.py) with its
    inputs regenerated from the seeds: fmaps, coords, convc1 weight and bias."""
    import datagen as dg
    with np.load(GOLDEN / f"{name}.npz") as z:
        d = {k: z[k] for k in z.files}
    B, D, H, W, r, cout, cin, i = (int(v) for v in d["case"])
    dist = str(d["dist"])
    d.update(B=B, D=D, H=H, W=W, radius=r, cout=cout, cin=cin)
    d["fmap1"] = dg.fmap(6000 + 10 * i, B, D, H, W, dist)
    d["fmap2"] = dg.fmap(6001 + 10 * i, B, D, H, W, dist)
    np.testing.assert_allclose([d["fmap1"].astype(np.float64).sum(),
                                d["fmap2"].astype(np.float64).sum()], d["fmap_checksum"],
                               rtol=0, atol=1e-6)
    mode, scale = (str(v) for v in d["coord"])
    d["coords"] = dg.coords(6002 + 10 * i, B, H, W, mode, float(scale))
    d["weight"], d["bias"] = dg.conv1x1_weights(i, cout, cin)
    return d
