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
