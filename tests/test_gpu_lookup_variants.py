"""Lookup kernel variants (DXR_LOOKUP_VARIANT, read by the launcher on every call)
must be bit-identical to the default wide kernel, which is itself pinned
bit-exact to the reference's lookup (tests/test_gpu_parity.py goldens).

Covered: the narrow form (1) and the 256 / 1024-thread wide forms (2, 3) over
odd level counts, row-major levels >= 4, radii 0..8, bf16 pyramids, far and
non-finite coords.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import datagen as dg

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
CASES = [  # B, D, H, W, levels, radius, dtype, coords
    (1, 64, 55, 128, 4, 4, torch.float32, "normal"),
    (2, 32, 23, 31, 5, 3, torch.float32, "uniform"),
    (1, 16, 40, 40, 1, 4, torch.float32, "far"),
    (1, 16, 33, 47, 3, 8, torch.float32, "normal"),
    (1, 16, 17, 19, 2, 0, torch.float32, "normal"),
    (2, 64, 30, 44, 4, 4, torch.bfloat16, "normal"),
    (1, 16, 64, 64, 6, 2, torch.float32, "uniform"),
]


@pytest.fixture(scope="module")
def dx():
    import dexiraft_amd
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dexiraft_amd.load_native()
    return dexiraft_amd


def _coords(seed, B, H, W, kind):
    if kind == "far":
        c = dg.coords(seed, B, H, W, "normal", 4.0)
        c[:, :, :2] += 1e4                  # whole rows far off the level
        c[:, 0, 3, :5] = np.nan
        c[:, 1, 4, :3] = np.inf
        return c
    return dg.coords(seed, B, H, W, kind, 6.0)


@pytest.mark.parametrize("variant", ["1", "2", "3"])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_lookup_variant_bit_identical(dx, variant, case, monkeypatch):
    B, D, H, W, L, r, dtype, kind = CASES[case]
    f1 = torch.from_numpy(dg.fmap(81 + case, B, D, H, W)).to(DEV).to(dtype)
    f2 = torch.from_numpy(dg.fmap(91 + case, B, D, H, W)).to(DEV).to(dtype)
    c = torch.from_numpy(_coords(101 + case, B, H, W, kind)).to(DEV)
    with torch.no_grad():
        cb = dx.CorrBlock(f1, f2, num_levels=L, radius=r)
        monkeypatch.delenv("DXR_LOOKUP_VARIANT", raising=False)
        ref = cb(c)
        monkeypatch.setenv("DXR_LOOKUP_VARIANT", variant)
        got = cb(c)
        monkeypatch.delenv("DXR_LOOKUP_VARIANT")
    torch.cuda.synchronize()
    assert torch.equal(torch.isnan(ref), torch.isnan(got))
    assert torch.equal(torch.nan_to_num(ref), torch.nan_to_num(got))
