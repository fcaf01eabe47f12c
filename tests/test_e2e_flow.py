"""End-to-end parity: final flow of the Dexi+RAFT refinement loop.

The golden (tests/golden/e2e_chairs.npz, made by tests/golden/make_e2e_golden.py)
is the reference's own CorrBlock + BasicUpdateBlock iterated 12 times
(core/raft.py:160-192) at config 1 (fmap 46x62, D=256, r=4, 4 levels) with
name-keyed deterministic weights.  Criteria (north_star): fp32 final flow EPE
< 1e-3 px; bf16 EPE < 1e-2 px (SURVEY.md §8(c) tolerance row).

CPU test: the harness (tests/e2e_flow.py) around the numpy oracle reproduces the
reference loop — this pins the harness itself.  GPU tests: the same harness
around the HIP CorrBlock / AlternateCorrBlock.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import e2e_flow as ef
from conftest import GOLDEN

EPE_F32 = 1e-3      # px, north_star fp32 criterion
EPE_BF16 = 1e-2     # px, SURVEY.md §8(c) proposed bf16 tolerance
EPE_HARNESS = 1e-4  # px, harness + oracle vs the reference loop on CPU


def golden():
    with np.load(GOLDEN / "e2e_chairs.npz") as z:
        return {k: z[k] for k in z.files}


def _run(block_cls, device, fmap_dtype=torch.float32):
    x = ef.e2e_inputs()
    W = ef.torch_weights(ef.update_weights(), device)
    t = {k: torch.from_numpy(v).to(device) for k, v in x.items()}
    f = {k: t[k].to(fmap_dtype) for k in ("fmap1", "fmap2", "fem1", "fem2")}
    with torch.no_grad():
        corr_fn = block_cls(f["fmap1"], f["fmap2"])
        corr_en = block_cls(f["fem1"], f["fem2"])
        return ef.refine(corr_fn, corr_en, W, t)


def _check(flows, up, eflow, tol):
    g = golden()
    per_iter = [ef.epe(fl, g["flows"][i]) for i, fl in enumerate(flows)]
    final = per_iter[-1]
    up_epe = ef.epe(up[:, :, ::4, ::4], g["flow_up_sub4"])
    e_epe = ef.epe(eflow, g["eflow"])
    print(f"final EPE {final:.3e} px, max over iters {max(per_iter):.3e}, "
          f"upsampled {up_epe:.3e}, edge flow {e_epe:.3e}")
    assert np.isfinite(final)
    assert final < tol, per_iter
    assert max(per_iter) < tol
    assert up_epe < 8 * tol          # full-res flow is 8x the low-res flow
    assert e_epe < tol


class _OracleBlock:
    """CorrBlock semantics from the numpy oracle (float32 volume, reference lookup)."""

    def __init__(self, fmap1, fmap2):
        from oracle import corr_oracle as co
        self._co = co
        self.pyr = co.corr_pyramid(fmap1.numpy(), fmap2.numpy(), ef.LEVELS, np.float32)

    def __call__(self, coords):
        return torch.from_numpy(self._co.corr_lookup(self.pyr, coords.numpy(), ef.RADIUS))


def test_golden_loop_is_well_conditioned():
    g = golden()
    assert g["flows"].shape == (ef.E2E["iters"], 1, 2, ef.E2E["H"], ef.E2E["W"])
    assert np.abs(g["flows"][-1]).max() > 8.0          # taps cross cells / leave the map
    assert float(g["epe_f32_vs_f64"]) < 1e-4           # fp32 rounding alone: ~6e-6 px


def test_harness_with_oracle_matches_reference_loop():
    torch.set_num_threads(8)
    flows, up, eflow = _run(_OracleBlock, "cpu")
    _check(flows, up, eflow, EPE_HARNESS)


@pytest.mark.gpu
def test_e2e_corrblock_f32():
    import dexiraft_amd
    flows, up, eflow = _run(dexiraft_amd.CorrBlock, "cuda")
    _check(flows, up, eflow, EPE_F32)


@pytest.mark.gpu
def test_e2e_alternate_corrblock_f32():
    import dexiraft_amd
    flows, up, eflow = _run(dexiraft_amd.AlternateCorrBlock, "cuda")
    _check(flows, up, eflow, EPE_F32)


@pytest.mark.gpu
def test_e2e_corrblock_bf16():
    import dexiraft_amd
    flows, up, eflow = _run(dexiraft_amd.CorrBlock, "cuda", torch.bfloat16)
    _check(flows, up, eflow, EPE_BF16)
