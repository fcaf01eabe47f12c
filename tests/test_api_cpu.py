"""CPU: the Python shell mirrors the reference interface and fails loudly
where it has no path (host tensors) instead of silently computing on the CPU."""
from __future__ import annotations

import inspect

import numpy as np
import pytest
import torch

import dexiraft_amd as dx


def test_public_surface_mirrors_reference():
    assert {"CorrBlock", "AlternateCorrBlock", "alt_cuda_corr", "coords_grid"} <= set(dx.__all__)
    for cls in (dx.CorrBlock, dx.AlternateCorrBlock):
        sig = inspect.signature(cls.__init__)
        assert list(sig.parameters) == ["self", "fmap1", "fmap2", "num_levels", "radius"]
        assert sig.parameters["num_levels"].default == 4
        assert sig.parameters["radius"].default == 4
        assert list(inspect.signature(cls.__call__).parameters) == ["self", "coords"]
    assert isinstance(inspect.getattr_static(dx.CorrBlock, "corr"), staticmethod)
    assert list(inspect.signature(dx.alt_cuda_corr.forward).parameters) == [
        "fmap1", "fmap2", "coords", "radius"]
    assert list(inspect.signature(dx.alt_cuda_corr.backward).parameters) == [
        "fmap1", "fmap2", "coords", "corr_grad", "radius"]


@pytest.mark.parametrize("ctor", [dx.CorrBlock, dx.AlternateCorrBlock])
def test_host_tensors_raise(ctor):
    f = torch.zeros(1, 8, 16, 16)
    with pytest.raises(RuntimeError, match="no CPU path"):
        ctor(f, f)


def test_host_tensors_raise_static_and_ffi():
    f = torch.zeros(1, 8, 16, 16)
    with pytest.raises(RuntimeError, match="no CPU path"):
        dx.CorrBlock.corr(f, f)
    with pytest.raises(RuntimeError, match="CUDA tensor"):
        dx.alt_cuda_corr.forward(torch.zeros(1, 4, 4, 8), torch.zeros(1, 4, 4, 8),
                                 torch.zeros(1, 1, 4, 4, 2), 4)
    with pytest.raises(RuntimeError, match="CUDA tensor"):
        z = torch.zeros(1, 4, 4, 8)
        dx.alt_cuda_corr.backward(z, z, torch.zeros(1, 1, 4, 4, 2), torch.zeros(1, 1, 81, 4, 4), 4)


def test_non_tensor_input_raises_type_error():
    with pytest.raises(TypeError):
        dx.CorrBlock(np.zeros((1, 8, 16, 16)), np.zeros((1, 8, 16, 16)))


def test_coords_grid_matches_reference_definition():
    # core/utils/utils.py:74-77: stack(meshgrid(arange(ht), arange(wd))[::-1]).float()
    ht, wd = 5, 7
    ys, xs = torch.meshgrid(torch.arange(ht), torch.arange(wd), indexing="ij")
    ref = torch.stack([xs, ys], dim=0).float()[None].repeat(3, 1, 1, 1)
    assert torch.equal(dx.coords_grid(3, ht, wd), ref)


@pytest.mark.parametrize("dim", [16, 64, 96, 128, 256, 324, 1000])
def test_sqrt_dim_is_the_references_float32_sqrt(dim):
    from dexiraft_amd.corr import _sqrt_dim
    assert _sqrt_dim(dim) == float(torch.sqrt(torch.tensor(dim).float()))


def test_channels_last_classification():
    """Which fmaps take the native layout path: NHWC-strided
    4-D tensors that are not also NCHW-contiguous (degenerate shapes are both)."""
    from dexiraft_amd.corr import _channels_last
    x = torch.zeros(2, 8, 5, 7)
    assert not _channels_last(x)
    assert _channels_last(x.contiguous(memory_format=torch.channels_last))
    assert not _channels_last(torch.zeros(2, 1, 5, 7).contiguous(memory_format=torch.channels_last))
    assert not _channels_last(x.transpose(2, 3))                      # other strides: .contiguous()


def test_host_channels_last_fmaps_raise():
    f = torch.zeros(1, 16, 16, 16).contiguous(memory_format=torch.channels_last)
    for ctor in (dx.CorrBlock, dx.AlternateCorrBlock):
        with pytest.raises(RuntimeError):
            ctor(f, f)


def test_bench_cpu_baseline_torch_restatement():
    """bench.py's cpu_baseline leg: the torch restatement of core/corr.py, bounded."""
    import bench
    res = bench.cpu_baseline(8, 12, 0.05, "torch")
    assert res["kind"] == "port" and res["unit"] == "pairs/s" and res["value"] > 0
    assert res["cores"] >= 1 and "torch_ref" in res["sample"]
