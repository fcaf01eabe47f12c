"""Coordinate helper of the lookup path (reference core/utils/utils.py:74-77)."""
from __future__ import annotations

import torch

__all__ = ["coords_grid"]


def coords_grid(batch: int, ht: int, wd: int, device=None) -> torch.Tensor:
    """``[batch, 2, ht, wd]`` float32 grid; channel 0 = x (column), 1 = y (row).

    Same values as the reference's ``coords_grid``; ``device`` lets callers build
    it directly on the GPU instead of the reference's host grid + copy
    (core/raft.py:81-82).
    """
    ys, xs = torch.meshgrid(torch.arange(ht, device=device, dtype=torch.float32),
                            torch.arange(wd, device=device, dtype=torch.float32),
                            indexing="ij")
    return torch.stack((xs, ys), dim=0)[None].repeat(batch, 1, 1, 1)
