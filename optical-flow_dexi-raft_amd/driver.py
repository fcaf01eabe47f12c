"""Inference driver around the correlation path.

Counterpart of the reference's evaluation loop (evaluate.py:37-57, 102-133):
pad a pair to a multiple of 8 (``InputPadder``, core/utils/utils.py:7-24), run
the model in test mode, unpad the full-resolution flow and write it as a
Middlebury ``.flo`` file (core/utils/frame_utils.py:70-99 ``writeFlow``).
The model is the caller's — the reference RAFT / Dexi+RAFT with this package's
``CorrBlock`` swapped in: the encoders, DexiNed and the
update block are outside this repository's scope.

Multi-GPU: one process per GPU (``torch.distributed.run``).  ``infer_pairs``
takes the full list of pairs, runs the contiguous share ``shard.pair_range``
gives this rank, and — when asked — all-gathers the unpadded flows to every
rank over RCCL/xGMI (``shard.gather_pairs``): the only collective, off the
correlation path.
"""
from __future__ import annotations

from pathlib import Path
from typing import Callable, Sequence

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

from .shard import gather_pairs, pair_range

__all__ = ["InputPadder", "write_flo", "read_flo", "infer_pairs", "FLO_TAG"]

FLO_TAG = 202021.25   # 'PIEH' as a little-endian float32 (frame_utils.py:9,88)


class InputPadder:
    """Pads images so that H and W are multiples of 8 (core/utils/utils.py:7-24).

    ``mode='sintel'`` splits the padding between both sides; any other mode
    (the reference's 'kitti') pads right and bottom only.  Padding replicates
    the border (``F.pad(mode='replicate')``).
    """

    def __init__(self, dims, mode: str = "sintel"):
        self.ht, self.wd = (int(d) for d in dims[-2:])
        pad_ht = (((self.ht // 8) + 1) * 8 - self.ht) % 8
        pad_wd = (((self.wd // 8) + 1) * 8 - self.wd) % 8
        if mode == "sintel":
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, pad_ht // 2, pad_ht - pad_ht // 2]
        else:
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, 0, pad_ht]

    def pad(self, *inputs: torch.Tensor) -> list[torch.Tensor]:
        return [F.pad(x, self._pad, mode="replicate") for x in inputs]

    def unpad(self, x: torch.Tensor) -> torch.Tensor:
        ht, wd = x.shape[-2:]
        c = [self._pad[2], ht - self._pad[3], self._pad[0], wd - self._pad[1]]
        return x[..., c[0]:c[1], c[2]:c[3]]


def write_flo(path: str | Path, flow) -> None:
    """Middlebury .flo (frame_utils.py:70-99): float32 tag 202021.25, int32 width,
    int32 height, then row-major interleaved (u, v) float32.  ``flow``: [H, W, 2]
    (as the reference's ``writeFlow(uv)``) or a [2, H, W] tensor/array."""
    a = flow.detach().cpu().numpy() if isinstance(flow, torch.Tensor) else np.asarray(flow)
    if a.ndim == 3 and a.shape[0] == 2 and a.shape[2] != 2:
        a = a.transpose(1, 2, 0)
    if a.ndim != 3 or a.shape[2] != 2:
        raise ValueError(f"flow must be [H, W, 2] or [2, H, W], got {a.shape}")
    h, w = a.shape[:2]
    with open(path, "wb") as f:
        np.array([FLO_TAG], dtype="<f4").tofile(f)
        np.array([w, h], dtype="<i4").tofile(f)
        np.ascontiguousarray(a, dtype="<f4").tofile(f)


def read_flo(path: str | Path) -> np.ndarray:
    """Inverse of ``write_flo`` (frame_utils.py:13-33 ``readFlow``): [H, W, 2] float32."""
    with open(path, "rb") as f:
        tag = np.fromfile(f, "<f4", 1)
        if tag.size != 1 or tag[0] != np.float32(FLO_TAG):
            raise ValueError(f"{path}: not a .flo file (magic {tag})")
        w, h = (int(v) for v in np.fromfile(f, "<i4", 2))
        data = np.fromfile(f, "<f4", 2 * w * h)
    if data.size != 2 * w * h:
        raise ValueError(f"{path}: truncated ({data.size} of {2 * w * h} values)")
    return data.reshape(h, w, 2)


def infer_pairs(model: Callable, image1: torch.Tensor, image2: torch.Tensor, iters: int = 12,
                mode: str = "sintel", gather: bool = True,
                flo_paths: Sequence[str | Path] | None = None) -> torch.Tensor:
    """Full-resolution flows of P image pairs, sharded over the process group.

    ``image1, image2``: [P, 3, H, W] (every rank passes the same list; each runs
    its ``pair_range`` share, one pair per forward as evaluate.py does).
    ``model(img1, img2, iters=iters, test_mode=True)`` returns ``(flow_low,
    flow_up)`` (core/raft.py:192-193).  Returns [P, 2, H, W] float32 flows on
    every rank when ``gather`` (RCCL all-gather), else this rank's [p, 2, H, W].
    ``flo_paths[i]``, when given, receives pair i's flow from the rank that
    computed it.
    """
    if image1.shape != image2.shape or image1.dim() != 4:
        raise ValueError(f"image pairs must be [P, 3, H, W] twins, got {tuple(image1.shape)} "
                         f"and {tuple(image2.shape)}")
    total = int(image1.shape[0])
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    start, stop = pair_range(total, world, rank)
    padder = InputPadder(image1.shape, mode=mode)
    flows = []
    with torch.no_grad():
        for i in range(start, stop):
            a, b = padder.pad(image1[i:i + 1], image2[i:i + 1])
            _, flow_up = model(a, b, iters=iters, test_mode=True)
            flow = padder.unpad(flow_up[0]).float()
            if flo_paths is not None:
                write_flo(flo_paths[i], flow)
            flows.append(flow)
    h, w = image1.shape[-2:]
    local = torch.stack(flows) if flows else image1.new_empty((0, 2, h, w), dtype=torch.float32)
    return gather_pairs(local.contiguous(), total) if gather else local
