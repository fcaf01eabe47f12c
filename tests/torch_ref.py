"""A plain-PyTorch fp32 statement of the reference CorrBlock (TEST INFRASTRUCTURE).

GPU numerics tests differentiate it with torch autograd on the same device and
compare the HIP backward against it (the numpy oracle has a backward too, pinned
to the reference's autograd in tests/test_oracle_golden.py; this module is the
device-side checker for shapes the numpy oracle is too slow for).

Semantics restated (reference paths):
  volume   core/corr.py:52-60   f1^T f2 (per pair, [N, N]) / sqrt(D) in float32
  pyramid  core/corr.py:19-27   levels [B*N, 1, H_l, W_l], F.avg_pool2d(2, 2)
  lookup   core/corr.py:29-50   per level, samples at coords / 2^l + (ox, oy),
                                ox added to x (first meshgrid index), channel
                                l*(2r+1)^2 + ox_idx*(2r+1) + oy_idx
  sampler  core/utils/utils.py:57-71  pixel -> [-1, 1], F.grid_sample bilinear,
                                zero padding, align_corners=True
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class TorchCorrBlock:
    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        B, D, H, W = fmap1.shape
        vol = torch.bmm(fmap1.reshape(B, D, H * W).transpose(1, 2), fmap2.reshape(B, D, H * W))
        vol = vol / torch.sqrt(torch.tensor(float(D), dtype=torch.float32))
        lvl = vol.reshape(B * H * W, 1, H, W)
        self.levels = [lvl]
        for _ in range(num_levels - 1):
            lvl = F.avg_pool2d(lvl, 2, stride=2)
            self.levels.append(lvl)
        self.radius = radius
        self.shape = (B, H, W)

    def __call__(self, coords):
        B, H, W = self.shape
        r = self.radius
        rd = 2 * r + 1
        off = torch.arange(-r, r + 1, dtype=torch.float32, device=coords.device)
        ox = off.view(rd, 1).expand(rd, rd)          # x offset varies with the first index
        oy = off.view(1, rd).expand(rd, rd)
        c = coords.permute(0, 2, 3, 1).reshape(B * H * W, 1, 1, 2)
        outs = []
        for i, img in enumerate(self.levels):
            hl, wl = img.shape[-2:]
            x = c[..., 0] / 2 ** i + ox
            y = c[..., 1] / 2 ** i + oy
            grid = torch.stack((2 * x / (wl - 1) - 1, 2 * y / (hl - 1) - 1), dim=-1)
            s = F.grid_sample(img, grid, align_corners=True)     # [BN, 1, rd, rd]
            outs.append(s.reshape(B, H, W, rd * rd))
        return torch.cat(outs, dim=-1).permute(0, 3, 1, 2).contiguous()
