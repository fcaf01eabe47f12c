"""Time alt_cuda_corr.forward / backward (reference FFI form) at a given size.

usage: python scripts/time_alt_backward.py [H W C r]   (default 1080p/8: 135 240 256 4)
"""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import dexiraft_amd as dx  # noqa: E402

H, W, C, r = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (135, 240, 256, 4)))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
f1 = torch.randn(1, H, W, C, device=dev, generator=g)
f2 = torch.randn(1, H, W, C, device=dev, generator=g)
ys, xs = torch.meshgrid(torch.arange(H, device=dev), torch.arange(W, device=dev), indexing="ij")
c = torch.stack([xs, ys], -1).float()[None, None] + torch.randn(1, 1, H, W, 2, device=dev,
                                                                generator=g) * 3
rd = 2 * r + 1
cg = torch.randn(1, 1, rd * rd, H, W, device=dev, generator=g)
for name, fn in (("forward", lambda: dx.alt_cuda_corr.forward(f1, f2, c, r)),
                 ("backward", lambda: dx.alt_cuda_corr.backward(f1, f2, c, cg, r))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / n * 1e3:.1f} us  (H={H} W={W} C={C} r={r})", flush=True)
