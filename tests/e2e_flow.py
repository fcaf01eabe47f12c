"""End-to-end flow harness: the Dexi+RAFT refinement loop around a correlation block.

Test infrastructure only.  It restates, with functional torch ops, the part of
the reference model that consumes the correlation lookups, so the north-star
criterion "final flow EPE < 1e-3 px (fp32)"  can be checked on
the GPU box without the reference:

  * BasicMotionEncoder / SepConvGRU / FlowHead / mask head
    (reference core/update.py:5-14, 35-60, 81-100, 121-140);
  * the two-volume iteration of RAFT.forward (core/raft.py:165-192): one
    correlation block over (fmap1, fmap2), one over the edge maps
    (fem1, fem2), a shared update block, ``coords1 += delta_flow +
    delta_eflow`` and ``ecoords1 += delta_eflow``;
  * convex 8x upsampling (core/raft.py:87-99).

The encoders (fnet/cnet/efnet/ecnet, DexiNed) are outside the hot path: their
outputs are synthesised by tests/datagen.py (fmaps: the fnet-like distribution;
context: tanh / relu of normals, as core/raft.py:151-158 applies them).
Weights are generated deterministically per reference parameter name (uniform
in +-1/sqrt(fan_in), PyTorch's default Conv2d bound), so the reference model
loaded with the same dict (tests/golden/make_e2e_golden.py) and this harness
compute the same function.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch
import torch.nn.functional as F

import datagen as dg

HDIM = CDIM = 128
RADIUS, LEVELS = 4, 4
CORR_PLANES = LEVELS * (2 * RADIUS + 1) ** 2

# reference BasicUpdateBlock(args(corr_levels=4, corr_radius=4), hidden_dim=128)
# state_dict names and shapes (core/update.py:81-88, 35-44, 6-10, 121-130).
PARAMS = {
    "encoder.convc1": (256, CORR_PLANES, 1, 1),
    "encoder.convc2": (192, 256, 3, 3),
    "encoder.convf1": (128, 2, 7, 7),
    "encoder.convf2": (64, 128, 3, 3),
    "encoder.conv": (126, 256, 3, 3),
    "gru.convz1": (128, 384, 1, 5),
    "gru.convr1": (128, 384, 1, 5),
    "gru.convq1": (128, 384, 1, 5),
    "gru.convz2": (128, 384, 5, 1),
    "gru.convr2": (128, 384, 5, 1),
    "gru.convq2": (128, 384, 5, 1),
    "flow_head.conv1": (256, 128, 3, 3),
    "flow_head.conv2": (2, 256, 3, 3),
    "mask.0": (256, 128, 3, 3),
    "mask.2": (576, 256, 1, 1),
}

# E2E case: config 1 (FlyingChairs 368x496 -> fmap 46x62), 12 iterations.
# ``flow_gain`` scales the flow head's output layer so that random weights give
# displacements of several pixels (taps crossing cells, some off the map).
E2E = {"H": 46, "W": 62, "D": 256, "iters": 12, "weight_seed": 5000, "input_seed": 6000,
       "flow_gain": 8.0}


def update_weights(seed: int = E2E["weight_seed"]) -> dict[str, np.ndarray]:
    """Reference-named state dict (float32 numpy) from the portable generator."""
    out = {}
    for name, shape in PARAMS.items():
        fan_in = shape[1] * shape[2] * shape[3]
        bound = 1.0 / np.sqrt(fan_in)
        if name == "flow_head.conv2":
            bound *= E2E["flow_gain"]
        key = seed + zlib.crc32(name.encode())
        n = int(np.prod(shape))
        out[name + ".weight"] = (bound * (2 * dg.uniform(key, n) - 1)).reshape(shape).astype(np.float32)
        out[name + ".bias"] = (bound * (2 * dg.uniform(key + 1, shape[0]) - 1)).astype(np.float32)
    return out


def e2e_inputs(seed: int = E2E["input_seed"], H: int = E2E["H"], W: int = E2E["W"],
               D: int = E2E["D"]) -> dict[str, np.ndarray]:
    """fmaps (fnet-like) for the image and edge volumes, and context features."""
    out = {k: dg.fmap(seed + i, 1, D, H, W, "fnet") for i, k in enumerate(("fmap1", "fmap2", "fem1", "fem2"))}
    for i, k in enumerate(("net", "inp", "enet", "einp")):
        z = dg.normal(seed + 10 + i, HDIM * H * W).reshape(1, HDIM, H, W)
        z = np.tanh(z) if k in ("net", "enet") else np.maximum(z, 0.0)
        out[k] = z.astype(np.float32)
    return out


def _conv(x, W, name, pad):
    return F.conv2d(x, W[name + ".weight"], W[name + ".bias"], padding=pad)


def update_block(W, net, inp, corr, flow):
    """BasicUpdateBlock.forward (core/update.py:132-140): (net, mask, delta_flow)."""
    # BasicMotionEncoder (core/update.py:90-100)
    cor = F.relu(_conv(corr, W, "encoder.convc1", 0))
    cor = F.relu(_conv(cor, W, "encoder.convc2", 1))
    flo = F.relu(_conv(flow, W, "encoder.convf1", 3))
    flo = F.relu(_conv(flo, W, "encoder.convf2", 1))
    out = F.relu(_conv(torch.cat([cor, flo], 1), W, "encoder.conv", 1))
    x = torch.cat([inp, out, flow], 1)
    # SepConvGRU (core/update.py:46-60): horizontal then vertical pass
    h = net
    for sfx, pad in (("1", (0, 2)), ("2", (2, 0))):
        hx = torch.cat([h, x], 1)
        z = torch.sigmoid(_conv(hx, W, "gru.convz" + sfx, pad))
        r = torch.sigmoid(_conv(hx, W, "gru.convr" + sfx, pad))
        q = torch.tanh(_conv(torch.cat([r * h, x], 1), W, "gru.convq" + sfx, pad))
        h = (1 - z) * h + z * q
    # FlowHead (core/update.py:13-14) and the mask head (core/update.py:126-129,139)
    delta = _conv(F.relu(_conv(h, W, "flow_head.conv1", 1)), W, "flow_head.conv2", 1)
    mask = 0.25 * _conv(F.relu(_conv(h, W, "mask.0", 1)), W, "mask.2", 0)
    return h, mask, delta


def upsample_flow(flow, mask):
    """Convex 8x upsampling (core/raft.py:87-99)."""
    N, _, H, W = flow.shape
    mask = torch.softmax(mask.view(N, 1, 9, 8, 8, H, W), dim=2)
    up = F.unfold(8 * flow, [3, 3], padding=1).view(N, 2, 9, 1, 1, H, W)
    up = torch.sum(mask * up, dim=2).permute(0, 1, 4, 2, 5, 3)
    return up.reshape(N, 2, 8 * H, 8 * W)


def coords_grid(B, H, W, device):
    ys, xs = torch.meshgrid(torch.arange(H, device=device, dtype=torch.float32),
                            torch.arange(W, device=device, dtype=torch.float32), indexing="ij")
    return torch.stack([xs, ys])[None].repeat(B, 1, 1, 1)


def refine(corr_fn, corr_en, W, ctx, iters=E2E["iters"]):
    """RAFT.forward's iteration (core/raft.py:160-192) with given correlation blocks.

    ``corr_fn`` / ``corr_en`` map coords [B,2,H,W] -> [B,324,H,W].  ``ctx`` holds
    net/inp/enet/einp tensors.  Returns (flow_lowres list per iteration,
    final upsampled flow, final edge flow).
    """
    net, inp, enet, einp = ctx["net"], ctx["inp"], ctx["enet"], ctx["einp"]
    B, _, H, Wd = net.shape
    coords0 = coords_grid(B, H, Wd, net.device)
    coords1 = coords0.clone()
    ecoords0 = coords_grid(B, H, Wd, net.device)
    ecoords1 = ecoords0.clone()
    flows = []
    up = None
    for _ in range(iters):
        corr = corr_fn(coords1)
        ecorr = corr_en(ecoords1)
        flow = coords1 - coords0
        eflow = ecoords1 - ecoords0
        net, up_mask, delta_flow = update_block(W, net, inp, corr, flow)
        enet, _, delta_eflow = update_block(W, enet, einp, ecorr, eflow)
        coords1 = coords1 + delta_flow + delta_eflow
        ecoords1 = ecoords1 + delta_eflow
        flows.append(coords1 - coords0)
        up = upsample_flow(coords1 - coords0, up_mask)
    return flows, up, ecoords1 - ecoords0


def epe(a, b) -> float:
    """Mean end-point error (px) between two flow fields [B,2,H,W]."""
    a = torch.as_tensor(a, dtype=torch.float64).cpu()
    b = torch.as_tensor(b, dtype=torch.float64).cpu()
    return float(torch.sqrt(((a - b) ** 2).sum(1)).mean())


def torch_weights(W: dict[str, np.ndarray], device) -> dict[str, torch.Tensor]:
    return {k: torch.from_numpy(v).to(device) for k, v in W.items()}


class E2EModel:
    """A ``model(image1, image2, iters=, test_mode=True) -> (flow_low, flow_up)``
    for ``driver.infer_pairs`` (the reference RAFT.forward signature,
    core/raft.py:101): the refinement loop above around ``block_cls`` blocks.
    The encoders are out of scope, so the "images" only select the synthetic
    encoder outputs: pair p is an image whose pixels all equal p, and its
    inputs are ``e2e_inputs(E2E['input_seed'] + 97 * p)`` (p = 0: the golden's)."""

    def __init__(self, block_cls, device, weights=None):
        self.block_cls = block_cls
        self.device = device
        self.W = torch_weights(weights or update_weights(), device)

    def inputs(self, p: int) -> dict[str, torch.Tensor]:
        x = e2e_inputs(E2E["input_seed"] + 97 * p)
        return {k: torch.from_numpy(v).to(self.device) for k, v in x.items()}

    def __call__(self, image1, image2, iters=E2E["iters"], test_mode=True):
        p = int(round(float(image1.reshape(-1)[0])))
        t = self.inputs(p)
        corr_fn = self.block_cls(t["fmap1"], t["fmap2"])
        corr_en = self.block_cls(t["fem1"], t["fem2"])
        flows, up, _ = refine(corr_fn, corr_en, self.W, t, iters)
        return flows[-1], up
