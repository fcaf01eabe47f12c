"""Generate the end-to-end flow golden by running the REFERENCE update loop on CPU.

Run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_e2e_golden.py
It imports the reference's ``CorrBlock`` (core/corr.py:12-50) and
``BasicUpdateBlock`` (core/update.py:121-140), loads the latter with the
name-keyed deterministic weights of tests/e2e_flow.py, and runs the
two-volume iteration of RAFT.forward (core/raft.py:160-192, restated here
line for line around the reference modules, since RAFT.__init__ needs the
absent DexiNed checkpoint) on the synthetic fmaps/context of
tests/e2e_flow.e2e_inputs.  Output: tests/golden/e2e_chairs.npz with the
low-res flow after every iteration, the final edge flow, and the final
upsampled flow (core/raft.py:87-99) subsampled every 4th pixel.

The fp64 run of the same loop is recorded too (``flow_f64``): its EPE to the
fp32 reference is the loop's own sensitivity to fp32 rounding, the floor any
fp32 implementation is judged against.
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
REFERENCE = Path("/root/reference/core")

import e2e_flow as ef  # noqa: E402


def run(dtype):
    sys.path.insert(0, str(REFERENCE))
    from corr import CorrBlock          # reference core/corr.py
    from update import BasicUpdateBlock  # reference core/update.py

    args = argparse.Namespace(corr_levels=ef.LEVELS, corr_radius=ef.RADIUS)
    block = BasicUpdateBlock(args, hidden_dim=ef.HDIM).to(dtype)
    block.load_state_dict({k: torch.from_numpy(v) for k, v in ef.update_weights().items()})
    block.eval()
    x = {k: torch.from_numpy(v).to(dtype) for k, v in ef.e2e_inputs().items()}
    with torch.no_grad():
        corr_fn = CorrBlock(x["fmap1"], x["fmap2"], radius=ef.RADIUS)
        corr_en = CorrBlock(x["fem1"], x["fem2"], radius=ef.RADIUS)
        # core/raft.py:160-192, verbatim semantics
        B, _, H, W = x["net"].shape
        net, inp, enet, einp = x["net"], x["inp"], x["enet"], x["einp"]
        coords0 = ef.coords_grid(B, H, W, "cpu").to(dtype)
        coords1 = coords0.clone()
        ecoords0 = coords0.clone()
        ecoords1 = coords0.clone()
        flows = []
        for _ in range(ef.E2E["iters"]):
            corr = corr_fn(coords1).to(dtype)
            ecorr = corr_en(ecoords1).to(dtype)
            flow = coords1 - coords0
            eflow = ecoords1 - ecoords0
            net, up_mask, delta_flow = block(net, inp, corr, flow)
            enet, _, delta_eflow = block(enet, einp, ecorr, eflow)
            coords1 = coords1 + delta_flow + delta_eflow
            ecoords1 = ecoords1 + delta_eflow
            flows.append((coords1 - coords0).clone())
        up = ef.upsample_flow(coords1 - coords0, up_mask)
    return [f.double().numpy() for f in flows], (ecoords1 - ecoords0).double().numpy(), up.double().numpy()


def main():
    torch.set_num_threads(8)
    flows, eflow, up = run(torch.float32)
    # fp64 loop: same modules and CorrBlock in double (core/corr.py:39 adds a float32
    # delta, promoted), i.e. the fp32 loop's own rounding sensitivity.
    flows64, _, _ = run(torch.float64)
    out = {
        "flows": np.stack(flows).astype(np.float32),       # [iters, 1, 2, H, W]
        "eflow": eflow.astype(np.float32),
        "flow_up_sub4": up[:, :, ::4, ::4].astype(np.float32),
        "flow_f64": flows64[-1],
        "epe_f32_vs_f64": np.float64(np.sqrt(((flows[-1] - flows64[-1]) ** 2).sum(1)).mean()),
    }
    np.savez_compressed(HERE / "e2e_chairs.npz", **out)
    f = flows[-1]
    print("final flow |mean| %.4f px, max %.3f px; eflow max %.3f; fp32-vs-fp64 EPE %.3e px"
          % (np.abs(f).mean(), np.abs(f).max(), np.abs(eflow).max(), out["epe_f32_vs_f64"]))


if __name__ == "__main__":
    main()
