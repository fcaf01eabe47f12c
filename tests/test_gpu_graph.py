"""The bench's measured step — one HIP graph holding the build and 12 lookups
(bench.py) — produces exactly what the eager calls produce, on replay after
replay, for both blocks.  Guards that the graph-timed number is valid work."""
from __future__ import annotations

import pytest
import torch

import datagen as dg

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def dx():
    import dexiraft_amd
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dexiraft_amd.load_native()
    return dexiraft_amd


@pytest.mark.parametrize("block", ["CorrBlock", "AlternateCorrBlock"])
def test_step_graph_matches_eager(dx, block):
    B, D, H, W, iters = 1, 256, 32, 48, 12
    f1 = torch.from_numpy(dg.fmap(201, B, D, H, W, "fnet")).to(DEV)
    f2 = torch.from_numpy(dg.fmap(202, B, D, H, W, "fnet")).to(DEV)
    cs = [torch.from_numpy(dg.coords(210 + k, B, H, W, "normal", 4.0)).to(DEV) for k in range(iters)]
    cls = getattr(dx, block)
    state = {}

    def step():
        blk = cls(f1, f2, radius=4)
        state["outs"] = [blk(c) for c in cs]

    stream = torch.cuda.Stream(device=DEV)
    with torch.no_grad(), torch.cuda.stream(stream):
        step()
        ref = [o.clone() for o in state["outs"]]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            step()
        for _ in range(3):
            for o in state["outs"]:
                o.zero_()
            g.replay()
            stream.synchronize()
            for a, b in zip(state["outs"], ref):
                assert torch.equal(a, b)


def test_multi_step_graph_matches_eager(dx):
    """bench.py's graph of G whole steps (--steps-per-graph): each step's block is
    released before the next is built, so later steps reuse the graph pool's
    memory; every step still produces its eager outputs, here over two pair sets."""
    B, D, H, W, iters, G = 1, 256, 24, 40, 12, 4
    sets = []
    for s in range(2):
        f1 = torch.from_numpy(dg.fmap(301 + 10 * s, B, D, H, W, "fnet")).to(DEV)
        f2 = torch.from_numpy(dg.fmap(302 + 10 * s, B, D, H, W, "fnet")).to(DEV)
        cs = [torch.from_numpy(dg.coords(310 + 10 * s + k, B, H, W, "normal", 4.0)).to(DEV)
              for k in range(iters)]
        sets.append((f1, f2, cs))
    state, kept = {}, {}

    def step(i):
        state.pop("cb", None)
        f1, f2, cs = sets[i % 2]
        state["cb"] = dx.CorrBlock(f1, f2, radius=4)
        kept[i] = [state["cb"](c) for c in cs]

    stream = torch.cuda.Stream(device=DEV)
    with torch.no_grad(), torch.cuda.stream(stream):
        ref = {}
        for i in range(2):
            step(i)
            ref[i] = [o.clone() for o in kept[i]]
        kept.clear()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for i in range(G):
                step(i)
        for _ in range(2):
            for outs in kept.values():
                for o in outs:
                    o.fill_(float("nan"))
            g.replay()
            stream.synchronize()
            for i in range(G):
                for a, b in zip(kept[i], ref[i % 2]):
                    assert torch.equal(a, b)
