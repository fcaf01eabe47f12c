#!/usr/bin/env python3
"""Same-process A/B of lookup variants inside the bench's step (profiles only).

The isolated back-to-back launches of scripts/xp_lookup.py replay one coordinate
set against a cache-warm pyramid; the bench's step (bench.py) runs the build and
then 12 lookups with 12 different coordinate sets.  This script captures that
step as one HIP graph per variant, with the same synthetic inputs as bench.py,
and times interleaved rounds of replays (HIP events, after a clock warm-up):

  --block corr  build (product CorrBlock; variant -4: the --prev-lib library's
                dxr_corr_pyramid_build_ws, product lookups; -5: the --prev-lib library's
                build and lookups, for A/Bs across a pyramid-layout change; -6: the experiments
                target's DMA build, product lookups) + 12 lookups by dxr_xp_lookup variant
                (libdexiraft_corr_exp.so: 0 spatial level-2/3 gathers, 32 query-major,
                64 the 256 x 16 shape, 128 1024 x 64) or the product's (-1);
  --block alt   12 on-the-fly lookups: dxr_alt_corr_lookup (-1, tile order),
                dxr_alt_corr_lookup_ws (-2, queries ordered first) or dxr_xp_alt_lookup
                variant v - 100 (100 the product's ordered form, 101 LDS-DMA cell staging).

Usage: python scripts/ab_step.py [--workload sintel] [--batch 1] [--variants -1 32 64]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))

SHAPES = {"sintel": (55, 128), "chairs": (46, 62), "kitti": (47, 156), "1080p": (136, 240)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="sintel", choices=sorted(SHAPES))
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--block", default="corr", choices=["corr", "alt"])
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--variants", type=int, nargs="+", default=[-1, 32, 64])
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--no-check", type=int, nargs="*", default=[],
                    help="variants whose outputs are not checked (timing ablations)")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--prev-lib", default=str(REPO / "scripts" / "libdexiraft_corr_r04.so"),
                    help="variant -3: dxr_corr_lookup of this earlier product library; "
                         "-4: its build")
    a = ap.parse_args()
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    lib = dexiraft_amd.load_native()
    xp = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    xp.dxr_xp_build_tail.restype = i32
    xp.dxr_xp_build_tail.argtypes = [vp, vp, i32, i32, i64, i64, i64, i64, vp, vp, i32, vp]
    xp.dxr_xp_lookup.restype = i32
    xp.dxr_xp_lookup.argtypes = [vp, i32, i64, i64, i64, i32, vp, vp, i32, vp, vp]
    xp.dxr_xp_alt_lookup.restype = i32
    xp.dxr_xp_alt_lookup.argtypes = [vp, ctypes.POINTER(vp), vp, vp, i64, i64, i64, i64, i32,
                                     ctypes.c_float, vp, i32, vp]
    prev = None
    if -3 in a.variants or -4 in a.variants or -5 in a.variants:
        prev = ctypes.CDLL(a.prev_lib)
        for name, (res, args) in nat.SIGNATURES.items():
            if hasattr(prev, name):
                getattr(prev, name).restype = res
                getattr(prev, name).argtypes = args
    dev = torch.device("cuda", 0)
    B, (H, W), D = a.batch, SHAPES[a.workload], 256
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    if a.dtype == "bf16":
        f1, f2 = f1.bfloat16(), f2.bfloat16()
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack((xs, ys))[None].expand(B, 2, H, W)
    coords = [(grid + 4.0 * torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous()
              for _ in range(12)]
    stream = torch.cuda.Stream(device=dev)
    with torch.no_grad(), torch.cuda.stream(stream):
        if a.block == "corr":
            cb = dexiraft_amd.CorrBlock(f1, f2)
            ref = [cb(c) for c in coords]
        else:
            ab = dexiraft_amd.AlternateCorrBlock(f1, f2)
            ref = [ab(c) for c in coords]
        outs = [torch.empty_like(r) for r in ref]
        nws = lib.dxr_alt_workspace_bytes(B, H, W, 4)
        ws = torch.empty(max(nws, 0), dtype=torch.uint8, device=dev)
        s = stream.cuda_stream

        bws = None
        if a.block == "corr":
            nb = lib.dxr_build_workspace_bytes(cb._in_dt, B, D, H, W)
            bws = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
            ppyr = torch.empty_like(cb._buf) if -5 in a.variants else None

        def step(v):
            if a.block == "corr" and v == -5:   # the previous library end to end, own buffer
                st = prev.dxr_corr_pyramid_build_ws(
                    f1.data_ptr(), f2.data_ptr(), cb._in_dt, nat.DXR_NCHW, B, D, H, W, 4,
                    float(D) ** 0.5, ppyr.data_ptr(), cb._pyr_dt, nat.DXR_BUILD_AUTO,
                    bws.data_ptr(), nb, s)
                assert st == 0
                for c, o in zip(coords, outs):
                    st = prev.dxr_corr_lookup(ppyr.data_ptr(), cb._pyr_dt, B, H, W, 4, 4, c.data_ptr(),
                                              o.data_ptr(), s)
                    assert st == 0
            elif a.block == "corr" and v == -6:   # the experiments target's DMA build (tail
                # policy 1, the product's), product lookups
                st = xp.dxr_xp_build_tail(f1.data_ptr(), f2.data_ptr(), cb._in_dt, nat.DXR_NCHW, B, D,
                                          H, W, cb._buf.data_ptr(), bws.data_ptr(), 1, s)
                assert st == 0
                for c, o in zip(coords, outs):
                    st = lib.dxr_corr_lookup(cb._buf.data_ptr(), cb._pyr_dt, B, H, W, 4, 4, c.data_ptr(),
                                             o.data_ptr(), s)
                    assert st == 0
            elif a.block == "corr":
                if v == -4:   # the previous library's build into the same buffer
                    st = prev.dxr_corr_pyramid_build_ws(
                        f1.data_ptr(), f2.data_ptr(), cb._in_dt, nat.DXR_NCHW, B, D, H, W, 4,
                        float(D) ** 0.5, cb._buf.data_ptr(), cb._pyr_dt, nat.DXR_BUILD_AUTO,
                        bws.data_ptr(), nb, s)
                else:
                    f_1, f_2, st = cb._launch_build(f1, f2)
                assert st == 0
                for c, o in zip(coords, outs):
                    if v in (-1, -3, -4):
                        fn = prev.dxr_corr_lookup if v == -3 else lib.dxr_corr_lookup
                        st = fn(cb._buf.data_ptr(), cb._pyr_dt, B, H, W, 4, 4, c.data_ptr(),
                                o.data_ptr(), s)
                    else:
                        st = xp.dxr_xp_lookup(cb._buf.data_ptr(), cb._pyr_dt, B, H, W, 4,
                                              c.data_ptr(), o.data_ptr(), v, None, s)
                    assert st == 0
            else:
                for c, o in zip(coords, outs):
                    args = (ab._f1_nhwc.data_ptr(), ab._f2_ptrs, c.data_ptr(), o.data_ptr(), B, H,
                            W, D, 4, 4, 16.0)
                    if v == -1:
                        st = lib.dxr_alt_corr_lookup(*args, s)
                    elif v == -2:
                        st = lib.dxr_alt_corr_lookup_ws(*args, ws.data_ptr(), nws, s)
                    else:   # experiments: dxr_xp_alt_lookup variant v - 100
                        st = xp.dxr_xp_alt_lookup(*args[:9], args[10], ws.data_ptr(), v - 100, s)
                    assert st == 0

        graphs = {}
        for v in a.variants:
            step(v)
            torch.cuda.synchronize()
            if v not in a.no_check:   # timing ablations compute something else
                for o, r in zip(outs, ref):
                    assert torch.equal(torch.nan_to_num(o, nan=1.5), torch.nan_to_num(r, nan=1.5)), v
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=stream):
                step(v)
            graphs[v] = gr
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            for v in a.variants:
                graphs[v].replay()
            torch.cuda.synchronize()
        res = {v: [] for v in a.variants}
        for _ in range(a.rounds):
            for v in a.variants:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    graphs[v].replay()
                e1.record(stream)
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    print(json.dumps({"workload": a.workload, "batch": B, "block": a.block, "dtype": a.dtype,
                      "what": "us per step graph (corr: build + 12 lookups; alt: 12 lookups), "
                              "min / median of rounds",
                      "us_per_step": {v: [round(min(t), 1), round(float(np.median(t)), 1)]
                                      for v, t in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
