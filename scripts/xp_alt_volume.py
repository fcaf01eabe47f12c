#!/usr/bin/env python3
"""Timing ablations of the coarse-level volume GEMM (alt_volume_gemm_kernel,
csrc/alt_corr.hip) through the experiments target's dxr_xp_alt_volume_gemm:
xa 0 the product kernel, 1 no stores, 2 no split VALU, 4 no MFMAs, 6 neither
split nor MFMAs, 7 none of the three (the skeleton: loads, LDS, barriers), each
in the register-split form (r) or the LDS-DMA form on pre-split planes (d); and
the FULL box form (dxr_xp_alt_coarse_volumes_full) for comparison.  HIP events
around back-to-back launches on one stream, per level.  Variant 0 is checked
bit for bit against the product entry point dxr_alt_coarse_volumes (r0, d0, full).

Usage: python scripts/xp_alt_volume.py [--workload 1080p] [--levels 2 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))

SHAPES = {"sintel": (55, 128), "chairs": (46, 62), "kitti": (47, 156), "1080p": (136, 240)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="1080p", choices=sorted(SHAPES))
    ap.add_argument("--levels", type=int, nargs="+", default=[2, 3])
    ap.add_argument("--variants", nargs="+", default=["r0", "d0", "d1", "d4", "d7"],
                    help="r<xa>: the register-split form, d<xa>: the LDS-DMA form on pre-split "
                         "planes (split passes included in its time)")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    lib = dexiraft_amd.load_native()
    xp = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    xp.dxr_xp_alt_volume_gemm.argtypes = [vp, vp, vp, i64, i64, i64, i64, i32, i32, vp, vp]
    xp.dxr_xp_alt_volume_gemm.restype = i32
    xp.dxr_xp_alt_coarse_volumes_full.argtypes = [vp, vp, i64, i64, i64, i64, i32, i32, vp, vp]
    xp.dxr_xp_alt_coarse_volumes_full.restype = i32

    H, W = SHAPES[a.workload]
    B, D, L = 1, 256, 4
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    f1 = torch.randn((B, D, H, W), device=dev, generator=g)
    f2 = torch.randn((B, D, H, W), device=dev, generator=g)
    dexiraft_amd.AlternateCorrBlock.COARSE_LEVEL_MAX_CELLS = 0
    ab = dexiraft_amd.AlternateCorrBlock(f1, f2, num_levels=L, radius=4)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    res = {"workload": a.workload, "what": "us per launch, HIP events over back-to-back launches"}
    for lvl in a.levels:
        n = lib.dxr_alt_volume_numel(B, H, W, lvl + 1, lvl)
        vol = torch.zeros((n,), device=dev)
        wsb = lib.dxr_alt_coarse_volumes_ws_bytes(B, H, W, D, lvl + 1, lvl)
        ws = torch.empty((wsb,), dtype=torch.uint8, device=dev)
        ref = torch.zeros((n,), device=dev)
        # the product entry point for this one level (num_levels = lvl + 1, first = lvl)
        assert lib.dxr_alt_coarse_volumes(ab._f1_nhwc.data_ptr(), ab._f2_ptrs, B, H, W, D, lvl + 1,
                                          lvl, ref.data_ptr(), sp.value) == 0

        def run(v, out):
            if v == "split":   # the DMA form's two split passes alone (d0 - split = its GEMM)
                return xp.dxr_xp_alt_volume_gemm(ab._f1_nhwc.data_ptr(),
                                                 ab._f2_nhwc[lvl].data_ptr(), out.data_ptr(), B,
                                                 H, W, D, lvl, 99, ws.data_ptr(), sp) * 0
            if v == "full":
                return xp.dxr_xp_alt_coarse_volumes_full(ab._f1_nhwc.data_ptr(),
                                                         ctypes.cast(ab._f2_ptrs, vp), B, H, W, D,
                                                         lvl + 1, lvl, out.data_ptr(), sp)
            return xp.dxr_xp_alt_volume_gemm(ab._f1_nhwc.data_ptr(), ab._f2_nhwc[lvl].data_ptr(),
                                             out.data_ptr(), B, H, W, D, lvl, int(v[1:]),
                                             ws.data_ptr() if v[0] == "d" else None, sp)

        for _ in range(300):    # clock warm-up (the GPU raises its clocks after ~ms of load)
            run("r0", vol)
        torch.cuda.synchronize()
        for v in list(a.variants) + ["full"]:
            vol.zero_()         # page padding: written as zeros by the GEMM, not by FULL
            for _ in range(3):
                assert run(v, vol) == 0
            torch.cuda.synchronize()
            if v in ("r0", "d0", "full"):
                assert torch.equal(vol, ref), (lvl, v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.reps):
                run(v, vol)
            e1.record(stream)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.reps * 1e3
            res[f"level{lvl}_xa{v}"] = round(us, 2)
            print(f"level {lvl} variant {v}: {us:.2f} us", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
