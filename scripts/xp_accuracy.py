#!/usr/bin/env python3
"""Accuracy of split-build variants (experiments target, never shipped).

Builds the paged f32 pyramid of one seeded pair with ``dxr_xp_build`` variants
and with the exact-f32 MFMA build (``DXR_BUILD_EXACT_F32``), unpacks every level
and compares each with a float64 reference (torch matmul + avg-pool in f64 on
the GPU).  Prints, per variant and level, max |err| and its ratio to the
exact-f32 build's max |err| — the bar of tests/test_gpu_parity.py
test_split_build_f32_accuracy (<= 2x).

Usage: python scripts/xp_accuracy.py [--H 55 --W 128] [--dist fnet] [--xp 0,1003]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--H", type=int, default=55)
    ap.add_argument("--W", type=int, default=128)
    ap.add_argument("--D", type=int, default=256)
    ap.add_argument("--dist", default="fnet", choices=["fnet", "normal", "small", "large"])
    ap.add_argument("--xp", default="0,1003")
    a = ap.parse_args()
    import dexiraft_amd
    nat = dexiraft_amd._native
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.dxr_xp_build.restype = ctypes.c_int
    lib.dxr_xp_build.argtypes = [vp, vp, i64, i64, i64, i64, vp, ctypes.c_int, vp]
    lib.dxr_pyramid_unpack.restype = ctypes.c_int
    lib.dxr_pyramid_unpack.argtypes = [vp, ctypes.c_int, i64, i64, i64, ctypes.c_int, ctypes.c_int,
                                       vp, vp]
    lib.dxr_corr_pyramid_build.restype = ctypes.c_int
    lib.dxr_corr_pyramid_build.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, i64, i64, i64, i64,
                                           ctypes.c_int, ctypes.c_float, vp, ctypes.c_int,
                                           ctypes.c_int, vp]
    dev = torch.device("cuda", 0)
    B, D, H, W = a.B, a.D, a.H, a.W
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    if a.dist == "fnet":
        f1, f2 = 1.1 + 1.45 * f1, 1.1 + 1.45 * f2
    elif a.dist == "small":
        f1, f2 = f1 * 1e-3, f2 * 1e-3
    elif a.dist == "large":
        f1 = f1 * 3e4            # some |x| above 65504: the H2 overflow fallback
    s = torch.cuda.current_stream().cuda_stream
    N = H * W
    ref = torch.matmul(f1.double().reshape(B, D, N).transpose(1, 2), f2.double().reshape(B, D, N))
    ref = (ref / D ** 0.5).reshape(B * N, 1, H, W)
    refs = [ref]
    for _ in range(3):
        refs.append(F.avg_pool2d(refs[-1], 2, stride=2))
    numel = nat.load().dxr_pyramid_numel(B, H, W, 4)
    pyr = torch.empty(numel, device=dev)

    def levels():
        out = []
        for lvl in range(4):
            h, w = H >> lvl, W >> lvl
            o = torch.empty((B * N, 1, h, w), device=dev)
            st = lib.dxr_pyramid_unpack(pyr.data_ptr(), 0, B, H, W, 4, lvl, o.data_ptr(), s)
            assert st == 0, st
            out.append(o)
        torch.cuda.synchronize()
        return out

    def errs(lv):
        return [(lv[i].double() - refs[i]).abs().max().item() for i in range(4)]

    pyr.fill_(float("nan"))
    st = lib.dxr_corr_pyramid_build(f1.data_ptr(), f2.data_ptr(), 0, 0, B, D, H, W, 4,
                                    float(D) ** 0.5, pyr.data_ptr(), 0, 1, s)
    assert st == 0, st
    base = errs(levels())
    print(json.dumps({"variant": "exact_f32", "max_err": base,
                      "max_ref": [r.abs().max().item() for r in refs]}), flush=True)
    for xp in (int(x) for x in a.xp.split(",")):
        pyr.fill_(float("nan"))
        st = lib.dxr_xp_build(f1.data_ptr(), f2.data_ptr(), B, D, H, W, pyr.data_ptr(), xp, s)
        assert st == 0, (xp, st)
        e = errs(levels())
        print(json.dumps({"variant": xp, "max_err": e,
                          "ratio_to_exact": [round(x / y, 3) for x, y in zip(e, base)]}), flush=True)


if __name__ == "__main__":
    main()
