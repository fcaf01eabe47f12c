#!/usr/bin/env python3
"""Can the split build's K loop and its pyramid writes overlap? (experiments target)

Times, in one process: (a) the f16-pair split build without epilogue stores
(dxr_xp_build xp 2001) alone, (b) a plain fill of a pyramid-sized buffer alone,
(c) both launched together on two streams, (d) the full build (xp 1003).
If (c) is close to max(a, b), the chip can overlap MFMA K loops with HBM writes
and the build's serialisation is a scheduling matter; if (c) is close to a + b,
the two contend for a shared resource.

Usage: python scripts/xp_overlap.py [--B 1]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    import dexiraft_amd
    nat = dexiraft_amd._native
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    fn = lib.dxr_xp_build
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                   ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    B, D, H, W = a.B, 256, 55, 128
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    n = nat.load().dxr_pyramid_numel(B, H, W, 4)
    pyr = torch.empty(n, device=dev)
    other = torch.empty(n, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def build(xp, s):
        assert fn(f1.data_ptr(), f2.data_ptr(), B, D, H, W, pyr.data_ptr(), xp, s.cuda_stream) == 0

    def timed(work):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            work()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps * 1e3

    cur = torch.cuda.current_stream()

    def both():
        ev = torch.cuda.Event()
        ev.record(cur)
        s1.wait_event(ev)
        s2.wait_event(ev)
        build(2001, s1)
        with torch.cuda.stream(s2):
            other.fill_(1.0)
        e1, e2 = torch.cuda.Event(), torch.cuda.Event()
        e1.record(s1)
        e2.record(s2)
        cur.wait_event(e1)
        cur.wait_event(e2)

    tasks = {
        "k_loop_only": lambda: build(2001, cur),
        "fill_only": lambda: other.fill_(1.0),
        "both_concurrent": both,
        "full_build": lambda: build(1003, cur),
    }
    for w in tasks.values():
        w()
    res = {k: [] for k in tasks}
    for _ in range(a.rounds):
        for k, w in tasks.items():
            res[k].append(timed(w))
    out = {k: round(float(np.median(v)), 2) for k, v in res.items()}
    out["pyramid_bytes"] = n * 4
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
