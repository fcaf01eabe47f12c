#!/usr/bin/env python3
"""Per-workgroup timeline of the split build (experiments target, never shipped).

Runs ``dxr_xp_build`` with XP bit 10 (code 3024; 3025 = the same without
epilogue stores), which makes wave 0 of every workgroup record its CU (HW_ID,
XCC_ID) and shader-clock stamps: t0 start, t1 K loop done, t2 epilogue stores
issued, t3 stores complete.  Reads them back with ``dxr_xp_trace_read`` and
reports, in clock cycles: phase durations, workgroups per CU, resident
workgroups per CU over time, the gap between a slot freeing and the next
workgroup starting on that CU, and the tail (time after the median CU's last
workgroup ends).

Usage: python scripts/xp_trace.py [--B 1] [--xp 3024] [--H 55 --W 128]
"""
from __future__ import annotations

import argparse
import collections
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def pct(x, q):
    return float(np.percentile(np.asarray(x, dtype=np.float64), q))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--H", type=int, default=55)
    ap.add_argument("--W", type=int, default=128)
    ap.add_argument("--xp", type=int, default=3024)
    a = ap.parse_args()
    import dexiraft_amd
    nat = dexiraft_amd._native
    lib = ctypes.CDLL(str(nat.LIB_PATH.with_name("libdexiraft_corr_exp.so")))
    fn = lib.dxr_xp_build
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                   ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    rd = lib.dxr_xp_trace_read
    rd.restype = ctypes.c_int
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    dev = torch.device("cuda", 0)
    B, D, H, W = a.B, 256, a.H, a.W
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    pyr = torch.empty(nat.load().dxr_pyramid_numel(B, H, W, 4), device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        assert fn(f1.data_ptr(), f2.data_ptr(), B, D, H, W, pyr.data_ptr(), a.xp, s) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    assert fn(f1.data_ptr(), f2.data_ptr(), B, D, H, W, pyr.data_ptr(), a.xp, s) == 0
    e1.record()
    torch.cuda.synchronize()
    wall_us = e0.elapsed_time(e1) * 1e3
    nwg = B * ((H * W + 127) // 128) * ((H + 7) // 8) * ((W + 15) // 16)
    nwg = min(nwg, 32768)
    buf = np.zeros(nwg * 5, dtype=np.uint64)
    assert rd(buf.ctypes.data, buf.nbytes) == 0
    t = buf.reshape(nwg, 5)
    hw = (t[:, 0] & 0xFFFFFFFF).astype(np.int64)
    xcc = (t[:, 0] >> 32).astype(np.int64) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    ts = t[:, 1:].astype(np.int64)
    out = {"xp": a.xp, "B": B, "workgroups": nwg, "wall_us": round(wall_us, 2)}
    # per-XCC clock origin (counters are per XCD)
    spans = []
    for x in np.unique(xcc):
        m = xcc == x
        ts[m] -= ts[m, 0].min()
        spans.append(int(ts[m, 3].max()))
    span = max(spans)
    out["span_cycles"] = span
    out["clock_ghz_est"] = round(span / wall_us / 1e3, 3)
    k, e, w = ts[:, 1] - ts[:, 0], ts[:, 2] - ts[:, 1], ts[:, 3] - ts[:, 2]
    for name, v in (("kloop", k), ("epi_issue", e), ("epi_drain", w)):
        out[name] = {"p10": int(pct(v, 10)), "p50": int(pct(v, 50)), "p90": int(pct(v, 90))}
    per_cu = collections.defaultdict(list)
    for i in range(nwg):
        per_cu[int(key[i])].append(i)
    counts = collections.Counter(len(v) for v in per_cu.values())
    out["cus"] = len(per_cu)
    out["wgs_per_cu"] = dict(sorted(counts.items()))
    # residency and dispatch gaps
    max_res, gaps, ends = [], [], []
    busy_epi_overlap = []
    for cuk, idx in per_cu.items():
        ev = sorted(idx, key=lambda i: ts[i, 0])
        starts = [ts[i, 0] for i in ev]
        stops = sorted(ts[i, 3] for i in ev)
        res = 0
        pts = sorted([(ts[i, 0], 1) for i in ev] + [(ts[i, 3], -1) for i in ev],
                     key=lambda p: (p[0], p[1]))
        for _, d in pts:
            res += d
            max_res.append(res)
        first = starts[0]
        for i in ev:
            if ts[i, 0] - first < 2000:
                continue  # first wave on this CU
            prev = [x for x in stops if x <= ts[i, 0]]
            if prev:
                gaps.append(ts[i, 0] - prev[-1])
        ends.append(max(stops))
        # while a WG is in its epilogue (t1..t3), how many other WGs of the CU are in K loop
        for i in ev:
            lo, hi = ts[i, 1], ts[i, 3]
            tot = 0
            for j in ev:
                if j == i:
                    continue
                a0, a1 = ts[j, 0], ts[j, 1]
                tot += max(0, min(hi, a1) - max(lo, a0))
            busy_epi_overlap.append(tot / max(1, hi - lo))
    out["max_resident_per_cu"] = int(max(max_res))
    out["dispatch_gap"] = {"p10": int(pct(gaps, 10)), "p50": int(pct(gaps, 50)),
                           "p90": int(pct(gaps, 90))} if gaps else None
    out["cu_end"] = {"min": int(min(ends)), "p50": int(pct(ends, 50)), "max": int(max(ends))}
    out["kloop_wgs_during_epilogue"] = {"p10": round(pct(busy_epi_overlap, 10), 2),
                                        "p50": round(pct(busy_epi_overlap, 50), 2),
                                        "p90": round(pct(busy_epi_overlap, 90), 2)}
    print(json.dumps(out), flush=True)
    # one CU's timeline (the first), relative to its first start
    cuk = sorted(per_cu)[0]
    ev = sorted(per_cu[cuk], key=lambda i: ts[i, 0])
    base = ts[ev[0], 0]
    print(json.dumps({"cu": cuk, "timeline": [[int(ts[i, c] - base) for c in range(4)] for i in ev]}),
          flush=True)


if __name__ == "__main__":
    main()
