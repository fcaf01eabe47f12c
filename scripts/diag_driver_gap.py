#!/usr/bin/env python3
"""Why does the driver's bench command (--steps 20 --warmup 5) read a slower build
than longer runs?  Same-process diagnostics on the bench's Sintel inputs.

Variants (raw C-ABI calls into preallocated buffers, same kernels as CorrBlock):
  ws   : dxr_corr_pyramid_build_ws  (split pass + LDS-DMA build, round 3 product)
  nows : dxr_corr_pyramid_build     (register-split build, round 2)
Each variant has a step graph (build + 12 lookups with 12 coordinate sets) and a
build-only graph of 20 back-to-back builds.

Protocols (interleaved over variants, --rounds times):
  driver : bench.py's sequence at K=20 W=5: 0.5 s clock warm-up of step replays,
           5 warmup replays, sync, then 20 timed replays (host clock, as bench.py);
  long   : the same with K=200;
  cold   : 50 ms idle, then 20 timed replays (no warm-up);
  build  : build-only graph replays (HIP events) right after a clock warm-up.
During every timed region a one-wave probe on a side stream samples the shader
clock (s_memtime / s_memrealtime, scripts/diag_clock.hip) every 20-200 us.
Also reports the host time spent enqueueing the replays.
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
sys.path.insert(0, str(REPO / "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", nargs="+", default=["ws", "nows"])
    a = ap.parse_args()
    import bench  # noqa: E402  (make_inputs: the bench's own synthetic inputs)
    import dexiraft_amd
    from dexiraft_amd import _native as nat
    lib = dexiraft_amd.load_native()
    diag = ctypes.CDLL(str(REPO / "scripts" / "libdxr_diag.so"))
    diag.dxr_diag_clock_probe.restype = ctypes.c_int
    diag.dxr_diag_clock_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_ulonglong,
                                          ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    B, H, W, D = 1, 55, 128, 256
    f1, f2, coords = bench.make_inputs(B, H, W, "f32", seed=1234, dev=dev)
    stream = torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)
    numel = lib.dxr_pyramid_numel(B, H, W, 4)
    pyr = torch.empty(numel, device=dev)
    wsb = lib.dxr_build_workspace_bytes(nat.DXR_F32, B, D, H, W)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    outs = [torch.empty((B, 324, H, W), device=dev) for _ in range(12)]
    div = float(np.sqrt(np.float32(D)))
    probe = torch.zeros(2 * 4096, dtype=torch.int64, device=dev)

    def build(v):
        s = stream.cuda_stream
        if v == "ws":
            st = lib.dxr_corr_pyramid_build_ws(f1.data_ptr(), f2.data_ptr(), nat.DXR_F32,
                                               nat.DXR_NCHW, B, D, H, W, 4, div, pyr.data_ptr(),
                                               nat.DXR_F32, nat.DXR_BUILD_AUTO, ws.data_ptr(),
                                               wsb, s)
        else:
            st = lib.dxr_corr_pyramid_build(f1.data_ptr(), f2.data_ptr(), nat.DXR_F32,
                                            nat.DXR_NCHW, B, D, H, W, 4, div, pyr.data_ptr(),
                                            nat.DXR_F32, nat.DXR_BUILD_AUTO, s)
        assert st == 0, (v, st)

    def step(v):
        build(v)
        for c, o in zip(coords, outs):
            st = lib.dxr_corr_lookup(pyr.data_ptr(), nat.DXR_F32, B, H, W, 4, 4, c.data_ptr(),
                                     o.data_ptr(), stream.cuda_stream)
            assert st == 0

    g_step, g_build = {}, {}
    with torch.cuda.stream(stream):
        for v in a.variants:
            step(v)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                step(v)
            g_step[v] = g
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                for _ in range(20):
                    build(v)
            g_build[v] = g
    torch.cuda.synchronize()

    def start_probe(n, interval_ticks):
        probe.zero_()
        torch.cuda.synchronize()
        st = diag.dxr_diag_clock_probe(probe.data_ptr(), n, interval_ticks, side.cuda_stream)
        assert st == 0
        time.sleep(0.0005)   # let the probe wave start

    def read_probe(n):
        torch.cuda.synchronize()
        p = probe[: 2 * n].view(n, 2).cpu().numpy().astype(np.float64)
        dt, dr = np.diff(p[:, 0]), np.diff(p[:, 1])
        ok = dr > 0
        mhz = dt[ok] / dr[ok] * 100.0
        return mhz

    def clock_warmup(v, seconds=0.5):
        t = time.perf_counter()
        while time.perf_counter() - t < seconds:
            for _ in range(20):
                g_step[v].replay()
            torch.cuda.synchronize()

    def timed_steps(v, k, probe_n, probe_iv):
        start_probe(probe_n, probe_iv)
        t0 = time.perf_counter()
        for _ in range(k):
            g_step[v].replay()
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        return el, t_enq, read_probe(probe_n)

    def summarize(mhz, el):
        # samples inside the timed region only (probe starts just before it)
        if mhz.size == 0:
            return {}
        return {"mhz_med": round(float(np.median(mhz)), 0), "mhz_min": round(float(mhz.min()), 0),
                "mhz_p10": round(float(np.percentile(mhz, 10)), 0),
                "mhz_max": round(float(mhz.max()), 0)}

    results = []
    with torch.cuda.stream(stream):
        for rnd in range(a.rounds):
            for v in a.variants:
                # driver protocol
                clock_warmup(v)
                for _ in range(5):
                    g_step[v].replay()
                torch.cuda.synchronize()
                el, enq, mhz = timed_steps(v, 20, 300, 2000)
                n_in = max(1, int(el * 1e6 / 20))
                results.append({"round": rnd, "variant": v, "protocol": "driver_k20",
                                "us_per_step": round(el / 20 * 1e6, 1),
                                "host_enqueue_us_per_step": round(enq / 20 * 1e6, 1),
                                **summarize(mhz[:n_in], el)})
                # long protocol
                clock_warmup(v)
                for _ in range(20):
                    g_step[v].replay()
                torch.cuda.synchronize()
                el, enq, mhz = timed_steps(v, 200, 400, 20000)
                n_in = max(1, int(el * 1e6 / 200))
                results.append({"round": rnd, "variant": v, "protocol": "long_k200",
                                "us_per_step": round(el / 200 * 1e6, 1),
                                "host_enqueue_us_per_step": round(enq / 200 * 1e6, 1),
                                **summarize(mhz[:n_in], el)})
                # cold protocol
                time.sleep(0.05)
                el, enq, mhz = timed_steps(v, 20, 300, 2000)
                n_in = max(1, int(el * 1e6 / 20))
                results.append({"round": rnd, "variant": v, "protocol": "cold_k20",
                                "us_per_step": round(el / 20 * 1e6, 1),
                                "host_enqueue_us_per_step": round(enq / 20 * 1e6, 1),
                                **summarize(mhz[:n_in], el)})
                # build-only graph, events
                clock_warmup(v)
                start_probe(300, 2000)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(5):
                    g_build[v].replay()
                e1.record(stream)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 100
                mhz = read_probe(300)
                n_in = max(1, int(us * 100 / 20))
                results.append({"round": rnd, "variant": v, "protocol": "build_only_bb100",
                                "us_per_build": round(us, 1), **summarize(mhz[:n_in], us)})
                for r in results[-4:]:
                    print(json.dumps(r), flush=True)
    # aggregate
    agg = {}
    for r in results:
        key = f"{r['variant']}:{r['protocol']}"
        val = r.get("us_per_step", r.get("us_per_build"))
        agg.setdefault(key, []).append(val)
    print(json.dumps({"summary_median_us": {k: round(float(np.median(v)), 1) for k, v in agg.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
