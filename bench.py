#!/usr/bin/env python3
"""Benchmark: frame pairs/s for one CorrBlock build + 12 lookups (BASELINE.json metric).

One "step" = for each of this rank's pairs, ``CorrBlock(fmap1, fmap2, radius=4)``
(the fused MFMA build of the 4-level pyramid) followed by 12 ``__call__(coords)``
lookups with 12 different coordinate sets, exactly the reference's per-forward
usage (core/raft.py:147, :169-173).  Inputs (fmaps [B,256,H/8,W/8] float32,
coords = grid + N(0, 4^2) px) are synthetic and resident in HBM before timing.

Launch: ``python bench.py [--gpus N --steps K --warmup W]``; for N > 1 the driver
runs it under torch.distributed.run, one rank per GPU.  Pairs are independent,
so each rank processes its own pairs (weak scaling, no collective on the data
path); ranks are bracketed by barriers and the max elapsed time over ranks is
used.  Rank 0 prints ONE JSON line.

Execution: the step is captured into two HIP graphs (build, lookups) and
replayed — the launch-bound lookups would otherwise be host-bound in Python.
HIP events between the two replays give the build kernel's duration inside the
timed region (the roofline's ``achieved``; it includes the graph launch, so it
reads a few percent above the rocprofv3 kernel duration — conservative).
(Event-record nodes inside one K-step graph would exclude it, but ROCm torch
refuses external events and raw hipEventRecord nodes did not record: r01.)
``--mode eager`` times plain Python calls instead.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

METRIC = "frame pairs/sec (corr build + 12 lookups) @436x1024, 1–8 GPU; % MFMA/HBM peak"
PEAK_F32_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
PEAK_BF16_TFLOPS = 2500.0    # dense BF16 MFMA
PEAK_HBM_GBS = 8000.0        # HBM3E spec

# name -> (image H, W after InputPadder, fmap H, W, default pairs per GPU, dtype)
WORKLOADS = {
    "sintel": ((440, 1024), (55, 128), 1, "f32"),
    "chairs": ((368, 496), (46, 62), 1, "f32"),
    "kitti": ((376, 1248), (47, 156), 8, "bf16"),
    "1080p": ((1088, 1920), (136, 240), 1, "f32"),
}
D, RADIUS, LEVELS, ITERS = 256, 4, 4, 12


def level_sizes(H, W, L=LEVELS):
    s = [(H, W)]
    for _ in range(L - 1):
        s.append((s[-1][0] // 2, s[-1][1] // 2))
    return s


def build_flops(B, H, W):
    n = H * W
    return 2.0 * B * n * n * D


def build_bytes(B, H, W, s_in=4, s_out=4):
    n = H * W
    cells = sum(h * w for h, w in level_sizes(H, W))
    return B * 2 * D * n * s_in + B * n * cells * s_out


def lookup_bytes(B, H, W, s_pyr=4):
    """Compulsory bytes of one lookup: window cells clipped to
    the level, the coords and the float32 output."""
    rd = 2 * RADIUS + 1
    win = sum(min(rd + 1, h) * min(rd + 1, w) for h, w in level_sizes(H, W))
    return B * H * W * (win * s_pyr + 8 + LEVELS * rd * rd * 4)


def build_kernel(dtype, H, W):
    """Which build kernel the library runs for this workload (csrc/corr_build.hip
    launch_build_f32 / launch_build_bf16), and the MFMA work it executes per
    algorithmic flop: the split f32 build issues six bf16 MFMA products per f32
    product (exact hi+mid+lo operand split, f32 accumulation)."""
    variant = os.environ.get("DXR_BUILD_VARIANT", "0")
    if dtype == "bf16":
        return "corr_build_bf16_kernel", 1, PEAK_BF16_TFLOPS, "bf16"
    if D % 16 == 0 and W % 2 == 0 and variant in ("0", "7", "8", "9", "40"):
        return ("corr_build_split_kernel (f32 operands split exactly into 3 bf16, "
                "bf16x6 MFMA, f32 accumulate)", 6, PEAK_BF16_TFLOPS, "bf16 MFMA, f32 accumulate")
    return "corr_build_f32_kernel", 1, PEAK_F32_TFLOPS, "f32"


def alt_lookup_flops(B, H, W):
    n = H * W
    return 2.0 * B * n * LEVELS * (2 * RADIUS + 2) ** 2 * D


def pmc_traffic(workload, kernel_prefix):
    """Per-launch HBM bytes of a kernel from the newest committed PMC summary of
    this workload (profiles/<round>/traffic*.json, written by
    scripts/pmc_traffic.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes
    of this bench), or None when that workload was not profiled."""
    files = sorted((REPO / "profiles").glob("*/traffic*.json"))
    for f in reversed(files):
        data = json.loads(f.read_text())
        if data.get("workload") != workload:
            continue
        for name, rec in data.get("kernels", {}).items():
            if name.split("::")[-1].startswith(kernel_prefix):
                return rec["traffic_bytes"], f"{f.relative_to(REPO)}: {rec['correction']}"
    return None, None


def init_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def make_inputs(B, H, W, dtype, seed, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    f1 = torch.randn((B, D, H, W), generator=g, device=dev)
    f2 = torch.randn((B, D, H, W), generator=g, device=dev)
    if dtype == "bf16":
        f1, f2 = f1.bfloat16(), f2.bfloat16()
    ys, xs = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    grid = torch.stack((xs, ys))[None].expand(B, 2, H, W)
    coords = [(grid + 4.0 * torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous()
              for _ in range(ITERS)]
    return f1, f2, coords


def cpu_baseline(H, W, budget_s, impl="torch"):
    """Time the reference's op sequence on host cores over a bounded sample.

    impl "torch" (default; SURVEY.md §8(d) "CPU reference timing"): the plain-PyTorch
    restatement tests/torch_ref.py (bmm, / sqrt(D), 3x F.avg_pool2d, 12 x 4
    F.grid_sample + cat + permute — core/corr.py's ops, pinned to the reference's
    goldens) on torch's CPU threads.  impl "numpy": the numpy oracle (oracle/,
    float32), matmul on BLAS threads, lookups single-threaded.
    """
    sys.path.insert(0, str(REPO / "tests"))
    import datagen as dg
    f1 = dg.fmap(0, 1, D, H, W)
    f2 = dg.fmap(1, 1, D, H, W)
    cs = [dg.coords(100 + k, 1, H, W, "normal", 4.0) for k in range(ITERS)]
    if impl == "torch":
        import torch_ref
        threads = torch.get_num_threads()
        t1, t2 = torch.from_numpy(f1), torch.from_numpy(f2)
        tc = [torch.from_numpy(c) for c in cs]

        def one_pair():
            blk = torch_ref.TorchCorrBlock(t1, t2, LEVELS, RADIUS)
            for c in tc:
                blk(c)
        what = f"torch CPU restatement of core/corr.py (tests/torch_ref.py), {threads} torch threads"
    else:
        import oracle
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])

        def one_pair():
            pyr = oracle.corr_pyramid(f1, f2, LEVELS, np.float32)
            for c in cs:
                oracle.corr_lookup(pyr, c, RADIUS)
        what = f"numpy float32 oracle; matmul on {threads} BLAS threads, lookups single-threaded"
    with torch.no_grad():
        one_pair()                                   # warm-up (allocator, thread pool)
        pairs, t0 = 0, time.perf_counter()
        while True:
            one_pair()
            pairs += 1
            el = time.perf_counter() - t0
            if el >= budget_s or pairs >= 50:
                break
    return {"value": pairs / el, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"{pairs} pair(s) of fmap {H}x{W}, D={D}: build + {ITERS} lookups, "
                      f"{el:.1f} s; {what}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="sintel", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=None, help="pairs per GPU per step (weak scaling)")
    ap.add_argument("--total-pairs", type=int, default=None,
                    help="strong scaling: this many pairs per step split over the ranks (C4: 64)")
    ap.add_argument("--dtype", default=None, choices=["f32", "bf16"])
    ap.add_argument("--mode", default="graph", choices=["graph", "eager"])
    ap.add_argument("--block", default="corr", choices=["corr", "alt"],
                    help="corr: CorrBlock (full pyramid); alt: AlternateCorrBlock (on the fly, C5)")
    ap.add_argument("--layout", default="nchw", choices=["nchw", "nhwc"],
                    help="fmap memory format: nchw (the reference's) or nhwc (channels-last "
                         "encoders, SURVEY §8(f) row 4)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-impl", default="torch", choices=["torch", "numpy"],
                    help="CPU baseline: torch restatement of core/corr.py (default) or numpy oracle")
    args = ap.parse_args()

    world, rank, local = init_dist()
    dev = torch.device("cuda", local if world > 1 else 0)
    import dexiraft_amd
    from dexiraft_amd.shard import max_over_ranks, pair_range
    dexiraft_amd.load_native()

    (img_h, img_w), (H, W), b_default, dt_default = WORKLOADS[args.workload]
    if args.total_pairs is not None:
        start, stop = pair_range(args.total_pairs, world, rank)
        B = stop - start
        if B < 1:
            raise SystemExit(f"--total-pairs {args.total_pairs} leaves rank {rank} without pairs")
    else:
        B = args.batch or b_default
    dtype = args.dtype or dt_default
    f1, f2, coords = make_inputs(B, H, W, dtype, seed=1234 + rank, dev=dev)
    if args.layout == "nhwc":
        f1 = f1.contiguous(memory_format=torch.channels_last)
        f2 = f2.contiguous(memory_format=torch.channels_last)
    stream = torch.cuda.Stream(device=dev)

    state = {}

    block_cls = dexiraft_amd.CorrBlock if args.block == "corr" else dexiraft_amd.AlternateCorrBlock

    def build():
        state["cb"] = block_cls(f1, f2, radius=RADIUS)

    def lookups():
        state["outs"] = [state["cb"](c) for c in coords]

    timing = "hip events between graph replays"
    with torch.no_grad(), torch.cuda.stream(stream):
        for _ in range(max(args.warmup, 1)):          # eager warmup (also JIT-free check)
            build()
            lookups()
        torch.cuda.synchronize()
        if args.mode == "graph":
            g_build, g_look = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_build, stream=stream):
                build()
            with torch.cuda.graph(g_look, stream=stream, pool=g_build.pool()):
                lookups()
            run_build, run_look = g_build.replay, g_look.replay
            # The whole step (build + 12 lookups) as ONE graph: what a serving loop
            # replays; `value` is timed on it.  The split graphs above give the
            # per-kernel durations (HIP events between their replays).
            g_step = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_step, stream=stream):
                build()
                lookups()
            for _ in range(max(args.warmup, 1)):
                run_build()
                run_look()
                g_step.replay()
        else:
            run_build, run_look = build, lookups
            timing = "hip events between eager launches"
        torch.cuda.synchronize()

        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
                torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        barrier(world)
        t0 = time.perf_counter()
        for e0, e1, e2 in evs:
            e0.record(stream)
            run_build()
            e1.record(stream)
            run_look()
            e2.record(stream)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        barrier(world)
        elapsed_split = elapsed
        if args.mode == "graph":
            barrier(world)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                g_step.replay()
            torch.cuda.synchronize()
            elapsed = time.perf_counter() - t0
            barrier(world)

    build_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in evs]))
    look_ms = float(np.mean([b.elapsed_time(c) for _, b, c in evs])) / ITERS
    elapsed = max_over_ranks(elapsed, device=dev)
    elapsed_split = max_over_ranks(elapsed_split, device=dev)
    if world > 1:
        # Correctness sanity outside the timed region: every rank's last lookup is finite.
        ok = torch.tensor([float(torch.isfinite(state["outs"][-1]).all())], device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        assert ok.item() == 1.0

    if rank == 0:
        pairs = (args.total_pairs if args.total_pairs is not None else world * B) * args.steps
        value = pairs / elapsed
        s_in = 2 if dtype == "bf16" else 4
        flops = build_flops(B, H, W)
        wl_key = f"{args.workload}_b{B}_{dtype}"
        lb = lookup_bytes(B, H, W, s_pyr=s_in)
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.total_pairs is not None else "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (torch.randn fmaps, coords = grid + N(0,4^2) px)",
            "config": {
                "workload": f"{'CorrBlock' if args.block == 'corr' else 'AlternateCorrBlock'} "
                            f"build + {ITERS} lookups, {args.workload} "
                            f"{img_h}x{img_w} (fmap {H}x{W}), D={D}, r={RADIUS}, L={LEVELS}",
                "pairs_per_gpu": B, "fmap_layout": args.layout, "mode": args.mode,
                "parallelism": f"pairs sharded x{world}",
                "kernel_timing": timing,
                "step_timing": ("one HIP graph per step (build + 12 lookups); "
                                f"{elapsed_split / args.steps * 1e3:.4f} ms/step with the build and "
                                "the lookups in two graphs (the kernel-timing pass)")
                               if args.mode == "graph" else "eager launches",
            },
        }
        if args.block == "corr":
            kname, mfma_per_flop, pipe_peak, mfma_dtype = build_kernel(dtype, H, W)
            # achieved = ALGORITHMIC flops (2*B*N^2*D) per launch / launch time, priced
            # against the dense MFMA peak of the path's arithmetic type: f32 (157.3 TF)
            # for f32 fmaps, bf16 (2.5 PF) for bf16 fmaps.  The split f32 build issues
            # 6 bf16 MFMA products per f32 product; its bf16-pipe occupancy is reported
            # beside it ("bf16_pipe"), not as the roofline.
            peak = PEAK_BF16_TFLOPS if dtype == "bf16" else PEAK_F32_TFLOPS
            achieved = flops / (build_ms * 1e-3) / 1e12
            b_traffic, b_src = pmc_traffic(wl_key, kname.split(" ")[0] + "<")
            l_traffic, l_src = pmc_traffic(wl_key, "corr_lookup_wide_kernel<")
            res["roofline"] = {
                "kernel": kname + " (stage a+b)",
                "bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                "traffic": b_traffic, "traffic_source": b_src,
                "mfma_dtype": mfma_dtype,
                "algorithmic_flops_per_launch": flops,
                "algorithmic_bytes_per_launch": build_bytes(B, H, W, s_in, s_in),
                "avg_launch_us": round(build_ms * 1e3, 2),
            }
            if mfma_per_flop > 1:
                issued = mfma_per_flop * flops / (build_ms * 1e-3) / 1e12
                res["roofline"]["bf16_pipe"] = {
                    "mfma_flops_per_launch": mfma_per_flop * flops,
                    "issued_tflops": round(issued, 2), "peak": pipe_peak,
                    "frac": round(issued / pipe_peak, 4)}
            res["lookup_roofline"] = {
                "kernel": "corr_lookup_wide_kernel (stage c)",
                "bound": "hbm", "achieved": round(lb / (look_ms * 1e-3) / 1e9, 1),
                "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(lb / (look_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                "algorithmic_bytes_per_launch": lb,
                "traffic": l_traffic, "traffic_source": l_src,
                "avg_launch_us": round(look_ms * 1e3, 2),
            }
        else:
            # on-the-fly lookups: (2r+2)^2 window dot products of length D per query
            # and level, f32-class arithmetic (SURVEY.md §8(d) stage d).  The default
            # kernel (D % 16 == 0, D <= 256) runs them as split-bf16 MFMA GEMMs over
            # each 4x8 query tile's union box of cells; the issued MFMA work depends on
            # the coordinates (box size), so the roofline prices the algorithmic window
            # FLOPs against the f32 peak, as for an f32 kernel.
            aflops = alt_lookup_flops(B, H, W)
            achieved = aflops / (look_ms * 1e-3) / 1e12
            mfma_alt = D % 16 == 0 and D <= 256 and os.environ.get("DXR_ALT_VARIANT") != "1"
            akern = "alt_corr_mfma_kernel" if mfma_alt else "alt_corr_kernel"
            a_traffic, a_src = pmc_traffic(wl_key, akern + "<")
            res["roofline"] = {
                "kernel": akern + (" (split-bf16 MFMA over the union box of 4x8-query windows, "
                                   "f32 accumulate)" if mfma_alt else " (per-query VALU)")
                + " (stage d, per lookup)",
                "bound": "mfma" if mfma_alt else "valu", "achieved": round(achieved, 2),
                "peak": PEAK_F32_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / PEAK_F32_TFLOPS, 4),
                "traffic": a_traffic, "traffic_source": a_src,
                "algorithmic_flops_per_launch": aflops,
                "avg_launch_us": round(look_ms * 1e3, 2),
                "pool_and_layout_us_per_step": round(build_ms * 1e3, 2),
            }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(H, W, args.cpu_seconds, args.cpu_impl)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
