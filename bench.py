#!/usr/bin/env python3
"""Benchmark: frame pairs/s for one CorrBlock build + 12 lookups (BASELINE.json metric).

One "step" = for each of this rank's pairs, ``CorrBlock(fmap1, fmap2, radius=4)``
(the fused MFMA build of the 4-level pyramid) followed by 12 ``__call__(coords)``
lookups with 12 different coordinate sets, exactly the reference's per-forward
usage (core/raft.py:147, :169-173).  Inputs (fmaps [B,256,H/8,W/8] float32,
coords = grid + N(0, 4^2) px) are synthetic and resident in HBM before timing.

Launch: ``python bench.py [--gpus N --steps K --warmup W]``.  With ``--gpus N > 1``
and no WORLD_SIZE in the environment, this process starts
``torch.distributed.run`` with N ranks (one per GPU, RCCL) as a child before it
touches any GPU, and exits with its status; under a launcher, WORLD_SIZE must
equal --gpus.  Pairs are independent, so each rank processes its own pairs (weak
scaling, no collective on the data path); ranks are bracketed by barriers and
the max elapsed time over ranks is used.  After timing, a float64 checksum of
every pair's 12th lookup output is all-gathered over RCCL (shard.gather_pairs)
and reported.  Rank 0 prints ONE JSON line.

Execution (``--mode graph``, default): ``value`` is timed on ONE HIP graph of
G = ``--steps-per-graph`` (4) consecutive whole steps (build + 12 lookups each),
replayed K / G times — the launch-bound lookups would otherwise be host-bound in
Python, and every replay of a graph pays the HIP runtime's graph-launch boundary
(~10 us on a Sintel step, round 5), which G steps per graph pay once.
Every step runs on the rank's synthetic pair set (fmaps + 12 coordinate sets), as
in rounds 1-4; ``--pair-sets S`` cycles S distinct sets over a graph's steps
instead (the fmaps then come from HBM, not from the caches a just-run encoder
leaves them in).  Before the W warmup steps the step is
replayed untimed for ``--clock-warmup-s`` (0.5 s): MI355X raises its clocks only
after some milliseconds of load, and 30 timed steps behind 3 warmups read 11 %
below the steady rate (round 2: 3,936 vs 4,414-4,454 pairs/s at 300-2,000 steps).
Kernel durations for the rooflines: lookup = HIP events on the launch stream
around back-to-back replays of a graph of the step's 12 lookups, / 12 (one
lookup plus its same-stream kernel boundary); build = the same around a graph
of 10 back-to-back builds, / 10 (the split pass, the build and their
boundaries); what the timed step spends beyond 12 lookups + one build (the
graph launch, the build -> lookup boundary) is reported as step_boundary_us.
``--mode eager`` times plain Python calls instead.
The line also carries ``box`` (host, GPU UUID) and ``calibration`` (a bf16 GEMM
and an HBM copy timed in this process before the clock warm-up: boxes differ by
up to ~18 % in the build kernel, round 5), and ``value_one_step_per_graph`` (the
same K steps replayed one graph per step, rounds 1-4's protocol).  Kernel-trace
step timelines are not in the line: they come from another run.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
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
SPLIT_PRODUCTS = 3           # f16 MFMA products per f32 product in the split build

# name -> (image H, W after InputPadder, fmap H, W, default pairs per GPU, dtype)
WORKLOADS = {
    "sintel": ((440, 1024), (55, 128), 1, "f32"),
    "chairs": ((368, 496), (46, 62), 1, "f32"),
    "kitti": ((376, 1248), (47, 156), 8, "bf16"),
    "1080p": ((1088, 1920), (136, 240), 1, "f32"),
}
D, RADIUS, LEVELS, ITERS = 256, 4, 4, 12
BUILDS_PER_GRAPH = 10        # back-to-back builds per graph in the build-timing pass


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


def lookup_line_floor_bytes(coords, H, W, s_pyr=4, line=128):
    """Line-granular floor of one lookup (scripts/lookup_lines.py
    restated vectorised): for the step's own coordinate sets, the 128-byte lines
    of the paged pyramid (§3.3) that hold each query's window cells (2r+2 per
    axis from floor(c / 2^l) - r, clipped to the level) — a query's map is its own
    page slice, so no line is shared between queries — plus the float32 output and
    the coords, which every layout must move.  Mean over the coordinate sets."""
    tx = (W + 15) // 16
    offs = np.arange(2 * RADIUS + 2)
    lines = []
    for c in coords:
        a = c.detach().float().cpu().numpy()
        B = a.shape[0]
        x = a[:, 0].reshape(-1).astype(np.float64)
        y = a[:, 1].reshape(-1).astype(np.float64)
        n = 0
        for lvl, (h, w) in enumerate(level_sizes(H, W)):
            th, tw = 8 >> lvl, 16 >> lvl
            fx, fy = np.floor(x / 2 ** lvl), np.floor(y / 2 ** lvl)
            ok = np.isfinite(fx) & np.isfinite(fy) & (np.abs(fx) < 1e8) & (np.abs(fy) < 1e8)
            cx = np.where(ok, fx, -1e6).astype(np.int64)[:, None] - RADIUS + offs
            cy = np.where(ok, fy, -1e6).astype(np.int64)[:, None] - RADIUS + offs
            vx, vy = (cx >= 0) & (cx < w), (cy >= 0) & (cy < h)
            tile = (cy // th)[:, :, None] * tx + (cx // tw)[:, None, :]
            elem = tile * (th * tw) + ((cy % th) * tw)[:, :, None] + (cx % tw)[:, None, :]
            key = np.where(vy[:, :, None] & vx[:, None, :], elem * s_pyr // line, -1)
            key = np.sort(key.reshape(key.shape[0], -1), axis=1)
            n += int(((key[:, 1:] != key[:, :-1]) & (key[:, 1:] >= 0)).sum() +
                     (key[:, 0] >= 0).sum())
        lines.append(n)
    rd = 2 * RADIUS + 1
    return float(np.mean(lines)) * line + B * H * W * (8 + LEVELS * rd * rd * 4)


def build_kernel(dtype, H, W):
    """The build kernel the library runs for this workload (csrc/corr_build.hip:
    CorrBlock passes a workspace, so dxr_corr_pyramid_build_ws takes its LDS-DMA
    builds) and the ceiling of the arithmetic it runs: the f32 build issues three
    f16 MFMA products per f32 product (operands pre-split into per-pixel
    power-of-two scaled f16 pairs hi + lo; lo*hi + hi*lo + hi*hi into one f32
    accumulator), so its binding ceiling is 2.5 PF / 3 = 833 TF f32-equivalent;
    the f32 peak (157.3 TF) is §8(d)'s.  bf16 fmaps run one bf16 MFMA product."""
    if dtype == "bf16":
        if D % 32 == 0:
            return ("corr_build_dma_kernel (bf16 operand records by LDS-DMA: channels-last fmaps "
                    "in place, NCHW fmaps after a pack pass; f32 accumulate)", 1,
                    PEAK_BF16_TFLOPS, "bf16")
        return "corr_build_bf16_q2_kernel", 1, PEAK_BF16_TFLOPS, "bf16"
    if D % 16 == 0:
        return ("corr_build_dma_kernel (after split_pairs_kernel: f32 operands pre-split into "
                "per-pixel power-of-two scaled f16 pairs hi + lo; LDS-DMA ring, "
                "3 f16 MFMA products, f32 accumulate)", SPLIT_PRODUCTS, PEAK_BF16_TFLOPS,
                "f16 MFMA, f32 accumulate")
    return "corr_build_f32_kernel", 1, PEAK_F32_TFLOPS, "f32"


def alt_lookup_flops(B, H, W):
    n = H * W
    return 2.0 * B * n * LEVELS * (2 * RADIUS + 2) ** 2 * D


def profile_config(workload, B, b_default, layout, block):
    """Directory name of this bench configuration under profiles/<round>/
    (scripts/gpu_final.sh): sintel, sintel_b8, chairs, kitti, kitti_nhwc, hd_alt,
    hd_full — workload key + non-default batch + layout + block."""
    name = {"1080p": "hd"}.get(workload, workload)
    if B != b_default:
        name += f"_b{B}"
    if layout == "nhwc":
        name += "_nhwc"
    if workload == "1080p":
        name += "_alt" if block == "alt" else "_full"
    return name


def _profile_files(pattern, cfg):
    """profiles/<round>/<cfg>/<pattern> newest round first, then every other
    match of profiles/*/<pattern> and profiles/*/*/<pattern>, newest round first."""
    root = REPO / "profiles"
    rnd = lambda f: f.relative_to(root).parts[0]  # noqa: E731
    own = sorted(root.glob(f"*/{cfg}/{pattern}"), key=rnd, reverse=True) if cfg else []
    rest = sorted((set(root.glob(f"*/{pattern}")) | set(root.glob(f"*/*/{pattern}"))) - set(own),
                  key=lambda f: (rnd(f), str(f)), reverse=True)
    return own + rest


def pmc_traffic(workload, kernel_prefix, cfg=None):
    """Per-launch HBM bytes of a kernel from the newest committed PMC summary of
    this configuration (profiles/<round>/<cfg>/traffic.json), else of this
    workload key (profiles/<round>/traffic*.json; written by scripts/pmc_traffic.py
    from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this bench), or None
    when that workload was not profiled."""
    for f in _profile_files("traffic*.json", cfg):
        data = json.loads(f.read_text())
        if data.get("workload") != workload:
            continue
        for name, rec in data.get("kernels", {}).items():
            if name.split("::")[-1].startswith(kernel_prefix):
                return rec["traffic_bytes"], f"{f.relative_to(REPO)}: {rec['correction']}"
    return None, None


def calibrate(dev, stream, reps=10):
    """In-process speed of this box, timed before the timed region (VERDICT r05
    item 4: boxes differ by up to ~18 % in the build kernel, so each result is
    recorded beside the box's own speed): a bf16 GEMM 8192^3 (torch -> hipBLASLt,
    MFMA-bound; its clock is the DVFS clock under MFMA load) and a 1 GiB
    device-to-device copy (HBM-bound), each as HIP events around `reps`
    back-to-back launches on the bench's stream after two untimed ones."""
    n = 8192
    out = {}
    with torch.cuda.stream(stream):
        a = torch.randn((n, n), device=dev, dtype=torch.bfloat16)
        b = torch.randn((n, n), device=dev, dtype=torch.bfloat16)
        c = torch.empty((n, n), device=dev, dtype=torch.bfloat16)
        src = torch.empty(1 << 28, device=dev, dtype=torch.float32)   # 1 GiB
        dst = torch.empty_like(src)
        src.fill_(1.0)

        def timed(fn):
            for _ in range(2):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e-3 / reps

        t_mm = timed(lambda: torch.matmul(a, b, out=c))
        t_cp = timed(lambda: dst.copy_(src))
        out["bf16_gemm_tflops"] = round(2.0 * n ** 3 / t_mm / 1e12, 1)
        out["hbm_copy_gbs"] = round(2.0 * src.numel() * 4 / t_cp / 1e9, 1)
        out["what"] = (f"bf16 GEMM {n}^3 (torch.matmul) and a 1 GiB device copy (read + write "
                       f"counted), HIP events around {reps} launches each, before the timed region")
        del a, b, c, src, dst
    torch.cuda.synchronize()
    return out


def box_identity(dev):
    """Which box produced the line (hostname, GPU name and UUID)."""
    p = torch.cuda.get_device_properties(dev)
    return {"host": socket.gethostname(), "gpu": p.name, "gpu_uuid": str(getattr(p, "uuid", ""))}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch_distributed(gpus: int, script: str | None = None,
                         argv: list[str] | None = None) -> int:
    """--gpus N > 1 without a launcher: run this script under torch.distributed.run
    (N ranks, rendezvous on 127.0.0.1) as a CHILD process — never exec: nothing in
    this process has touched the GPU — and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", script or str(Path(__file__).resolve()),
           *(sys.argv[1:] if argv is None else argv)]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def init_dist(gpus: int):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {gpus}; they must agree")
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


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _nproc() -> int:
    """What coreutils ``nproc`` reports: the processing units this process may
    use (its CPU affinity, capped by OMP_NUM_THREADS / OMP_THREAD_LIMIT) — on
    the GPU box the harness's per-GPU CPU share, not the whole host."""
    try:
        return int(subprocess.run(["nproc"], capture_output=True, text=True,
                                  check=True).stdout.strip())
    except (OSError, ValueError, subprocess.CalledProcessError):
        return len(os.sched_getaffinity(0))


def cpu_baseline(H, W, budget_s, impl="torch", reps=5):
    """Time the reference's op sequence on host cores: warm-up 1,
    then the median of ``reps`` repetitions, each timing as many single pairs as
    fit in budget_s / reps (at least one), on ``torch.set_num_threads(nproc)``
    threads (nproc as coreutils reports it, see _nproc).

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
    nproc = _nproc()
    prev_threads = torch.get_num_threads()
    if impl == "torch":
        import torch_ref
        torch.set_num_threads(nproc)
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
    rates, pairs, total = [], 0, 0.0
    with torch.no_grad():
        one_pair()                                   # warm-up (allocator, thread pool)
        for _ in range(reps):
            n, t0 = 0, time.perf_counter()
            while n == 0 or time.perf_counter() - t0 < budget_s / reps:
                one_pair()
                n += 1
            dt = time.perf_counter() - t0
            rates.append(n / dt)
            pairs += n
            total += dt
    torch.set_num_threads(prev_threads)
    med = float(np.median(rates))
    return {"value": round(med, 4), "unit": "pairs/s", "cores": threads,
            "nproc": nproc, "host_cpus": os.cpu_count(), "cpu_model": _cpu_model(),
            "kind": "port",
            "median_of": reps, "median_s_per_pair": round(1.0 / med, 4),
            "sample": f"median of {reps} reps ({pairs} single pairs in {total:.1f} s) of fmap "
                      f"{H}x{W}, D={D}: build + {ITERS} lookups each; {what}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="sintel", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=None, help="pairs per GPU per step (weak scaling)")
    ap.add_argument("--total-pairs", type=int, default=None,
                    help="strong scaling: this many pairs per step split over the ranks (C4: 64)")
    ap.add_argument("--dtype", default=None, choices=["f32", "bf16"])
    ap.add_argument("--mode", default="graph", choices=["graph", "eager"])
    ap.add_argument("--steps-per-graph", type=int, default=4,
                    help="graph mode: consecutive steps (each its own pair set) captured in one "
                         "HIP graph; reduced to gcd(--steps, this) so exactly K steps are timed")
    ap.add_argument("--pair-sets", type=int, default=1,
                    help="distinct synthetic pair sets cycled over a graph's steps (default 1: "
                         "every step on the rank's one pair set, as rounds 1-4; DESIGN §6)")
    ap.add_argument("--block", default="corr", choices=["corr", "alt"],
                    help="corr: CorrBlock (full pyramid); alt: AlternateCorrBlock (on the fly, C5)")
    ap.add_argument("--alt-coarse-cells", type=int, default=None,
                    help="--block alt: AlternateCorrBlock.COARSE_LEVEL_MAX_CELLS (levels of at most "
                         "this many cells computed once per block as whole volumes; 0: none)")
    ap.add_argument("--alt-coarse-min-queries", type=int, default=None,
                    help="--block alt: AlternateCorrBlock.COARSE_MIN_QUERIES (volumes only on maps "
                         "of at least this many query pixels)")
    ap.add_argument("--alt-volume-planes", type=int, default=None, choices=[0, 1],
                    help="--block alt: AlternateCorrBlock.COARSE_VOLUME_PLANES (1: the volume "
                         "GEMM's LDS-DMA form on pre-split f16 pair planes; 0: its register form)")
    ap.add_argument("--layout", default="nchw", choices=["nchw", "nhwc"],
                    help="fmap memory format: nchw (the reference's) or nhwc (channels-last "
                         "encoders, SURVEY §8(f) row 4)")
    ap.add_argument("--clock-warmup-s", type=float, default=0.5,
                    help="untimed replays of the step for this long before the W warmup steps: "
                         "the GPU raises its clocks only after ~ms of load (30 timed steps after "
                         "3 warmups read 11 %% low on MI355X)")
    ap.add_argument("--no-calibration", action="store_true",
                    help="skip the in-process box calibration (bf16 GEMM + HBM copy)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-impl", default="torch", choices=["torch", "numpy"],
                    help="CPU baseline: torch restatement of core/corr.py (default) or numpy oracle")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args.gpus))
    world, rank, local = init_dist(args.gpus)
    dev = torch.device("cuda", local if world > 1 else 0)
    import dexiraft_amd
    from dexiraft_amd.shard import gather_pairs, max_over_ranks, pair_range
    dexiraft_amd.load_native()

    (img_h, img_w), (H, W), b_default, dt_default = WORKLOADS[args.workload]
    if args.total_pairs is not None:
        start, stop = pair_range(args.total_pairs, world, rank)
        B = stop - start
        if B < 1:
            raise SystemExit(f"--total-pairs {args.total_pairs} leaves rank {rank} without pairs")
        total = args.total_pairs
    else:
        B = args.batch or b_default
        total = world * B
    dtype = args.dtype or dt_default
    # steps per graph replay; each step of a replay runs on its own pair set
    G = math.gcd(args.steps, max(args.steps_per_graph, 1)) if args.mode == "graph" else 1
    sets = []
    for i in range(min(G, max(args.pair_sets, 1))):
        f1, f2, coords = make_inputs(B, H, W, dtype, seed=1234 + rank + 7919 * i, dev=dev)
        if args.layout == "nhwc":
            f1 = f1.contiguous(memory_format=torch.channels_last)
            f2 = f2.contiguous(memory_format=torch.channels_last)
        sets.append((f1, f2, coords))
    sets = [sets[i % len(sets)] for i in range(G)]
    f1, f2, coords = sets[0]
    stream = torch.cuda.Stream(device=dev)

    state = {}
    block_cls = dexiraft_amd.CorrBlock if args.block == "corr" else dexiraft_amd.AlternateCorrBlock
    if args.block == "alt" and args.alt_coarse_cells is not None:
        block_cls.COARSE_LEVEL_MAX_CELLS = args.alt_coarse_cells
    if args.block == "alt" and args.alt_coarse_min_queries is not None:
        block_cls.COARSE_MIN_QUERIES = args.alt_coarse_min_queries
    if args.block == "alt" and args.alt_volume_planes is not None:
        block_cls.COARSE_VOLUME_PLANES = bool(args.alt_volume_planes)

    def build(i=0):
        # the previous step's block and outputs go first (one pyramid alive at a time)
        state.pop("outs", None)
        state.pop("cb", None)
        state["cb"] = block_cls(sets[i][0], sets[i][1], radius=RADIUS)

    def lookups(i=0):
        state["outs"] = [state["cb"](c) for c in sets[i][2]]

    def step(i=0):
        build(i)
        lookups(i)

    timing = ("lookup = hip events around back-to-back replays of a graph of the step's 12 "
              "lookups / 12; build = hip events around back-to-back replays of a graph of "
              f"{BUILDS_PER_GRAPH} builds / {BUILDS_PER_GRAPH} (each incl. its same-stream "
              "boundaries); boundary = timed step - 12 lookups - build")
    with torch.no_grad(), torch.cuda.stream(stream):
        for _ in range(max(min(args.warmup, 3), 1)):  # eager warmup (also a JIT-free check)
            step()
        torch.cuda.synchronize()
        if args.mode == "graph":
            # G whole steps (build + 12 lookups each, G pair sets) as ONE graph: what
            # a serving loop over a stream of pairs replays; `value` is timed on it.
            g_step = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_step, stream=stream):
                for i in range(G):
                    step(i)
            run_step = g_step.replay
        else:
            run_step = step
            timing = "hip events around eager launches"
        torch.cuda.synchronize()
        # box calibration first, so that its GEMM burst is followed by the whole
        # clock warm-up on the step itself (placed after the warm-up it left the
        # driver's 5-replay timed region ~5 % below the same steps re-timed later,
        # round 6: 5,300 vs 5,585 pairs/s on one box)
        calib = calibrate(dev, stream) if not args.no_calibration else None
        # clock warm-up: replay the full step (same work, same outputs) until the
        # chip has been under load for --clock-warmup-s, then the W warmup steps
        t_w = time.perf_counter()
        n_clock = 0
        while time.perf_counter() - t_w < args.clock_warmup_s:
            for _ in range(20):
                run_step()
            n_clock += 20
            torch.cuda.synchronize()
        for _ in range(-(-args.warmup // G)):
            run_step()
        torch.cuda.synchronize()

        barrier(world)
        t0 = time.perf_counter()
        for _ in range(args.steps // G):     # exactly K steps
            run_step()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        barrier(world)

        # correctness record: float64 checksum of each pair's 12th lookup (of the
        # last timed replay), gathered from every rank over RCCL (the only
        # collective; outside the timed region)
        local_sums = state["outs"][-1].double().sum(dim=(1, 2, 3))
        sums = gather_pairs(local_sums, total)
        finite = bool(torch.isfinite(sums).all().item())

        # Kernel-timing pass (outside the timed region): the 12 lookups as one graph,
        # replayed back to back after the timed steps (steady clocks): lookup = that
        # time / 12, i.e. one lookup plus its same-stream kernel boundary; build
        # (stage a+b, or the on-the-fly block's pools/layout) = the timed step time
        # - 12 lookups, i.e. the build plus its boundary and the graph launch.
        # Compare with the rocprofv3 kernel durations and the idle time per step of
        # the same command's kernel trace (scripts/trace_gaps.py, profiles/).
        if args.mode == "graph":
            keep = dict(state)            # the step graph's own tensors stay allocated
            cb = state["cb"]              # the last step's block, with its pair set's coords
            g_look = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_look, stream=stream, pool=g_step.pool()):
                [cb(c) for c in sets[G - 1][2]]
            # the build alone, as a graph of back-to-back builds (each block freed
            # before the next is built, as in the step); in the step graph's pool,
            # so its blocks reuse that pool's free memory (a private
            # pool held another pyramid + workspace, ~5.7 GB at 1080p)
            g_build = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_build, stream=stream, pool=g_step.pool()):
                for _ in range(BUILDS_PER_GRAPH):
                    block_cls(f1, f2, radius=RADIUS)
            # the captures left the GPU idle: bring the clocks back up first
            t_w = time.perf_counter()
            while time.perf_counter() - t_w < min(args.clock_warmup_s, 0.25):
                for _ in range(10):
                    g_step.replay()
                torch.cuda.synchronize()
            for _ in range(5):
                g_look.replay()
                g_build.replay()
            torch.cuda.synchronize()
            reps = max(50, min(args.steps, 100))

            def events(graph, n):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(n):
                    graph.replay()
                e1.record(stream)
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / n

            look_ms = events(g_look, reps) / ITERS
            build_ms = events(g_build, max(5, reps // 4)) / BUILDS_PER_GRAPH
            one_ms = None
            if G > 1:
                # the same K steps as one graph per step (rounds 1-4's protocol;
                # each replay pays the runtime's replay boundary), for comparison
                g_one = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g_one, stream=stream, pool=g_step.pool()):
                    step(G - 1)
                for _ in range(5):
                    g_one.replay()
                one_ms = events(g_one, args.steps)
                del g_one
            boundary_ms = elapsed / args.steps * 1e3 - ITERS * look_ms - build_ms
            del keep, g_build
        else:
            one_ms = None
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(stream)
            build()
            ev[1].record(stream)
            lookups()
            ev[2].record(stream)
            torch.cuda.synchronize()
            build_ms, look_ms = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]) / ITERS
            boundary_ms = elapsed / args.steps * 1e3 - ITERS * look_ms - build_ms

    elapsed = max_over_ranks(elapsed, device=dev)
    if not finite:
        raise SystemExit("bench.py: non-finite lookup output")

    if rank == 0:
        pairs = total * args.steps
        value = pairs / elapsed
        s_in = 2 if dtype == "bf16" else 4
        flops = build_flops(B, H, W)
        wl_key = f"{args.workload}_b{B}_{dtype}"
        cfg = profile_config(args.workload, B, b_default, args.layout, args.block)
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
            "value_one_step_per_graph": (round(total / (one_ms * 1e-3), 3) if one_ms else None),
            "dtype": dtype,
            "data": "synthetic (torch.randn fmaps, coords = grid + N(0,4^2) px)",
            "config": {
                "workload": f"{'CorrBlock' if args.block == 'corr' else 'AlternateCorrBlock'} "
                            f"build + {ITERS} lookups, {args.workload} "
                            f"{img_h}x{img_w} (fmap {H}x{W}), D={D}, r={RADIUS}, L={LEVELS}",
                "pairs_per_gpu": B, "fmap_layout": args.layout, "mode": args.mode,
                "parallelism": f"pairs sharded x{world}",
                "step_timing": (f"one HIP graph per {G} consecutive whole steps (build + 12 "
                                f"lookups each); {args.steps // G} replays"
                                if args.mode == "graph" else "eager launches"),
                "steps_per_graph": G, "pair_sets": len({id(t[0]) for t in sets}),
                "kernel_timing": timing,
                "clock_warmup": f"{n_clock} untimed step replays ({args.clock_warmup_s} s) before "
                                f"the {args.warmup} warmup steps",
            },
            "box": box_identity(dev),
            "calibration": calib,
            "pair_checksums": {
                "what": "float64 sum of each pair's 12th lookup output, all-gathered over "
                        f"{'RCCL' if world > 1 else 'no collective (1 rank)'}",
                "pairs": int(sums.numel()), "sum_of_sums": float(sums.sum().item()),
                "first": [round(float(v), 3) for v in sums[:4].tolist()],
            },
        }
        if args.block == "corr":
            kname, mfma_per_flop, pipe_peak, mfma_dtype = build_kernel(dtype, H, W)
            # achieved = ALGORITHMIC flops (2*B*N^2*D) per launch / launch time.
            # Ceiling = the dense MFMA peak of the arithmetic actually run: bf16 fmaps
            # 2.5 PF; f32 fmaps on the split build 2.5 PF / 3 = 833 TF f32-equivalent
            # (its f16 pipe, same dense peak as bf16); the exact-f32 build 157.3 TF.  frac_f32_peak keeps
            # SURVEY §8(d)'s f32 pricing beside it.
            achieved = flops / (build_ms * 1e-3) / 1e12
            ceiling = pipe_peak / mfma_per_flop
            b_traffic, b_src = pmc_traffic(wl_key, kname.split(" ")[0] + "<", cfg)
            l_traffic, l_src = pmc_traffic(wl_key, "corr_lookup_qm_kernel<", cfg)
            bb = build_bytes(B, H, W, s_in, s_in)
            res["roofline"] = {
                "kernel": kname + " (stage a+b)",
                "bound": "mfma", "achieved": round(achieved, 2), "peak": round(ceiling, 1),
                "unit": "TFLOP/s", "frac": round(achieved / ceiling, 4),
                "peak_basis": (f"dense f16 MFMA 2.5 PF / {mfma_per_flop} products per f32 product"
                               if mfma_per_flop > 1 else f"dense {mfma_dtype} MFMA peak"),
                "frac_f32_peak": None if dtype == "bf16" else round(achieved / PEAK_F32_TFLOPS, 4),
                "traffic": b_traffic, "traffic_source": b_src,
                "mfma_dtype": mfma_dtype,
                "algorithmic_flops_per_launch": flops,
                "algorithmic_bytes_per_launch": bb,
                "hbm_frac": round(bb / (build_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                "avg_launch_us": round(build_ms * 1e3, 2),
                "step_boundary_us": round(boundary_ms * 1e3, 2),
            }
            lf = lookup_line_floor_bytes(sets[G - 1][2], H, W, s_pyr=s_in)
            res["lookup_roofline"] = {
                "kernel": "corr_lookup_qm_kernel (stage c; window cells staged query-minor in LDS)",
                "bound": "hbm", "achieved": round(lb / (look_ms * 1e-3) / 1e9, 1),
                "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(lb / (look_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                "algorithmic_bytes_per_launch": lb,
                # the achievable floor of this layout: whole 128-B lines holding the
                # taps' cells + output + coords, and the time at 8 TB/s
                "line_floor_bytes": round(lf),
                "frac_of_line_floor": round(lf / (look_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                "traffic": l_traffic, "traffic_source": l_src,
                "avg_launch_us": round(look_ms * 1e3, 2),
            }
        else:
            # on-the-fly lookups: (2r+2)^2 window dot products of length D per query
            # and level, f32-class arithmetic (SURVEY.md §8(d) stage d), priced at
            # the f32 peak; the default kernel runs them as f16-pair split MFMA GEMMs.
            aflops = alt_lookup_flops(B, H, W)
            achieved = aflops / (look_ms * 1e-3) / 1e12
            akern = "alt_corr_mfma_kernel"
            # the windowed instantiation (radius 4; the FULL one, radius 0, builds the
            # coarse-level volumes once per block), plus the volume lookup when the
            # block answers its coarse levels from volumes
            a_traffic, a_src = pmc_traffic(wl_key, f"{akern}<{RADIUS},", cfg)
            vol_first = getattr(state.get("cb"), "coarse_first_level", None)
            if a_traffic is not None and vol_first is not None:
                v_traffic, _ = pmc_traffic(wl_key, "corr_lookup_qm_kernel<", cfg)
                if v_traffic is None:
                    a_traffic = a_src = None
                else:
                    a_traffic += v_traffic
                    a_src += f" (+ corr_lookup_qm_kernel ALT: levels >= {vol_first} from volumes)"
            pipe = PEAK_BF16_TFLOPS / SPLIT_PRODUCTS   # the f16-pair split's own ceiling (833 TF)
            res["roofline"] = {
                "kernel": akern + " (f16-pair split MFMA over the window boxes of 32 queries "
                                  "grouped by window position (alt_bin_*_kernel order) or by "
                                  "4 x 8 tile, f32 accumulate; stage d; avg_launch_us = one "
                                  "lookup incl. its three ordering launches)",
                "bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_F32_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / PEAK_F32_TFLOPS, 4),
                "frac_pipe_ceiling": round(achieved / pipe, 4), "pipe_ceiling_tflops": round(pipe, 1),
                "traffic": a_traffic, "traffic_source": a_src,
                "algorithmic_flops_per_launch": aflops,
                "avg_launch_us": round(look_ms * 1e3, 2),
                "pool_and_layout_us_per_step": round(build_ms * 1e3, 2),
                "step_boundary_us": round(boundary_ms * 1e3, 2),
            }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(H, W, args.cpu_seconds, args.cpu_impl)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
