"""CPU, world_size 2 (gloo): the multi-GPU structure of the path — pairs sharded
contiguously per rank, max-over-ranks timing, all-gather of per-pair results —
exercised with the same functions bench.py uses (RCCL replaces gloo on GPUs)."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dexiraft_amd.shard import gather_pairs, max_over_ranks, pair_range


@pytest.mark.parametrize("total,world", [(64, 1), (64, 2), (64, 8), (5, 2), (3, 8), (0, 4)])
def test_pair_range_partitions_exactly(total, world):
    spans = [pair_range(total, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0 and a0 <= a1
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def test_pair_range_rejects_bad_requests():
    for args in ((4, 0, 0), (4, 2, 2), (-1, 2, 0)):
        with pytest.raises(ValueError):
            pair_range(*args)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, total: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, stop = pair_range(total, world, rank)
        # each rank "computes" its pairs: a per-pair result tensor [2, 3, 4]
        local = torch.stack([torch.full((2, 3, 4), float(p)) for p in range(start, stop)]) \
            if stop > start else torch.empty((0, 2, 3, 4))
        full = gather_pairs(local, total)
        ok_gather = full.shape == (total, 2, 3, 4) and all(
            bool((full[p] == p).all()) for p in range(total))
        t = max_over_ranks(0.5 + rank)
        q.put((rank, ok_gather, t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [6, 5, 1])
def test_gloo_world2_shard_gather_and_max(total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert [r[0] for r in res] == [0, 1]
    assert all(r[1] for r in res), "gathered pairs wrong"
    assert all(r[2] == 1.5 for r in res), "max over ranks wrong"


def test_single_process_gather_is_identity():
    x = torch.arange(12.0).reshape(3, 4)
    assert gather_pairs(x, 3) is x
    assert max_over_ranks(2.5) == 2.5


_RANK_SCRIPT = r'''
import json, os, sys
import torch.distributed as dist
sys.path.insert(0, {repo!r})
from dexiraft_amd.shard import gather_pairs, pair_range
import torch
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
total = int(sys.argv[sys.argv.index("--total-pairs") + 1])
start, stop = pair_range(total, world, rank)
local = torch.arange(start, stop, dtype=torch.float64) * 10.0
sums = gather_pairs(local, total)
with open(os.path.join({out!r}, f"rank{{rank}}.json"), "w") as f:
    json.dump({{"rank": rank, "world": world, "local_rank": int(os.environ["LOCAL_RANK"]),
               "span": [start, stop], "sums": sums.tolist()}}, f)
dist.destroy_process_group()
'''


def test_bench_launcher_builds_n_ranks(tmp_path):
    """``bench.py --gpus N`` without a launcher starts torch.distributed.run with N
    ranks as a child (bench.relaunch_distributed); each rank owns its pair_range
    share and the per-pair checksums come back whole from gather_pairs (gloo here,
    RCCL in bench.py)."""
    import json
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(repo))
    import bench
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT.format(repo=str(repo), out=str(tmp_path)))
    rc = bench.relaunch_distributed(2, script=str(script), argv=["--gpus", "2",
                                                                  "--total-pairs", "5"])
    assert rc == 0
    recs = sorted((json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(2)),
                  key=lambda d: d["rank"])
    assert [d["span"] for d in recs] == [[0, 3], [3, 5]]
    assert all(d["world"] == 2 and d["local_rank"] == d["rank"] for d in recs)
    assert all(d["sums"] == [0.0, 10.0, 20.0, 30.0, 40.0] for d in recs)


def test_bench_refuses_world_size_mismatch(monkeypatch):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="must agree"):
        bench.init_dist(4)
