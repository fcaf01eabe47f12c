"""Frame-pair sharding across GPUs.

Pairs are independent (the volume of pair b depends only on fmap1[b], fmap2[b],
coords[b]: core/corr.py:53-60), so the only multi-GPU structure is a partition of
the pair batch, one process per GPU, plus — where a caller needs the results on
one rank — a gather of the per-pair outputs (flows) over RCCL (xGMI) or gloo.
There is no collective on the data path.  The reference's only parallelism,
``nn.DataParallel`` (train.py:139, evaluate.py:221), replicates in one process;
this replaces it for inference.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

__all__ = ["pair_range", "max_over_ranks", "gather_pairs"]


def pair_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, stop) of ``total`` pairs owned by ``rank``; the first
    ``total % world`` ranks take one extra pair."""
    if world < 1 or not 0 <= rank < world or total < 0:
        raise ValueError(f"bad partition request total={total} world={world} rank={rank}")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def max_over_ranks(value: float, device: torch.device | str = "cpu", group=None) -> float:
    """Max of a per-rank scalar (e.g. elapsed seconds) over the group."""
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def gather_pairs(local: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """All-gather per-pair results sharded by ``pair_range`` into [total, ...] on
    every rank (one ``all_gather_into_tensor`` over padded shards; RCCL on GPUs).

    ``local`` holds this rank's pairs along dim 0 (possibly 0 of them).
    """
    if not (dist.is_available() and dist.is_initialized()):
        if local.shape[0] != total:
            raise ValueError("single process: local must hold every pair")
        return local
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    start, stop = pair_range(total, world, rank)
    if local.shape[0] != stop - start:
        raise ValueError(f"rank {rank} holds {local.shape[0]} pairs, expected {stop - start}")
    per = -(-total // world) if total else 0
    padded = local.new_zeros((per,) + tuple(local.shape[1:]))
    padded[: local.shape[0]] = local
    out = local.new_empty((per * world,) + tuple(local.shape[1:]))
    if per:
        dist.all_gather_into_tensor(out, padded.contiguous(), group=group)
    pieces = []
    for r in range(world):
        s, e = pair_range(total, world, r)
        pieces.append(out[r * per: r * per + (e - s)])
    return torch.cat(pieces, dim=0)
