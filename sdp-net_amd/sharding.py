"""Batch sharding of the SdP-Net forward across GPUs.

Images never interact in ``MainModel.forward`` (model.py:129-149: LayerNorm, the
depthwise conv and attention are all per image), so a global batch splits into
contiguous per-rank shards with no collective on the data path.  One process per
GPU (torch.distributed.run); the only communication is the timing barrier and the
max-over-ranks of the elapsed time that bench.py reports.
"""
from typing import Callable, Tuple

import torch
import torch.distributed as dist


def shard_bounds(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of the images rank `rank` owns; shards differ in size by at most one."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(global_batch, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def world_info() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank scalar (the step time) over all ranks; identity at world 1."""
    world, _ = world_info()
    if world == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device=None) -> float:
    world, _ = world_info()
    if world == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def sharded_forward(fn: Callable[[torch.Tensor], torch.Tensor], x_global: torch.Tensor) -> torch.Tensor:
    """Run fn on this rank's shard of x_global (no communication)."""
    world, rank = world_info()
    lo, hi = shard_bounds(x_global.shape[0], world, rank)
    return fn(x_global[lo:hi])
