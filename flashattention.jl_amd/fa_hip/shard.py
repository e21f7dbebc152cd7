"""Multi-GPU sharding of the hot path over (batch × head) slabs.

The reference layout is column-major (N, d, B·H): the batch dimension is the
slowest-varying, so a contiguous range of slabs is a contiguous byte range.
Each rank (one process per GPU, ``torch.distributed`` over RCCL/xGMI or gloo
on CPU) owns the slabs ``shard_range(BH, world, rank)`` and calls
``dense_fa`` / ``dense_fa_backward`` on them with NO data-path collective:
slabs are independent.  ``gather_slabs`` is an optional, untimed all-gather
for callers that need the whole result on every rank.
"""
from __future__ import annotations

from typing import Tuple

import torch

__all__ = ["shard_range", "local_slabs", "gather_slabs"]


def shard_range(n_slabs: int, world: int, rank: int) -> Tuple[int, int]:
    """[start, stop) of the slabs rank `rank` owns: contiguous, sizes differ by ≤ 1."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(n_slabs, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def local_slabs(x: torch.Tensor, world: int, rank: int) -> torch.Tensor:
    """The rank's slabs of a Julia-layout (…, B) array, as a zero-copy view
    (contiguous in memory because B is the last, slowest dimension)."""
    a, b = shard_range(x.shape[-1], world, rank)
    return x[..., a:b]


def gather_slabs(local: torch.Tensor, n_slabs: int, group=None) -> torch.Tensor:
    """All-gather every rank's slabs into the full (…, n_slabs) array (column-major).
    One collective of ~1/world of the data per rank (ranks' slab counts differ
    by at most one, so each part is padded to the largest); not on any timed path."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    ranges = [shard_range(n_slabs, world, r) for r in range(world)]
    cap = max(b - a for a, b in ranges)
    inner = tuple(reversed(local.shape[:-1]))                 # row-major trailing dims
    mine = torch.zeros((cap,) + inner, dtype=local.dtype, device=local.device)
    mine[: local.shape[-1]] = local.permute(*reversed(range(local.dim())))
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    full = torch.cat([p[: b - a] for p, (a, b) in zip(parts, ranges)], dim=0)   # (B, …) row-major
    return full.permute(*reversed(range(full.dim())))          # == (…, B) column-major
