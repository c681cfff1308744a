"""Multi-GPU frame split: image rows shard across ranks, the canvas is gathered.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).
Every pixel of the reference's render is independent (renderer.c:216-237), so
rank r renders the interleaved rows r, r+N, r+2N, ... (interleaving balances
the spatially skewed cost of scenes such as cornell_box). The only exchange is
the final canvas placement on rank 0 — a gather, not a reduction, so N-GPU
canvases are bit-identical to the 1-GPU canvas.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def rows_of(rank: int, world: int, height: int) -> range:
    """Rows rendered by `rank` (interleaved, stride = world)."""
    return range(rank, height, world)


def shard_capacity(world: int, height: int) -> int:
    """Rows per shard after padding every shard to the same size (equal-size collectives)."""
    return (height + world - 1) // world


def gather_canvas(shard: torch.Tensor, rank: int, world: int, height: int, dst: int = 0):
    """Gather interleaved row shards into the full (height, width, 4) canvas on `dst`.

    `shard` is (shard_capacity, width, 4) holding this rank's rows first (padded).
    Returns the canvas on dst, None elsewhere.
    """
    cap = shard_capacity(world, height)
    assert shard.shape[0] == cap, (shard.shape, cap)
    if world == 1:
        return shard[:height]
    gathered = [torch.empty_like(shard) for _ in range(world)] if rank == dst else None
    dist.gather(shard, gather_list=gathered, dst=dst)
    if rank != dst:
        return None
    canvas = torch.empty((height,) + tuple(shard.shape[1:]), dtype=shard.dtype, device=shard.device)
    for r in range(world):
        n = len(rows_of(r, world, height))
        canvas[r::world] = gathered[r][:n]
    return canvas
