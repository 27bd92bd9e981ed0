"""Multi-GPU frame assembly: one process per GPU, pixel rows sharded y % world == rank.

Each rank renders its rows into a full-size zero-initialised float3 framebuffer (the
library writes zeros everywhere else), then one ``reduce(SUM)`` to rank 0 assembles the
image.  Pixels are independent in the reference (per-pixel seed j + width*i, per-pixel
accumulation: Src/renderer.cpp:35-36, 75), so the sum is exact: every pixel receives one
rank's value plus zeros.  On ROCm the "nccl" backend is RCCL over xGMI; the tests use
"gloo" on CPU.
"""
from __future__ import annotations


def shard_rows(height: int, rank: int, world: int):
    """Rows owned by `rank` (same rule as the library's shard_index/shard_count)."""
    return list(range(rank, height, world))


def reduce_framebuffer(fb, dist, dst: int = 0):
    """Sum the per-rank framebuffers into rank `dst` (in place)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return fb
    dist.reduce(fb, dst=dst, op=dist.ReduceOp.SUM)
    return fb


def max_over_ranks(value: float, dist, device=None) -> float:
    """Slowest rank's time (the bench reports whole-job throughput against it)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
