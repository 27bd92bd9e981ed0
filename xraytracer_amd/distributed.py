"""Multi-GPU frame assembly: one process per GPU, pixel rows sharded y % world == rank.

Each rank renders its rows into a full-size zero-initialised float3 framebuffer (the
library writes zeros everywhere else), then one ``reduce(SUM)`` to rank 0 assembles the
image.  Pixels are independent in the reference (per-pixel seed j + width*i, per-pixel
accumulation: Src/renderer.cpp:35-36, 75), so the sum is exact: every pixel receives one
rank's value plus zeros.  On ROCm the "nccl" backend is RCCL over xGMI; the tests use
"gloo" on CPU.

``ShardedRenderer`` is the torchrun-side counterpart of the reference's ParallelRenderer
(Src/renderer.cpp:83-99, a thread pool over the rows of one machine): the same row split,
one process per GPU instead of one thread per row, and the frame assembled by a collective
instead of shared memory.  C/C++ callers get the same split inside the library
(``xrt_create_multi``; ``HipRenderer(spp, cam, integ, devices)``).
"""
from __future__ import annotations

# counters of XrtStats that are per-rank work and sum over ranks (the rest are per-rank
# launch statistics: schedule, iterations, kernel times)
SUMMED_COUNTERS = ("segments", "shadow_rays", "draws", "samples", "rejected")


def shard_rows(height: int, rank: int, world: int):
    """Rows owned by `rank` (same rule as the library's shard_index/shard_count)."""
    return list(range(rank, height, world))


def _world(dist):
    if dist is None or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(), dist.get_world_size()


def reduce_framebuffer(fb, dist, dst: int = 0):
    """Sum the per-rank framebuffers into rank `dst` (in place).

    With async_op=False torch makes the caller's current stream wait for the collective, so
    a later render that waits on that stream (xrt_render_device_after) cannot overwrite `fb`
    while the reduce still reads it."""
    if _world(dist)[1] == 1:
        return fb
    dist.reduce(fb, dst=dst, op=dist.ReduceOp.SUM)
    return fb


def max_over_ranks(value: float, dist, device=None) -> float:
    """Slowest rank's time (the bench reports whole-job throughput against it)."""
    if _world(dist)[1] == 1:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_counters(counters: dict, dist, device=None) -> dict:
    """Whole-job totals of the SUMMED_COUNTERS present in `counters` (other keys unchanged)."""
    out = dict(counters)
    if _world(dist)[1] == 1:
        return out
    import torch
    keys = [k for k in SUMMED_COUNTERS if k in counters]
    t = torch.tensor([float(counters[k]) for k in keys], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    out.update(zip(keys, t.tolist()))
    return out


class ShardedRenderer:
    """One rank's share of a frame rendered by every rank of `dist` (ParallelRenderer shape).

    renderer: anything with HipRenderer.render_device's signature (one GPU per rank).
    render(scene, W, H, fb) renders this rank's rows into the device tensor `fb` (H, W, 3)
    float32 — zeros elsewhere — after the work already queued on torch's current stream,
    then reduces the frame into rank `dst`.  Only rank `dst`'s `fb` holds the image.

    Only the overwrite mode is supported: with accumulate=True every rank's unowned rows would
    keep their old contents and the SUM reduce would add them once per rank, so render()
    raises ValueError for it."""

    def __init__(self, renderer, dist=None, dst: int = 0, time_reduce: bool = False):
        self.renderer = renderer
        self.dist = dist
        self.dst = dst
        self.rank, self.world = _world(dist)
        # time_reduce: wait for each framebuffer reduce to complete and record its host time
        # (bench.py); off by default, so callers can overlap the reduce with later work
        self.time_reduce = time_reduce
        self.last_reduce_s = 0.0   # host time of the last render()'s framebuffer reduce (time_reduce)
        if not 0 <= dst < self.world:
            raise ValueError(f"dst rank {dst} outside world of {self.world}")

    def rows(self, height: int):
        return shard_rows(height, self.rank, self.world)

    def render(self, scene, width: int, height: int, fb, after_stream=None, **kw):
        if tuple(fb.shape) != (height, width, 3) or not fb.is_contiguous():
            raise ValueError(f"framebuffer must be a contiguous ({height}, {width}, 3) tensor, got {tuple(fb.shape)}")
        if kw.get("accumulate"):
            raise ValueError("ShardedRenderer supports only the overwrite mode (accumulate=False): a SUM reduce "
                             "of row shards would add every rank's stale unowned rows")
        import torch
        if after_stream is None and fb.is_cuda:
            after_stream = torch.cuda.current_stream(fb.device).cuda_stream
        st = self.renderer.render_device(scene, width, height, fb.data_ptr(), shard_index=self.rank,
                                         shard_count=self.world, after_stream=after_stream, **kw)
        # the render has returned with the image complete; with time_reduce the reduce is
        # timed on its own (host clock to its completion: the next render would wait for it)
        import time
        t0 = time.perf_counter()
        reduce_framebuffer(fb, self.dist, self.dst)
        if self.time_reduce:
            if self.world > 1 and fb.is_cuda:
                torch.cuda.synchronize(fb.device)
            self.last_reduce_s = time.perf_counter() - t0
        return st
