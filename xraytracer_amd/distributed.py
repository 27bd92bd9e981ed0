"""Multi-GPU frame assembly: one process per GPU, pixel rows sharded y % world == rank.

Each rank renders its rows into a full-size float3 framebuffer (the library writes zeros
everywhere else).  Pixels are independent in the reference (per-pixel seed j + width*i,
per-pixel accumulation: Src/renderer.cpp:35-36, 75), so rank 0's image is assembled from the
ranks' rows alone, two ways:

* ``gather`` (default): every rank packs its rows y % world == rank into a (ceil(H/world), W, 3)
  buffer and one ``gather`` brings them to rank 0, which writes them into their rows — each
  rank sends 1/world of the frame over its own xGMI link to rank 0 (a point-to-point hop per
  rank) instead of a ring pass over the whole frame.
* ``reduce``: one ``reduce(SUM)`` of the full framebuffers — exact too, every pixel receives
  one rank's value plus zeros, but it moves world times the bytes.

On ROCm the "nccl" backend is RCCL over xGMI; the tests use "gloo" on CPU.

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


def gather_framebuffer(fb, dist, dst: int = 0):
    """Assemble the row shards into rank `dst`'s `fb` (in place): each rank sends only its
    rows y % world == rank, packed into ceil(H / world) rows (the last one padding when H is not
    a multiple of world); rank `dst` writes every other rank's rows into place.  Bit-identical
    to reduce_framebuffer: both leave each pixel the value of the one rank that owns it.

    With async_op=False torch makes the caller's current stream wait for the collective, so a
    later render that waits on that stream cannot overwrite `fb` (or the send buffer's source
    rows) while the gather still reads them."""
    rank, world = _world(dist)
    if world == 1:
        return fb
    height = fb.shape[0]
    rmax = (height + world - 1) // world
    send = fb.new_zeros((rmax,) + tuple(fb.shape[1:]))
    mine = fb[rank::world]
    send[: mine.shape[0]] = mine
    if rank == dst:
        bufs = [send if r == dst else fb.new_empty(send.shape) for r in range(world)]
        dist.gather(send, gather_list=bufs, dst=dst)
        for r in range(world):
            if r != dst:
                n = len(range(r, height, world))
                fb[r::world] = bufs[r][:n]
    else:
        dist.gather(send, dst=dst)
    return fb


def assembly_bytes(height: int, width: int, world: int, mode: str = "gather") -> int:
    """Framebuffer bytes sent per frame, all ranks together: gather — every other rank's packed
    rows into rank 0; reduce — (world - 1) full framebuffers' worth (each rank's frame is
    combined once on its way to rank 0, whatever the algorithm's chunking)."""
    if world == 1:
        return 0
    if mode == "gather":
        return (world - 1) * ((height + world - 1) // world) * width * 12
    return (world - 1) * height * width * 12


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
    then assembles the frame in rank `dst`'s `fb` (only that one holds the image).

    assembly: "gather" (each rank sends its owned rows; default) or "reduce" (a SUM reduce of
    the full framebuffers).  Only the overwrite mode is supported: with accumulate=True every
    rank's unowned rows would keep their old contents (and the SUM reduce would add them once
    per rank), so render() raises ValueError for it."""

    def __init__(self, renderer, dist=None, dst: int = 0, time_reduce: bool = False, assembly: str = "gather"):
        if assembly not in ("gather", "reduce"):
            raise ValueError(f"assembly must be 'gather' or 'reduce', got {assembly!r}")
        self.renderer = renderer
        self.dist = dist
        self.dst = dst
        self.assembly = assembly
        self.rank, self.world = _world(dist)
        # time_reduce: wait for each framebuffer reduce to complete and record its host time
        # (bench.py); off by default, so callers can overlap the reduce with later work
        self.time_reduce = time_reduce
        self.last_reduce_s = 0.0   # host time of the last render()'s frame assembly (time_reduce)
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
        if self.assembly == "gather":
            gather_framebuffer(fb, self.dist, self.dst)
        else:
            reduce_framebuffer(fb, self.dist, self.dst)
        if self.time_reduce:
            if self.world > 1 and fb.is_cuda:
                torch.cuda.synchronize(fb.device)
            self.last_reduce_s = time.perf_counter() - t0
        return st
