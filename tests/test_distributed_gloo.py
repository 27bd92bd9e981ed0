"""N>1 path on CPU: world_size-2 gloo run of the frame-assembly code bench.py uses.

Each rank renders its row shard (here with the CPU oracle standing in for the device
shard render, since this container has no GPU; the device shard render itself is covered
by tests/test_gpu_parity.py::test_shards_reassemble_exactly) into a zero framebuffer, and
xraytracer_amd.distributed.reduce_framebuffer sums them to rank 0.  The assembled image
must equal the single-process render bit for bit.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, SPP = 40, 23, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import pyoracle
    from xraytracer_amd import distributed, scenes
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = scenes.cornell(W, H)
    part, _ = pyoracle.render(s, W, H, SPP, nthreads=1, shard_index=rank, shard_count=world)
    rows = set(distributed.shard_rows(H, rank, world))
    assert all(np.all(part[y] == 0) for y in range(H) if y not in rows)
    fb = torch.from_numpy(part.copy())
    distributed.reduce_framebuffer(fb, dist)
    t = distributed.max_over_ranks(float(rank + 1), dist)
    if rank == 0:
        np.save(out_path, fb.numpy())
        assert t == float(world)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_row_shards_reduce_to_full_image(tmp_path, world):
    import pyoracle
    from xraytracer_amd import scenes
    out = str(tmp_path / "fb.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    full, _ = pyoracle.render(scenes.cornell(W, H), W, H, SPP, nthreads=1)
    assert np.array_equal(got, full)


class _OracleShardRenderer:
    """Stand-in for HipRenderer.render_device on CPU: writes the oracle's shard into the
    framebuffer's memory through the pointer, as the library writes a device buffer."""

    def __init__(self, spp):
        self.spp = spp
        self.calls = []

    def render_device(self, scene, width, height, out_ptr, shard_index=0, shard_count=1, after_stream=None, **kw):
        import pyoracle
        part, _ = pyoracle.render(scene, width, height, self.spp, nthreads=1, shard_index=shard_index,
                                  shard_count=shard_count)
        part = np.ascontiguousarray(part, dtype=np.float32)
        ctypes.memmove(out_ptr, part.ctypes.data, part.nbytes)
        self.calls.append((shard_index, shard_count, after_stream))
        return {"samples": width * len(range(shard_index, height, shard_count)) * self.spp}


def _sharded_worker(rank, world, port, out_path, steps, assembly="gather", dst=0):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    from xraytracer_amd import distributed, scenes
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = scenes.cornell(W, H)
    r = _OracleShardRenderer(SPP)
    sr = distributed.ShardedRenderer(r, dist, dst=dst, assembly=assembly)
    assert sr.rows(H) == distributed.shard_rows(H, rank, world)
    fb = torch.full((H, W, 3), 7.0)   # stale contents: every step overwrites the whole buffer
    frames = []
    for _ in range(steps):
        st = sr.render(s, W, H, fb)
        if rank == dst:
            frames.append(fb.numpy().copy())
        elif assembly == "gather":   # a sender's own buffer is untouched: its rows, zeros elsewhere
            mine = np.zeros(H, bool)
            mine[rank::world] = True
            assert np.all(fb.numpy()[~mine] == 0) and np.any(fb.numpy()[mine] != 0)
    assert r.calls == [(rank, world, None)] * steps
    tot = distributed.sum_counters({"samples": st["samples"], "iterations": 5}, dist)
    assert tot["samples"] == W * H * SPP and tot["iterations"] == 5
    if rank == dst:
        np.save(out_path, np.stack(frames))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,assembly,dst", [(2, "gather", 0), (3, "gather", 0), (3, "gather", 1),
                                                (2, "reduce", 0), (3, "reduce", 0)])
def test_sharded_renderer_every_step_exact(tmp_path, world, assembly, dst):
    """ShardedRenderer (bench.py's step): several frames in a row into the same buffer, each
    assembled on rank `dst` equal to the one-process render, by the owned-rows gather (the
    default: each rank sends only rows y % world == rank, packed) and by the SUM reduce of full
    framebuffers; world 3 leaves uneven row counts (H = 23: 8, 8, 7 rows, so one packed buffer
    carries a padding row)."""
    import pyoracle
    from xraytracer_amd import scenes
    out = str(tmp_path / "frames.npy")
    mp.spawn(_sharded_worker, args=(world, _free_port(), out, 3, assembly, dst), nprocs=world, join=True)
    got = np.load(out)
    full, _ = pyoracle.render(scenes.cornell(W, H), W, H, SPP, nthreads=1)
    assert got.shape[0] == 3
    for f in got:
        assert np.array_equal(f, full)


def test_sharded_renderer_rejects_bad_buffer():
    from xraytracer_amd import distributed
    sr = distributed.ShardedRenderer(_OracleShardRenderer(1), None)
    assert (sr.rank, sr.world) == (0, 1)
    with pytest.raises(ValueError):
        sr.render(None, W, H, torch.zeros((H, W + 1, 3)))
    with pytest.raises(ValueError):
        distributed.ShardedRenderer(_OracleShardRenderer(1), None, dst=1)
    # row shards + SUM reduce cannot accumulate in place
    with pytest.raises(ValueError):
        sr.render(None, W, H, torch.zeros((H, W, 3)), accumulate=True)
    with pytest.raises(ValueError):
        distributed.ShardedRenderer(_OracleShardRenderer(1), None, assembly="allreduce")


def test_assembly_bytes():
    from xraytracer_amd import distributed
    # C3 1280x720 at 8 ranks: 7 packed 90-row shards vs 7 full 11 MB framebuffers
    assert distributed.assembly_bytes(720, 1280, 8) == 7 * 90 * 1280 * 12
    assert distributed.assembly_bytes(720, 1280, 8, "reduce") == 7 * 720 * 1280 * 12
    assert distributed.assembly_bytes(23, 40, 3) == 2 * 8 * 40 * 12
    assert distributed.assembly_bytes(600, 800, 1) == 0
