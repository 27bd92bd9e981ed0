"""N>1 path on CPU: world_size-2 gloo run of the frame-assembly code bench.py uses.

Each rank renders its row shard (here with the CPU oracle standing in for the device
shard render, since this container has no GPU; the device shard render itself is covered
by tests/test_gpu_parity.py::test_shards_reassemble_exactly) into a zero framebuffer, and
xraytracer_amd.distributed.reduce_framebuffer sums them to rank 0.  The assembled image
must equal the single-process render bit for bit.
"""
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
