"""CPU stand-in for HipRenderer in bench.py's multi-rank plumbing test (tests/test_bench_launch.py),
selected with bench.py --test-standin bench_standin:make.  Not the oracle and not a renderer: it
writes a known value into the rows a shard owns (zeros elsewhere), so the reduced frame can be
checked, and returns counters shaped like xrt_stats.  XRT_BENCH_STANDIN_FAIL_RANK=r makes
rank r raise in its render, to test that a failing rank fails the job."""
import ctypes
import os
from types import SimpleNamespace

import numpy as np


class StandIn:
    def __init__(self, spp, device):
        self.spp = spp
        self.device = device
        self.frames = 0
        self.reduced_ok = 0   # rank 0: frames whose reduced image (read back at the next render) was whole

    def upload(self, scene):
        pass

    def render_device(self, scene, width, height, ptr, shard_index=0, shard_count=1, **kw):
        if str(shard_index) == os.environ.get("XRT_BENCH_STANDIN_FAIL_RANK"):
            raise RuntimeError(f"stand-in rank {shard_index} fails on purpose")
        fb = np.ctypeslib.as_array((ctypes.c_float * (height * width * 3)).from_address(ptr))
        fb = fb.reshape(height, width, 3)
        if shard_index == 0 and self.frames > 0:   # bench renders into the tensor rank 0 reduced into
            want = np.broadcast_to((np.arange(height, dtype=np.float32) + 1)[:, None, None], fb.shape)
            self.reduced_ok += int(np.array_equal(fb, want))
        fb[:] = 0.0
        rows = np.arange(shard_index, height, shard_count)
        fb[rows] = (rows[:, None, None] + 1).astype(np.float32)   # row y holds y + 1
        self.frames += 1
        n = len(rows) * width
        k = [0.0] * 7
        return SimpleNamespace(segments=n * self.spp, shadow_rays=0, draws=2 * n * self.spp, samples=n * self.spp,
                               iterations=1, rejected=0, kernel_ms=k, launches=[0] * 7, schedule=5)

    def close(self):
        out = os.environ.get("XRT_BENCH_STANDIN_OUT")
        if out:
            with open(f"{out}.{os.environ.get('RANK', '0')}", "w") as f:
                f.write(f"{self.frames} {self.reduced_ok}")


def make(spp, device):
    return StandIn(spp, device)
