"""Multi-GPU inside the library (xrt_create_multi; the C++ HipRenderer(spp, cam, integ,
devices) of ParallelRenderer, Src/renderer.cpp:83-99): row shards rendered concurrently
per device and assembled on the first device by strided peer copies.

The GPU box has one MI355X, so the device list names GPU 0 several times: every device
context, host thread, stream and the row gather run exactly as on a node, only on one
card.  The frame must be bit-identical to the one-GPU render and to the oracle.
"""
import os
import subprocess

import numpy as np
import pytest

import pyoracle
from xraytracer_amd import abi, scenes
from xraytracer_amd.renderer import HipRenderer

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def single():
    r = HipRenderer(4, device=0)
    yield r
    r.close()


@pytest.mark.parametrize("n", [2, 3])
def test_multi_matches_single_and_oracle(single, n):
    s = scenes.cornell(96, 71)
    m = HipRenderer(4, devices=[0] * n)
    assert abi.lib().xrt_device_count(m.ctx) == n
    img = m.render(s, 96, 71, timing=True)
    ref, st = pyoracle.render(s, 96, 71, 4)
    assert np.array_equal(img, ref)
    g = m.stats
    assert (g.samples, g.segments, g.shadow_rays, g.draws) == (96 * 71 * 4, st["segments"], st["shadow_rays"],
                                                               st["draws"])
    single.spp = 4
    assert np.array_equal(single.render(s, 96, 71), img)
    # the caller's own row shard, split again over the devices
    part = m.render(s, 96, 71, shard_index=1, shard_count=2)
    assert np.array_equal(part[1::2], ref[1::2]) and np.all(part[0::2] == 0)
    m.close()


def test_multi_device_output_accumulate_and_media():
    import torch

    m = HipRenderer(3, devices=[0, 0])
    s = scenes.cornell(64, 48)
    init = np.random.default_rng(1).uniform(0, 2, (48, 64, 3)).astype(np.float32)
    ref, _ = pyoracle.render(s, 64, 48, 3, initial=init)
    assert np.array_equal(m.render(s, 64, 48, initial=init), ref)
    fb = torch.from_numpy(init).to("cuda:0")
    m.render_device(s, 64, 48, fb.data_ptr(), accumulate=True)
    assert np.array_equal(fb.cpu().numpy(), ref)
    fb.fill_(9.0)
    m.render_device(s, 64, 48, fb.data_ptr(), after_stream=torch.cuda.current_stream().cuda_stream)
    plain, _ = pyoracle.render(s, 64, 48, 3)
    assert np.array_equal(fb.cpu().numpy(), plain)
    # the medium is uploaded to every device (VolumePathTracing, fused k_step<VPT>)
    v = scenes.smoke(40, 30, n=32)
    ref, st = pyoracle.render(v, 40, 30, 3)
    assert np.array_equal(m.render(v, 40, 30), ref)
    assert m.stats.draws == st["draws"]
    m.close()


def test_cpp_multi_gpu_renderer(tmp_path):
    """examples/cornellbox.cpp with a device list: HipRenderer(spp, cam, integ, {0, 0})."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "examples", "bin", "cornellbox")
    out = tmp_path / "fb.raw"
    env = dict(os.environ, XRT_DATA_DIR=os.path.join(root, "xraytracer_amd", "data") + "/")
    subprocess.check_call([exe, "64", "48", "4", "gi", str(out), "0,0"], env=env)
    img = np.fromfile(out, dtype=np.float32).reshape(48, 64, 3)
    ref, _ = pyoracle.render(scenes.cornell(64, 48), 64, 48, 4)
    assert np.array_equal(img, ref)


def test_sharded_renderer_device_frames(single):
    """bench.py's step on one GPU: distributed.ShardedRenderer over HipRenderer.render_device
    into one torch tensor, frame after frame (the render waits on torch's current stream, so
    a stale buffer and queued torch work are overwritten in order), each frame equal to the
    oracle; a row shard of the same tensor holds the oracle's shard rows and zeros."""
    import torch
    from xraytracer_amd import distributed

    W, H = 72, 40
    s = scenes.cornell(W, H)
    single.spp = 4
    sr = distributed.ShardedRenderer(single, None)
    fb = torch.full((H, W, 3), 3.0, dtype=torch.float32, device="cuda:0")
    ref, st = pyoracle.render(s, W, H, 4)
    for _ in range(2):
        fb.mul_(2.0)   # torch work queued on the current stream before the render
        got = sr.render(s, W, H, fb)
        assert np.array_equal(fb.cpu().numpy(), ref)
        assert (got.samples, got.segments, got.draws) == (W * H * 4, st["segments"], st["draws"])
    part, _ = pyoracle.render(s, W, H, 4, shard_index=1, shard_count=3)
    got = single.render_device(s, W, H, fb.data_ptr(), shard_index=1, shard_count=3,
                               after_stream=torch.cuda.current_stream().cuda_stream)
    assert np.array_equal(fb.cpu().numpy(), part)
    assert got.samples == W * len(distributed.shard_rows(H, 1, 3)) * 4


def _slow_then_fill(stream, fb, value):
    """Queue ~tens of ms of GPU work on `stream`, then overwrite fb: a render that does not
    wait for `stream` would run before the fill and be clobbered by it."""
    import torch

    with torch.cuda.stream(stream):
        if hasattr(torch.cuda, "_sleep"):
            torch.cuda._sleep(50_000_000)
        else:   # pragma: no cover - older torch
            x = torch.randn(4096, 4096, device=fb.device)
            for _ in range(8):
                x = x @ x
                x = x / x.norm()
        fb.fill_(value)


@pytest.mark.parametrize("which", ["side", "legacy_null"])
def test_sharded_render_waits_for_long_work_on_after_stream(single, which):
    """ShardedRenderer's render must start only after the work queued on
    the stream it is given.  Long work (a device sleep) followed by a fill of the framebuffer
    is queued on a side stream (or the legacy null stream, handle 0); the render is told to
    wait on that stream and must still produce the oracle's image, not the fill value."""
    import torch
    from xraytracer_amd import distributed

    W, H = 64, 40
    s = scenes.cornell(W, H)
    single.spp = 3
    ref, _ = pyoracle.render(s, W, H, 3)
    sr = distributed.ShardedRenderer(single, None)
    fb = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    if which == "side":
        stream = torch.cuda.Stream(device="cuda:0")
        handle = stream.cuda_stream
    else:
        stream = torch.cuda.default_stream("cuda:0")
        handle = 0
        assert stream.cuda_stream == 0
    for _ in range(2):
        _slow_then_fill(stream, fb, 9.0)
        sr.render(s, W, H, fb, after_stream=handle)
        torch.cuda.synchronize()
        assert np.array_equal(fb.cpu().numpy(), ref)
    if which == "side":
        # control: told to wait on an idle stream, the render finishes first and the queued
        # fill lands on top of it — so the queued work above was long enough to matter
        idle = torch.cuda.Stream(device="cuda:0")
        _slow_then_fill(stream, fb, 9.0)
        sr.render(s, W, H, fb, after_stream=idle.cuda_stream)
        torch.cuda.synchronize()
        assert np.all(fb.cpu().numpy() == 9.0)


def test_sharded_render_rejects_accumulate(single):
    """row shards + a SUM reduce cannot accumulate (each rank's unowned rows would
    be added once per rank), so ShardedRenderer refuses accumulate=True."""
    import torch
    from xraytracer_amd import distributed

    sr = distributed.ShardedRenderer(single, None)
    fb = torch.zeros((8, 8, 3), dtype=torch.float32, device="cuda:0")
    with pytest.raises(ValueError):
        sr.render(scenes.cornell(8, 8), 8, 8, fb, accumulate=True)


def _device_count():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_device_count() < 2, reason="needs two physical GPUs (the round's GPU box has one)")
def test_two_physical_devices_match_oracle():
    """xrt_create_multi over two physical devices — peer access enabled
    between them and the row gather a cross-device strided copy — bit-exact, including the
    two-level C4 family on the fused schedule."""
    n = min(_device_count(), 4)
    m = HipRenderer(3, devices=list(range(n)))
    assert abi.lib().xrt_device_count(m.ctx) == n
    for s, w, h in ((scenes.cornell(96, 71), 96, 71),
                    (scenes.cornell_spheremesh(64, 36, n_theta=40, n_phi=40), 64, 36)):
        img = m.render(s, w, h)
        ref, _ = pyoracle.render(s, w, h, 3)
        assert np.array_equal(img, ref)
    m.close()


@pytest.mark.skipif(_device_count() < 2, reason="needs two physical GPUs (the round's GPU box has one)")
def test_bench_runs_ranks_over_rccl(tmp_path):
    """`bench.py --gpus 2` without a launcher starts two ranks (one per GPU, RCCL reduce of
    the framebuffer) and reports n_gpus 2; the reduce time is reported on its own."""
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--spp", "8", "--no-cpu"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["config"]["assembly_ms_per_step"] >= 0.0 and d["config"]["assembly"] == "gather"
