"""GPU parity at every BASELINE.json workload's own geometry, through
the same entry point, flags and launch geometry the bench times — no overrides.

The oracle cannot render the full spp in a test (C2 is 491 M samples), but a pixel's
samples run in order on one RNG stream, so the first k samples of the full-spp render are
exactly a k-spp render: the bench's launch geometry (slots per wave, group traces,
live-list partitions, segments per launch) depends only on the image size and the scene,
which are the workload's own.  Each test asserts that geometry, then compares the image
bit for bit (C3 and C4, whose oracle is the reference's linear scan over 1,001 spheres or
51,236 triangles, on a subset of the GPU frame's rows) and the path counters exactly.
C4 is also rendered as the row shard one rank of its 8-GPU configuration renders.
"""
import functools
import numpy as np
import pytest

import pyoracle
from xraytracer_amd import abi, scenes
from xraytracer_amd.renderer import HipRenderer

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-3  # BASELINE.json north_star: per-channel RMSE < 1e-3 at matched seeds


def compare(img, ref):
    assert img.shape == ref.shape
    rmse = np.sqrt(np.mean((img.astype(np.float64) - ref.astype(np.float64)) ** 2, axis=(0, 1)))
    assert np.all(rmse < RMSE_TOL), rmse
    bad = np.argwhere(~np.all(img == ref, axis=-1))
    assert len(bad) == 0, (len(bad), bad[:5], rmse)


def partitions(n_slots, merged=False):
    """The library's live-list partition count for a shard of n_slots (xrt_api.cpp): the merged
    schedule takes >= 2048 slots per partition (at most 256), the others >= 512 (at most 1024)."""
    max_parts, min_slots = (256, 2048) if merged else (1024, 512)
    n = min(max_parts, max(1, n_slots // min_slots))
    return n & ~7 if n >= 8 else n


def counters_equal(g, st):
    assert (g.segments, g.shadow_rays, g.draws, g.rejected, g.stalled) == \
        (st["segments"], st["shadow_rays"], st["draws"], st["rejected"], st["stalled"])


@pytest.fixture(scope="module")
def renderer():
    r = HipRenderer(1, device=0)
    yield r
    r.close()


def render_like_bench(r, cfg, spp, schedule="auto"):
    """bench.py's step: xrt_render_device into a torch tensor on cuda:0, schedule auto,
    HIP-event timing on, shard 0 of 1."""
    import torch

    c = scenes.CONFIGS[cfg]
    w, h = c["width"], c["height"]
    scene = scenes.build(cfg)
    r.spp = spp
    r.upload(scene)
    fb = torch.full((h, w, 3), 7.0, dtype=torch.float32, device="cuda:0")   # overwritten, not added to
    r.render_device(scene, w, h, fb.data_ptr(), after_stream=torch.cuda.current_stream().cuda_stream,
                    timing=True, schedule=schedule)
    img = fb.cpu().numpy()
    ref, st = pyoracle.render(scene, w, h, spp)
    return img, ref, st, r.stats


def test_c2_headline_geometry(renderer):
    """C2 (Cornell 800x600, GI(3)): the headline kernel k_step_merged with full waves (64
    slots per wave, pair passes, no group traces) over 232 live-list partitions, 64
    segments per launch — the instantiation the bench's number comes from."""
    img, ref, st, g = render_like_bench(renderer, "C2", 4)
    assert g.schedule == abi.XRT_SCHED_STEP_MERGED
    assert (g.slots_per_wave, g.group_lanes, g.partitions, g.visits_per_launch) == (64, 1, partitions(480000, merged=True), 64)
    assert g.samples == 800 * 600 * 4
    compare(img, ref)
    counters_equal(g, st)


def test_c2_headline_across_launches(renderer):
    """the benched instantiation k_step_merged<GI, 1, 64, 1, false> across
    launch boundaries.  At 64 spp a C2 pixel needs ~114 visits (1.78 segments per sample) and
    the worst ~175, so every slot resumes its path state from HBM at least once and the
    frame takes >= 3 step launches; 64 spp draw ~396 words per pixel on average against a
    520-word refill threshold, so most slots' rings are twisted in-launch (wave_refill).
    Full frame, bit-exact, counters equal (Src/renderer.cpp:29-81, Src/sampler.h:16-50)."""
    img, ref, st, g = render_like_bench(renderer, "C2", 64)
    assert g.schedule == abi.XRT_SCHED_STEP_MERGED
    assert (g.slots_per_wave, g.group_lanes, g.partitions, g.visits_per_launch) == (64, 1, partitions(480000, merged=True), 64)
    assert g.launches[abi.XRT_K_STEP] >= 3, g.launches[abi.XRT_K_STEP]
    assert g.launches[abi.XRT_K_REFILL] == 1    # only the first twist of every slot is a launch
    # in-launch refills ran (measured: 258,950 for 480,000 slots — pixels whose samples end
    # after one segment draw ~2.5 words per sample and never run low)
    assert g.rng_twists - g.path_slots > g.path_slots // 4, (g.rng_twists, g.path_slots)
    compare(img, ref)
    counters_equal(g, st)


def test_c3_geometry_across_launches(renderer):
    """VERDICT r2 #1 for C3 (1,000 spheres, 1280x720, Direct) under the per-slot schedule
    (XRT_FLAG_NO_PIXEL; the default is k_pixel, tests/test_gpu_pixel.py): at 96 spp every
    slot needs 96 visits, three rounds of k_step (32 visits per launch), each twisting its
    slots' RNG rings at its end (in-line refills: no k_refill launch after the seeding one).
    The oracle's linear sphere scan is slow, so a row subset (rows y % 64 == 21) of the
    full-frame GPU image is compared bit for bit."""
    import torch

    c = scenes.CONFIGS["C3"]
    w, h, spp = c["width"], c["height"], 96
    scene = scenes.build("C3")
    renderer.spp = spp
    renderer.upload(scene)
    fb = torch.full((h, w, 3), 7.0, dtype=torch.float32, device="cuda:0")
    renderer.render_device(scene, w, h, fb.data_ptr(), after_stream=torch.cuda.current_stream().cuda_stream,
                           timing=True, schedule="step")
    g = renderer.stats
    img = fb.cpu().numpy()
    assert g.schedule == abi.XRT_SCHED_STEP and g.partitions == partitions(w * h)
    assert g.launches[abi.XRT_K_STEP] >= 3 and g.launches[abi.XRT_K_REFILL] == 1, list(g.launches)
    assert g.rng_twists > g.path_slots   # twists beyond each slot's first: done inside k_step
    assert g.segments == w * h * spp   # Direct: one Scene::intersect per sample
    k, n = 21, 64
    ref, st = pyoracle.render(scene, w, h, spp, shard_index=k, shard_count=n)
    compare(img[k::n], ref[k::n])


def test_c3_row_shard(renderer):
    """C3 as one rank of 8 renders it under the per-slot schedule (rows y % 8 == 3: 90 x 1280
    slots, 224 partitions — a grid that is not a power-of-two multiple of the partitions),
    8 spp, zeros elsewhere, rows y % 64 == 3 bit-exact against the oracle."""
    import torch

    c = scenes.CONFIGS["C3"]
    w, h, spp = c["width"], c["height"], 8
    scene = scenes.build("C3")
    renderer.spp = spp
    renderer.upload(scene)
    fb = torch.full((h, w, 3), 7.0, dtype=torch.float32, device="cuda:0")
    renderer.render_device(scene, w, h, fb.data_ptr(), after_stream=torch.cuda.current_stream().cuda_stream,
                           timing=True, schedule="step", shard_index=3, shard_count=8)
    g = renderer.stats
    img = fb.cpu().numpy()
    assert g.schedule == abi.XRT_SCHED_STEP and g.partitions == partitions(90 * 1280) == 224
    assert g.samples == 90 * 1280 * spp
    owned = np.zeros(h, bool)
    owned[3::8] = True
    assert np.all(img[~owned] == 0)
    ref, _ = pyoracle.render(scene, w, h, spp, shard_index=3, shard_count=64)
    compare(img[3::64], ref[3::64])


@pytest.mark.parametrize("schedule", ["auto", "step"])
def test_c3_geometry(renderer, schedule):
    """C3 (1,000 spheres + sphere light, 1280x720, Direct), full frame at 1 spp: the pixel
    schedule (the bench's) and the per-slot fused k_step with the LDS skip-link sphere BVH
    over 1024 partitions."""
    img, ref, st, g = render_like_bench(renderer, "C3", 1, schedule=schedule)
    assert g.schedule == (abi.XRT_SCHED_PIXEL if schedule == "auto" else abi.XRT_SCHED_STEP)
    assert g.partitions == partitions(1280 * 720)
    compare(img, ref)
    counters_equal(g, st)


@pytest.mark.parametrize("sched,deep", [("auto", "auto"), ("wavefront", "auto"), ("wavefront", "single"),
                                        ("wavefront", "quad")])
def test_c4_mesh_geometry(renderer, sched, deep):
    """C4's own mesh: SphereMesh(nTheta = nPhi = 160) = 51,200 triangles + the Cornell box
    (51,236), at C4's 16:9 aspect (160x90): the fused two-level schedule (merged kernel, the
    small objects by pair passes, the BVH walked by the wave's quads — what the bench runs)
    and the wavefront schedule with the BVH walked with four lanes per queued ray and with
    one (XRT_FLAG_DEEP_SINGLE)."""
    s = scenes.cornell_spheremesh(160, 90)
    assert s.desc.n_tris == 51200 + 36
    renderer.spp = 2
    renderer.upload(s)
    img = renderer.render(s, 160, 90, timing=True, deep=deep, schedule=sched)
    g = renderer.stats
    if sched == "auto":
        assert g.schedule == abi.XRT_SCHED_STEP_BVH and g.launches[abi.XRT_K_STEP] > 0
        assert g.launches[abi.XRT_K_TRACE] == g.launches[abi.XRT_K_DEEP] == g.launches[abi.XRT_K_SHADE] == 0
    else:
        assert g.schedule == abi.XRT_SCHED_WAVEFRONT and g.launches[abi.XRT_K_STEP] == 0
        assert g.launches[abi.XRT_K_DEEP] == g.launches[abi.XRT_K_TRACE] > 0
    ref, st = pyoracle.render(s, 160, 90, 2)
    compare(img, ref)
    counters_equal(g, st)


# rows y % 64 == 3 of C4 at 2 spp: a subset of the full frame and of the row shard 3 of 8
C4_SUB = (3, 64)


@functools.lru_cache(maxsize=1)
def c4_reference():
    c = scenes.CONFIGS["C4"]
    k, n = C4_SUB
    return pyoracle.render(scenes.build("C4"), c["width"], c["height"], 2, shard_index=k, shard_count=n)


def render_c4(renderer, **kw):
    import torch

    c = scenes.CONFIGS["C4"]
    w, h = c["width"], c["height"]
    scene = scenes.build("C4")
    assert scene.desc.n_tris == 51200 + 36
    renderer.spp = 2
    renderer.upload(scene)
    fb = torch.full((h, w, 3), 7.0, dtype=torch.float32, device="cuda:0")
    renderer.render_device(scene, w, h, fb.data_ptr(), after_stream=torch.cuda.current_stream().cuda_stream,
                           timing=True, schedule="auto", **kw)
    return fb.cpu().numpy(), renderer.stats


def test_c4_full_geometry(renderer):
    """C4 at its own 1920x1080 through the bench's entry point (auto schedule,
    device output): the fused two-level kernel over 256 live-list partitions across several
    launches; rows y % 64 == 3 bit-exact against the oracle (Src/renderer.cpp:29-81,
    Src/primitive.cpp:83-168)."""
    img, g = render_c4(renderer)
    assert g.schedule == abi.XRT_SCHED_STEP_BVH
    assert g.partitions == partitions(1920 * 1080, merged=True) == 256
    assert g.samples == 1920 * 1080 * 2
    assert g.launches[abi.XRT_K_STEP] >= 2 and g.layout_launches[0] >= 1   # full waves first
    ref, _ = c4_reference()
    k, n = C4_SUB
    compare(img[k::n], ref[k::n])


def test_c4_row_shard(renderer):
    """C4's multi-GPU configuration: the row shard rank 3 of 8 renders (rows y % 8 == 3, 135 x
    1920 slots, 120 partitions); zeros elsewhere, and rows y % 64 == 3 (inside the shard)
    bit-exact against the oracle."""
    img, g = render_c4(renderer, shard_index=3, shard_count=8)
    assert g.schedule == abi.XRT_SCHED_STEP_BVH
    assert g.samples == 135 * 1920 * 2 and g.path_slots == 135 * 1920
    assert g.partitions == partitions(135 * 1920, merged=True) == 120
    owned = np.zeros(1080, bool)
    owned[3::8] = True
    assert np.all(img[~owned] == 0)
    ref, _ = c4_reference()
    k, n = C4_SUB
    compare(img[k::n], ref[k::n])


C4_TWIST_SPP = 96


@functools.lru_cache(maxsize=1)
def c4_twist_reference():
    s = scenes.cornell_spheremesh(64, 36, n_theta=24, n_phi=24)
    return s, pyoracle.render(s, 64, 36, C4_TWIST_SPP)


@pytest.mark.parametrize("spw,shard", [(0, None), (64, None), (32, None), (16, None), (0, 3)])
def test_c4_kernel_twists_in_launch(renderer, spw, shard):
    """the benched C4 kernel k_step_merged<GI, ..., BVH> twisting its slots'
    RNG rings at the end of a launch (wave_refill staged through the MergedWave LDS it shares
    with the BVH top nodes and the quads' stacks).  A slot asks for a twist once fewer than
    rng_keep = 64 * 8 + 8 = 520 words are left, i.e. after ~104 draws, ~15 samples of C4's
    ~7 draws each, so at 96 spp nearly every slot twists in-launch at least once.  The C4 scene
    family with a 24 x 24 sphere mesh (1,152 + 36 triangles: the mesh goes into the BVH), at
    every slots-per-wave layout the library picks from (64, 32, 16; auto = 16 for 2,304
    slots) and as row shard 3 of 8: bit-exact, counters equal (Src/sampler.h:16-50,
    Src/renderer.cpp:29-81)."""
    s, (ref, st) = c4_twist_reference()
    assert s.desc.n_tris == 24 * 24 * 2 + 36
    renderer.spp = C4_TWIST_SPP
    renderer.upload(s)
    kw = {} if shard is None else dict(shard_index=shard, shard_count=8)
    img = renderer.render(s, 64, 36, timing=True, schedule="auto", slots_per_wave=spw, **kw)
    g = renderer.stats
    assert g.schedule == abi.XRT_SCHED_STEP_BVH
    assert g.launches[abi.XRT_K_REFILL] == 1 and g.launches[abi.XRT_K_STEP] >= 2, list(g.launches)
    assert g.rng_twists - g.path_slots > g.path_slots // 4, (g.rng_twists, g.path_slots)
    if spw:
        assert g.layout_launches[abi.LAYOUTS.index(spw)] == g.launches[abi.XRT_K_STEP]
    if shard is None:
        compare(img, ref)
        counters_equal(g, st)
    else:
        owned = np.zeros(36, bool)
        owned[shard::8] = True
        assert np.all(img[~owned] == 0)
        compare(img[owned], ref[owned])


def test_c5_full_frame(renderer):
    """C5 (smoke VPT(10) on the 128^3 grid) at its own 800x600 through the
    bench's entry point, 8 spp: 936 partitions, walks carried across several k_step launches
    with refills, full frame bit-exact and counters equal (Src/integrator.h:409-473,
    Src/medium.cpp:45-133)."""
    img, ref, st, g = render_like_bench(renderer, "C5", 8)
    assert g.schedule == abi.XRT_SCHED_STEP
    assert g.partitions == partitions(800 * 600) == 936
    assert g.launches[abi.XRT_K_STEP] >= 2, list(g.launches)   # 128 events per launch: walks carried over
    compare(img, ref)
    counters_equal(g, st)
    assert st["segments"] > 0


def test_c5_grid_geometry(renderer):
    """C5's own medium: the 128^3 synthetic smoke grid under VolumePathTracing(10), at C5's
    4:3 aspect (200x150, 8 spp) — fused k_step<VPT> with walks that suspend across refills."""
    s = scenes.smoke(200, 150)
    assert s.medium.density.shape == (128, 128, 128)
    renderer.spp = 8
    renderer.upload(s)
    img = renderer.render(s, 200, 150, timing=True)
    g = renderer.stats
    assert g.schedule == abi.XRT_SCHED_STEP
    ref, st = pyoracle.render(s, 200, 150, 8)
    compare(img, ref)
    counters_equal(g, st)
    assert st["segments"] > 0 and st["draws"] > 8 * 200 * 150 * 2


def test_render_device_repeated_steps_ordered_after_caller_stream(renderer):
    """bench.py renders into the same tensor every step while torch work queued on the
    caller's stream still touches it: xrt_render_device_after waits for that work, so every
    step's image is the fresh render, bit-exact (stream ordering)."""
    import torch

    s = scenes.cornell(160, 120)
    renderer.spp = 3
    renderer.upload(s)
    ref, _ = pyoracle.render(s, 160, 120, 3)
    fb = torch.zeros((120, 160, 3), dtype=torch.float32, device="cuda:0")
    junk = torch.randn(2048, 2048, device="cuda:0")
    for step in range(3):
        # queue slow work that writes fb on the caller's stream, then render at once
        for _ in range(4):
            junk = junk @ junk
            junk = junk / junk.norm()
        fb.add_(1000.0 + junk[0, 0])
        renderer.render_device(s, 160, 120, fb.data_ptr(), after_stream=torch.cuda.current_stream().cuda_stream)
        compare(fb.cpu().numpy(), ref)
    # the device-wide form (no stream given) orders the same way
    fb.fill_(5.0)
    renderer.render_device(s, 160, 120, fb.data_ptr())
    compare(fb.cpu().numpy(), ref)


@pytest.mark.parametrize("schedule", ["auto", "wavefront"])
def test_accumulates_into_a_nonzero_image(renderer, schedule):
    """Renderer::render fills the caller's Image in place: samples are added to what the
    pixels hold, then divided (Src/renderer.cpp:75,98).  Host and device entry points."""
    import torch

    s = scenes.cornell(64, 48)
    rng = np.random.default_rng(5)
    init = rng.uniform(0.0, 3.0, (48, 64, 3)).astype(np.float32)
    renderer.spp = 4
    renderer.upload(s)
    img = renderer.render(s, 64, 48, initial=init, schedule=schedule)
    ref, st = pyoracle.render(s, 64, 48, 4, initial=init)
    compare(img, ref)
    plain, _ = pyoracle.render(s, 64, 48, 4)
    assert not np.array_equal(ref, plain)
    fb = torch.from_numpy(init).to("cuda:0")
    renderer.render_device(s, 64, 48, fb.data_ptr(), accumulate=True, schedule=schedule)
    compare(fb.cpu().numpy(), ref)
    # a shard accumulates its own rows and leaves the others as they were
    fb = torch.from_numpy(init).to("cuda:0")
    renderer.render_device(s, 64, 48, fb.data_ptr(), accumulate=True, shard_index=1, shard_count=2,
                           schedule=schedule)
    out = fb.cpu().numpy()
    compare(out[1::2], ref[1::2])
    assert np.array_equal(out[0::2], init[0::2])


@pytest.mark.parametrize("schedule", ["auto", "wavefront"])
def test_rejected_samples(renderer, schedule):
    """The NaN / Inf / negative sample check (Src/renderer.cpp:57-73) with a nonzero count:
    a light whose green radiance is negative makes every sample that sees it negative."""
    s = scenes.SceneBundle()
    s.load_obj(scenes.CORNELL_OBJ)
    s.add_quad_light("QuadLight", (343.0, 548.0, 227.0), (343.0, 548.0, 332.0), (213.0, 548.0, 227.0),
                     (25.0, -1.0, 25.0))
    s.flatten()
    s.camera = scenes.pinhole(scenes.CORNELL_C2W, 60.0, 64, 48)
    renderer.spp = 6
    renderer.upload(s)
    for integ in ("gi", "direct"):
        img = renderer.render(s, 64, 48, integrator=integ, schedule=schedule)
        ref, st = pyoracle.render(s, 64, 48, 6, integrator=integ)
        compare(img, ref)
        assert st["rejected"] > 1000
        counters_equal(renderer.stats, st)


def test_shard_without_rows(renderer):
    """A rank that owns no rows (shard_index >= height) returns an all-zero image."""
    s = scenes.cornell(8, 2)
    renderer.spp = 2
    renderer.upload(s)
    img = renderer.render(s, 8, 2, shard_index=3, shard_count=4)
    assert np.all(img == 0)
    assert renderer.stats.samples == 0
