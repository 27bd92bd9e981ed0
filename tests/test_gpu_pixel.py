"""Pixel-parallel sample chains (k_pixel, xraytracer_amd/csrc/pixel.hip) against the oracle.

The schedule evaluates 64 candidate samples of one pixel at once (every even stream offset
of a window) and keeps the ones on the pixel's chain o -> o + 2 + 2·NL·hit(o): DirectIntegrator
(Src/integrator.h:82-119) draws 2 words per area light only after a surface hit, Normal
(:22-74) never.  Bar: the framebuffer bit for bit and every counter — Scene::intersect calls,
shadow rays, RNG draws (the final stream cursor of every pixel, summed), rejects — equal to the
reference's sequential NormalRenderer::doRender (Src/renderer.cpp:29-81) as restated by the
oracle.  Cases: spp around the window size (chains that end mid-window, windows that end
inside a sample's light words), one and two lights, streams long enough to wrap the wave's
624-word LDS window many times, tie-breaking sphere BVHs, triangle and mixed scenes, the
in-place accumulate contract, rejected samples, row shards and C3's own 1280x720 geometry.
"""
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


def counters_equal(g, st):
    assert (g.segments, g.shadow_rays, g.draws, g.rejected, g.stalled) == \
        (st["segments"], st["shadow_rays"], st["draws"], st["rejected"], st["stalled"])


@pytest.fixture(scope="module")
def renderer():
    r = HipRenderer(1, device=0)
    yield r
    r.close()


def render_pixel(r, scene, w, h, spp, integrator=None, **kw):
    r.spp = spp
    r._uploaded = None
    img = r.render(scene, w, h, integrator=integrator, timing=True, **kw)
    g = r.stats
    okw = {k: v for k, v in kw.items() if k in ("shard_index", "shard_count", "initial")}
    ref, st = pyoracle.render(scene, w, h, spp, integrator=integrator, **okw)
    assert g.schedule == abi.XRT_SCHED_PIXEL, g.schedule
    assert g.launches[abi.XRT_K_STEP] == 1 and g.launches[abi.XRT_K_REFILL] == 0, list(g.launches)
    return img, ref, st, g


def two_light_cornell(w, h):
    s = scenes.SceneBundle()
    s.load_obj(scenes.CORNELL_OBJ)
    s.add_quad_light("QuadLight", (343.0, 548.0, 227.0), (343.0, 548.0, 332.0), (213.0, 548.0, 227.0),
                     (25.0, 25.0, 25.0))
    s.add_triangle_light("TriLight", (100.0, 500.0, 100.0), (150.0, 500.0, 100.0), (100.0, 500.0, 150.0),
                         (10.0, 5.0, 2.0))
    s.flatten()
    s.camera = scenes.pinhole(scenes.CORNELL_C2W, 60.0, w, h)
    return s


def dup_spheres(w, h):
    """Every sphere twice (equal hit distances): the BVH must keep the reference's in-order
    tie break."""
    s = scenes.SceneBundle()
    for k in range(24):
        x, z = -3.0 + (k % 6) * 1.2, -2.0 - (k // 6) * 1.2
        s.add_sphere(f"a{k:02d}", (x, 0.0, z), 0.5, (0.9, 0.2, 0.2))
        s.add_sphere(f"b{k:02d}", (x, 0.0, z), 0.5, (0.2, 0.9, 0.2))
    s.add_sphere_light("SphereLight", (0.0, 6.0, -4.0), 1.5, (20.0, 20.0, 20.0))
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 3, 4, 1), 60.0, w, h)
    return s


def test_c3_family_long_chains(renderer):
    """C3's scene (1,000 spheres + a sphere light, Direct) at C3's own 512 spp on a 48x27
    image: ~1,000-2,000 words per pixel, so every wave regenerates its 624-word LDS window
    many times and walks ~8-16 windows per pixel."""
    s = scenes.spheres(48, 27)
    img, ref, st, g = render_pixel(renderer, s, 48, 27, 512)
    compare(img, ref)
    counters_equal(g, st)
    assert g.segments == 48 * 27 * 512
    assert st["draws"] > 48 * 27 * 512 * 2   # some samples hit surfaces and draw light words
    assert g.rng_twists >= g.path_slots * 2


@pytest.mark.parametrize("wh", [(4, 3), (9, 5), (23, 13)])
def test_frustum_lists_and_their_overflow(renderer, wh):
    """Sphere-BVH scenes trace a pixel's camera rays against the spheres its widened jitter
    pyramid meets (pix_frustum).  At 4x3 a pixel's pyramid holds far more than the list's 64
    entries, so those pixels walk the BVH instead; at 23x13 the pixels build lists."""
    w, h = wh
    s = scenes.spheres(w, h)
    img, ref, st, g = render_pixel(renderer, s, w, h, 150)
    compare(img, ref)
    counters_equal(g, st)
    # which of k_pixel's paths ran (xrt_stats pix_*): every pixel builds a list or overflows
    assert g.pix_frustum + g.pix_frustum_overflow == w * h
    if wh == (4, 3):
        assert g.pix_frustum_overflow > 0   # pyramids holding more than 64 spheres walk the BVH
    if wh == (23, 13):
        assert g.pix_frustum > 0


def far_cluster(w, h, n=300, seed=11):
    """n small spheres in a 12-unit cluster around (5000, 2000, -8000) with a sphere light and
    the camera 15 units away: coordinates ~1e4 against a ~20-unit scene, so the float error of
    the list tests' dot products is a few times 1e-4, near the BVH margin (sph_pad)."""
    rng = np.random.default_rng(seed)
    s = scenes.SceneBundle()
    base = np.array([5000.0, 2000.0, -8000.0])
    for k in range(n):
        c = base + rng.uniform(-6.0, 6.0, 3)
        s.add_sphere(f"s{k:03d}", tuple(float(x) for x in c), float(rng.uniform(0.2, 0.6)),
                     tuple(float(x) for x in rng.uniform(0.2, 0.9, 3)))
    s.add_sphere_light("SphereLight", tuple(float(x) for x in base + [0.0, 12.0, 0.0]), 2.0, (30.0, 30.0, 30.0))
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, base[0], base[1] + 1.0, base[2] + 15.0, 1), 50.0, w, h)
    s.integrator, s.max_depth = "direct", 1
    return s


@pytest.mark.parametrize("wh", [(40, 30), (160, 90)])
def test_block_culled_lists_far_from_origin(renderer, wh):
    """The frustum and shadow lists are built from 64-sphere blocks whose bounding ball meets
    the pixel's pyramid / the shadow hulls (KParams::sblk): a cluster far from the origin (float
    error of the tests near the margin) with 5 blocks, at a coarse and a fine pixel size."""
    w, h = wh
    s = far_cluster(w, h)
    img, ref, st, g = render_pixel(renderer, s, w, h, 48)
    compare(img, ref)
    counters_equal(g, st)
    assert st["shadow_rays"] > 0
    assert g.pix_frustum > 0 and g.pix_shadow_list > 0 and g.pix_flushes > 0


@pytest.mark.parametrize("spp", [1, 2, 21, 31, 32, 33, 63, 64, 65, 127, 129, 300])
def test_window_edges_two_lights(renderer, spp):
    """Two area lights (NL = 2: a surface hit draws 4 light words, so a chain skips 2
    candidates): spp below, at and above the 64-candidate window, chains that end inside
    a window and windows whose last sample's light words run past the window."""
    s = two_light_cornell(24, 18)
    img, ref, st, g = render_pixel(renderer, s, 24, 18, spp, integrator="direct")
    compare(img, ref)
    counters_equal(g, st)


@pytest.mark.parametrize("spp", [1, 64, 65, 200])
def test_cornell_direct_one_light(renderer, spp):
    s = scenes.cornell(40, 30)
    img, ref, st, g = render_pixel(renderer, s, 40, 30, spp, integrator="direct")
    compare(img, ref)
    counters_equal(g, st)


@pytest.mark.parametrize("integ", ["direct", "normal"])
def test_sphere_bvh_ties(renderer, integ):
    s = dup_spheres(48, 36)
    img, ref, st, g = render_pixel(renderer, s, 48, 36, 96, integrator=integ)
    compare(img, ref)
    counters_equal(g, st)


@pytest.mark.parametrize("spp", [1, 63, 64, 65, 150])
def test_normal_integrator_scenes(renderer, spp):
    """NormalIntegrator: every candidate is a sample (2 words each); triangle, sphere and
    mixed (medium box) scenes."""
    for s, w, h in ((scenes.cornell(32, 24), 32, 24), (dup_spheres(24, 18), 24, 18), (scenes.smoke(16, 12), 16, 12)):
        img, ref, st, g = render_pixel(renderer, s, w, h, spp, integrator="normal")
        compare(img, ref)
        counters_equal(g, st)


def test_accumulate_and_rejects(renderer):
    """Renderer::render's in-place contract (samples added to the Image's prior contents,
    Src/renderer.cpp:75) and the NaN / Inf / negative check (:57-73) with a nonzero reject
    count: a light whose green radiance is negative."""
    s = scenes.SceneBundle()
    s.load_obj(scenes.CORNELL_OBJ)
    s.add_quad_light("QuadLight", (343.0, 548.0, 227.0), (343.0, 548.0, 332.0), (213.0, 548.0, 227.0),
                     (25.0, -1.0, 25.0))
    s.flatten()
    s.camera = scenes.pinhole(scenes.CORNELL_C2W, 60.0, 32, 24)
    init = np.random.default_rng(3).uniform(0.0, 2.0, (24, 32, 3)).astype(np.float32)
    img, ref, st, g = render_pixel(renderer, s, 32, 24, 70, integrator="direct", initial=init)
    compare(img, ref)
    counters_equal(g, st)
    assert st["rejected"] > 1000


def test_deferred_shading_rejects_and_accumulate(renderer):
    """Direct on a sphere scene queues its surface hits and shades three windows at once
    (pixel.hip deferred shading); the pending samples keep their order through the flush:
    a sphere light with negative green radiance makes every sample that sees it (directly or
    through a light sample) rejected, samples are added to a nonzero image, and spp values
    end the chain at every point of a flush cycle."""
    s = scenes.SceneBundle()
    for k in range(30):
        x, z = -3.0 + (k % 6) * 1.2, -2.0 - (k // 6) * 1.2
        s.add_sphere(f"s{k:02d}", (x, 0.0, z), 0.5, (0.7, 0.5, 0.3))
    s.add_sphere_light("SphereLight", (0.5, 2.5, -4.0), 1.0, (20.0, -1.0, 20.0))
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 3, 4, 1), 60.0, 32, 24)
    init = np.random.default_rng(4).uniform(0.0, 2.0, (24, 32, 3)).astype(np.float32)
    for spp in (5, 64, 130, 191, 257):
        img, ref, st, g = render_pixel(renderer, s, 32, 24, spp, integrator="direct", initial=init)
        compare(img, ref)
        counters_equal(g, st)
        assert st["rejected"] > 0


@pytest.mark.parametrize("light", ["quad", "triangle", "sphere"])
def test_shadow_occluder_lists(renderer, light):
    """Direct on a sphere scene with one sphere light traces a pixel's shadow rays against the
    occluders that meet the hull of its camera-list spheres and the light's bounding ball
    (pix_shadow_list) instead of walking the BVH, at sizes where pixels see 1-4 spheres (lists)
    and more (BVH walks).  Under a quad or a triangle light the scene holds a mesh (the light's
    object), so it is not a sphere-BVH scene and every window walks the scene: the same images,
    with the list counters at zero."""
    s = scenes.SceneBundle()
    for k in range(48):
        x, z = -3.5 + (k % 8) * 1.0, -2.0 - (k // 8) * 1.0
        s.add_sphere(f"s{k:02d}", (x, 0.1 * (k % 3), z), 0.45, (0.6, 0.6, 0.6))
    if light == "quad":
        s.add_quad_light("L", (-1.0, 4.0, -3.0), (1.0, 4.0, -3.0), (-1.0, 4.0, -5.0), (12.0, 12.0, 12.0))
    elif light == "triangle":
        s.add_triangle_light("L", (-1.0, 4.0, -3.0), (1.5, 4.0, -3.5), (0.0, 4.5, -6.0), (12.0, 9.0, 6.0))
    else:
        s.add_sphere_light("L", (0.5, 4.0, -4.0), 0.8, (15.0, 15.0, 15.0))
    s.flatten()
    for w, h in ((48, 27), (13, 7)):
        s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 2.5, 3, 1), 60.0, w, h)
        img, ref, st, g = render_pixel(renderer, s, w, h, 70, integrator="direct")
        compare(img, ref)
        counters_equal(g, st)
        # the lists are built for pure sphere scenes (SCN_SPHERE): a quad or triangle light
        # adds a mesh object, and those scenes trace their shadow rays through the scene walk
        # instead (the counters show which path ran)
        if light == "sphere" and (w, h) == (48, 27):
            assert g.pix_shadow_list > 0 and g.pix_frustum > 0
        if light != "sphere":
            assert g.pix_shadow_list == 0 and g.pix_frustum == 0


def covered_block(w, h):
    """A big sphere filling the whole view (every camera ray of every pixel hits it), a
    sphere light beside the camera and 20 small occluders between them, outside the view (so
    the scene has its sphere BVH and every pixel's frustum list is the big sphere alone): every
    window of every pixel is all surface hits, so after each pixel's first window the chain runs
    in stride-4 windows (pixel.hip), with one-sphere frustum lists and shadow-occluder lists."""
    s = scenes.SceneBundle()
    s.add_sphere("big", (0.0, 0.0, -12.0), 6.0, (0.6, 0.5, 0.4))
    for k in range(20):
        s.add_sphere(f"occ{k:02d}", (2.0 + 0.3 * k, 3.0 + 0.15 * k, -4.0 - 0.25 * k), 0.3, (0.5, 0.5, 0.5))
    s.add_sphere_light("SphereLight", (6.0, 6.0, -2.0), 1.0, (25.0, 25.0, 25.0))
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1), 20.0, w, h)
    s.integrator, s.max_depth = "direct", 1
    return s


def test_stride4_windows_on_a_covered_block(renderer):
    """Stride-4 windows forced: 512 spp on pixels whose every sample hits a surface.  Per
    pixel: one stride-2 window (32 samples), then 7 stride-4 windows of 64 samples each while
    at least 64 samples remain, then the last 32 at stride 2.  Bit-exact, counters equal."""
    w, h = 16, 12
    s = covered_block(w, h)
    img, ref, st, g = render_pixel(renderer, s, w, h, 512)
    compare(img, ref)
    counters_equal(g, st)
    assert st["draws"] == w * h * 512 * 4   # every sample: 2 jitter + 2 light words
    assert g.pix_stride4 == 7 * w * h and g.pix_windows == 9 * w * h
    assert g.pix_frustum == w * h and g.pix_shadow_list == w * h and g.pix_flushes > 0
    assert st["shadow_rays"] > 0 and img.mean() > 0


def test_shards_and_step_schedule_agree(renderer):
    """Row shards of the pixel schedule reassemble the whole frame bit for bit, and the
    per-slot fused schedule (XRT_FLAG_NO_PIXEL) renders the same image."""
    s = scenes.spheres(40, 22)
    renderer.spp = 40
    renderer._uploaded = None
    full = renderer.render(s, 40, 22)
    assert renderer.stats.schedule == abi.XRT_SCHED_PIXEL
    acc = np.zeros_like(full)
    for k in range(3):
        part = renderer.render(s, 40, 22, shard_index=k, shard_count=3)
        assert renderer.stats.schedule == abi.XRT_SCHED_PIXEL
        rows = np.arange(22) % 3 != k
        assert np.all(part[rows] == 0)
        acc += part
    assert np.array_equal(acc, full)
    step = renderer.render(s, 40, 22, schedule="step")
    assert renderer.stats.schedule == abi.XRT_SCHED_STEP
    assert np.array_equal(step, full)


def render_c3(r, spp, **kw):
    import torch

    c = scenes.CONFIGS["C3"]
    w, h = c["width"], c["height"]
    scene = scenes.build("C3")
    r.spp = spp
    r.upload(scene)
    fb = torch.full((h, w, 3), 7.0, dtype=torch.float32, device="cuda:0")
    r.render_device(scene, w, h, fb.data_ptr(), after_stream=torch.cuda.current_stream().cuda_stream,
                    timing=True, schedule="auto", **kw)
    return scene, fb.cpu().numpy(), r.stats


def test_c3_headline_geometry(renderer):
    """C3 at its own 1280x720 through the bench's entry point (auto schedule, device output):
    the pixel schedule, 96 spp (2-3 windows per pixel), rows y % 64 == 21 bit-exact (the
    oracle's linear scan over 1,001 spheres is slow)."""
    scene, img, g = render_c3(renderer, 96)
    assert g.schedule == abi.XRT_SCHED_PIXEL and g.launches[abi.XRT_K_STEP] == 1
    assert g.samples == 1280 * 720 * 96 and g.segments == 1280 * 720 * 96
    k, n = 21, 64
    ref, st = pyoracle.render(scene, 1280, 720, 96, shard_index=k, shard_count=n)
    compare(img[k::n], ref[k::n])


def test_c3_fast_paths_in_compared_rows(renderer):
    """C3 at 1280x720, 96 spp, rendered as the row shard y % 64 == 29 (rows 29 ... 669, most
    of them >= 405, where the sphere field fills the pixels), so the counters describe exactly
    the compared rows: frustum lists, shadow-occluder lists, deferred flushes and stride-4
    windows all ran there, and the rows are bit-exact."""
    scene, img, g = render_c3(renderer, 96, shard_index=29, shard_count=64)
    assert g.schedule == abi.XRT_SCHED_PIXEL
    npx = 11 * 1280
    assert g.samples == npx * 96
    assert g.pix_frustum > 0 and g.pix_shadow_list > 0 and g.pix_flushes > 0 and g.pix_stride4 > 0
    assert g.pix_frustum + g.pix_frustum_overflow == npx
    ref, st = pyoracle.render(scene, 1280, 720, 96, shard_index=29, shard_count=64)
    compare(img[29::64], ref[29::64])
    assert (g.shadow_rays, g.draws) == (st["shadow_rays"], st["draws"])


def test_c3_row_shard(renderer):
    """C3 as rank 3 of 8 renders it (rows y % 8 == 3), 24 spp: zeros elsewhere, rows
    y % 64 == 3 bit-exact."""
    scene, img, g = render_c3(renderer, 24, shard_index=3, shard_count=8)
    assert g.schedule == abi.XRT_SCHED_PIXEL
    assert g.samples == 90 * 1280 * 24
    owned = np.zeros(720, bool)
    owned[3::8] = True
    assert np.all(img[~owned] == 0)
    ref, _ = pyoracle.render(scene, 1280, 720, 24, shard_index=3, shard_count=64)
    compare(img[3::64], ref[3::64])
