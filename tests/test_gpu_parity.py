"""GPU parity: libxrt_hip.so (through the C ABI) against the oracle and the reference's
golden vectors.  Bar: bit-exact pixels (the device path restates every float op of the
reference, incl. glibc sinf/cosf); RMSE < 1e-3 per channel is the north-star tolerance and
is asserted as a backstop on every image.
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from xraytracer_amd import abi, scenes
from xraytracer_amd.renderer import HipRenderer

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-3  # BASELINE.json north_star: per-channel RMSE < 1e-3 at matched seeds


def compare(img, ref, min_exact=1.0):
    assert img.shape == ref.shape
    assert np.all(np.isfinite(img))
    exact = float(np.mean(np.all(img == ref, axis=-1)))
    rmse = np.sqrt(np.mean((img.astype(np.float64) - ref.astype(np.float64)) ** 2, axis=(0, 1)))
    assert np.all(rmse < RMSE_TOL), rmse
    assert exact >= min_exact, (exact, rmse, np.argwhere(~np.all(img == ref, axis=-1))[:5])
    return exact, rmse


@pytest.fixture(scope="module")
def renderer():
    r = HipRenderer(16, device=0)
    yield r
    r.close()


@pytest.fixture(params=["auto", "step_tri", "wavefront"])
def sched(request):
    """Every device schedule: "auto" runs the fused LDS-resident kernels for scenes that fit
    (every scene below except the C4 sphere mesh) — small triangle scenes with merged
    shadow + extension traces (k_step_merged), Direct / Normal as pixel-parallel sample
    chains (k_pixel); "step_tri" forces the per-slot kernels with per-ray-kind cooperative
    traces (k_step_tri) for triangle scenes and k_step for the others; "wavefront" forces
    k_shade + k_trace."""
    return request.param


EXPECT_TRI = {"auto": abi.XRT_SCHED_STEP_MERGED, "step_tri": abi.XRT_SCHED_STEP_TRI,
              "wavefront": abi.XRT_SCHED_WAVEFRONT}


GPU_ONLY = ("slots_per_wave", "visits_per_launch", "group", "deep", "timing")   # launch geometry, not semantics


def render_both(r, scene, w, h, spp, schedule="auto", **kw):
    r.spp = spp
    r._uploaded = None
    img = r.render(scene, w, h, schedule=schedule, **kw)
    ref, st = pyoracle.render(scene, w, h, spp, **{k: v for k, v in kw.items() if k not in GPU_ONLY})
    steps = r.stats.launches[abi.XRT_K_STEP]
    if schedule == "wavefront":
        assert steps == 0
    return img, ref, st


# ------------------------------------------------------------------ RNG / trig ----
def test_rng_matches_reference_streams(gpu, golden):
    seeds = np.asarray(golden["rng_seeds"], dtype=np.uint32)
    out = np.zeros(len(seeds) * 2000, np.float32)
    rc = abi.lib().xrt_test_rng(gpu, abi.u32ptr(seeds), len(seeds), 0, 2000, abi.fptr(out))
    assert rc == 0
    ref = np.asarray(golden["rng_draws_2000"], dtype=np.uint32)
    assert np.array_equal(out.view(np.uint32), ref)


def test_rng_deep_stream_and_many_slots(gpu, golden):
    out = np.zeros(100, np.float32)
    seeds = np.array([7], np.uint32)
    assert abi.lib().xrt_test_rng(gpu, abi.u32ptr(seeds), 1, 100000, 100, abi.fptr(out)) == 0
    assert np.array_equal(out.view(np.uint32), np.asarray(golden["rng_seed7_skip100000"], np.uint32))
    # 4096 streams at once, crossing several wave-cooperative refills in one launch
    seeds = np.arange(4096, dtype=np.uint32) * 7919
    out = np.zeros(4096 * 64, np.float32)
    assert abi.lib().xrt_test_rng(gpu, abi.u32ptr(seeds), 4096, 3000, 64, abi.fptr(out)) == 0
    out = out.reshape(4096, 64)
    for s in (0, 1, 63, 64, 1000, 4095):
        assert np.array_equal(out[s], pyoracle.draws(int(seeds[s]), 64, skip=3000)), s


def test_trig_restatement_matches_host_libm_on_every_sampled_phi(gpu):
    """Every phi = 2*PI*r for all 83,886,080 reachable draw values r (Lambert, HG and
    SphereLight all use this domain): device glibc_sinf/cosf == host libm, bit for bit."""
    lib = abi.lib()
    one = np.float32(1.0).view(np.uint32)
    chunk = 1 << 24
    total, bad = 0, 0
    for first in range(0, int(one), chunk):
        cnt = min(chunk, int(one) - first)
        s = np.empty(cnt, np.float32)
        c = np.empty(cnt, np.float32)
        r = np.empty(cnt, np.float32)
        assert lib.xrt_test_trig_draw_domain(gpu, first, cnt, abi.fptr(s), abi.fptr(c), abi.fptr(r)) == 0
        keep = ~np.isnan(r)
        phi = np.float32(2.0 * np.float32(3.14159265359)) * r[keep]
        hs, hc = pyoracle.libm_sincosf(phi)
        bad += int(np.sum(hs.view(np.uint32) != s[keep].view(np.uint32)))
        bad += int(np.sum(hc.view(np.uint32) != c[keep].view(np.uint32)))
        total += int(keep.sum())
    assert total == 83886080
    assert bad == 0


def test_trig_general_arguments(gpu):
    x = np.concatenate([np.linspace(-100, 100, 20001, dtype=np.float32),
                        np.array([0.0, -0.0, 1e-30, 0.7853981, 0.7853982, 1e-4], np.float32)])
    out = np.zeros(2 * len(x), np.float32)
    assert abi.lib().xrt_test_trig(gpu, abi.fptr(x), len(x), abi.fptr(out)) == 0
    hs, hc = pyoracle.libm_sincosf(x)
    assert np.array_equal(out[0::2].view(np.uint32), hs.view(np.uint32))
    assert np.array_equal(out[1::2].view(np.uint32), hc.view(np.uint32))


def test_logf_restatement_on_vpt_domain(gpu):
    """-log(max(1 - u, 0)) over every reachable draw u (VolumePathTracing free flights)."""
    one = int(np.float32(1.0).view(np.uint32))
    bits = np.arange(0, one, dtype=np.uint32)
    r = bits.view(np.float32)
    r = r[(r.astype(np.float64) * 4294967296.0) == np.floor(r.astype(np.float64) * 4294967296.0)]
    x = np.maximum(np.float32(1.0) - r, np.float32(0.0)).astype(np.float32)
    assert len(x) == 83886080
    bad = 0
    for k in range(0, len(x), 1 << 24):
        xs = np.ascontiguousarray(x[k:k + (1 << 24)])
        out = np.zeros(2 * len(xs), np.float32)
        assert abi.lib().xrt_test_logexp(gpu, abi.fptr(xs), len(xs), abi.fptr(out)) == 0
        lg, _ = pyoracle.libm_logexpf(xs)
        bad += int(np.sum(out[0::2].view(np.uint32) != lg.view(np.uint32)))
    assert bad == 0


def test_expf_restatement_negative_range(gpu):
    """expf over every 7th negative float down to -104 plus edge values (exp(-sigma*t))."""
    lo = int(np.float32(-0.0).view(np.uint32))
    hi = int(np.float32(-104.0).view(np.uint32))
    bits = np.arange(lo, hi + 1, 7, dtype=np.uint64).astype(np.uint32)
    edge = [0.0, -0.0, -np.inf, 1.0, 88.0, -103.5, float.fromhex("-0x1.f8cbb2p+5")]   # last: FMA-variant case
    x = np.concatenate([bits.view(np.float32), np.array(edge, np.float32)])
    bad = 0
    for k in range(0, len(x), 1 << 24):
        xs = np.ascontiguousarray(x[k:k + (1 << 24)])
        out = np.zeros(2 * len(xs), np.float32)
        assert abi.lib().xrt_test_logexp(gpu, abi.fptr(xs), len(xs), abi.fptr(out)) == 0
        _, ex = pyoracle.libm_logexpf(xs)
        bad += int(np.sum(out[1::2].view(np.uint32) != ex.view(np.uint32)))
    assert bad == 0


@pytest.mark.parametrize("mode,c", [(0, 0.0), (1, "bsdf_pdf"), (1, 3.0)])
def test_fast_division_is_ieee_on_every_float(gpu, mode, c):
    """The kernels' fast reciprocal (Moller-Trumbore 1/det, orthonormalBasis) and divisions
    by constants (Lambert pdf 1/(2*PI), Russian roulette /3) equal IEEE division on all 2^32
    inputs (device_math.h rcp_rn / div_const)."""
    if c == "bsdf_pdf":
        c = np.float32(1.0) / (np.float32(2.0) * np.float32(3.14159265359))   # Src/material.h pdf
    c = np.float32(c)
    rc = np.float32(1.0) / c if mode == 1 else np.float32(0.0)
    n = C.c_uint64(0)
    bad = np.zeros(16, np.uint32)
    assert abi.lib().xrt_test_fastdiv(gpu, mode, C.c_float(c), C.c_float(rc), C.byref(n), abi.u32ptr(bad)) == 0
    assert n.value == 0, [hex(int(b)) for b in bad if b != 0xFFFFFFFF]


@pytest.mark.parametrize("y", [1.0 / 1.2, 1.0 / 2.2, 0.5, 2.0, 3.0, -1.5])
def test_powf_restatement_matches_host_libm(gpu, y):
    """glibc powf restatement (device_math.h, Image::gammaCorrection's std::pow) against the
    host libm on every 131st positive float bit pattern (zero, subnormals, normals, inf,
    NaN) and on negative x for integer and non-integer y."""
    y = float(np.float32(y))
    pos = np.arange(0, 0x7fffffff, 131, dtype=np.uint32).view(np.float32)
    neg = -np.linspace(1e-3, 50.0, 20011, dtype=np.float32)
    x = np.concatenate([pos, neg, np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan], np.float32)])
    out = np.zeros_like(x)
    assert abi.lib().xrt_test_powf(gpu, abi.fptr(x), len(x), C.c_float(y), abi.fptr(out)) == 0
    ref = pyoracle.libm_powf(x, y)
    same = (out.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(out) & np.isnan(ref))
    assert same.all(), (y, x[~same][:8], out[~same][:8], ref[~same][:8])


def test_tonemap_matches_reference_output_stage(renderer):
    """Image::gammaCorrection + writePPM quantisation on the device (xrt_tonemap) equals the
    restatement of the reference's host code, on a rendered Cornell image and on edge
    values (0, subnormal, 1, large, inf, NaN) through the device-pointer path."""
    import torch

    s = scenes.cornell(64, 48)
    img, ref, _ = render_both(renderer, s, 64, 48, 4)
    compare(img, ref)
    for gamma in (1.2, 2.2):
        assert np.array_equal(renderer.tonemap(64, 48, gamma), pyoracle.tonemap(ref, gamma))
    edge = np.array([0.0, 1e-40, 1e-3, 0.5, 1.0, 1.0001, 7.5, 3e9, 1e30, np.inf, np.nan, 1e-7], np.float32)
    vals = np.resize(edge, 4 * 3 * 3).reshape(3, 4, 3).astype(np.float32)
    dev = torch.from_numpy(vals).to("cuda:0")
    got = renderer.tonemap(4, 3, 1.2, device_ptr=dev.data_ptr())
    assert np.array_equal(got, pyoracle.tonemap(vals, 1.2)), (got, pyoracle.tonemap(vals, 1.2))


# ------------------------------------------------------------------ images ----
def test_c1_cornell_gi_bit_exact(renderer, sched):
    """Config C1 (Cornell 256x256x16, GIIntegrator(3)) — full framebuffer vs oracle."""
    s = scenes.cornell(256, 256)
    img, ref, st = render_both(renderer, s, 256, 256, 16, schedule=sched)
    compare(img, ref)
    g = renderer.stats
    assert (g.launches[abi.XRT_K_STEP] > 0) == (sched != "wavefront")
    assert g.schedule == EXPECT_TRI[sched]
    assert (g.segments, g.shadow_rays, g.draws, g.rejected) == (st["segments"], st["shadow_rays"], st["draws"],
                                                                st["rejected"])


def test_cornell_gi_nonsquare_and_depths(renderer, sched):
    s = scenes.cornell(80, 60)
    for depth in (1, 2, 5):
        img, ref, st = render_both(renderer, s, 80, 60, 8, max_depth=depth, schedule=sched)
        compare(img, ref)
        assert renderer.stats.draws == st["draws"]


def test_cornell_direct(renderer, sched):
    s = scenes.cornell(96, 72)
    img, ref, _ = render_both(renderer, s, 96, 72, 8, integrator="direct", schedule=sched)
    compare(img, ref)


def test_deep_streams_wrap_the_ring(renderer, sched):
    """~2,000-2,500 draws per pixel: every slot's stream position passes the ring's end
    (1,248 words) more than once, so the vector RNG loads take their wrap-around branch
    (a window that straddles the end) in every schedule, across many refills."""
    s = scenes.cornell(16, 12)
    for spp, kw in ((400, {}), (640, {"integrator": "direct"})):
        img, ref, st = render_both(renderer, s, 16, 12, spp, schedule=sched, **kw)
        compare(img, ref)
        assert renderer.stats.draws == st["draws"]
        assert st["draws"] / (16 * 12) > 2 * 1248 - 624   # the stream starts at word 624


@pytest.mark.parametrize("wh", [(1, 1), (7, 3), (65, 33)])
def test_edge_sizes(renderer, wh, sched):
    w, h = wh
    s = scenes.cornell(w, h)
    img, ref, _ = render_both(renderer, s, w, h, 3, schedule=sched)
    compare(img, ref)


def test_spp_one_and_depth_zero(renderer, sched):
    s = scenes.cornell(40, 30)
    img, ref, _ = render_both(renderer, s, 40, 30, 1, schedule=sched)
    compare(img, ref)
    img, ref, _ = render_both(renderer, s, 40, 30, 4, max_depth=0, schedule=sched)
    assert np.all(img == 0) and np.all(ref == 0)


@pytest.mark.parametrize("visits", [1, 2, 3, 7])
def test_merged_segments_per_launch(renderer, visits):
    """The merged-trace kernel drains its shadow rays at every launch boundary and resumes
    paths across launches: any number of segments per launch gives the same image and
    counters (GI and Direct; one and two lights)."""
    s = scenes.cornell(24, 18)
    for kw in ({}, {"integrator": "direct"}, {"max_depth": 5}):
        img, ref, st = render_both(renderer, s, 24, 18, 6, visits_per_launch=visits, schedule="step", **kw)
        compare(img, ref)
        g = renderer.stats
        assert g.schedule == abi.XRT_SCHED_STEP_MERGED and g.visits_per_launch == visits
        assert (g.segments, g.shadow_rays, g.draws) == (st["segments"], st["shadow_rays"], st["draws"])


@pytest.mark.parametrize("spw,group", [(4, True), (16, True), (32, True), (64, True), (16, False), (32, False)])
def test_merged_slots_per_wave(renderer, spw, group):
    """The merged kernel's layouts for small pixel shards — 16 or 32 slots per wave, their
    traces shared by 4 or 2 lanes per slot (group trace) or spread over idle lanes
    (cooperative passes) — render the same image and counters as full waves."""
    s = scenes.cornell(40, 30)
    for kw in ({}, {"integrator": "direct"}):
        img, ref, st = render_both(renderer, s, 40, 30, 5, slots_per_wave=spw, group=group, schedule="step", **kw)
        compare(img, ref)
        g = renderer.stats
        assert g.schedule == abi.XRT_SCHED_STEP_MERGED
        assert (g.slots_per_wave, g.group_lanes) == (spw, 64 // spw if group and spw < 64 else 1)
        assert (g.segments, g.shadow_rays, g.draws) == (st["segments"], st["shadow_rays"], st["draws"])


def test_shards_reassemble_exactly(renderer):
    """Row-interleaved pixel shards (the multi-GPU split) sum to the 1-shard image bit-exactly."""
    s = scenes.cornell(48, 37)
    renderer.spp = 4
    renderer._uploaded = None
    full = renderer.render(s, 48, 37)
    acc = np.zeros_like(full)
    for k in range(3):
        part = renderer.render(s, 48, 37, shard_index=k, shard_count=3)
        rows = np.arange(37) % 3 != k
        assert np.all(part[rows] == 0)
        acc += part
    assert np.array_equal(acc, full)


def test_c3_spheres_direct(renderer, sched):
    """Config C3 scene (1000 spheres + sphere light, DirectIntegrator) at reduced size."""
    s = scenes.spheres(160, 90)
    img, ref, st = render_both(renderer, s, 160, 90, 4, schedule=sched)
    compare(img, ref)
    assert renderer.stats.schedule == {"wavefront": abi.XRT_SCHED_WAVEFRONT, "step_tri": abi.XRT_SCHED_STEP,
                                       "auto": abi.XRT_SCHED_PIXEL}[sched]
    assert renderer.stats.shadow_rays == st["shadow_rays"]


def dup_spheres(w, h):
    """Sphere scene with every sphere present twice (same centre and radius, different
    albedo): equal hit distances, so the sphere BVH must reproduce the reference's
    in-order tie break (the first object in iteration order wins)."""
    s = scenes.SceneBundle()
    for k in range(24):
        x, z = -3.0 + (k % 6) * 1.2, -2.0 - (k // 6) * 1.2
        s.add_sphere(f"a{k:02d}", (x, 0.0, z), 0.5, (0.9, 0.2, 0.2))
        s.add_sphere(f"b{k:02d}", (x, 0.0, z), 0.5, (0.2, 0.9, 0.2))
    s.add_sphere_light("SphereLight", (0.0, 6.0, -4.0), 1.5, (20.0, 20.0, 20.0))
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 3, 4, 1), 60.0, w, h)
    s.integrator, s.max_depth = "gi", 3
    return s


@pytest.mark.parametrize("integ", ["direct", "gi"])
def test_sphere_bvh_ties_and_gi(renderer, sched, integ):
    """Sphere BVH (fused schedule) vs the oracle's linear scan: duplicated spheres (ties
    broken by iteration order), GI bounces between spheres, Direct."""
    s = dup_spheres(64, 48)
    img, ref, st = render_both(renderer, s, 64, 48, 4, integrator=integ, schedule=sched)
    compare(img, ref)
    assert renderer.stats.segments == st["segments"]
    assert renderer.stats.shadow_rays == st["shadow_rays"]


@pytest.mark.parametrize("integ,depth", [("indirect", 3), ("indirect", 5), ("normal", 1)])
def test_indirect_and_normal_integrators(renderer, sched, integ, depth):
    """IndirectIntegrator (Src/integrator.h:122-190) and NormalIntegrator (:22-74) on the
    Cornell box (triangles) and the sphere scene, bit-exact against the oracle."""
    for s, w, h in ((scenes.cornell(64, 48), 64, 48), (dup_spheres(48, 36), 48, 36)):
        img, ref, st = render_both(renderer, s, w, h, 4, integrator=integ, max_depth=depth, schedule=sched)
        compare(img, ref)
        assert renderer.stats.segments == st["segments"]
        assert renderer.stats.draws == st["draws"]


def test_normal_integrator_on_medium_box(renderer, sched):
    """NormalIntegrator over the smoke scene: a BoxMesh hit leaves the shading normal at its
    default (0), so the pixel is 0.5 — as in the reference."""
    s = scenes.smoke(32, 24)
    img, ref, _ = render_both(renderer, s, 32, 24, 2, integrator="normal", schedule=sched)
    compare(img, ref)


@pytest.mark.parametrize("integ,schedule", [("indirect", "auto"), ("normal", "step"), ("gi", "step_tri")])
def test_kstep_refill_staging_beside_a_large_scene(renderer, integ, schedule):
    """k_step stages its in-line RNG refill through LDS right after the scene carve
    (kstep_refill_off).  A 520-triangle scene (Cornell + two 242-triangle sphere meshes, none
    large enough for the BVH) fills ~59 KB of the 64 KiB scene budget, so scene + staging
    exceed 64 KiB; the launch is sized for both.  Rings are twisted in-launch."""
    s = scenes.SceneBundle()
    s.load_obj(scenes.CORNELL_OBJ)
    s.add_quad_light("QuadLight", (343.0, 548.0, 227.0), (343.0, 548.0, 332.0), (213.0, 548.0, 227.0),
                     (25.0, 25.0, 25.0))
    s.add_sphere_mesh("mesh_a", (150.0, 420.0, 400.0), 90.0, 11, 11, (0.58, 0.58, 0.58))
    s.add_sphere_mesh("mesh_b", (400.0, 120.0, 300.0), 70.0, 11, 11, (0.3, 0.6, 0.5))
    s.flatten()
    s.camera = scenes.pinhole(scenes.CORNELL_C2W, 60.0, 40, 30)
    assert s.desc.n_tris == 36 + 2 * 242
    spp = 160 if integ == "normal" else 64   # Normal draws 2 words per sample: 160 spp to run low
    img, ref, st = render_both(renderer, s, 40, 30, spp, integrator=integ, max_depth=3, schedule=schedule,
                               timing=True)
    compare(img, ref)
    g = renderer.stats
    assert g.schedule == abi.XRT_SCHED_STEP   # the layout leaves no room for k_step_tri's scratch
    assert (g.segments, g.shadow_rays, g.draws) == (st["segments"], st["shadow_rays"], st["draws"])
    assert g.launches[abi.XRT_K_REFILL] == 1 and g.rng_twists - g.path_slots > g.path_slots // 4


@pytest.mark.parametrize("deep", ["fused", "single", "quad"])
@pytest.mark.parametrize("nt,w,h,spp", [(24, 64, 36, 4), (80, 48, 30, 3), (380, 12, 9, 2)])
def test_c4_sphere_mesh_gi(renderer, nt, w, h, spp, deep):
    """Config C4 scene family (Cornell + tessellated sphere; 1,152, 12,800 and 288,800 mesh
    triangles) at reduced size, bit-exact against the oracle's linear scan, counters
    included: the fused two-level schedule (merged kernel + the wave's quad BVH walk) and
    the wavefront schedule with one or four lanes per deep ray.  The largest binary tree has
    more than 65,536 nodes, so the wavefront traversal stack takes 32-bit entries."""
    s = scenes.cornell_spheremesh(w, h, n_theta=nt, n_phi=nt)
    if deep == "fused":
        img, ref, st = render_both(renderer, s, w, h, spp, schedule="auto")
    else:
        img, ref, st = render_both(renderer, s, w, h, spp, deep=deep, schedule="wavefront")
    compare(img, ref)
    g = renderer.stats
    if deep == "fused":
        assert g.schedule == abi.XRT_SCHED_STEP_BVH and g.launches[abi.XRT_K_DEEP] == 0
    else:
        assert g.launches[abi.XRT_K_STEP] == 0   # multi-pass schedule
        assert g.schedule == abi.XRT_SCHED_WAVEFRONT
    assert (g.segments, g.shadow_rays, g.draws) == (st["segments"], st["shadow_rays"], st["draws"])


@pytest.mark.parametrize("integ", ["gi", "direct"])
@pytest.mark.parametrize("spw", [0, 16, 32, 64])
def test_two_level_fused_layouts_and_lights(renderer, integ, spw):
    """The fused two-level kernel (k_step_merged<..., BVH>) with two area lights (a quad and a
    triangle light: NL = 2), GI and Direct, at every slots-per-wave layout, and a few visits
    per launch so paths and their RNG windows cross launches: bit-exact with counters equal."""
    s = scenes.SceneBundle()
    s.load_obj(scenes.CORNELL_OBJ)
    s.add_quad_light("QuadLight", (343.0, 548.0, 227.0), (343.0, 548.0, 332.0), (213.0, 548.0, 227.0),
                     (25.0, 25.0, 25.0))
    s.add_triangle_light("TriLight", (100.0, 500.0, 100.0), (150.0, 500.0, 100.0), (100.0, 500.0, 150.0),
                         (10.0, 5.0, 2.0))
    s.add_sphere_mesh("sphere_mesh", (150.0, 420.0, 400.0), 90.0, 60, 60, (0.58, 0.58, 0.58))
    s.flatten()
    s.camera = scenes.pinhole(scenes.CORNELL_C2W, 60.0, 72, 40)
    img, ref, st = render_both(renderer, s, 72, 40, 5, integrator=integ, schedule="auto", slots_per_wave=spw,
                               visits_per_launch=3)
    compare(img, ref)
    g = renderer.stats
    assert g.schedule == abi.XRT_SCHED_STEP_BVH and g.launches[abi.XRT_K_STEP] > 2
    if spw:
        assert g.layout_launches[abi.LAYOUTS.index(spw)] == g.launches[abi.XRT_K_STEP]
    assert (g.segments, g.shadow_rays, g.draws) == (st["segments"], st["shadow_rays"], st["draws"])


def test_triangle_light_and_two_lights(renderer, sched):
    s = scenes.SceneBundle()
    s.load_obj(scenes.CORNELL_OBJ)
    s.add_quad_light("QuadLight", (343.0, 548.0, 227.0), (343.0, 548.0, 332.0), (213.0, 548.0, 227.0),
                     (25.0, 25.0, 25.0))
    s.add_triangle_light("TriLight", (100.0, 500.0, 100.0), (150.0, 500.0, 100.0), (100.0, 500.0, 150.0),
                         (10.0, 5.0, 2.0))
    s.flatten()
    s.camera = scenes.pinhole(scenes.CORNELL_C2W, 60.0, 64, 48)
    img, ref, _ = render_both(renderer, s, 64, 48, 4, schedule=sched)
    compare(img, ref)
    img, ref, _ = render_both(renderer, s, 64, 48, 4, integrator="direct", schedule=sched)
    compare(img, ref)


def test_c5_smoke_vpt(renderer, sched):
    """Config C5 family (synthetic density grid in a BoxMesh + quad light,
    VolumePathTracing(10)) at reduced grid and image size."""
    s = scenes.smoke(48, 36, n=32)
    img, ref, st = render_both(renderer, s, 48, 36, 4, schedule=sched)
    compare(img, ref)
    g = renderer.stats
    assert g.draws == st["draws"] and g.segments == st["segments"] and g.stalled == st["stalled"] == 0


def test_grid_signed_zeros_and_denormals(renderer, sched):
    """A density grid with +0 and -0 zeros mixed, a block of -0 only and a lone denormal:
    the device's interpolation (float index path for origin 0 / power-of-two voxels, double
    otherwise) renders as the oracle reads it."""
    s = scenes.smoke(40, 30, n=32)
    g = s.medium.density
    z = g == 0.0
    g[z & (np.indices(g.shape).sum(axis=0) % 3 == 0)] = -0.0
    g[:8, :8, :8] = -0.0
    g[20:28, 0:8, 0:8] = 0.0
    g[23, 5, 6] = np.float32(1e-40)
    img, ref, st = render_both(renderer, s, 40, 30, 4, schedule=sched)
    compare(img, ref)
    assert renderer.stats.draws == st["draws"]


def test_vpt_medium_walk_suspends_and_resumes(renderer, sched):
    """Many spp per pixel forces delta-tracking walks to cross RNG refills (suspend/resume)."""
    s = scenes.smoke(12, 9, n=32)
    img, ref, st = render_both(renderer, s, 12, 9, 96, schedule=sched)
    compare(img, ref)
    assert renderer.stats.draws == st["draws"]


@pytest.mark.parametrize("visits", [1, 3, 128])
@pytest.mark.parametrize("integ", ["vpt", "vpt_nee"])
def test_vpt_events_resume_across_launches(renderer, visits, integ):
    """The fused VPT kernel runs one event (a trace or ONE collision) per iteration and a walk
    carries over in registers; with 1-3 events per launch almost every walk is saved at a
    launch end and resumed by the next launch.  Bit-exact, same draws and segments."""
    s = dense_smoke(20, 15) if integ == "vpt_nee" else scenes.smoke(20, 15, n=32)
    img, ref, st = render_both(renderer, s, 20, 15, 6, integrator=integ, visits_per_launch=visits)
    compare(img, ref)
    g = renderer.stats
    assert g.visits_per_launch == visits
    assert g.draws == st["draws"] and g.segments == st["segments"]


def dense_smoke(w, h, n=24, g=0.4):
    """Smoke scene with a denser, anisotropic medium: more scattering events, more NEE ratio
    tracking steps per light sample, HenyeyGreenstein with g != 0."""
    s = scenes.SceneBundle()
    med = scenes.Medium(scenes.smoke_grid(n, seed=3), (0.0, 0.0, 0.0), 1.0, g, (0.05, 0.02, 0.01), (0.4, 0.5, 0.6),
                        multiplier=1.5)
    c = (n - 1) / 2.0
    s.add_quad_light("QuadLight", (c + 10, n + 15.0, c + 10), (c - 10, n + 15.0, c + 10), (c + 10, n + 15.0, c - 10),
                     (20.0, 20.0, 20.0))
    s.add_medium("medium", med)
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, c, c, c + 2.2 * n, 1), 45.0, w, h)
    s.integrator, s.max_depth = "vpt_nee", 10
    return s


def homog_scene(kind, w, h, g=0.3):
    """A homogeneous medium box (HomogeneousMedium{MIS,Achromatic,NoMIS}, Src/medium.h:
    122-277) under a quad light."""
    s = scenes.SceneBundle()
    a = (0.02, 0.02, 0.02) if kind == "achromatic" else (0.02, 0.03, 0.01)
    sc = (0.08, 0.08, 0.08) if kind == "achromatic" else (0.06, 0.09, 0.12)
    s.add_quad_light("QuadLight", (18.0, 25.0, 18.0), (2.0, 25.0, 18.0), (18.0, 25.0, 2.0), (20.0, 20.0, 20.0))
    s.add_medium("medium", scenes.HomogeneousMedium(kind, g, a, sc, (0.0, 0.0, 0.0), (20.0, 12.0, 20.0)))
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 10, 6, 55, 1), 45.0, w, h)
    s.integrator, s.max_depth = "vpt", 10
    return s


@pytest.mark.parametrize("kind", ["mis", "achromatic", "nomis"])
@pytest.mark.parametrize("integ", ["vpt", "vpt_nee"])
def test_homogeneous_media(renderer, sched, kind, integ):
    """Homogeneous media under VolumePathTracing and VolumePathTracingNEE (analytic
    transmittance on the NEE shadow ray), bit-exact against the oracle."""
    s = homog_scene(kind, 40, 30)
    img, ref, st = render_both(renderer, s, 40, 30, 4, integrator=integ, schedule=sched)
    compare(img, ref)
    g = renderer.stats
    assert g.draws == st["draws"] and g.segments == st["segments"] and g.shadow_rays == st["shadow_rays"]


@pytest.mark.parametrize("dense", [False, True])
def test_vpt_nee(renderer, sched, dense):
    """VolumePathTracingNEE (Src/integrator.h:481-636): light sample at every scattering
    event, shadow ray's closest hit, ratio-tracking transmittance through the medium."""
    s = dense_smoke(40, 30) if dense else scenes.smoke(40, 30, n=32)
    img, ref, st = render_both(renderer, s, 40, 30, 4, integrator="vpt_nee", schedule=sched)
    compare(img, ref)
    g = renderer.stats
    assert g.draws == st["draws"] and g.segments == st["segments"] and g.shadow_rays == st["shadow_rays"]
    assert st["shadow_rays"] > 0


def test_vpt_nee_ratio_tracking_suspends_and_resumes(renderer, sched):
    """Many spp on a few pixels of the dense medium: NEE ratio tracking (and delta tracking)
    runs out of RNG words mid-walk and resumes after the refill."""
    s = dense_smoke(8, 6)
    img, ref, st = render_both(renderer, s, 8, 6, 160, integrator="vpt_nee", schedule=sched)
    compare(img, ref)
    assert renderer.stats.draws == st["draws"]


@pytest.mark.parametrize("kind", ["gi", "direct"])
def test_cpp_api_example_matches_oracle(tmp_path, kind):
    """examples/cornellbox.cpp — the reference example written against include/xrt/*.h with
    HipRenderer — renders the same image as the oracle, bit for bit."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "examples", "bin", "cornellbox")
    out = tmp_path / "fb.raw"
    env = dict(os.environ, XRT_DATA_DIR=os.path.join(root, "xraytracer_amd", "data") + "/")
    subprocess.check_call([exe, "64", "48", "4", kind, str(out)], env=env)
    img = np.fromfile(out, dtype=np.float32).reshape(48, 64, 3)
    s = scenes.cornell(64, 48)
    ref, _ = pyoracle.render(s, 64, 48, 4, integrator=kind)
    compare(img, ref)
