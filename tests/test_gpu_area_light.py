"""SphereLight built with AREA_SAMPLING (Src/light.h:131-135,185-191; UniformSampleSphere,
Src/light.cpp:99-105) on the GPU against the oracle.

The reference compiles SphereLight::sample's uniform-point-on-the-sphere branch when
AREA_SAMPLING is defined (its build leaves it off, Src/cmakelists.txt:63); here it is a light
kind of its own (XRT_LIGHT_SPHERE_AREA, SphereLight::Sampling::Area).  The oracle's restatement
is pinned by the reference-compiled KAT `sphere_area_*` (tests/test_oracle_kats.py).  Bar:
framebuffers bit for bit and the path counters equal, under every schedule that samples
lights: pixel-parallel chains (k_pixel, with the camera-frustum and shadow-occluder lists of a
sphere field), the per-slot fused kernel (k_step) and the wavefront (k_shade + k_trace), for
DirectIntegrator, GIIntegrator and VolumePathTracingNEE.
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


@pytest.fixture(scope="module")
def renderer():
    r = HipRenderer(1, device=0)
    yield r
    r.close()


def render_both(r, scene, w, h, spp, **kw):
    r.spp = spp
    r._uploaded = None
    img = r.render(scene, w, h, **kw)
    okw = {k: v for k, v in kw.items() if k in ("integrator", "max_depth", "shard_index", "shard_count")}
    ref, st = pyoracle.render(scene, w, h, spp, **okw)
    g = r.stats
    assert (g.segments, g.shadow_rays, g.draws, g.rejected) == \
        (st["segments"], st["shadow_rays"], st["draws"], st["rejected"])
    return img, ref, st


def sphere_field(w, h, area=True):
    """A 12 x 8 field of Lambert spheres under one sphere light (C3's layout, smaller): the
    pixel schedule builds camera-frustum lists and, with one light, shadow-occluder lists."""
    s = scenes.SceneBundle()
    k = 0
    for iz in range(8):
        for ix in range(12):
            s.add_sphere(f"sphere_{k:03d}", (-5.5 + ix, 0.0, -2.0 - iz), 0.4, (0.58, 0.58, 0.58))
            k += 1
    s.add_sphere_light("SphereLight", (0.0, 6.0, -6.0), 1.5, (30.0, 30.0, 30.0), area=area)
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 3, 5, 1), 60.0, w, h)
    s.integrator, s.max_depth = "direct", 1
    return s


@pytest.mark.parametrize("schedule,expect", [("auto", abi.XRT_SCHED_PIXEL), ("step", abi.XRT_SCHED_STEP),
                                             ("wavefront", abi.XRT_SCHED_WAVEFRONT)])
def test_direct_area_sphere_light(renderer, schedule, expect):
    s = sphere_field(96, 64)
    img, ref, st = render_both(renderer, s, 96, 64, 24, schedule=schedule)
    compare(img, ref)
    assert renderer.stats.schedule == expect
    assert st["shadow_rays"] > 0
    # the two samplings draw the same words but place the light samples differently
    cone, _ = pyoracle.render(sphere_field(96, 64, area=False), 96, 64, 24)
    assert not np.array_equal(cone, ref)


@pytest.mark.parametrize("schedule,expect", [("auto", abi.XRT_SCHED_STEP), ("wavefront", abi.XRT_SCHED_WAVEFRONT)])
def test_gi_area_sphere_light(renderer, schedule, expect):
    s = sphere_field(64, 48)
    img, ref, st = render_both(renderer, s, 64, 48, 8, integrator="gi", max_depth=3, schedule=schedule)
    compare(img, ref)
    assert renderer.stats.schedule == expect
    assert st["segments"] > 64 * 48 * 8


def cornell_area_sphere_light(w, h):
    """Triangles and an analytic light sphere: the Cornell box lit by an area-sampled
    SphereLight under its ceiling (a mixed scene)."""
    s = scenes.SceneBundle()
    s.load_obj(scenes.CORNELL_OBJ)
    s.add_sphere_light("SphereLight", (278.0, 480.0, 280.0), 40.0, (12.0, 12.0, 12.0), area=True)
    s.flatten()
    s.camera = scenes.pinhole(scenes.CORNELL_C2W, 60.0, w, h)
    s.integrator, s.max_depth = "gi", 3
    return s


@pytest.mark.parametrize("schedule", ["auto", "wavefront"])
def test_cornell_gi_area_sphere_light(renderer, schedule):
    s = cornell_area_sphere_light(48, 36)
    img, ref, st = render_both(renderer, s, 48, 36, 8, schedule=schedule)
    compare(img, ref)


def test_vpt_nee_area_sphere_light(renderer):
    """VolumePathTracingNEE (Src/integrator.h:481-636): light samples from inside and outside
    the medium through ratio tracking, towards an area-sampled sphere light."""
    n = 24
    s = scenes.SceneBundle()
    med = scenes.Medium(scenes.smoke_grid(n, seed=3), (0.0, 0.0, 0.0), 1.0, 0.4, (0.05, 0.02, 0.01),
                        (0.4, 0.5, 0.6), multiplier=1.5)
    c = (n - 1) / 2.0
    s.add_sphere_light("SphereLight", (c, n + 12.0, c), 6.0, (20.0, 20.0, 20.0), area=True)
    s.add_medium("medium", med)
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, c, c, c + 2.2 * n, 1), 45.0, 24, 18)
    s.integrator, s.max_depth = "vpt_nee", 10
    img, ref, st = render_both(renderer, s, 24, 18, 6)
    compare(img, ref)
    assert st["shadow_rays"] > 0
