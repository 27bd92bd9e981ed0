"""Speculative sample starts (k_step_spec, xraytracer_amd/csrc/spec.hip) against the oracle.

In the merged schedule's group layouts (16 slots of 4 lanes; the 4-slot tail, 16 lanes; 8
slots of 8 lanes when forced) every GIIntegrator sample (Src/integrator.h:205-287)
is started beside its predecessor's last trace: the slot's other lanes trace the camera rays of
the three stream offsets where the successor can start, and the lane whose offset the trace
confirms shades the successor's first hit in the same visit.  Bar: framebuffers bit for bit
and every counter (Scene::intersect calls, shadow rays, draws, rejects) equal to the
reference's sequential NormalRenderer::doRender (Src/renderer.cpp:29-81) as restated by the
oracle.  The variant is the default (XRT_FLAG_NO_SPEC turns it off: same image, no speculative
launch).  Cases force it on every launch (slots_per_wave=16, 8 or 4) and let the library mix
it with the other layouts; cover launch boundaries (1-3 visits per launch: samples and
pending shadow rays cross launches), depths 2-5, rejects with the in-place accumulate
contract, the camera lists' covered / multi-triangle / empty pixels, and C2's own geometry
as one row shard of an 8-GPU frame.
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


def render_spec(r, scene, w, h, spp, force=True, spw=16, **kw):
    r.spp = spp
    r._uploaded = None
    img = r.render(scene, w, h, timing=True, slots_per_wave=spw if force else 0, **kw)
    g = r.stats
    okw = {k: v for k, v in kw.items() if k in ("integrator", "max_depth", "shard_index", "shard_count", "initial")}
    ref, st = pyoracle.render(scene, w, h, spp, **okw)
    assert g.schedule == abi.XRT_SCHED_STEP_MERGED
    assert (g.segments, g.shadow_rays, g.draws, g.rejected) == \
        (st["segments"], st["shadow_rays"], st["draws"], st["rejected"])
    return img, ref, st, g


@pytest.mark.parametrize("spp", [1, 2, 7, 33])
def test_cornell_every_launch_speculative(renderer, spp):
    s = scenes.cornell(64, 48)
    img, ref, st, g = render_spec(renderer, s, 64, 48, spp)
    compare(img, ref)
    assert g.spec_launches == g.launches[abi.XRT_K_STEP] > 0


@pytest.mark.parametrize("spw", [8, 4])
def test_wider_groups(renderer, spw):
    """8 and 16 lanes per slot (k_step_spec<8, 8>, <4, 16>: the quad and replicas of it that
    widen the group trace), across launch boundaries."""
    s = scenes.cornell(40, 30)
    img, ref, st, g = render_spec(renderer, s, 40, 30, 11, spw=spw, visits_per_launch=3)
    compare(img, ref)
    assert g.spec_launches == g.launches[abi.XRT_K_STEP] > 5


@pytest.mark.parametrize("visits", [1, 2, 3, 7])
def test_samples_and_shadow_rays_cross_launches(renderer, visits):
    """1-7 visits per launch: most launches end with a sample in progress, an ended sample
    whose shadow ray is in flight, or a successor started and ended at its camera ray — all
    drained or saved at the launch end and resumed by the next launch."""
    s = scenes.cornell(40, 30)
    img, ref, st, g = render_spec(renderer, s, 40, 30, 9, visits_per_launch=visits)
    compare(img, ref)
    assert g.visits_per_launch == visits and g.spec_launches > 5


@pytest.mark.parametrize("depth", [2, 3, 5])
def test_depths(renderer, depth):
    s = scenes.cornell(48, 36)
    img, ref, st, g = render_spec(renderer, s, 48, 36, 12, max_depth=depth)
    compare(img, ref)


def test_mixed_layouts_frame(renderer):
    """The library's own layout choice for a 120k-pixel frame at 4 visits per launch: 32 slots
    per wave while more than 90k slots live, then the speculative 16-slot launches and, below
    20k, the speculative 4-slot ones — slots move between the kernels mid-sample."""
    s = scenes.cornell(400, 300)
    img, ref, st, g = render_spec(renderer, s, 400, 300, 24, force=False, visits_per_launch=4)
    compare(img, ref)
    ll = g.layout_launches
    assert g.spec_launches == ll[2] + ll[4] and ll[2] > 0 and ll[4] > 0 and ll[0] + ll[1] > 0


def test_rejects_and_accumulate(renderer):
    """A light with negative green radiance (every sample that sees it is rejected) and
    samples added in place to a nonzero image (Src/renderer.cpp:57-75)."""
    s = scenes.SceneBundle()
    s.load_obj(scenes.CORNELL_OBJ)
    s.add_quad_light("QuadLight", (343.0, 548.0, 227.0), (343.0, 548.0, 332.0), (213.0, 548.0, 227.0),
                     (25.0, -1.0, 25.0))
    s.flatten()
    s.camera = scenes.pinhole(scenes.CORNELL_C2W, 60.0, 40, 30)
    s.integrator, s.max_depth = "gi", 3
    init = np.random.default_rng(5).uniform(0.0, 2.0, (30, 40, 3)).astype(np.float32)
    img, ref, st, g = render_spec(renderer, s, 40, 30, 20, initial=init)
    compare(img, ref)
    assert st["rejected"] > 100


def test_c2_row_shard(renderer):
    """C2's own geometry (800x600, the Cornell box, GI(3)) as rank 3 of an 8-GPU frame, 64 spp,
    speculative starts on every launch: every owned row bit-exact, zeros elsewhere."""
    import torch
    c = scenes.CONFIGS["C2"]
    w, h = c["width"], c["height"]
    scene = scenes.build("C2")
    renderer.spp = 64
    renderer.upload(scene)
    fb = torch.full((h, w, 3), 7.0, dtype=torch.float32, device="cuda:0")
    renderer.render_device(scene, w, h, fb.data_ptr(), shard_index=3, shard_count=8, slots_per_wave=16,
                           timing=True)
    g = renderer.stats
    assert g.spec_launches == g.launches[abi.XRT_K_STEP] > 0
    img = fb.cpu().numpy()
    owned = np.zeros(h, bool)
    owned[3::8] = True
    assert np.all(img[~owned] == 0)
    ref, st = pyoracle.render(scene, w, h, 64, shard_index=3, shard_count=8)
    compare(img[owned], ref[owned])
    assert (g.segments, g.shadow_rays, g.draws) == (st["segments"], st["shadow_rays"], st["draws"])


def test_no_spec_flag_same_image(renderer):
    """XRT_FLAG_NO_SPEC keeps the 16-slot launches on k_step_merged: the same image and counters."""
    s = scenes.cornell(48, 36)
    renderer.spp = 16
    renderer._uploaded = None
    a = renderer.render(s, 48, 36, slots_per_wave=16)
    ga = renderer.stats
    b = renderer.render(s, 48, 36, slots_per_wave=16, spec=False)
    gb = renderer.stats
    assert ga.spec_launches > 0 and gb.spec_launches == 0
    assert np.array_equal(a, b) and (ga.segments, ga.draws) == (gb.segments, gb.draws)
