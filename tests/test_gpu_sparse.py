"""Sparse (NanoVDB-layout) density: the C5 smoke grid cut into 8^3 leaf bricks with the
empty leaves dropped (xrt_set_medium_bricks), rendered under every schedule
and compared bit for bit with the oracle on the dense grid it was cut from — OpenVDB's
BoxSampler reads inactive voxels as background 0, so the two are the same density field.
"""
import dataclasses

import numpy as np
import pytest

import pyoracle
from xraytracer_amd import scenes
from xraytracer_amd.renderer import HipRenderer

pytestmark = pytest.mark.gpu


def sparse_smoke(w, h, n):
    s = scenes.smoke(w, h, n=n)
    s.medium = dataclasses.replace(s.medium, sparse=True)
    return s


def test_brick_cut_drops_empty_leaves():
    s = sparse_smoke(8, 6, 128)
    table, bricks = s.medium.bricks()
    assert table.shape == (16, 16, 16)
    assert 0 < len(bricks) < table.size            # empty leaves carry no storage
    # every voxel reads back through the table
    g = s.medium.density
    z, y, x = 37, 64, 90
    b = table[z // 8, y // 8, x // 8]
    assert b >= 0 and bricks[b, z % 8, y % 8, x % 8] == g[z, y, x]


@pytest.mark.parametrize("schedule", ["auto", "wavefront"])
@pytest.mark.parametrize("integ", ["vpt", "vpt_nee"])
def test_sparse_grid_renders_like_dense(schedule, integ):
    w, h, spp = 80, 60, 4
    s = sparse_smoke(w, h, 128)
    r = HipRenderer(spp, device=0)
    img = r.render(s, w, h, integrator=integ, schedule=schedule)
    ref, st = pyoracle.render(s, w, h, spp, integrator=integ)
    assert np.array_equal(img, ref), np.argwhere(~np.all(img == ref, axis=-1))[:5]
    assert r.stats.draws == st["draws"] and r.stats.segments == st["segments"]
    r.close()


def test_sparse_grid_with_odd_dims_and_multiplier():
    """A grid whose sides are not multiples of 8 (partial leaves at the far faces) and a
    density multiplier; delta tracking crosses leaf boundaries everywhere."""
    rng = np.random.default_rng(9)
    g = scenes.smoke_grid(40, seed=5)[:37, :29, :33].copy()
    g[:, :, :9] = 0.0
    med = scenes.Medium(g, (-3.0, 1.0, 2.0), 1.5, 0.3, (0.05, 0.03, 0.02), (0.3, 0.4, 0.5), multiplier=2.0,
                        sparse=True)
    s = scenes.SceneBundle()
    s.add_quad_light("QuadLight", (40.0, 70.0, 40.0), (-10.0, 70.0, 40.0), (40.0, 70.0, -10.0), (20.0, 20.0, 20.0))
    s.add_medium("medium", med)
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 22, 22, 120, 1), 45.0, 48, 36)
    s.integrator, s.max_depth = "vpt_nee", 10
    r = HipRenderer(4, device=0)
    img = r.render(s, 48, 36)
    ref, st = pyoracle.render(s, 48, 36, 4)
    assert np.array_equal(img, ref)
    assert st["shadow_rays"] > 0
    r.close()
