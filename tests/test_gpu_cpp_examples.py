"""The reference's volumetric examples ported to the drop-in C++ API (examples/vpt.cpp ←
Src/examples/vpt.cpp:20-83, examples/nee.cpp ← Src/examples/nee.cpp:20-82), rendered by
HipRenderer through HipRenderer::render's medium branches (csrc/host/hip_renderer.cpp) and
compared bit for bit with the oracle on the same scene built through the Python layer.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import pyoracle
from xraytracer_amd import scenes

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(exe, args):
    return subprocess.run([os.path.join(ROOT, "examples", "bin", exe)] + [str(a) for a in args], check=True,
                          capture_output=True, text=True).stdout


def test_vpt_example_homogeneous_mis(tmp_path):
    """HomogeneousMediumMIS box + QuadLight, VolumePathTracing(10), camera at z = 5 with
    FOV = 2 * 180 * atanf(1/3) / PI."""
    w, h, spp = 64, 64, 8
    out = tmp_path / "vpt.raw"
    log = run("vpt", [w, h, spp, out])
    img = np.fromfile(out, dtype=np.float32).reshape(h, w, 3)
    fov = float.fromhex(re.search(r"FOV (\S+)", log).group(1))
    # GCC folds atanf(1.0f / 3.0f) at compile time: the correctly rounded value
    a = np.float32(np.arctan(np.float64(np.float32(1.0) / np.float32(3.0))))
    assert np.float32(fov) == np.float32(np.float32(np.float32(360.0) * a) / np.float32(3.14159265359))
    s = scenes.SceneBundle()
    s.add_medium("medium", scenes.HomogeneousMedium("mis", 0.0, (0.5, 0.5, 0.5), (0.5, 0.5, 0.5), (-1.0, -1.0, -1.0),
                                                    (1.0, 1.0, 1.0)))
    s.add_quad_light("QuadLight", (0.5, 1.4, 0.5), (-0.5, 1.4, 0.5), (0.5, 1.4, -0.5), (10.0, 10.0, 10.0))
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 5, 1), fov, w, h)
    s.integrator, s.max_depth = "vpt", 10
    ref, st = pyoracle.render(s, w, h, spp)
    assert st["segments"] > w * h * spp
    assert np.array_equal(img, ref), np.argwhere(~np.all(img == ref, axis=-1))[:5]


@pytest.mark.parametrize("layout", ["dense", "sparse"])
def test_nee_example_heterogeneous_dense_grid(tmp_path, layout):
    """HeterogeneousMedium over a DenseGrid + SphereLight(r 50, at y 400 through its
    lightToWorld), VolumePathTracingNEE(32), camera at (0, 70, 550), FOV 60: delta tracking,
    NEE ratio tracking, cone sampling of the sphere light."""
    w, h, spp = 48, 36, 4
    n, origin, voxel = 48, (-190.0, -190.0, -190.0), 8.0
    grid = scenes.smoke_grid(n, seed=11)
    gpath = tmp_path / "grid.raw"
    np.ascontiguousarray(grid, dtype=np.float32).tofile(gpath)
    out = tmp_path / "nee.raw"
    run("nee", [gpath, n, n, n, *origin, voxel, w, h, spp, out, layout])
    img = np.fromfile(out, dtype=np.float32).reshape(h, w, 3)
    s = scenes.SceneBundle()
    s.add_medium("medium", scenes.Medium(grid, origin, voxel, 0.0, (0.01, 0.01, 0.01), (0.05, 0.05, 0.05)))
    s.add_sphere_light("SphereLight", (0.0, 400.0, 0.0), 50.0, (30.0, 30.0, 30.0))
    s.flatten()
    s.camera = scenes.pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 70, 550, 1), 60.0, w, h)
    s.integrator, s.max_depth = "vpt_nee", 32
    ref, st = pyoracle.render(s, w, h, spp)
    assert st["shadow_rays"] > 0 and st["segments"] > 0
    assert np.array_equal(img, ref), np.argwhere(~np.all(img == ref, axis=-1))[:5]
