"""Scene::intersect / Scene::occluded (Src/scene.cpp:190-211) as GPU queries (xrt_query) —
the render's own trace kernels (small-scene LDS trace, sphere scan, BVH, mixed box scenes)
answer caller rays — against the oracle's restatement of the reference, field by field and
bit for bit; and the reference's host API (Sampler, PinholeCamera::sampleRay,
Scene::sampleAreaLight, single-ray and batched Scene queries) through examples/scene_query.cpp.
"""
import os
import subprocess

import numpy as np
import pytest

import pyoracle
from xraytracer_amd import scenes
from xraytracer_amd.renderer import HipRenderer

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("hit", "object", "primitive", "t", "t1", "position", "ng", "ns", "dpdu", "dpdv", "barycentric")


def record(h):
    out = []
    for f in FIELDS:
        v = getattr(h, f)
        vals = list(v) if hasattr(v, "__len__") else [v]
        out += [np.float32(x).view(np.uint32) if isinstance(x, float) else np.uint32(np.int32(x).view(np.uint32))
                for x in vals]
    return np.array(out, np.uint32)


def random_rays(rng, n, lo, hi, outside=None):
    o = rng.uniform(lo, hi, (n, 3))
    if outside is not None:
        o[::5] = outside
    d = rng.normal(size=(n, 3))
    d[::3] /= np.linalg.norm(d[::3], axis=1, keepdims=True)
    d[7::11, 1] = 0.0   # axis-parallel components
    return np.concatenate([o, d], axis=1).astype(np.float32)


SCENES = {
    "cornell": (lambda: scenes.cornell(32, 32), (0.0, 0.0, 0.0), (556.0, 548.0, 559.0), (278.0, 274.4, -750.0)),
    "spheres": (lambda: scenes.spheres(32, 18), (-20.0, -1.0, -27.0), (20.0, 11.0, 1.0), (0.0, 4.0, 8.0)),
    "spheremesh": (lambda: scenes.cornell_spheremesh(32, 18, n_theta=40, n_phi=40), (0.0, 0.0, 0.0),
                   (556.0, 548.0, 559.0), (278.0, 274.4, -750.0)),
    "smoke": (lambda: scenes.smoke(32, 24, n=32), (-10.0, -10.0, -10.0), (42.0, 110.0, 42.0), (15.5, 15.5, 85.7)),
}


@pytest.mark.parametrize("name", sorted(SCENES))
def test_query_matches_oracle(name):
    make, lo, hi, outside = SCENES[name]
    s = make()
    rng = np.random.default_rng(hash(name) % 1000)
    rays = random_rays(rng, 4000, lo, hi, outside)
    tmax = rng.uniform(0.0, 800.0, len(rays)).astype(np.float32)
    r = HipRenderer(1, device=0)
    got = r.query(s, rays)
    ref = pyoracle.query(s, rays)
    assert sum(h.hit for h in ref) > 500
    for k in range(len(rays)):
        assert np.array_equal(record(got[k]), record(ref[k])), (name, k, rays[k])
    got = r.query(s, rays, tmax=tmax, occluded=True)
    ref = pyoracle.query(s, rays, tmax=tmax, occluded=True)
    assert [h.hit for h in got] == [h.hit for h in ref]
    assert sum(h.hit for h in ref) > 0
    r.close()


def test_cpp_host_query_api(tmp_path):
    """Sampler, PinholeCamera::sampleRay, Scene::intersect/occluded (single and batched) and
    Scene::sampleAreaLight through the C++ headers, on the Cornell box."""
    rng = np.random.default_rng(3)
    n = 500
    rays = random_rays(rng, n, (0.0, 0.0, 0.0), (556.0, 548.0, 559.0), (278.0, 274.4, -750.0))
    tmax = rng.uniform(0.0, 800.0, n).astype(np.float32)
    raw = tmp_path / "rays.raw"
    np.concatenate([rays, tmax[:, None]], axis=1).astype(np.float32).tofile(raw)
    out = tmp_path / "out.raw"
    subprocess.check_call([os.path.join(ROOT, "examples", "bin", "scene_query"),
                           os.path.join(ROOT, "xraytracer_amd", "data") + "/", str(raw), str(n), str(out)])
    got = np.fromfile(out, np.float32)
    s = scenes.cornell(800, 600)
    ref = pyoracle.query(s, rays)
    occ = pyoracle.query(s, rays, tmax=tmax, occluded=True)
    rec = 21
    single = got[:n * rec].reshape(n, rec)
    batch = got[n * rec:2 * n * rec].reshape(n, rec)
    for k in range(n):
        h = ref[k]
        exp = np.array([float(h.hit), float(h.object), h.t, h.t1, *h.position, *h.ng, *h.ns, *h.dpdu, *h.dpdv,
                        *(h.barycentric if h.primitive >= 0 else (0.0, 0.0))], np.float32)
        assert np.array_equal(single[k].view(np.uint32), exp.view(np.uint32)), k
        assert np.array_equal(batch[k].view(np.uint32), exp.view(np.uint32)), k
    p = 2 * n * rec
    assert np.array_equal(got[p:p + n], [float(h.hit) for h in occ])
    assert np.array_equal(got[p + n:p + 2 * n], [float(h.hit) for h in occ])
    p += 2 * n
    d = pyoracle.draws(12345, 128).reshape(-1, 2)
    assert np.array_equal(got[p:p + 128].reshape(-1, 2), d[:, ::-1])   # getNext2D = (2nd, 1st) under GCC
    p += 128
    d0 = pyoracle.draws(0, 64 + 32 + 64)
    assert np.array_equal(got[p:p + 64], d0[:64])
    p += 64
    cam = pyoracle.camera(scenes.pinhole(scenes.CORNELL_C2W, 60.0, 800, 600))
    import ctypes as C
    for k in range(16):
        o = np.zeros(3, np.float32)
        dd = np.zeros(3, np.float32)
        pyoracle.lib().orc_kat_camera(C.byref(cam), C.c_float(d0[64 + 2 * k]), C.c_float(d0[65 + 2 * k]),
                                      pyoracle.fp(o), pyoracle.fp(dd))
        assert np.array_equal(got[p:p + 7], np.concatenate([o, dd, [1.0]]).astype(np.float32)), k
        p += 7
    assert np.all(got[p:p + 128].reshape(-1, 2) == [1.0, 1.0])


def test_occluded_query_lightless_two_level():
    """an occluded query on a two-level scene (a big mesh among small
    objects) with no area light queues every deep ray as a shadow ray of light 0; the deep
    queues must hold them (part_cap per light of the trace kernel, at least one).  More rays
    than several partitions' worth, bit-exact hit flags against the oracle."""
    from xraytracer_amd import scenes as S
    s = S.SceneBundle()
    s.load_obj(S.CORNELL_OBJ)
    s.add_sphere_mesh("sphere_mesh", (150.0, 420.0, 400.0), 90.0, 40, 40, (0.58, 0.58, 0.58))
    s.flatten()
    s.camera = S.pinhole(S.CORNELL_C2W, 60.0, 32, 18)
    assert s.desc.n_lights == 0
    rng = np.random.default_rng(11)
    n = 20000
    o = rng.uniform((60.0, 330.0, 310.0), (240.0, 510.0, 490.0), (n, 3))   # around the sphere mesh
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d], axis=1).astype(np.float32)
    tmax = rng.uniform(0.0, 600.0, n).astype(np.float32)
    r = HipRenderer(1, device=0)
    got = r.query(s, rays, tmax=tmax, occluded=True)
    ref = pyoracle.query(s, rays, tmax=tmax, occluded=True)
    hits = [h.hit for h in ref]
    assert [h.hit for h in got] == hits
    assert 1000 < sum(hits) < n - 1000
    # and the closest-hit query of the same rays
    got = r.query(s, rays)
    ref = pyoracle.query(s, rays)
    for k in range(0, n, 7):
        assert np.array_equal(record(got[k]), record(ref[k])), k
    r.close()
