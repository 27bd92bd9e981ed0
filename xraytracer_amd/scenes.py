"""Scene builders for the benchmark configurations (BASELINE.json ``configs``).

Every scene is built through the C++ host layer (``Scene`` of include/xrt/scene.h, via the
``xrt_hscene_*`` C facade), i.e. with the same object/light constructors, tinyobjloader-v2
OBJ semantics and ``std::unordered_map`` object order that a C++ user of the reference API
gets.  ``SceneBundle.desc`` is the flattened C-ABI description; the oracle and the GPU
path both consume exactly that.

  C1  Cornell box, 256x256, 16 spp, GIIntegrator(3)          (Src/examples/cornellbox.cpp)
  C2  Cornell box, 800x600, 1024 spp, GIIntegrator(3)
  C3  1000 spheres + sphere light, 1280x720, 512 spp, DirectIntegrator
  C4  Cornell + 51,200-triangle SphereMesh, 1920x1080, 2048 spp, GIIntegrator(3)
  C5  synthetic 128^3 smoke + quad light, 800x600, 512 spp, VolumePathTracing(10)
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import math
import os

import numpy as np

from . import abi

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
CORNELL_OBJ = os.path.join(DATA, "cornell_box.obj")


@dataclasses.dataclass
class Camera:
    """PinholeCamera(aspect, c2w, FOV) (Src/camera.h:37-47)."""
    c2w: np.ndarray          # (16,) float32, row-major, row-vector convention
    scale: float             # tan(0.5*deg2rad(FOV)), computed by the C++ host layer
    aspect: float            # float(width) / height


def pinhole(c2w_rows, fov_deg: float, width: int, height: int) -> Camera:
    c2w = np.ascontiguousarray(np.asarray(c2w_rows, dtype=np.float32).reshape(16))
    scale = float(abi.lib().xrt_pinhole_scale(C.c_float(fov_deg)))
    aspect = float(np.float32(np.float32(width) / np.float32(height)))
    return Camera(c2w, scale, aspect)


@dataclasses.dataclass
class Medium:
    """HeterogeneousMedium over a dense grid (include/xrt/medium.h, grid.h)."""
    density: np.ndarray      # (nz, ny, nx) float32
    origin: tuple
    voxel_size: float
    g: float
    absorption: tuple
    scattering: tuple
    multiplier: float = 1.0
    sparse: bool = False     # upload as 8^3 leaf bricks (xrt_set_medium_bricks), same image

    def bricks(self):
        """(table [nbz, nby, nbx] int32 brick index or -1, bricks [n, 8, 8, 8] float32): the
        grid cut into XRT_BRICK^3 leaves, all-zero leaves dropped (SparseGrid::fromDense)."""
        B = abi.XRT_BRICK
        nz, ny, nx = self.density.shape
        nb = [(n + B - 1) // B for n in (nz, ny, nx)]
        pad = np.zeros([n * B for n in nb], np.float32)
        pad[:nz, :ny, :nx] = self.density
        leaves = pad.reshape(nb[0], B, nb[1], B, nb[2], B).transpose(0, 2, 4, 1, 3, 5).reshape(-1, B, B, B)
        keep = np.any(leaves != 0.0, axis=(1, 2, 3))
        table = np.full(len(leaves), -1, np.int32)
        table[keep] = np.arange(int(keep.sum()), dtype=np.int32)
        return table.reshape(nb), np.ascontiguousarray(leaves[keep])

    def bounds(self):
        nz, ny, nx = self.density.shape
        o = np.asarray(self.origin, dtype=np.float64)
        n = np.array([nx - 1, ny - 1, nz - 1], dtype=np.float64)
        return (o.astype(np.float32), (n * self.voxel_size + o).astype(np.float32))

    def desc(self) -> abi.XrtMediumDesc:
        d = abi.XrtMediumDesc()
        nz, ny, nx = self.density.shape
        self._dens = np.ascontiguousarray(self.density, dtype=np.float32)
        d.nx, d.ny, d.nz = nx, ny, nz
        d.density = abi.fptr(self._dens)
        lo, hi = self.bounds()
        for i in range(3):
            d.origin[i] = self.origin[i]
            d.bbox_min[i] = lo[i]
            d.bbox_max[i] = hi[i]
            d.absorption[i] = self.absorption[i]
            d.scattering[i] = self.scattering[i]
        d.voxel_size = self.voxel_size
        d.max_density = float(self._dens.max())
        d.g = self.g
        d.density_multiplier = self.multiplier
        return d


@dataclasses.dataclass
class HomogeneousMedium:
    """HomogeneousMedium{MIS, Achromatic, NoMIS}(g, a, s, box) (Src/medium.h:122-277).
    kind: "mis" | "achromatic" | "nomis"; Achromatic takes scalar a, s (pass (a, a, a))."""
    kind: str
    g: float
    absorption: tuple
    scattering: tuple
    box_min: tuple
    box_max: tuple

    KINDS = {"mis": abi.XRT_MEDIUM_HOMOGENEOUS_MIS, "achromatic": abi.XRT_MEDIUM_HOMOGENEOUS_ACHROMATIC,
             "nomis": abi.XRT_MEDIUM_HOMOGENEOUS_NOMIS}

    def bounds(self):
        return (np.asarray(self.box_min, np.float32), np.asarray(self.box_max, np.float32))

    def desc(self) -> abi.XrtMediumDesc:
        d = abi.XrtMediumDesc()
        lo, hi = self.bounds()
        for i in range(3):
            d.bbox_min[i] = lo[i]
            d.bbox_max[i] = hi[i]
            d.absorption[i] = self.absorption[i]
            d.scattering[i] = self.scattering[i]
        d.g = self.g
        d.kind = self.KINDS[self.kind]
        return d


class SceneBundle:
    """A host Scene (C++), its flattened description, camera and optional medium."""

    def __init__(self):
        self._lib = abi.lib()
        self.h = self._lib.xrt_hscene_create()
        if not self.h:
            raise abi.XrtError("xrt_hscene_create failed")
        self.desc = abi.XrtSceneDesc()
        self.camera: Camera | None = None
        self.medium: Medium | None = None
        self.integrator = "gi"
        self.max_depth = 3

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h:
            self._lib.xrt_hscene_destroy(h)

    def _check(self, rc, what):
        if rc != 0:
            err = self._lib.xrt_hscene_last_error(self.h).decode()
            raise abi.XrtError(f"{what} failed ({rc}): {err}")

    # --- Scene API mirror -----------------------------------------------------------
    def load_obj(self, path):
        self._check(self._lib.xrt_hscene_load_obj(self.h, path.encode()), f"loadObj({path})")

    def add_mesh(self, name, tri_v, albedo, tri_n=None):
        tv = np.ascontiguousarray(np.asarray(tri_v, dtype=np.float32).reshape(-1, 9))
        tn = None if tri_n is None else np.ascontiguousarray(np.asarray(tri_n, dtype=np.float32).reshape(-1, 9))
        self._check(self._lib.xrt_hscene_add_mesh(self.h, name.encode(), abi.fptr(tv),
                                                  None if tn is None else abi.fptr(tn), len(tv),
                                                  abi.fptr(abi.f3(albedo))), f"add_mesh({name})")

    def add_sphere_mesh(self, name, center, radius, n_theta, n_phi, albedo):
        self._check(self._lib.xrt_hscene_add_sphere_mesh(self.h, name.encode(), abi.fptr(abi.f3(center)),
                                                         C.c_float(radius), n_theta, n_phi,
                                                         abi.fptr(abi.f3(albedo))), f"SphereMesh({name})")

    def add_sphere(self, name, center, radius, albedo):
        self._check(self._lib.xrt_hscene_add_sphere(self.h, name.encode(), abi.fptr(abi.f3(center)),
                                                    C.c_float(radius), abi.fptr(abi.f3(albedo))),
                    f"Sphere({name})")

    def add_quad_light(self, name, v0, v1, v2, Le):
        self._check(self._lib.xrt_hscene_add_quad_light(self.h, name.encode(), abi.fptr(abi.f3(v0)),
                                                        abi.fptr(abi.f3(v1)), abi.fptr(abi.f3(v2)),
                                                        abi.fptr(abi.f3(Le))), f"QuadLight({name})")

    def add_triangle_light(self, name, v0, v1, v2, Le):
        self._check(self._lib.xrt_hscene_add_triangle_light(self.h, name.encode(), abi.fptr(abi.f3(v0)),
                                                            abi.fptr(abi.f3(v1)), abi.fptr(abi.f3(v2)),
                                                            abi.fptr(abi.f3(Le))), f"TriangleLight({name})")

    def add_sphere_light(self, name, center, radius, Le, area=False):
        """SphereLight; area=True: the reference's AREA_SAMPLING build (Src/light.h:131-135)"""
        fn = self._lib.xrt_hscene_add_sphere_light_area if area else self._lib.xrt_hscene_add_sphere_light
        self._check(fn(self.h, name.encode(), abi.fptr(abi.f3(center)), C.c_float(radius), abi.fptr(abi.f3(Le))),
                    f"SphereLight({name})")

    def add_medium(self, name, medium: Medium):
        lo, hi = medium.bounds()
        self.medium = medium
        self._check(self._lib.xrt_hscene_add_medium_box(self.h, name.encode(), abi.fptr(abi.f3(lo)),
                                                        abi.fptr(abi.f3(hi))), f"medium box({name})")

    def flatten(self):
        self._check(self._lib.xrt_hscene_flatten(self.h, C.byref(self.desc)), "flatten")
        return self.desc

    def object_names(self):
        out, i = [], 0
        while True:
            n = self._lib.xrt_hscene_object_name(self.h, i)
            if n is None:
                return out
            out.append(n.decode())
            i += 1

    def triangles(self):
        d = self.desc
        if d.n_tris == 0:
            return np.zeros((0, 3, 3), np.float32)
        return np.ctypeslib.as_array(d.tri_v, shape=(d.n_tris * 9,)).reshape(-1, 3, 3).copy()


# ------------------------------------------------------------------ configs ----
CONFIGS = {
    "C1": dict(scene="cornell", width=256, height=256, spp=16, integrator="gi", max_depth=3),
    "C2": dict(scene="cornell", width=800, height=600, spp=1024, integrator="gi", max_depth=3),
    "C3": dict(scene="spheres", width=1280, height=720, spp=512, integrator="direct", max_depth=1),
    "C4": dict(scene="cornell_spheremesh", width=1920, height=1080, spp=2048, integrator="gi", max_depth=3),
    "C5": dict(scene="smoke", width=800, height=600, spp=512, integrator="vpt", max_depth=10),
}

CORNELL_C2W = (-1.0, 0, 0, 0, 0, 1.0, 0, 0, 0, 0, -1.0, 0, 278, 274.4, -750.0, 1)   # cornellbox.cpp:29-34


def cornell(width, height, obj_path=CORNELL_OBJ) -> SceneBundle:
    """Src/examples/cornellbox.cpp:19-47: loadObj + QuadLight(Le = 25), FOV 60."""
    s = SceneBundle()
    s.load_obj(obj_path)
    s.add_quad_light("QuadLight", (343.0, 548.0, 227.0), (343.0, 548.0, 332.0), (213.0, 548.0, 227.0),
                     (25.0, 25.0, 25.0))
    s.flatten()
    s.camera = pinhole(CORNELL_C2W, 60.0, width, height)
    return s


def cornell_spheremesh(width, height, n_theta=160, n_phi=160) -> SceneBundle:
    """C4: Cornell + SphereMesh(c=(150,420,400), r=90, 160x160, Lambert(0.58))."""
    s = SceneBundle()
    s.load_obj(CORNELL_OBJ)
    s.add_quad_light("QuadLight", (343.0, 548.0, 227.0), (343.0, 548.0, 332.0), (213.0, 548.0, 227.0),
                     (25.0, 25.0, 25.0))
    s.add_sphere_mesh("sphere_mesh", (150.0, 420.0, 400.0), 90.0, n_theta, n_phi, (0.58, 0.58, 0.58))
    s.flatten()
    s.camera = pinhole(CORNELL_C2W, 60.0, width, height)
    return s


def spheres(width, height, nx=40, nz=25) -> SceneBundle:
    """C3: 1000 Lambert(0.58) spheres r=0.4 on a 40x25 xz grid + SphereLight."""
    s = SceneBundle()
    k = 0
    for iz in range(nz):
        for ix in range(nx):
            x = -19.5 + ix
            z = -2.0 - iz
            s.add_sphere(f"sphere_{k:04d}", (x, 0.0, z), 0.4, (0.58, 0.58, 0.58))
            k += 1
    s.add_sphere_light("SphereLight", (0.0, 10.0, -12.0), 2.0, (30.0, 30.0, 30.0))
    s.flatten()
    s.camera = pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 4, 8, 1), 60.0, width, height)
    s.integrator, s.max_depth = "direct", 1
    return s


def smoke_grid(n=128, seed=7) -> np.ndarray:
    """Deterministic synthetic density in [0,1]: Gaussian blobs + fixed-seed value noise."""
    rng = np.random.default_rng(seed)
    ax = (np.arange(n, dtype=np.float64) + 0.5) / n
    z, y, x = np.meshgrid(ax, ax, ax, indexing="ij")
    d = np.zeros((n, n, n), np.float64)
    for _ in range(12):
        c = rng.uniform(0.25, 0.75, 3)
        r = rng.uniform(0.06, 0.16)
        d += np.exp(-(((x - c[0]) ** 2 + (y - c[1]) ** 2 + (z - c[2]) ** 2) / (2 * r * r)))
    coarse = rng.random((9, 9, 9))
    idx = np.clip((ax * 8).astype(int), 0, 7)
    fr = ax * 8 - idx
    def lerp_axis(a, axis):
        a0 = np.take(a, idx, axis=axis)
        a1 = np.take(a, idx + 1, axis=axis)
        sh = [1, 1, 1]
        sh[axis] = n
        w = fr.reshape(sh)
        return a0 * (1 - w) + a1 * w
    noise = lerp_axis(lerp_axis(lerp_axis(coarse, 0), 1), 2)
    d = d * (0.6 + 0.4 * noise)
    d = d / d.max()
    d[d < 0.02] = 0.0
    return d.astype(np.float32)


def smoke(width, height, n=128) -> SceneBundle:
    """C5: synthetic n^3 grid, voxel 1, g=0, sigma_a 0.01, sigma_s 0.05
    (Src/examples/nee.cpp:54) + QuadLight above the box; VolumePathTracing(10)."""
    s = SceneBundle()
    med = Medium(smoke_grid(n), (0.0, 0.0, 0.0), 1.0, 0.0, (0.01, 0.01, 0.01), (0.05, 0.05, 0.05))
    c = (n - 1) / 2.0
    s.add_quad_light("QuadLight", (c + 40, n + 60.0, c + 40), (c - 40, n + 60.0, c + 40), (c + 40, n + 60.0, c - 40),
                     (20.0, 20.0, 20.0))
    s.add_medium("medium", med)
    s.flatten()
    s.camera = pinhole((1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, c, c, c + 2.2 * n, 1), 45.0, width, height)
    s.integrator, s.max_depth = "vpt", 10
    return s


def build(config: str, width=None, height=None) -> SceneBundle:
    cfg = CONFIGS[config]
    w = width or cfg["width"]
    h = height or cfg["height"]
    kind = cfg["scene"]
    if kind == "cornell":
        s = cornell(w, h)
    elif kind == "cornell_spheremesh":
        s = cornell_spheremesh(w, h)
    elif kind == "spheres":
        s = spheres(w, h)
    else:
        s = smoke(w, h)
    s.integrator, s.max_depth = cfg["integrator"], cfg["max_depth"]
    return s
