"""ctypes binding of the C ABI in include/xrt.h (libxrt_hip.so).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C xraytracer_amd/csrc``)
and loaded from ``xraytracer_amd/libxrt_hip.so``.  There is no fallback: if the shared
library is missing, importing the renderer raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libxrt_hip.so")
if os.environ.get("XRT_LIB"):   # experiment builds (csrc/Makefile `variant` -> variants/), same ABI
    _v = os.path.join(HERE, "variants", os.environ["XRT_LIB"])
    LIB_PATH = _v if os.path.exists(_v) else os.path.join(HERE, os.environ["XRT_LIB"])

XRT_ABI_VERSION = 12  # include/xrt.h XRT_ABI_VERSION
XRT_OK = 0
XRT_OBJ_MESH, XRT_OBJ_SPHERE, XRT_OBJ_BOX = 0, 1, 2
XRT_LIGHT_QUAD, XRT_LIGHT_TRIANGLE, XRT_LIGHT_SPHERE, XRT_LIGHT_SPHERE_AREA = 0, 1, 2, 3
XRT_MAT_NONE, XRT_MAT_LAMBERT = 0, 1
XRT_INTEGRATOR_GI, XRT_INTEGRATOR_DIRECT, XRT_INTEGRATOR_VPT = 0, 1, 2
XRT_INTEGRATOR_INDIRECT, XRT_INTEGRATOR_NORMAL, XRT_INTEGRATOR_VPT_NEE = 3, 4, 5
XRT_MEDIUM_HETEROGENEOUS, XRT_MEDIUM_HOMOGENEOUS_MIS, XRT_MEDIUM_HOMOGENEOUS_ACHROMATIC, XRT_MEDIUM_HOMOGENEOUS_NOMIS = 0, 1, 2, 3
XRT_FLAG_TIMING, XRT_FLAG_WAVEFRONT, XRT_FLAG_NO_MERGED, XRT_FLAG_NO_GROUP, XRT_FLAG_ACCUMULATE = 1, 2, 4, 8, 16
XRT_FLAG_DEEP_SINGLE, XRT_FLAG_DEEP_QUAD, XRT_FLAG_NO_PIXEL = 32, 64, 128
XRT_FLAG_NO_SPEC = 256
XRT_SCHED_WAVEFRONT, XRT_SCHED_STEP, XRT_SCHED_STEP_TRI, XRT_SCHED_STEP_MERGED, XRT_SCHED_STEP_BVH = 0, 1, 2, 3, 4
XRT_SCHED_PIXEL = 5
SCHEDULE_NAMES = ("wavefront", "step", "step_tri", "step_merged", "step_bvh", "pixel")
XRT_K_SEED, XRT_K_TRACE, XRT_K_SHADE, XRT_K_FINISH, XRT_K_STEP, XRT_K_REFILL, XRT_K_DEEP, XRT_K_COUNT = \
    0, 1, 2, 3, 4, 5, 6, 7
LAYOUTS = (64, 32, 16, 8, 4)   # xrt_stats.layout_launches: slots per wave
KERNEL_NAMES = ("seed", "trace", "shade", "finish", "step", "refill", "trace_deep4")

INTEGRATORS = {"gi": XRT_INTEGRATOR_GI, "direct": XRT_INTEGRATOR_DIRECT, "vpt": XRT_INTEGRATOR_VPT,
               "indirect": XRT_INTEGRATOR_INDIRECT, "normal": XRT_INTEGRATOR_NORMAL, "vpt_nee": XRT_INTEGRATOR_VPT_NEE}

f32p = C.POINTER(C.c_float)
u32p = C.POINTER(C.c_uint32)


class XrtObject(C.Structure):
    _fields_ = [("kind", C.c_int32), ("first", C.c_int32), ("count", C.c_int32),
                ("material", C.c_int32), ("albedo", C.c_float * 3), ("light", C.c_int32),
                ("medium", C.c_int32)]


class XrtLight(C.Structure):
    _fields_ = [("kind", C.c_int32), ("v0", C.c_float * 3), ("v1", C.c_float * 3),
                ("v2", C.c_float * 3), ("center", C.c_float * 3), ("radius", C.c_float),
                ("Le", C.c_float * 3)]


class XrtSceneDesc(C.Structure):
    _fields_ = [("n_objects", C.c_uint32), ("objects", C.POINTER(XrtObject)),
                ("n_tris", C.c_uint32), ("tri_v", f32p), ("tri_n", f32p),
                ("n_spheres", C.c_uint32), ("spheres", f32p),
                ("n_boxes", C.c_uint32), ("boxes", f32p),
                ("n_lights", C.c_uint32), ("lights", C.POINTER(XrtLight))]


class XrtMediumDesc(C.Structure):
    _fields_ = [("nx", C.c_uint32), ("ny", C.c_uint32), ("nz", C.c_uint32), ("density", f32p),
                ("origin", C.c_float * 3), ("voxel_size", C.c_float),
                ("bbox_min", C.c_float * 3), ("bbox_max", C.c_float * 3),
                ("max_density", C.c_float), ("g", C.c_float),
                ("absorption", C.c_float * 3), ("scattering", C.c_float * 3),
                ("density_multiplier", C.c_float), ("kind", C.c_int32)]


class XrtBrickGrid(C.Structure):
    _fields_ = [("nbx", C.c_uint32), ("nby", C.c_uint32), ("nbz", C.c_uint32), ("table", C.POINTER(C.c_int32)),
                ("n_bricks", C.c_uint32), ("bricks", f32p)]


XRT_BRICK = 8


class XrtRenderParams(C.Structure):
    _fields_ = [("integrator", C.c_int32), ("max_depth", C.c_uint32), ("width", C.c_uint32),
                ("height", C.c_uint32), ("spp", C.c_uint32), ("shard_index", C.c_uint32),
                ("shard_count", C.c_uint32), ("flags", C.c_uint32), ("slots_per_wave", C.c_uint32),
                ("visits_per_launch", C.c_uint32)]


class XrtStats(C.Structure):
    _fields_ = [("wall_ms", C.c_double), ("kernel_ms", C.c_double * XRT_K_COUNT),
                ("launches", C.c_uint64 * XRT_K_COUNT), ("samples", C.c_uint64),
                ("segments", C.c_uint64), ("shadow_rays", C.c_uint64), ("draws", C.c_uint64),
                ("rejected", C.c_uint64), ("iterations", C.c_uint64), ("path_slots", C.c_uint64),
                ("schedule", C.c_uint64), ("stalled", C.c_uint64), ("slots_per_wave", C.c_uint32),
                ("group_lanes", C.c_uint32), ("partitions", C.c_uint32), ("visits_per_launch", C.c_uint32),
                ("rng_twists", C.c_uint64), ("layout_launches", C.c_uint64 * 5),
                ("pix_windows", C.c_uint64), ("pix_stride4", C.c_uint64), ("pix_frustum", C.c_uint64),
                ("pix_frustum_overflow", C.c_uint64), ("pix_shadow_list", C.c_uint64),
                ("pix_shadow_overflow", C.c_uint64), ("pix_flushes", C.c_uint64), ("spec_launches", C.c_uint64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("kernel_ms", "launches", "layout_launches")}
        d["layout_launches"] = dict(zip(LAYOUTS, (int(x) for x in self.layout_launches)))
        d["kernel_ms"] = {n: self.kernel_ms[i] for i, n in enumerate(KERNEL_NAMES)}
        d["launches"] = {n: int(self.launches[i]) for i, n in enumerate(KERNEL_NAMES)}
        return d


class XrtHit(C.Structure):
    _fields_ = [("hit", C.c_int32), ("object", C.c_int32), ("primitive", C.c_int32), ("t", C.c_float),
                ("t1", C.c_float), ("position", C.c_float * 3), ("ng", C.c_float * 3), ("ns", C.c_float * 3),
                ("dpdu", C.c_float * 3), ("dpdv", C.c_float * 3), ("barycentric", C.c_float * 2)]


XRT_QUERY_INTERSECT, XRT_QUERY_OCCLUDED = 0, 1


# Every symbol include/xrt.h declares, with its ctypes signature.
SIGNATURES = {
    "xrt_abi_version": (C.c_int, []),
    "xrt_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "xrt_create_multi": (C.c_int, [C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_void_p)]),
    "xrt_device_count": (C.c_int, [C.c_void_p]),
    "xrt_destroy": (None, [C.c_void_p]),
    "xrt_last_error": (C.c_char_p, [C.c_void_p]),
    "xrt_upload_scene": (C.c_int, [C.c_void_p, C.POINTER(XrtSceneDesc)]),
    "xrt_set_camera": (C.c_int, [C.c_void_p, f32p, C.c_float, C.c_float]),
    "xrt_set_medium": (C.c_int, [C.c_void_p, C.POINTER(XrtMediumDesc)]),
    "xrt_set_medium_bricks": (C.c_int, [C.c_void_p, C.POINTER(XrtMediumDesc), C.POINTER(XrtBrickGrid)]),
    "xrt_render": (C.c_int, [C.c_void_p, C.POINTER(XrtRenderParams), f32p, C.POINTER(XrtStats)]),
    "xrt_render_device": (C.c_int, [C.c_void_p, C.POINTER(XrtRenderParams), C.c_void_p, C.POINTER(XrtStats)]),
    "xrt_render_device_after": (C.c_int, [C.c_void_p, C.POINTER(XrtRenderParams), C.c_void_p, C.c_void_p,
                                          C.POINTER(XrtStats)]),
    "xrt_hscene_create": (C.c_void_p, []),
    "xrt_hscene_destroy": (None, [C.c_void_p]),
    "xrt_hscene_last_error": (C.c_char_p, [C.c_void_p]),
    "xrt_hscene_load_obj": (C.c_int, [C.c_void_p, C.c_char_p]),
    "xrt_hscene_add_mesh": (C.c_int, [C.c_void_p, C.c_char_p, f32p, f32p, C.c_uint32, f32p]),
    "xrt_hscene_add_sphere_mesh": (C.c_int, [C.c_void_p, C.c_char_p, f32p, C.c_float, C.c_int, C.c_int, f32p]),
    "xrt_hscene_add_sphere": (C.c_int, [C.c_void_p, C.c_char_p, f32p, C.c_float, f32p]),
    "xrt_hscene_add_quad_light": (C.c_int, [C.c_void_p, C.c_char_p, f32p, f32p, f32p, f32p]),
    "xrt_hscene_add_triangle_light": (C.c_int, [C.c_void_p, C.c_char_p, f32p, f32p, f32p, f32p]),
    "xrt_hscene_add_sphere_light": (C.c_int, [C.c_void_p, C.c_char_p, f32p, C.c_float, f32p]),
    "xrt_hscene_add_sphere_light_area": (C.c_int, [C.c_void_p, C.c_char_p, f32p, C.c_float, f32p]),
    "xrt_hscene_add_medium_box": (C.c_int, [C.c_void_p, C.c_char_p, f32p, f32p]),
    "xrt_hscene_flatten": (C.c_int, [C.c_void_p, C.POINTER(XrtSceneDesc)]),
    "xrt_hscene_object_name": (C.c_char_p, [C.c_void_p, C.c_uint32]),
    "xrt_pinhole_scale": (C.c_float, [C.c_float]),
    "xrt_test_rng": (C.c_int, [C.c_void_p, u32p, C.c_uint32, C.c_uint32, C.c_uint32, f32p]),
    "xrt_test_trig": (C.c_int, [C.c_void_p, f32p, C.c_uint32, f32p]),
    "xrt_test_trig_draw_domain": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, f32p, f32p, f32p]),
    "xrt_test_logexp": (C.c_int, [C.c_void_p, f32p, C.c_uint32, f32p]),
    "xrt_test_powf": (C.c_int, [C.c_void_p, f32p, C.c_uint32, C.c_float, f32p]),
    "xrt_query": (C.c_int, [C.c_void_p, C.c_uint32, f32p, f32p, C.c_int32, C.POINTER(XrtHit)]),
    "xrt_tonemap": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_float, C.POINTER(C.c_uint8)]),
    "xrt_test_fastdiv": (C.c_int, [C.c_void_p, C.c_uint32, C.c_float, C.c_float, C.POINTER(C.c_uint64), u32p]),
}

_lib = None


def lib():
    """Load libxrt_hip.so (raises if it has not been built — there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() "
                              "(the HIP path has no CPU fallback)")
        # PyTorch-ROCm wheels bundle their own HIP runtime.  Once /opt/rocm's runtime (which
        # libxrt_hip links) is loaded, torch's own fails to initialise later in the same
        # process ("No HIP GPUs are available"; measured on the MI355X box), while the other
        # order works.  Load torch first when it is installed, so callers can render into
        # torch tensors (xrt_render_device) in any import order.
        # A torch that is installed but broken (its bundled HIP libraries raise OSError /
        # RuntimeError) must not stop the C path from loading.
        try:
            import torch  # noqa: F401
        except Exception as e:  # noqa: BLE001
            if not isinstance(e, ImportError):
                import warnings
                warnings.warn(f"torch failed to import ({e!r}); loading libxrt_hip without it")
        l = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def fptr(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(f32p)


def u32ptr(a: np.ndarray):
    assert a.dtype == np.uint32 and a.flags.c_contiguous
    return a.ctypes.data_as(u32p)


def f3(v):
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32).reshape(3))


class XrtError(RuntimeError):
    pass
