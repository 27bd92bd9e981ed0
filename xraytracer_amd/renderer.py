"""Python mirror of HipRenderer (include/xrt/renderer.h) over the C ABI.

``HipRenderer(spp, device).render(scene)`` has the contract of the reference's
``Renderer::render(scene, Uniform, image)`` (Src/renderer.h:15, renderer.cpp:29-99): it
returns the per-pixel mean of ``spp`` samples, seeds ``j + width*i`` per pixel, and drops
NaN / Inf / negative samples.  Everything runs on the GPU through libxrt_hip.so; there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .scenes import SceneBundle


class HipRenderer:
    def __init__(self, spp: int, device: int = 0, devices=None):
        """device: one GPU; devices: a list of GPUs rendered as one (xrt_create_multi —
        row shards per GPU, frame assembled on devices[0])."""
        self.spp = int(spp)
        self._lib = abi.lib()
        ctx = C.c_void_p()
        if devices is not None:
            devs = (C.c_int * len(devices))(*[int(d) for d in devices])
            rc = self._lib.xrt_create_multi(devs, len(devices), C.byref(ctx))
            what = f"xrt_create_multi(devices={list(devices)})"
        else:
            rc = self._lib.xrt_create(int(device), C.byref(ctx))
            what = f"xrt_create(device={device})"
        if rc != 0:
            raise abi.XrtError(f"{what} failed ({rc}): {self._lib.xrt_last_error(None).decode()}")
        self.ctx = ctx
        self.stats = None
        self._uploaded = None

    def close(self):
        ctx, self.ctx = getattr(self, "ctx", None), None
        if ctx:
            self._lib.xrt_destroy(ctx)

    __del__ = close

    def _check(self, rc, what):
        if rc != 0:
            raise abi.XrtError(f"{what} failed ({rc}): {self._lib.xrt_last_error(self.ctx).decode()}")

    def upload(self, scene: SceneBundle):
        self._check(self._lib.xrt_upload_scene(self.ctx, C.byref(scene.desc)), "xrt_upload_scene")
        cam = scene.camera
        self._check(self._lib.xrt_set_camera(self.ctx, abi.fptr(cam.c2w), C.c_float(cam.scale),
                                             C.c_float(cam.aspect)), "xrt_set_camera")
        if scene.medium is not None:
            md = scene.medium.desc()
            if getattr(scene.medium, "sparse", False):
                table, bricks = scene.medium.bricks()
                self._bricks = (table, bricks)   # alive until the library has copied them
                nbz, nby, nbx = table.shape
                bg = abi.XrtBrickGrid(nbx, nby, nbz, table.ctypes.data_as(C.POINTER(C.c_int32)), len(bricks),
                                      abi.fptr(bricks.reshape(-1)))
                self._check(self._lib.xrt_set_medium_bricks(self.ctx, C.byref(md), C.byref(bg)),
                            "xrt_set_medium_bricks")
            else:
                self._check(self._lib.xrt_set_medium(self.ctx, C.byref(md)), "xrt_set_medium")
        self._uploaded = scene

    def params(self, scene, width, height, shard_index=0, shard_count=1, timing=False, integrator=None,
               max_depth=None, schedule="auto", slots_per_wave=0, visits_per_launch=0, group=True,
               accumulate=False, deep="auto", spec=True):
        """schedule: "auto" (fused k_step when the scene fits in LDS — for small triangle
        scenes with merged shadow + extension traces, for Direct / Normal pixel-parallel
        sample chains (k_pixel) — else the multi-pass wavefront), "step" (the per-slot fused
        schedule also for Direct / Normal), "wavefront" (always k_shade + k_trace) or
        "step_tri" (per-slot fused, one cooperative trace per ray kind instead of the merged
        traces).  slots_per_wave / visits_per_launch /
        group fix the merged schedule's launch geometry (0 / True = the library's choice);
        results never depend on them.  accumulate: add the samples to the output buffer's
        current contents before the divide (XRT_FLAG_ACCUMULATE, Renderer::render's contract).
        deep: the two-level trace's BVH walk, "auto", "single" (one lane per queued ray) or
        "quad" (four); results never depend on it.  spec: speculative sample starts in the merged
        schedule's 16-slot launches (GI with one light; spec=False sets XRT_FLAG_NO_SPEC); results
        never depend on it."""
        if schedule not in ("auto", "step", "wavefront", "step_tri"):
            raise ValueError(f"unknown schedule {schedule!r}")
        if deep not in ("auto", "single", "quad"):
            raise ValueError(f"unknown deep walk {deep!r}")
        p = abi.XrtRenderParams()
        p.integrator = abi.INTEGRATORS[integrator or scene.integrator]
        p.max_depth = scene.max_depth if max_depth is None else max_depth
        p.width, p.height, p.spp = width, height, self.spp
        p.shard_index, p.shard_count = shard_index, shard_count
        p.flags = ((abi.XRT_FLAG_TIMING if timing else 0) | (abi.XRT_FLAG_WAVEFRONT if schedule == "wavefront" else 0) |
                   (abi.XRT_FLAG_NO_MERGED if schedule == "step_tri" else 0) | (0 if group else abi.XRT_FLAG_NO_GROUP) |
                   (abi.XRT_FLAG_NO_PIXEL if schedule in ("step", "step_tri") else 0) |
                   (abi.XRT_FLAG_ACCUMULATE if accumulate else 0) | (0 if spec else abi.XRT_FLAG_NO_SPEC) |
                   {"auto": 0, "single": abi.XRT_FLAG_DEEP_SINGLE, "quad": abi.XRT_FLAG_DEEP_QUAD}[deep])
        p.slots_per_wave, p.visits_per_launch = slots_per_wave, visits_per_launch
        return p

    def render(self, scene: SceneBundle, width: int, height: int, initial=None, **kw) -> np.ndarray:
        """Render into a host (H, W, 3) float32 image.  initial: the Image's prior contents,
        accumulated into in place as Renderer::render does (XRT_FLAG_ACCUMULATE)."""
        if self._uploaded is not scene:
            self.upload(scene)
        p = self.params(scene, width, height, accumulate=initial is not None, **kw)
        img = np.zeros((height, width, 3), np.float32)
        if initial is not None:
            img[...] = initial
        st = abi.XrtStats()
        self._check(self._lib.xrt_render(self.ctx, C.byref(p), abi.fptr(img), C.byref(st)), "xrt_render")
        self.stats = st
        return img

    def query(self, scene: SceneBundle, rays: np.ndarray, tmax=None, occluded: bool = False):
        """Scene::intersect (or, with occluded=True, Scene::occluded(ray, tmax)) for rays
        (n, 6) = origin, direction, on the GPU with the render's trace kernels (xrt_query).
        Returns an array of abi.XrtHit."""
        if self._uploaded is not scene:
            self.upload(scene)
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        n = len(r)
        out = (abi.XrtHit * max(1, n))()
        tm = None if tmax is None else np.ascontiguousarray(np.broadcast_to(np.asarray(tmax, np.float32), (n,)))
        self._check(self._lib.xrt_query(self.ctx, n, abi.fptr(r), abi.fptr(tm) if tm is not None else None,
                                        abi.XRT_QUERY_OCCLUDED if occluded else abi.XRT_QUERY_INTERSECT, out),
                    "xrt_query")
        return out[:n]

    def tonemap(self, width: int, height: int, gamma: float, device_ptr: int = 0) -> np.ndarray:
        """Image::gammaCorrection(gamma) + writePPM's 8-bit quantisation on the GPU, of the
        last render() (device_ptr 0) or of a device float3 buffer: (H, W, 3) uint8."""
        out = np.empty((height, width, 3), np.uint8)
        self._check(self._lib.xrt_tonemap(self.ctx, C.c_void_p(device_ptr or None), width * height, C.c_float(gamma),
                                          out.ctypes.data_as(C.POINTER(C.c_uint8))), "xrt_tonemap")
        return out

    @staticmethod
    def write_ppm(path: str, rgb8: np.ndarray):
        """Image::writePPM's text format (Src/image.h:92-114): P3, width height, 255, one
        "R G B" line per pixel."""
        h, w, _ = rgb8.shape
        with open(path, "w") as f:
            f.write(f"P3\n{w} {h}\n255\n")
            f.write("".join(f"{r} {g} {b}\n" for r, g, b in rgb8.reshape(-1, 3).tolist()))

    def render_device(self, scene: SceneBundle, width: int, height: int, out_ptr: int, after_stream=None, **kw):
        """Render into a device buffer (e.g. torch tensor .data_ptr()) of H*W*3 float32.
        after_stream: a HIP stream handle (torch.cuda.current_stream().cuda_stream) whose
        queued work must finish before the buffer is overwritten; None = wait for the whole
        device.  Returns when the image is complete."""
        if self._uploaded is not scene:
            self.upload(scene)
        p = self.params(scene, width, height, **kw)
        st = abi.XrtStats()
        if after_stream is None:
            rc = self._lib.xrt_render_device(self.ctx, C.byref(p), C.c_void_p(out_ptr), C.byref(st))
        else:
            rc = self._lib.xrt_render_device_after(self.ctx, C.byref(p), C.c_void_p(out_ptr),
                                                   C.c_void_p(after_stream or None), C.byref(st))
        self._check(rc, "xrt_render_device")
        self.stats = st
        return st
