"""xraytracer_amd — MI355X-native backend for xRayTracer's path-tracing hot path.

The product is libxrt_hip.so (C ABI: include/xrt.h; C++ API: include/xrt/*.h).  This
package is its Python binding: scene builders for the benchmark configurations and a
HipRenderer mirror.  See DESIGN.md.
"""
from . import abi  # noqa: F401

__all__ = ["abi", "scenes", "renderer"]
