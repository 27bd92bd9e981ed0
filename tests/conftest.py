import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libxrt_hip.so on the GPU)")


def _ensure_built():
    lib = os.path.join(ROOT, "xraytracer_amd", "libxrt_hip.so")
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "xraytracer_amd", "csrc")])
    if not os.path.exists(orc):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_ensure_built()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "ref_kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu():
    """A HipRenderer-independent device context for self-tests."""
    import ctypes as C
    from xraytracer_amd import abi
    ctx = C.c_void_p()
    rc = abi.lib().xrt_create(0, C.byref(ctx))
    if rc != 0:
        pytest.fail(f"xrt_create failed on the GPU box ({rc}): {abi.lib().xrt_last_error(None).decode()}")
    yield ctx
    abi.lib().xrt_destroy(ctx)
