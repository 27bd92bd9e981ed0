"""The C-ABI library loads and exports every symbol include/xrt.h declares (no GPU needed)."""
import ctypes as C
import os
import re

from xraytracer_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "xrt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(xrt_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    lib = C.CDLL(abi.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(declared_functions()) == set(abi.SIGNATURES)


def test_abi_version():
    assert abi.lib().xrt_abi_version() == abi.XRT_ABI_VERSION


def test_null_arguments_are_rejected_without_a_gpu():
    lib = abi.lib()
    assert lib.xrt_create(0, None) == -1
    assert lib.xrt_render(None, None, None, None) != 0
    assert lib.xrt_upload_scene(None, None) == -1
    assert lib.xrt_last_error(None)
    assert lib.xrt_create_multi(None, 0, None) == -1
    assert lib.xrt_device_count(None) == 0
